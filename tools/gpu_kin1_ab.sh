#!/bin/bash
# The forward computing K's tiles and writing them into K's band for the backward
# (GPX_B16_INLINE_K=1) against both sweeps computing them (3, the default): the bit-identity
# test first, then the Q = 3 device ceiling and bench lines on one box.
TAG=${1:-k1ab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inline_k_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 3 1; do
  for e in 1.18 1.9; do
    GPX_B16_INLINE_K=$k timeout -k 10 180 python tools/band_throughput.py --b 512 --g 4 --reps 10 --ell $e \
      > gpurun_out/${TAG}_tp.tmp 2>&1 || { tail -5 gpurun_out/${TAG}_tp.tmp; exit 1; }
    echo "kin=$k ell=$e $(tail -1 gpurun_out/${TAG}_tp.tmp | cut -c1-120)" | tee -a gpurun_out/${TAG}_throughput.txt
  done
done
bash tools/ab_env.sh $TAG "GPX_B16_INLINE_K=3" "GPX_B16_INLINE_K=1" "GPX_B16_INLINE_K=1 GPX_B16_INLINE_K_WIDE=3" \
  "GPX_B16_INLINE_K=3"
