#!/bin/bash
# The inline-K sweeps' exps four at a time (exp4) against the previous build (GPX_LIB=$OLD):
# bit-identity tests first, then the Q = 3 device ceiling and bench lines on one box.
TAG=${1:-e4ab}
OLD=${2:-portfoliooptgp_amd/libgpx_prev.so}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inline_k_gpu.py tests/test_deferred_gpu.py tests/test_band16_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for lib in "$OLD" portfoliooptgp_amd/libgpx.so; do
  for e in 1.18 1.9; do
    GPX_LIB=$lib timeout -k 10 180 python tools/band_throughput.py --b 512 --g 4 --reps 10 --ell $e > gpurun_out/${TAG}_tp.tmp 2>&1 \
      || { tail -5 gpurun_out/${TAG}_tp.tmp; exit 1; }
    echo "$lib ell=$e $(tail -1 gpurun_out/${TAG}_tp.tmp | cut -c1-110)" | tee -a gpurun_out/${TAG}_throughput.txt
  done
done
bash tools/ab_env.sh $TAG "GPX_LIB=$OLD" "GPX_LIB=portfoliooptgp_amd/libgpx.so" "GPX_LIB=$OLD" "GPX_LIB=portfoliooptgp_amd/libgpx.so"
