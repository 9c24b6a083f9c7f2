#!/bin/bash
# Kernel A/B on one box: the GPU parity tests with the current library, then the device ceiling
# (tools/band_throughput.py, per width class and for the headline's class mix) and bench lines
# for an older library build (GPX_LIB=$OLD) against the current one.
# usage: tools/gpu_kernel_ab.sh TAG OLD_LIB
TAG=${1:-kab}
OLD=${2:-portfoliooptgp_amd/libgpx_r04k.so}
mkdir -p gpurun_out
MIX="1.18:0.88,1.6:0.052,1.9:0.06,2.3:0.008"
timeout -k 10 600 python -u -m pytest tests/test_band16_gpu.py tests/test_deferred_gpu.py tests/test_band_storage_gpu.py \
  tests/test_c2_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
for lib in "$OLD" portfoliooptgp_amd/libgpx.so; do
  for e in 1.18 1.6 1.9 mix; do
    if [ $e = mix ]; then args="--ells $MIX"; else args="--ell $e"; fi
    GPX_LIB=$lib timeout -k 10 180 python tools/band_throughput.py --b 512 --g 4 --reps 10 $args > gpurun_out/${TAG}_tp.tmp 2>&1 \
      || { echo "throughput failed: $lib $e"; tail -5 gpurun_out/${TAG}_tp.tmp; exit 1; }
    echo "$lib $e $(tail -1 gpurun_out/${TAG}_tp.tmp)" | tee -a gpurun_out/${TAG}_throughput.txt
  done
done
bash tools/ab_env.sh $TAG "GPX_LIB=$OLD GPX_DEFER_Q=-1" "GPX_DEFER_Q=-1" "GPX_LIB=$OLD GPX_DEFER_Q=3" "GPX_DEFER_Q=3" \
  "GPX_DEFER_Q=-1 GPX_B16_INLINE_K=3" "GPX_DEFER_Q=3 GPX_B16_INLINE_K=3" "GPX_DEFER_Q=3 GPX_DEFER_LANES=1"
