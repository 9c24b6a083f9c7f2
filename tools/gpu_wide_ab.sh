#!/bin/bash
# The inline-K GPU test, then bench lines for the deferred part's wide launch with and without
# inline K tiles (GPX_B16_INLINE_K_WIDE) and the own-stream deferral, on one box.
# usage: tools/gpu_wide_ab.sh TAG
TAG=${1:-wab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inline_k_gpu.py tests/test_deferred_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tools/ab_env.sh $TAG "GPX_B16_INLINE_K_WIDE=3" "GPX_B16_INLINE_K_WIDE=0" "GPX_B16_INLINE_K_WIDE=2" \
  "GPX_B16_INLINE_K_WIDE=0 GPX_DEFER_STREAM=1" "GPX_B16_INLINE_K_WIDE=3"
