#!/bin/bash
# End-of-round A/B on one box: fused sweeps and the forward-writes-K variant with the final kernels.
TAG=${1:-lab}
bash tools/ab_env.sh $TAG "GPX_B16_FUSED=0" "GPX_B16_FUSED=1" "GPX_B16_INLINE_K=1" "GPX_B16_FUSED=0" "GPX_B16_FUSED=1" \
  "GPX_B16_INLINE_K=1"
