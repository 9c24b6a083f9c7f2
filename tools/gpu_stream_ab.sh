#!/bin/bash
# Same-box A/B: the driver's own stream for a single device batch (default now) against the
# caller's default stream (GPX_DRIVER_CALLER_STREAM=1), each with the deferred part on the call's
# stream (default) or on a stream of its own (GPX_DEFER_STREAM=1).
TAG=${1:-sab}
bash tools/ab_env.sh $TAG "GPX_DRIVER_CALLER_STREAM=0" "GPX_DRIVER_CALLER_STREAM=1" \
  "GPX_DEFER_STREAM=1" "GPX_DEFER_STREAM=1 GPX_DRIVER_CALLER_STREAM=1" "GPX_DEFER_STREAM=1"
