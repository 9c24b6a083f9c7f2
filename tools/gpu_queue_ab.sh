#!/bin/bash
# Same-box A/B of the process / hardware-queue layout and the deferral width with the deferred
# part on its own stream.
TAG=${1:-qab}
bash tools/ab_env.sh $TAG "GPX_HW_QUEUES=2" "GPX_HW_QUEUES=3" "GPX_HW_QUEUES=3 GPX_BENCH_PROCS=6" \
  "GPX_DEFER_Q=4" "GPX_HW_QUEUES=2"
