#!/bin/bash
# Same-box A/B of the deferred part's stream priority (GPX_SLOW_PRIORITY: -1 lowest, 1 highest).
TAG=${1:-pab}
bash tools/ab_env.sh $TAG "GPX_SLOW_PRIORITY=0" "GPX_SLOW_PRIORITY=1" "GPX_SLOW_PRIORITY=-1" "GPX_SLOW_PRIORITY=0"
