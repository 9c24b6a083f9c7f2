#!/bin/bash
# The deferred part's band16 classes as one wide launch (default) or per-class launches.
TAG=${1:-w2ab}
bash tools/ab_env.sh $TAG "GPX_DEFER_WIDE=1" "GPX_DEFER_WIDE=0" "GPX_DEFER_WIDE=1" "GPX_DEFER_WIDE=0"
