#!/bin/bash
# Device batches per host process with the end-of-round defaults (one stream per batch).
TAG=${1:-gab}
bash tools/ab_env.sh $TAG "GPX_BENCH_GROUPS=1" "GPX_BENCH_GROUPS=2" "GPX_BENCH_GROUPS=1" "GPX_BENCH_GROUPS=2"
