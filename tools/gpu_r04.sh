#!/bin/bash
# Round-4 GPU pass: the gate (tests, smoke, bench line), then A/B bench lines for switches given
# as extra args "NAME=VALUE" (each one bench run with that environment), all under time limits.
# usage: tools/gpu_r04.sh TAG [ENV=VAL ...]
TAG=${1:-r04}
shift
bash tools/gpu_check.sh "$TAG" || exit 1
for kv in "$@"; do
  env "$kv" timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary > "gpurun_out/${TAG}_bench_${kv}.log" 2>&1 \
    || { tail -20 "gpurun_out/${TAG}_bench_${kv}.log"; exit 1; }
  python tools/bench_summary.py "$kv" "gpurun_out/${TAG}_bench_${kv}.log"
done
