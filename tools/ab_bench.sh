#!/bin/bash
# A/B bench runs on one GPU box (repo root, via gpurun): each argument is one variant, written
# "NAME:ENV1=v1,ENV2=v2:bench args" (ENV part and args part may be empty). Every variant runs the
# bench (no CPU baseline, no secondary lines) under its own time limit; the chain stops at the
# first failure. Summary lines: gpurun_out/<TAG>_ab.txt, raw lines gpurun_out/<TAG>_<NAME>.json
# usage: tools/ab_bench.sh TAG "base::" "nolanes:GPX_BAND_LANES=0:" "q4:GPX_HW_QUEUES=4:--steps 10"
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  NAME=${v%%:*}; REST=${v#*:}; ENVS=${REST%%:*}; ARGS=${REST#*:}
  ENVARGS=()
  if [ -n "$ENVS" ]; then IFS=',' read -ra ENVARGS <<< "$ENVS"; fi
  env "${ENVARGS[@]}" timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary $ARGS \
    > gpurun_out/${TAG}_${NAME}.log 2>&1 || { echo "variant $NAME failed"; tail -20 gpurun_out/${TAG}_${NAME}.log; exit 1; }
  tail -1 gpurun_out/${TAG}_${NAME}.log > gpurun_out/${TAG}_${NAME}.json
  python3 tools/bench_summary.py "$NAME" gpurun_out/${TAG}_${NAME}.json | tee -a gpurun_out/${TAG}_ab.txt
done
