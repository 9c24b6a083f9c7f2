#!/bin/bash
# Steady state of the headline: the driver's --steps 20 against a 3x longer run, same box.
TAG=${1:-steady}
mkdir -p gpurun_out
for st in 20 60 20; do
  i=$((i + 1))
  echo "# env: --steps $st" > gpurun_out/${TAG}_$i.log
  timeout -k 10 400 python bench.py --steps $st --no-cpu-baseline --no-secondary >> gpurun_out/${TAG}_$i.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
  python tools/bench_summary.py "steps $st" gpurun_out/${TAG}_$i.log
done
