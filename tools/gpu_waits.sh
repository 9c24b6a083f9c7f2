#!/bin/bash
# Where the host threads wait (GPX_SUBMIT_STATS=1: per-batch submit / predict wait timers on
# stderr) in the default bench and with the deferred part on its own stream.
TAG=${1:-waits}
mkdir -p gpurun_out
for kv in "GPX_SUBMIT_STATS=1" "GPX_SUBMIT_STATS=1 GPX_DEFER_STREAM=1"; do
  i=$((i + 1))
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/${TAG}_$i.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
  python tools/bench_summary.py "$kv" gpurun_out/${TAG}_$i.log
  grep "gpx submit stats" gpurun_out/${TAG}_$i.log | tail -8 | cut -c1-400
done
