#!/bin/bash
# 20-step bench over band-storage slot layouts (driver stats on).
# usage: tools/bench_sweep3.sh TAG "groups:width[:hwqueues]" ...
set -e
TAG=${1:-s3}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sweep_$TAG
mkdir -p "$OUT"
export GPX_DRIVER_STATS=1
for gw in "$@"; do
  IFS=: read g w q <<< "$gw"
  export GPX_HW_QUEUES=${q:-8}
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --groups $g --width $w > "$OUT/g${g}w${w}q${GPX_HW_QUEUES}.log" 2>&1
  tail -1 "$OUT/g${g}w${w}q${GPX_HW_QUEUES}.log" > "$OUT/g${g}w${w}q${GPX_HW_QUEUES}.json"
  python3 -c "import json; d=json.load(open('$OUT/g${g}w${w}q${GPX_HW_QUEUES}.json')); s=d['driver_stats_last_call']; print('g${g}w${w}q${GPX_HW_QUEUES}', round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), round(d['band_path']['problems_per_call'],1), 'wait', round(s['device_wait'],3), 'steps', round(s['steps'],3))"
done
