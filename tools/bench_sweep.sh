#!/bin/bash
# Bench configuration sweep on the GPU box (run from the repo root via gpurun): host-side
# cProfile of one step, then short bench runs over device-batch layouts, driver stats on.
# Outputs: gpurun_out/sweep_<tag>/{host_profile.txt, <variant>.json}
# usage: tools/bench_sweep.sh TAG
set -e
TAG=${1:-sweep}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sweep_$TAG
mkdir -p "$OUT"
export GPX_DRIVER_STATS=1
timeout -k 10 240 python3 tools/prof_host.py > "$OUT/host_profile.txt" 2>&1
run() {  # name, then bench args
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" > "$OUT/$name.log" 2>&1
  tail -1 "$OUT/$name.log" > "$OUT/$name.json"
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value'],1), d['ms_per_step'])"
}
run g3w576
run g4w640 --groups 4 --width 640
run g3w640wide64 --groups 3 --width 640 --wide-slots 64
GPX_HW_QUEUES=12 run g4w640q12 --groups 4 --width 640
