#!/bin/bash
# Band-storage parity tests, then bench over slot counts with band storage (driver stats on).
# usage: tools/bench_sweep2.sh TAG [widths...]
set -e
TAG=${1:-s2}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sweep_$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_band_storage_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
export GPX_DRIVER_STATS=1
for w in "${@:-576 960 1344}"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --width $w > "$OUT/w$w.log" 2>&1
  tail -1 "$OUT/w$w.log" > "$OUT/w$w.json"
  python3 -c "import json; d=json.load(open('$OUT/w$w.json')); print('w$w', round(d['value'],1), round(d['ms_per_step'],2), d['roofline']['frac'], d['band_path']['problems_per_call'], d['driver_stats_last_call'])"
done
