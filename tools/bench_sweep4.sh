#!/bin/bash
# bench over host-process / device-batch / slot layouts (GPU box, repo root)
# usage: tools/bench_sweep4.sh TAG "procs:groups:width:hwqueues" ...
TAG=${1:-s4}; shift
mkdir -p gpurun_out/sweep_$TAG
for cfg in "$@"; do
  IFS=: read p g w q <<< "$cfg"
  GPX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 60 --warmup 3 \
    --procs $p --groups $g --width $w > gpurun_out/sweep_$TAG/p${p}g${g}w${w}q${q}.log 2>&1 \
    || { tail -5 gpurun_out/sweep_$TAG/p${p}g${g}w${w}q${q}.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep_$TAG/p${p}g${g}w${w}q${q}.log').read().strip().splitlines()[-1]); print('$cfg', round(d['value'],1), 'evals/s', round(d['evals_per_s']), 'host', [round(h['host_share'],2) for h in d['host']], 'ppc', round(d['band_path']['problems_per_call'],1), 'ms/call', round(d['band_path']['ms_per_call'],2), 'b16share', round(d['roofline'].get('band16_share_of_band_evals',0),4))"
done
