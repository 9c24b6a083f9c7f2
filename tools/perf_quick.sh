#!/bin/bash
# Quick device check after a kernel change (GPU box, repo root): the band16 parity tests, the
# band sweeps' throughput ceiling at two lengthscales, then a shorter bench line.
# usage: tools/perf_quick.sh TAG [bench args]
TAG=${1:-q}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_band16_gpu.py tests/test_c2_parity_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for ell in 1.18 1.6; do
  timeout -k 10 200 python tools/band_throughput.py --b 512 --g 4 --reps 20 --ell $ell > gpurun_out/${TAG}_tp_$ell.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_tp_$ell.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tp_$ell.log
done
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary --steps 100 "$@" > gpurun_out/${TAG}_bench.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_bench.log').read().strip().splitlines()[-1]); print('fits/s', round(d['value'],1), 'evals/s', round(d['evals_per_s']), 'host_share', [round(h['host_share'],2) for h in d['host']], 'frac', round(d['roofline']['frac'],4), 'chip', round(d['roofline']['chip_frac'],4))"
