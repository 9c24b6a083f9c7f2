#!/bin/bash
# band16 iteration check: parity tests, throughput at Q = 3 / 4 / 5 lengthscales, a 100-step bench
T=${1:-y}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_band16_gpu.py tests/test_c2_parity_gpu.py tests/test_band_storage_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for ell in 1.18 1.6 1.9; do
  timeout -k 10 120 python tools/band_throughput.py --b 512 --g 4 --reps 20 --ell $ell > gpurun_out/${T}_tp_$ell.log 2>&1 || { tail -20 gpurun_out/${T}_tp_$ell.log; exit 1; }
  echo "ell=$ell $(tail -1 gpurun_out/${T}_tp_$ell.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["evals_per_s"]), round(d["ms_per_round"],2), round(d.get("b16_fwd_avg_ms",0),3), round(d.get("b16_bwd_avg_ms",0),3), round(d.get("band16_mean_q",0),2))')"
done
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary --steps 100 > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1]); print('fits/s', round(d['value'],1), 'evals/s', round(d['evals_per_s']), 'host_share', [round(h['host_share'],2) for h in d['host']], 'frac', round(d['roofline']['frac'],4), 'chip', round(d['roofline']['chip_frac'],4))"
timeout -k 10 120 python tools/band16_phases.py 2048 1.18 > gpurun_out/${T}_ph_2048.log 2>&1 || { tail -20 gpurun_out/${T}_ph_2048.log; exit 1; }
grep -v amdgpu gpurun_out/${T}_ph_2048.log | cut -c1-700
