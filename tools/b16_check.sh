#!/bin/bash
# band16 kernel iteration on the GPU box (repo root): parity tests, throughput ceiling at two
# lengthscales, per-phase cycles at one and two waves per SIMD.
# usage: tools/b16_check.sh TAG
TAG=${1:-b16}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_band16_gpu.py tests/test_c2_parity_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for ell in 1.18 1.6; do
  timeout -k 10 120 python tools/band_throughput.py --b 512 --g 4 --reps 20 --ell $ell > gpurun_out/${TAG}_tp_$ell.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_tp_$ell.log; exit 1; }
  echo "ell=$ell $(tail -1 gpurun_out/${TAG}_tp_$ell.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["evals_per_s"]), round(d["b16_fwd_avg_ms"],3), round(d["b16_bwd_avg_ms"],3))')"
done
for b in 1024 2048; do
  timeout -k 10 120 python tools/band16_phases.py $b 1.18 > gpurun_out/${TAG}_ph_$b.log 2>&1 || { tail -20 gpurun_out/${TAG}_ph_$b.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_ph_$b.log
done
