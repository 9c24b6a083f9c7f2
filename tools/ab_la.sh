mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_band16_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for la in 0 1; do for ell in 1.18 1.6; do
  GPX_B16_LA=$la timeout -k 10 120 python tools/band_throughput.py --b 512 --g 4 --reps 20 --ell $ell > gpurun_out/ab_tp_${la}_$ell.log 2>&1 || { tail -20 gpurun_out/ab_tp_${la}_$ell.log; exit 1; }
  echo "LA=$la ell=$ell $(tail -1 gpurun_out/ab_tp_${la}_$ell.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["evals_per_s"]), round(d["b16_fwd_avg_ms"],3), round(d["b16_bwd_avg_ms"],3))')"
done; done
for la in 0 1; do for b in 1024 2048 4096; do
  GPX_B16_LA=$la timeout -k 10 120 python tools/band16_phases.py $b 1.18 > gpurun_out/ab_ph_${la}_$b.log 2>&1 || { tail -20 gpurun_out/ab_ph_${la}_$b.log; exit 1; }
done; done
cat gpurun_out/ab_ph_*.log
