#!/bin/bash
# A/B of an alternate library build (portfoliooptgp_amd/libgpx_alt.so) against the in-tree one on
# the band16 throughput tool, interleaved; usage: tools/ab_lib.sh TAG ell...
TAG=${1:-ab}; shift
mkdir -p gpurun_out
for rep in 1 2; do for lib in base alt; do for ell in "$@"; do
  if [ $lib = alt ]; then export GPX_LIB=$PWD/portfoliooptgp_amd/libgpx_alt.so; else unset GPX_LIB; fi
  timeout -k 10 120 python tools/band_throughput.py --b 512 --g 4 --reps 20 --ell $ell > gpurun_out/${TAG}_${lib}_${ell}_$rep.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_${lib}_${ell}_$rep.log; exit 1; }
  echo "$lib ell=$ell rep=$rep $(tail -1 gpurun_out/${TAG}_${lib}_${ell}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["evals_per_s"]), round(d["b16_fwd_avg_ms"],3), round(d["b16_bwd_avg_ms"],3))')"
done; done; done
