#!/bin/bash
# Round-6 evidence on the GPU box (repo root, via gpurun), into gpurun_out/prof_<tag>/ — round 5's
# passes (tools/profile_round5.sh: the default bench line, 8 traced single-process instances in
# the headline's layout, one instance's kernel stats, FETCH_SIZE and WRITE_SIZE passes) plus
#   5. the fp64 pass: MFMA MOPS, the fp64 VALU instruction counts, MFMA busy, GUI_ACTIVE
#      (7 counters: 6 SQ + 1 GRBM, within one pass's limits) -> tools/mfma_summary.py: per kernel
#      the fp64 work of the MFMAs AND of the VALU (exps, the 16x16 leaf's uniform chain) and the
#      fp64 datapath's busy share (gfx950: the two share one datapath, profiles/r06_ab.md)
# usage: [SKIP_BENCH=1] [SKIP_TRACE=1] tools/profile_round6.sh TAG
set -e
TAG=${1:-r06}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.log" 2>&1
  tail -1 "$OUT/bench.log" | cut -c1-200
fi
cd /tmp && export TMPDIR=/tmp
INST="--no-cpu-baseline --no-secondary --procs 1 --width 1024 --fits 768 --steps 8 --warmup 1"
if [ -z "$SKIP_TRACE" ]; then
  pids=()
  for i in 0 1 2 3 4 5 6 7; do
    timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_p$i" -o run -- \
      python3 "$ROOT/bench.py" $INST > "$OUT/trace_p$i.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p"; done
  cd "$ROOT"
  python3 tools/trace_multi.py "$OUT/trace_multi.json" "$OUT/bench.log" $(for i in 0 1 2 3 4 5 6 7; do echo "$OUT/trace_p$i"; done) \
    | head -60
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" $INST > "$OUT/stats.log" 2>&1
fi
SHORT="--no-cpu-baseline --no-secondary --procs 1 --width 1024 --fits 768 --steps 1 --warmup 1"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" $SHORT > "$OUT/fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" $SHORT > "$OUT/write.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
  SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/fp64" -o run -- python3 "$ROOT/bench.py" $SHORT > "$OUT/fp64.log" 2>&1
cd "$ROOT"
for K in band16_fwd_kernel band16_bwd_kernel band16_wide_kernel; do
  python3 tools/pmc_summary.py "$OUT/fetch" "$OUT/write" 4096 "$OUT/${K}_traffic.json" $K > /dev/null || true
done
python3 tools/mfma_summary.py "$OUT/fp64" "$OUT/fp64_summary.csv" | tee "$OUT/fp64_summary.txt"
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
ls "$OUT"
