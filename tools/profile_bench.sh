#!/bin/bash
# Round profile of the default bench command on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats            -> per-kernel time summary
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE         -> HBM traffic of the contraction (separate passes)
#   4. --pmc MFMA busy / fp64 MOPS / GUI_ACTIVE      -> MFMA utilisation per kernel
# Outputs land in gpurun_out/prof_<tag>/; copy the summaries into profiles/ afterwards.
# usage: tools/profile_bench.sh TAG [bench args...]
set -e
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/write.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/mfma" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/mfma.log" 2>&1
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT/fetch" "$OUT/write" 4096 "$OUT/contract_traffic.json" > /dev/null
python3 tools/mfma_summary.py "$OUT/mfma" "$OUT/mfma_summary.csv"
python3 tools/trace_check.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace.log" "$OUT/trace_check.json"
tail -1 "$OUT/trace.log"
# raw per-dispatch CSVs are large: keep them compressed
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
