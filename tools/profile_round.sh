#!/bin/bash
# Round evidence on the GPU box (run from the repo root via gpurun):
#   0. the bench line itself (python bench.py: the defaults, CPU baseline and secondary lines included)
#   1. rocprofv3 --kernel-trace --stats of a shorter bench (20 steps) -> per-kernel summary + trace check
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (separate passes) -> HBM bytes of the roofline kernel
#   4. --pmc MFMA busy / fp64 MOPS / GUI_ACTIVE               -> MFMA utilisation per kernel
# Outputs land in gpurun_out/prof_<tag>/; copy the summaries into profiles/ afterwards.
# usage: tools/profile_round.sh TAG
set -e
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
# counter passes serialise every dispatch: one host process and a short run (bytes and MFMA
# counts per problem do not depend on the process count)
SHORT="--no-cpu-baseline --no-secondary --steps 3 --warmup 1 --procs 1 --width 1024"
# the kernel trace over 40 steps of one host process (the profiler's output files are per
# process; the trace check compares this run's own bench line with its own trace)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --no-secondary --steps 40 --warmup 1 --procs 1 --width 2048 > "$OUT/trace.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" $SHORT > "$OUT/fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" $SHORT > "$OUT/write.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/mfma" -o run -- python3 "$ROOT/bench.py" $SHORT > "$OUT/mfma.log" 2>&1
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT/fetch" "$OUT/write" 4096 "$OUT/band16_bwd_traffic.json" band16_bwd_kernel > /dev/null
python3 tools/pmc_summary.py "$OUT/fetch" "$OUT/write" 4096 "$OUT/band16_fwd_traffic.json" band16_fwd_kernel > /dev/null
python3 tools/mfma_summary.py "$OUT/mfma" "$OUT/mfma_summary.csv" > "$OUT/mfma_summary.txt"
python3 tools/trace_check.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace.log" "$OUT/trace_check.json" > /dev/null
python3 tools/trace_util.py "$OUT/trace/run_kernel_trace.csv" 0.2 > "$OUT/trace_util.txt"
tail -1 "$OUT/bench.log"
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
