#!/bin/bash
# Round-5 evidence on the GPU box (repo root, via gpurun), into gpurun_out/prof_<tag>/:
#   0. the default bench line (the headline's layout: 8 host processes x 1024 slots)
#   1. the headline's layout under the kernel trace: 8 concurrent single-process bench instances
#      (1024 slots each), each under its own rocprofv3 --kernel-trace (a profiled program may not
#      spawn the bench's helper processes, so the shell starts the 8) -> tools/trace_multi.py: per
#      sweep kernel the trace's average launch vs the instances' HIP events and vs line 0
#   2. rocprofv3 --kernel-trace --stats of one instance -> per-kernel summary
#   3. --pmc FETCH_SIZE, 4. --pmc WRITE_SIZE (separate passes, one instance of 1024 slots) -> HBM
#      bytes per problem of the band16 sweeps and the wide launch (tools/pmc_summary.py)
# usage: [SKIP_BENCH=1] tools/profile_round5.sh TAG
set -e
TAG=${1:-r05}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.log" 2>&1
  tail -1 "$OUT/bench.log" | cut -c1-200
fi
cd /tmp && export TMPDIR=/tmp
INST="--no-cpu-baseline --no-secondary --procs 1 --width 1024 --fits 768 --steps 8 --warmup 1"
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
SHORT="--no-cpu-baseline --no-secondary --procs 1 --width 1024 --fits 768 --steps 1 --warmup 1"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" $SHORT > "$OUT/fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" $SHORT > "$OUT/write.log" 2>&1
cd "$ROOT"
for K in band16_fwd_kernel band16_bwd_kernel band16_wide_kernel; do
  python3 tools/pmc_summary.py "$OUT/fetch" "$OUT/write" 4096 "$OUT/${K}_traffic.json" $K > /dev/null || true
done
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
ls "$OUT"
