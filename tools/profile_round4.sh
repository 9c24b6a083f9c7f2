#!/bin/bash
# Round-4 evidence on the GPU box (run from the repo root via gpurun), into gpurun_out/prof_<tag>/:
#   0. the bench line with the defaults (CPU baseline and secondary lines included)
#   1. the wave trace of the bench's own 8-process layout: occupancy timeline + per-call timeline
#   2. rocprofv3 --kernel-trace --stats of one host process (the bench's helpers are spawned
#      processes, which must not start under the profiler) -> per-kernel summary + trace check
#   3. --pmc FETCH_SIZE, 4. --pmc WRITE_SIZE (separate passes) -> HBM bytes per problem of the
#      band16 sweeps, for the K-band path (GPX_B16_INLINE_K=0) and the inline-K path (3, the default)
# usage: [SKIP_BENCH=1] tools/profile_round4.sh TAG
set -e
TAG=${1:-r04}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
if [ -z "$SKIP_BENCH" ]; then  # (SKIP_BENCH=1: the caller has just run the default bench line)
  timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.log" 2>&1
  tail -1 "$OUT/bench.log" | cut -c1-300
fi
GPX_WAVE_TRACE=1 GPX_WAVE_TRACE_OUT="$OUT/wave_trace.npz" timeout -k 10 300 python3 "$ROOT/bench.py" \
  --no-cpu-baseline --no-secondary > "$OUT/wave_bench.log" 2>&1
python3 "$ROOT/tools/call_timeline.py" "$OUT/wave_trace.npz" > "$OUT/call_timeline.txt"
python3 "$ROOT/tools/wave_overlap.py" "$OUT/wave_trace.npz" > "$OUT/wave_overlap.txt"
rm -f "$OUT/wave_trace.npz"
cd /tmp && export TMPDIR=/tmp
SHORT="--no-cpu-baseline --no-secondary --steps 1 --warmup 1 --procs 1 --width 1024 --fits 1024"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --no-secondary --steps 3 --warmup 1 --procs 1 --width 2048 --fits 2048 \
  > "$OUT/trace.log" 2>&1
for K in 0 3; do
  GPX_B16_INLINE_K=$K timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_k$K" -o run -- \
    python3 "$ROOT/bench.py" $SHORT > "$OUT/fetch_k$K.log" 2>&1
  GPX_B16_INLINE_K=$K timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_k$K" -o run -- \
    python3 "$ROOT/bench.py" $SHORT > "$OUT/write_k$K.log" 2>&1
done
cd "$ROOT"
for K in 0 3; do
  python3 tools/pmc_summary.py "$OUT/fetch_k$K" "$OUT/write_k$K" 4096 "$OUT/band16_bwd_traffic_k$K.json" band16_bwd_kernel > /dev/null
  python3 tools/pmc_summary.py "$OUT/fetch_k$K" "$OUT/write_k$K" 4096 "$OUT/band16_fwd_traffic_k$K.json" band16_fwd_kernel > /dev/null
done
python3 tools/trace_check.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace.log" "$OUT/trace_check.json" > /dev/null || true
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
ls "$OUT"
