#!/bin/bash
# A/B bench lines on one box: each argument is a space-separated list of VAR=VALUE settings for
# one bench.py run (no CPU baseline, no secondary lines). Summaries via tools/bench_summary.py.
# usage: tools/ab_env.sh TAG "GPX_X=1 GPX_Y=2" "GPX_X=0" ...
TAG=${1:-ab}
shift
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i + 1))
  log="gpurun_out/${TAG}_${i}.log"
  echo "# env: $kv" > "$log"
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary >> "$log" 2>&1 \
    || { echo "[$kv] failed"; tail -20 "$log"; exit 1; }
  python tools/bench_summary.py "$kv" "$log"
  python - "$log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d.get("wave_trace")
if w:
    print("   wave trace: mean resident %.0f (occ %.3f) fwd %.3f ms bwd %.3f ms share %s" % (
        w["mean_resident_waves"], w["occupancy_2048"], w["fwd_wave_ms_mean"], w["bwd_wave_ms_mean"],
        {k: round(v, 3) for k, v in w["share_of_span_by_resident_waves"].items()}))
st = d.get("driver_stats_last_call") or {}
print("   driver:", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()})
PY
  # a raw trace: its call timeline here, then the file goes (gpurun copies back <= 64 MiB)
  tr=$(echo "$kv" | tr ' ' '\n' | sed -n 's/^GPX_WAVE_TRACE_OUT=//p')
  if [ -n "$tr" ] && [ -f "$tr" ]; then
    python tools/call_timeline.py "$tr" > "${tr%.npz}_timeline.txt" 2>&1 && sed 's/^/   /' "${tr%.npz}_timeline.txt"
    [ -n "$KEEP_TRACE" ] || rm -f "$tr"
  fi
done
