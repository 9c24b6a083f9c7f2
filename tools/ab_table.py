"""Markdown table of bench A/B runs (gpurun_out/<tag>_<i>.log from tools/ab_env.sh, which also
prints the environment of each run): python tools/ab_table.py [--env MAP.json] LOG_GLOB ... >
profiles/r04_ab.md. MAP.json = {"<tag>_<i>": "VAR=VALUE ..."} labels logs written without their
"# env:" line."""
import glob
import json
import sys

args = sys.argv[1:]
envmap = {}
if args[:1] == ["--env"]:
    envmap = json.load(open(args[1]))
    args = args[2:]
rows = []
for pat in args:
    for f in sorted(glob.glob(pat)):
        try:
            lines = open(f).read().strip().splitlines()
            d = json.loads(lines[-1])
        except Exception:
            continue
        env = next((l[len("# env: "):] for l in lines if l.startswith("# env: ")), "")
        env = env or envmap.get(f.rsplit("/", 1)[-1][:-len(".log")], "")
        c = d.get("config", {})
        w = d.get("wave_trace") or {}
        st = d.get("driver_stats_last_call") or {}
        dc = st.get("device_call") or st.get("device_wait")
        rows.append((f + (f" `{env}`" if env else ""), d["value"], d["evals_per_s"], d["ms_per_step"] * d["steps"] / 1e3, c.get("host_processes_per_gpu"),
                     w.get("mean_resident_waves"), w.get("fwd_wave_ms_mean"), w.get("bwd_wave_ms_mean"),
                     (dc / st["rounds"] * 1e3) if dc and st.get("rounds") else None))
print("| run log | fits/s | evals/s | region s | procs | mean resident waves | fwd wave ms | bwd wave ms | device ms per call |")
print("|---|---|---|---|---|---|---|---|---|")
f = lambda v, fmt: (fmt % v) if v is not None else ""
for r in rows:
    print(f"| {r[0]} | {r[1]:.0f} | {r[2]:.0f} | {r[3]:.2f} | {r[4]} | {f(r[5], '%.0f')} | {f(r[6], '%.3f')} | "
          f"{f(r[7], '%.3f')} | {f(r[8], '%.1f')} |")
