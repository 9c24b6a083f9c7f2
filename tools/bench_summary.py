"""One-line summary of a bench.py JSON line: python tools/bench_summary.py NAME file.json"""
import json
import sys

name, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
r = d.get("roofline", {})
bp = d.get("band_path", {})
hs = [h.get("host_share") for h in d.get("host", [])]
print(f"{name}: fits/s {d['value']:.1f} evals/s {d['evals_per_s']:.0f} nfev {d['nfev_mean']:.2f} "
      f"region {d['ms_per_step'] * d['steps'] / 1e3:.2f}s slot_demand {r.get('slot_demand', r.get('occupancy'))} frac {r.get('frac', 0):.4f} "
      f"chip {r.get('chip_frac', 0):.4f} launch_ms {r.get('avg_launch_ms', 0):.3f} "
      f"ms/call {bp.get('ms_per_call', 0):.2f} prob/call {bp.get('problems_per_call', 0):.0f} "
      f"host_share {[round(x, 2) for x in hs if x is not None]}", flush=True)
