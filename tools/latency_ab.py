"""A/B of the few-problem latency lines (bench.secondary_c3 and secondary_solo) between the in-tree
library and GPX_LIB_ALT, alternating, each run in its own process.
usage: python tools/latency_ab.py [reps]   (GPU box; JSON lines)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import bench
c3 = bench.secondary_c3(0)
solo = bench.secondary_solo(0)
print(json.dumps({"c3_wall_ms": c3["wall_s_all_series_1gpu"] * 1e3, "c3_share_ms": c3["wall_s_per_gpu_share_at_8gpus"] * 1e3,
                  "solo_ms": solo["bcr"]["fit_ms_median"]}))
'''
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for tag, lib in (("base", None), ("alt", os.environ.get("GPX_LIB_ALT"))):
        env = dict(os.environ, REPO=repo)
        env.pop("GPX_LIB", None)
        if lib:
            env["GPX_LIB"] = lib
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(json.dumps({"lib": tag, "rep": rep, **{k: round(v, 2) for k, v in d.items()}}), flush=True)
