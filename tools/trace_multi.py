"""The bench's banded sweep kernels timed two ways in the headline's own layout: N concurrent
single-process bench instances on one GPU (each its own 1024 slots, as the bench's N host
processes), every instance under its own `rocprofv3 --kernel-trace` (tools/profile_round5.sh).
Per kernel of the bench line's roofline.sweeps: the trace's average launch duration over every
instance's timed region (between its two spin-kernel markers) against the instances' own HIP-event
averages, and against a reference bench line (the default 8-process command) when given.

usage: python tools/trace_multi.py OUT.json REF_BENCH_LOG DIR1 [DIR2 ...]
  DIRi: a rocprofv3 output directory (run_kernel_trace.csv[.gz]) with the instance's bench log beside
  it as DIRi.log"""
import csv
import gzip
import json
import os
import sys

TAGS = ("band16_fwd_kernel", "band16_bwd_kernel", "band16_wide_kernel", "band_fwd1_kernel", "band_bwd1_kernel",
        "band_fwd_kernel", "band_bwd_kernel")


def tag_of(key):
    for t in TAGS:
        if key.startswith(t):
            return t
    return None


def bench_line(path):
    line = [l for l in open(path) if '"metric"' in l][-1]
    return json.loads(line[line.index("{"):])


def main():
    out, ref_log, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    per = {}
    bench_avgs = {}
    for d in dirs:
        p = os.path.join(d, "run_kernel_trace.csv")
        op = open
        if not os.path.exists(p):
            p += ".gz"
            op = gzip.open
        rows = list(csv.DictReader(op(p, "rt")))
        marks = sorted(int(r["Start_Timestamp"]) for r in rows if "spin_kernel" in r["Kernel_Name"])
        t0, t1 = marks[-2], marks[-1]
        b = bench_line(d + ".log")
        for key, v in b["roofline"].get("sweeps", {}).items():
            t = tag_of(key)
            if t is None or not v.get("launches"):
                continue
            bench_avgs.setdefault(t, []).append((v["avg_launch_ms"], v["launches"]))
        for r in rows:
            s = int(r["Start_Timestamp"])
            if not (t0 <= s <= t1):
                continue
            name = r["Kernel_Name"]
            for t in TAGS:
                if t + "<" in name or t + "(" in name:
                    per.setdefault(t, []).append((int(r["End_Timestamp"]) - s) / 1e6)
                    break
    ref = bench_line(ref_log)
    ref_sw = {tag_of(k): v for k, v in ref["roofline"].get("sweeps", {}).items() if tag_of(k)}
    res = {"instances": len(dirs), "reference_bench": os.path.basename(ref_log),
           "reference_fits_per_s": ref["value"], "kernels": {}}
    for t, ds in per.items():
        avg = sum(ds) / len(ds)
        ba = bench_avgs.get(t, [])
        bavg = sum(a * n for a, n in ba) / max(sum(n for _, n in ba), 1) if ba else None
        r = ref_sw.get(t)
        res["kernels"][t] = {"trace_launches": len(ds), "trace_avg_launch_ms": avg,
                             "instances_hip_event_avg_ms": bavg,
                             "rel_diff_trace_vs_instances": (avg / bavg - 1.0) if bavg else None,
                             "reference_bench_avg_launch_ms": r["avg_launch_ms"] if r else None,
                             "rel_diff_trace_vs_reference_bench": (avg / r["avg_launch_ms"] - 1.0) if r else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
