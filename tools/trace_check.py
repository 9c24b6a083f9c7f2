"""Cross-check of bench.py's live timing of its roofline kernel against a rocprofv3 kernel trace
of the same command: that kernel's dispatches between the bench's two timed-region markers (the
spin kernel of torch.cuda._sleep) are averaged and compared with the bench line's
roofline.avg_launch_ms / launches. The kernel is the one the bench line names: the fused
banded sweep (band16_bwd/fwd_kernel, band_bwd1/fwd1_kernel) or the dense fused contraction.

usage: python tools/trace_check.py TRACE_CSV[.gz] BENCH_LOG OUT.json
"""
import csv
import gzip
import json
import sys


def is_contract(name: str) -> bool:
    return "gemm_kernel<" in name and ("true, false, 1>" in name or "true, false, 3>" in name)


def matcher(bench_kernel: str):
    """Trace-name predicate for the kernel a bench line's roofline names."""
    for tag in ("band16_bwd_kernel", "band16_fwd_kernel", "band16_wide_kernel", "band_bwd1_kernel", "band_fwd1_kernel",
                "band_bwd_kernel", "band_fwd_kernel"):
        if bench_kernel.startswith(tag):
            return lambda name, tag=tag: tag + "<" in name or tag + "(" in name
    return is_contract


def main():
    tpath, blog, out = sys.argv[1], sys.argv[2], sys.argv[3]
    op = gzip.open if tpath.endswith(".gz") else open
    rows = list(csv.DictReader(op(tpath, "rt")))
    marks = sorted(int(r["Start_Timestamp"]) for r in rows if "spin_kernel" in r["Kernel_Name"])
    if len(marks) < 2:
        sys.exit(f"expected 2 timed-region markers, found {len(marks)}")
    t0, t1 = marks[-2], marks[-1]
    line = [l for l in open(blog) if '"metric"' in l][-1]
    bench = json.loads(line[line.index("{"):])
    rf = bench["roofline"]
    match = matcher(rf["kernel"])
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
          if match(r["Kernel_Name"]) and t0 <= int(r["Start_Timestamp"]) <= t1]
    avg = sum(e - s for s, e in ks) / len(ks) / 1e6
    res = {
        "kernel": rf["kernel"],
        "timed_region_ms_trace": (t1 - t0) / 1e6,
        "trace_launches": len(ks),
        "trace_avg_launch_ms": avg,
        "bench_launches": rf.get("launches"),
        "bench_avg_launch_ms": rf["avg_launch_ms"],
        "rel_diff": avg / rf["avg_launch_ms"] - 1.0,
        "bench_value_fits_per_s": bench["value"],
        "sources": [tpath, blog],
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
