"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for the gradient-contraction
kernel into profiles/<round>_contract_traffic.json (read by bench.py for roofline.traffic).

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3 section): counters are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled;
WRITE_SIZE is taken as is. Each dispatch's problem count is its workgroup count divided by
the lower-tile count of one problem (exact when the active count is a multiple of 8, the
XCD-hybrid grid adds < 8 idle-tail workgroups otherwise).

usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR NP OUT.json [KERNEL_TAG]

With KERNEL_TAG (e.g. band_bwd1_kernel) the fused banded kernel of that name is summarised
instead: one workgroup per problem, so a dispatch's problem count is its workgroup count.
"""
import csv
import json
import sys


def is_contract(name: str) -> bool:
    # gemm_kernel<BM, TA=true, TB=false, EPI_CONTRACT(1) | EPI_CONTRACT1(3)>
    return "gemm_kernel<" in name and ("true, false, 1>" in name or "true, false, 3>" in name)


def collect(d, counter, match=None):
    match = match or is_contract
    tot, wgs, n, names = 0.0, 0, 0, set()
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter or not match(r["Kernel_Name"]):
            continue
        tot += float(r["Counter_Value"])
        wgs += int(r["Grid_Size"]) // int(r["Workgroup_Size"])
        n += 1
        names.add(r["Kernel_Name"])
    return tot, wgs, n, sorted(names)


def main():
    fdir, wdir, np_, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    tag = sys.argv[5] if len(sys.argv) > 5 else None
    if tag:
        match = lambda name: tag + "<" in name or tag + "(" in name  # noqa: E731
        ntl = 1  # one workgroup per problem
    else:
        match = None
        nt = np_ // 128
        ntl = nt * (nt + 1) // 2
    f_kb, f_wgs, f_n, names = collect(fdir, "FETCH_SIZE", match)
    w_kb, w_wgs, w_n, _ = collect(wdir, "WRITE_SIZE", match)
    fb = f_kb * 1024 * 2
    wb = w_kb * 1024
    res = {
        "kernel": names,
        "Np": np_, "tiles_per_problem": ntl,
        "fetch_dispatches": f_n, "write_dispatches": w_n,
        "fetch_bytes_per_problem": fb / (f_wgs / ntl),
        "write_bytes_per_problem": wb / (w_wgs / ntl),
        "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
        "sources": [fdir, wdir],
    }
    res["hbm_bytes_per_problem"] = res["fetch_bytes_per_problem"] + res["write_bytes_per_problem"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
