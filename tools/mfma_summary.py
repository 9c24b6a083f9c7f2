"""Per-kernel MFMA utilisation from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE (csv output).

* issued fp64 MFMA flops = MOPS_F64 x 512 (one v_mfma_f64_16x16x4_f64 = 2048 flops = 4 MOPS;
  checked against the launcher's own issued-flop count);
* MFMA-busy fraction = MFMA_BUSY_CYCLES (summed over the 1024 SIMDs) / (GUI_ACTIVE / 8 XCDs x
  1024 SIMDs) — the share of SIMD-cycles the matrix pipe was busy while the kernel ran (PMC
  collection serialises dispatches, so each kernel runs alone);
* issued TFLOP/s over the dispatches' own durations;
* when the pass also holds SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 (wave instructions): the fp64
  VALU flops (64 lanes x 1, or 2 for FMA) beside the MFMA flops, and the fp64 datapath's busy
  share. On gfx950 the fp64 MFMA and the fp64 VALU share one datapath (round 6,
  tools/micro/mfma_valu_overlap.hip: an MFMA + FMA mix costs the sum of the two), so the sweeps'
  fp64 roofline counts both: a v_mfma_f64_16x16x4_f64 holds it 64 cycles (4 MOPS: 16 per MOP),
  a fp64 VALU instruction ~4 (3.5 measured at two waves per SIMD).

usage: python tools/mfma_summary.py PMC_DIR OUT.csv
"""
import csv
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def main():
    d, out = sys.argv[1], sys.argv[2]
    agg = defaultdict(lambda: defaultdict(float))
    seen = set()
    rd = csv.DictReader(open(f"{d}/run_counter_collection.csv"))
    need = {"Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"}
    if not need <= set(rd.fieldnames or []):
        sys.exit(f"unexpected columns: {rd.fieldnames}")
    for r in rd:
        k = r["Kernel_Name"]
        a = agg[k]
        a[r["Counter_Name"]] += float(r["Counter_Value"])
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
        if (k, disp) not in seen:
            seen.add((k, disp))
            a["dispatches"] += 1
            a["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    rows = []
    for k, a in agg.items():
        gui = a.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        flops = a.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512.0
        vf = 64.0 * (a.get("SQ_INSTS_VALU_ADD_F64", 0.0) + a.get("SQ_INSTS_VALU_MUL_F64", 0.0)
                     + a.get("SQ_INSTS_VALU_TRANS_F64", 0.0) + 2.0 * a.get("SQ_INSTS_VALU_FMA_F64", 0.0))
        vi = (a.get("SQ_INSTS_VALU_ADD_F64", 0.0) + a.get("SQ_INSTS_VALU_MUL_F64", 0.0)
              + a.get("SQ_INSTS_VALU_TRANS_F64", 0.0) + a.get("SQ_INSTS_VALU_FMA_F64", 0.0))
        dp = 16.0 * a.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) + 4.0 * vi
        extra = {}
        if vi > 0:
            extra = {"VALU_fp64_TFLOP": vf / 1e12,
                     "fp64_TFLOPs_per_s_mfma_plus_valu": (flops + vf) / a["ns"] / 1e3 if a["ns"] else 0.0,
                     "valu_over_mfma_flops": vf / flops if flops else 0.0,
                     "fp64_datapath_busy_est": dp / (gui * SIMDS) if gui else 0.0}
        rows.append({
            "Kernel_Name": k,
            "Dispatches": int(a["dispatches"]),
            "Total_ms": a["ns"] / 1e6,
            "Issued_fp64_TFLOP": flops / 1e12,
            "Issued_TFLOPs_per_s": flops / a["ns"] / 1e3 if a["ns"] else 0.0,
            "MFMA_busy_frac": busy / (gui * SIMDS) if gui else 0.0,
            **extra,
        })
    rows.sort(key=lambda r: -r["Total_ms"])
    with open(out, "w", newline="") as f:
        keys = list(dict.fromkeys(k for r in rows for k in r))
        w = csv.DictWriter(f, fieldnames=keys, restval="")
        w.writeheader()
        for r in rows:
            w.writerow({k: (f"{v:.4f}" if isinstance(v, float) else v) for k, v in r.items()})
    tot_ns = sum(r["Total_ms"] for r in rows)
    tot_fl = sum(r["Issued_fp64_TFLOP"] for r in rows)
    for r in rows[:8]:
        more = (f"  +VALU {r['fp64_TFLOPs_per_s_mfma_plus_valu']:6.1f} TF/s  datapath {r['fp64_datapath_busy_est']:.3f}"
                if "fp64_datapath_busy_est" in r else "")
        print(f"{r['Total_ms']:10.1f} ms  {r['Issued_TFLOPs_per_s']:6.1f} TF/s  busy {r['MFMA_busy_frac']:.3f}{more}  {r['Kernel_Name'][:70]}")
    print(f"all kernels (serialised): {tot_ns:.1f} ms, {tot_fl / tot_ns * 1e3:.1f} TF/s issued")


if __name__ == "__main__":
    main()
