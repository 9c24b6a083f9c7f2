"""Per-kernel averages (per dispatch) of every counter of a rocprofv3 --pmc pass (csv output):
python tools/pmc_table.py PMC_DIR [kernel-substring]. Also per-wave figures when SQ_WAVES is in
the pass (instruction counts / SQ_WAVES; SQ_*_CYCLES-type counters are quad-cycles)."""
import csv
import json
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = defaultdict(lambda: defaultdict(float))
    seen = set()
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        if flt not in k:
            continue
        a = agg[k]
        a[r["Counter_Name"]] += float(r["Counter_Value"])
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
        if (k, disp) not in seen:
            seen.add((k, disp))
            a["dispatches"] += 1
            a["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        n = a["dispatches"]
        row = {"kernel": k[:90], "dispatches": int(n), "avg_ms": a["ns"] / n / 1e6}
        for c, v in a.items():
            if c not in ("dispatches", "ns"):
                row[c] = v / n
        w = a.get("SQ_WAVES")
        if w:
            row["per_wave"] = {c: v / w for c, v in a.items() if c.startswith("SQ_") and c != "SQ_WAVES"}
        print(json.dumps(row))


if __name__ == "__main__":
    main()
