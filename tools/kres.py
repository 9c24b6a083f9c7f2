"""Per-kernel VGPR / AGPR / scratch / occupancy of a .hip file (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/kres.py portfoliooptgp_amd/csrc/gpx_band16.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
                      "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True, cwd=".")
cur = None
rows = []
for line in out.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f'{r["name"][:60]:60s} V={r.get("VGPRs")} A={r.get("AGPRs")} scr={r.get("ScratchSize [bytes/lane]")} '
              f'occ={r.get("Occupancy [waves/SIMD]")} lds={r.get("LDS Size [bytes/block]")}')
