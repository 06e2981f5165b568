"""Print per-kernel resource usage (VGPR/AGPR/spill/scratch/occupancy/LDS) of a HIP source file.
usage: python tools/kres.py file.hip [name-filter]"""
import re, subprocess, sys
f = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I../../include", "-I.",
                      "-c", f, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.rsplit(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} spill={r.get('VGPRs Spill')} "
              f"sspill={r.get('SGPRs Spill')} scratch={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')} "
              f"lds={r.get('LDS Size [bytes/block]')}")
