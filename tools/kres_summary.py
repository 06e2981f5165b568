"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel (VGPRs, spills, LDS).
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres_summary.py [name-filter]"""
import re, sys
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key in ("VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "LDS Size \\[bytes/block\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(r"remark:\s+" + key + r": (\d+)", line)
        if m:
            cur[key.split(" ")[0] + ("_spill" if "Spill" in key else "")] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:80]:80s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>4} "
              f"vspill {r.get('VGPRs_spill','?'):>4} sspill {r.get('SGPRs_spill','?'):>4} lds {r.get('LDS','?'):>6} "
              f"occ {r.get('Occupancy','?')}")
