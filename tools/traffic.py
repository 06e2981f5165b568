"""profiles/traffic.json from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over bench.py.

python tools/traffic.py <pmc FETCH dir> <pmc WRITE dir> <suffix> [<family>=<kernel-name substring> ...]

Every family gets bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB per dispatch x 1024; FETCH_SIZE doubled: gfx950
counts half of the bytes of wide coalesced streaming reads, MI355X_MICROARCH.md HBM/rocprofv3 section), averaged over
the dispatches whose kernel name contains the substring.  <suffix> (e.g. "@512x1" or "") is appended to each family
key so the C3 and C5 workloads keep separate entries; existing entries of traffic.json are kept."""
import csv
import glob
import json
import sys
from pathlib import Path

d1, d2, suffix = sys.argv[1:4]
fams = dict(a.split("=", 1) for a in sys.argv[4:])


def per_dispatch(d, cname, sub):
    rows = list(csv.DictReader(open(glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0])))
    tot, ids = 0.0, set()
    alts = sub.split("|")     # 'a|b': kernels whose name contains any alternative (the bench's conv family)
    for r in rows:
        if any(a in r["Kernel_Name"] for a in alts) and r["Counter_Name"] == cname:
            tot += float(r["Counter_Value"])
            ids.add(r["Dispatch_Id"])
    return tot / max(1, len(ids)) * 1024.0, len(ids)


path = Path("profiles/traffic.json")
out = json.loads(path.read_text()) if path.exists() else {}
for fam, sub in fams.items():
    f, nf = per_dispatch(d1, "FETCH_SIZE", sub)
    w, nw = per_dispatch(d2, "WRITE_SIZE", sub)
    if not nf:
        continue
    out[fam + suffix] = {"bytes_per_launch": round(2 * f + w), "fetch_bytes": round(2 * f), "write_bytes": round(w),
                         "launches_sampled": nf,
                         "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py "
                                   f"(kernels matching '{sub}'); FETCH_SIZE x2 (gfx950 correction)"}
path.write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
