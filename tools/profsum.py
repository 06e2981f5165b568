"""Summarise rocprofv3 kernel timing: python tools/profsum.py <dir> [steps] [top]

Reads <dir>/*kernel_stats.csv (rocprofv3 --stats --output-format csv), or aggregates
<dir>/*kernel_trace.csv itself (e.g. after rocpd2csv on a .db run)."""
import csv, sys, glob, collections

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
stats = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
if stats:
    rows = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(stats[0]))]
else:
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])):
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    rows = [(k, v[0], v[1]) for k, v in agg.items()]
tot = sum(r[2] for r in rows)
for name, calls, ns in sorted(rows, key=lambda r: -r[2])[:top]:
    print(f"{ns/1e6/steps:8.3f} ms/step {100*ns/tot:6.2f}% n/step={calls/steps:6.1f} avg={ns/calls/1e3:8.1f}us  {name[:100]}")
print(f"total {tot/1e6/steps:.2f} ms/step")
# optional family summary: argv[4] = regex of the family's launch kernels, argv[5] = regex of companion kernels
# whose time belongs to those launches (the split-K finisher of conv5's small-map form): avg = (family +
# companion time) / family launches — what bench.py's probe (HIP events around the whole unet_conv call) measures
if len(sys.argv) > 4:
    import re
    fam = re.compile(sys.argv[4])
    comp = re.compile(sys.argv[5]) if len(sys.argv) > 5 else None
    n = sum(c for nm, c, _ in rows if fam.search(nm))
    t_f = sum(ns for nm, _, ns in rows if fam.search(nm))
    t_c = sum(ns for nm, _, ns in rows if comp and comp.search(nm) and not fam.search(nm))
    if n:
        print(f"family /{sys.argv[4]}/: {n / steps:.1f} launches/step, {t_f / 1e6 / steps:.3f} ms/step"
              f" + companions {t_c / 1e6 / steps:.3f} ms/step; avg {(t_f + t_c) / n / 1e3:.2f} us per launch")
