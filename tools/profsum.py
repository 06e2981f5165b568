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
