"""Aggregate rocprofv3 --pmc counter_collection.csv per kernel: python tools/pmcsum.py <dir> [name-regex]"""
import csv, glob, re, sys, collections
d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = list(csv.DictReader(open(glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
dur = collections.defaultdict(dict)
for r in rows:
    k = r["Kernel_Name"]
    if flt and not re.search(flt, k):
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
    dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, c in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]].values())):
    n = len(disp[k])
    t = sum(dur[k].values()) / n
    print(f"{k[:90]}  n={n} avg_dur={t/1e3:.1f}us")
    print("   " + "  ".join(f"{cn}={v/n:.4g}" for cn, v in sorted(c.items())))
