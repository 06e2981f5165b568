"""Per-basic-block instruction mix of one kernel in a hipcc -S listing.
usage: python tools/asmstat.py file.s symbol_substring"""
import re, sys, collections
lines = open(sys.argv[1]).read().split("\n")
sym = sys.argv[2]
start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(sym) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or re.match(r"^\.Lfunc_end", lines[i]))
blocks = []
cur = ["entry", collections.Counter(), start]
for i in range(start + 1, end):
    l = lines[i].strip()
    if re.match(r"^\.LBB\S+:", l):
        blocks.append(cur)
        cur = [l[:-1], collections.Counter(), i]
        continue
    if not l or l.startswith(";") or l.startswith("."):
        continue
    op = l.split()[0]
    c = cur[1]
    if op.startswith("v_mfma"): c["mfma"] += 1
    elif op.startswith("v_accvgpr"): c["accmov"] += 1
    elif op.startswith("v_"): c["valu"] += 1
    elif op.startswith("ds_read") or op.startswith("ds_load"): c["ds_rd"] += 1
    elif op.startswith("ds_"): c["ds_wr"] += 1
    elif op.startswith("global_load") or op.startswith("buffer_load"): c["vmem_ld"] += 1
    elif op.startswith("global_store") or op.startswith("buffer_store"): c["vmem_st"] += 1
    elif op.startswith("s_waitcnt"): c["waitcnt"] += 1
    elif op.startswith("s_barrier"): c["barrier"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"): c["branch"] += 1
    elif op.startswith("s_"): c["salu"] += 1
    else: c["other"] += 1
blocks.append(cur)
tot = collections.Counter()
for name, c, ln in blocks:
    tot.update(c)
    if c["mfma"] or sum(c.values()) > 60:
        print(f"{name:14s} line {ln:7d}: " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
print("TOTAL:", " ".join(f"{k}={v}" for k, v in sorted(tot.items())))
