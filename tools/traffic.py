"""profiles/traffic.json from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over bench.py.

python tools/traffic.py <pmc FETCH dir> <pmc WRITE dir> <suffix> [<family>=<kernel-name substring> ...]
python tools/traffic.py --all <pmc FETCH dir> <pmc WRITE dir> [<suffix>]

Every family gets bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB per dispatch x 1024; FETCH_SIZE doubled: gfx950
counts half of the bytes of wide coalesced streaming reads, MI355X_MICROARCH.md HBM/rocprofv3 section), averaged over
the dispatches whose kernel name matches.  <suffix> (e.g. "@512x1" or "") is appended to each family key so the C3
and C5 workloads keep separate entries; existing entries of traffic.json are kept.

--all: the conv family of the bench line, every conv5 / conv3 instantiation on its own, and the
HBM-bound kernel families under the names bench.py's `hbm` block uses (C-ABI entry points / kernel families), so that
its measured_bytes_per_launch is filled.  Kernel names appear mangled (_ZN4unet...) or demangled in the CSV; the
patterns below match either form."""
import collections
import csv
import glob
import json
import re
import sys
from pathlib import Path

POOL = r"(Lb1E|, true>)"
NOPOOL = r"(Lb0E|, false>)"
# bench.py hbm-family name -> regex over the kernel name
HBM_FAMILIES = {
    "unet_bn_bwd_apply": r"bn_bwd_apply_vec_kernel.*" + NOPOOL,
    "unet_bn_bwd_apply_pool": r"bn_bwd_apply_vec_kernel.*" + POOL,
    "unet_bn_bwd_reduce": r"bn_bwd_reduce_vec_kernel.*" + NOPOOL,
    "unet_bn_bwd_reduce_pool": r"bn_bwd_reduce_vec_kernel.*" + POOL,
    "unet_gate_bwd1": r"gate_bwd1",
    "unet_gate_bwd2": r"gate_bwd2",
    "unet_gate_bwd3": r"gate_bwd3",
    "unet_gate_psi": r"psi_vec_kernel",
    "unet_upsample_bwd": r"upsample_bwd",
    "unet_materialize": r"materialize_(fast_)?kernel",
    "unet_materialize_pool": r"materialize_pool_kernel",
    "smallcin_fwd_mfma_kernel": r"smallcin_fwd_mfma_kernel",
    # template <T, NA, NB, OMK, XD> (round 6: XD, the x prefetch depth, after OMK)
    "pw_conv_kernel": r"pw_conv_kernel(IDF16.?Li\d+ELi\d+ELi0E|<[^>]*, 0, \d+>)",        # OMK 0: y + BN sums
    "pw_conv_kernel(dgrad)": r"pw_conv_kernel(IDF16.?Li\d+ELi\d+ELi[12]E|<[^>]*, [12], \d+>)",  # OMK 1/2: fp32
}
CONV_FAMILY = {"bf16": r"(conv3_kernel<bf16,3,|conv5_kernel<bf16,|conv3_kernelIDF16bLi3E|conv5w?_kernelIDF16b)",
               "fp16": r"(conv3_kernel<fp16,3,|conv5_kernel<fp16,|conv3_kernelIDF16_Li3E|conv5w?_kernelIDF16_)"}


def rows_of(d):
    return list(csv.DictReader(open(glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0])))


def per_kernel(rows, cname):
    """kernel name -> (sum of counter over dispatches, set of dispatch ids)"""
    tot = collections.defaultdict(float)
    ids = collections.defaultdict(set)
    for r in rows:
        if r["Counter_Name"] == cname:
            tot[r["Kernel_Name"]] += float(r["Counter_Value"])
            ids[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return tot, ids


def family(fetch, write, rx):
    f = sum(v for k, v in fetch[0].items() if re.search(rx, k))
    nf = sum(len(v) for k, v in fetch[1].items() if re.search(rx, k))
    w = sum(v for k, v in write[0].items() if re.search(rx, k))
    nw = sum(len(v) for k, v in write[1].items() if re.search(rx, k))
    if not nf or not nw:
        return None
    fb, wb = f / nf * 1024.0, w / nw * 1024.0
    return {"bytes_per_launch": round(2 * fb + wb), "fetch_bytes": round(2 * fb), "write_bytes": round(wb),
            "launches_sampled": nf,
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py (kernels matching "
                      f"'{rx}'); FETCH_SIZE x2 (gfx950 correction)"}


def main():
    path = Path("profiles/traffic.json")
    out = json.loads(path.read_text()) if path.exists() else {}
    if sys.argv[1] == "--all":
        d1, d2 = sys.argv[2:4]
        suffix = sys.argv[4] if len(sys.argv) > 4 else ""
        fetch, write = per_kernel(rows_of(d1), "FETCH_SIZE"), per_kernel(rows_of(d2), "WRITE_SIZE")
        fams = dict(HBM_FAMILIES)
        for prec, rx in CONV_FAMILY.items():
            key = f"conv3_kernel<{prec},3,|conv5_kernel<{prec},|conv5w_kernel<{prec}"   # bench.py's family key
            fams[key] = rx
        # every conv5 / conv3 instantiation separately (the conv family's traffic split)
        for k in set(fetch[0]) | set(write[0]):
            m = re.search(r"(conv5w_kernel|conv5_kernel|conv3_kernel)\S*", k)
            if m:
                fams["inst:" + m.group(0)] = re.escape(m.group(0))
        for fam, rx in sorted(fams.items()):
            ent = family(fetch, write, rx)
            if ent is not None:
                out[fam + suffix] = ent
    else:
        d1, d2, suffix = sys.argv[1:4]
        fams = dict(a.split("=", 1) for a in sys.argv[4:])
        fetch, write = per_kernel(rows_of(d1), "FETCH_SIZE"), per_kernel(rows_of(d2), "WRITE_SIZE")
        for fam, sub in fams.items():
            ent = family(fetch, write, "|".join(re.escape(a) for a in sub.split("|")))
            if ent is not None:
                out[fam + suffix] = ent
    path.write_text(json.dumps(out, indent=1))
    for k, v in out.items():
        print(f"{v['bytes_per_launch'] / 1e6:10.2f} MB/launch  fetch {v['fetch_bytes'] / 1e6:9.2f}  write "
              f"{v['write_bytes'] / 1e6:9.2f}  n={v['launches_sampled']:5d}  {k}")


if __name__ == "__main__":
    main()
