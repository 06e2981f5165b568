"""Measured vs algorithmic HBM bytes per conv5 / conv3 instantiation.

python tools/conv_traffic.py <layerprof.txt> [profiles/traffic.json]

Algorithmic bytes of one launch, from the layer list of tools/layerprof.py (one training step, forward
lines before the first weight gradient):
  forward y:  x (+ the gate pre-activation, fp32 per pixel) + y (+ act_out, the stored transformed input, on
              BN-activation sources of maps up to 256^2)
  dgrad y (BN-backward sums, OM5_BNB): dy + the activation y1 it masks + g
  dgrad fp32: dy + the fp32 gradient (accumulated outputs read too are not counted: the network's fp32
              dgrads through conv5 / conv3 store without accumulation)
Measured: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per dispatch (tools/traffic.py --all, "inst:" entries).  The
kernel instantiation of each line follows the host dispatch: conv5 <T, MI, OM, SK, GATE, ABL, PIPE[, NWV]>
(OM 0 y, 1 fp32, 2 y + BN-backward sums; SK 1 plain, 2 one BN activation, 3 activation + stored)."""
import collections
import json
import re
import sys

LINE = re.compile(r"^\s*([\d.]+) us\s+[\d.]+ TF/s\s+(conv|wgrad)\s*(\w*)\s+(\d+)x(\d+)x(\d+)\s+(\d+)->\s*(\d+) k(\d) "
                  r"\[([^\]]+)\] (\S+)")


def main():
    lp = open(sys.argv[1]).read().splitlines()
    tr = json.load(open(sys.argv[2] if len(sys.argv) > 2 else "profiles/traffic.json"))
    fwd = True
    groups = collections.defaultdict(list)
    for ln in lp:
        m = LINE.match(ln)
        if not m:
            continue
        us, kind, mode, N, H, W, cin, cout, k, srcs, var = m.groups()
        if kind == "wgrad":
            fwd = False
            continue
        N, H, W, cin, cout, k = map(int, (N, H, W, cin, cout, k))
        if k != 3 or not var.startswith(("conv5", "conv3")):
            continue
        P = N * H * W
        kinds = srcs.split("+")
        if mode == "y" and fwd:
            b = P * cin * 2 + P * cout * 2
            act = kinds[0].startswith("act")
            if act and H * W <= 256 * 256:
                b += P * int(re.sub(r"\D", "", kinds[0])) * 2          # act_out
            om = 0
            sk = 1 if not act else (2 if len(kinds) == 1 else 3)
        elif mode == "y":
            b = P * cin * 2 + P * cout * 2 * 2                           # dy + y1 + g
            om, sk = 2, 1
        else:
            b = P * cin * 2 + P * cout * 4
            om, sk = 1, 1
        fam = "conv5" if var.startswith("conv5") else "conv3"
        # the traffic model of a conv5 launch: each 16 x 32 tile DMAs its (16 + 2) x 34 input halo, once per
        # 64-channel output block (gy = Cout / 64 blocks read the same halo; adjacent tiles run on other XCDs,
        # so the overlap and the re-reads leave the XCD's L2: FETCH_SIZE counts Infinity-Cache hits too)
        gy = -(-cout // 64)
        xin = P * cin * 2
        model = b + xin * (18 / 16 * 34 / 32 * gy - 1)
        groups[(fam, om, sk)].append((b, float(us), model))
    print(f"{'instantiation':22s} {'launches/step':>13s} {'algorithmic MB':>15s} {'model MB':>9s} {'measured MB':>12s} "
          f"{'meas/alg':>9s} {'meas/model':>10s}")
    for (fam, om, sk), v in sorted(groups.items()):
        alg = sum(x[0] for x in v) / len(v)
        mod = sum(x[2] for x in v) / len(v)
        meas = None
        if fam == "conv5":
            pat = f"inst:conv5_kernelIDF16bLi4ELi{om}ELi{sk}E"
            ms = [e["bytes_per_launch"] for key, e in tr.items() if key.startswith(pat)]
            meas = sum(ms) / len(ms) if ms else None
        name = f"{fam} OM{om} SK{sk}"
        nan = float("nan")
        print(f"{name:22s} {len(v):13d} {alg / 1e6:15.1f} {mod / 1e6:9.1f} {meas / 1e6 if meas else nan:12.1f} "
              f"{meas / alg if meas else nan:9.2f} {meas / mod if meas else nan:10.2f}")


if __name__ == "__main__":
    main()
