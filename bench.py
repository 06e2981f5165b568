#!/usr/bin/env python3
"""Benchmark: 512x512 CT slices/sec fwd+bwd, AttentionUNet bs=4/GPU (BASELINE.json metric).

One step = the reference's training micro-step (scripts/train.py:127-143) on one synthetic batch per
GPU: forward -> DiceBCELoss -> backward -> (DDP all-reduce) -> clip_grad_norm_(1.0) -> AdamW.step
-> zero_grad.  Inputs are generated once and stay resident in HBM.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints one JSON line (value = whole-job images/s, max-over-ranks time).  The line carries
`roofline` (the dominant kernel, timed live with HIP events on its launch stream) and
`cpu_baseline` (the CPU oracle timed on a bounded sample on this host, rank 0 at N=1 only).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}   # MI355X dense peaks (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
FLOPS_PER_IMAGE = {"attention_unet": 983.4e9, "unet": 957.5e9}   # fwd+bwd, 1ch 512^2
FLOPS_PER_IMAGE_C5 = 3938.3e9                                      # AttentionUNet 3ch 1024^2 fwd+bwd
METRIC = "512x512 CT slices/sec fwd+bwd, AttentionUNet bs=4/GPU, 1/2/4/8 MI355X"   # BASELINE.json


def cpu_model() -> str:
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def disc_targets(n: int, h: int, w: int, gen: torch.Generator) -> torch.Tensor:
    """1-3 discs of radius 6-20 px per image (≈0.36 % foreground on average)."""
    t = torch.zeros(n, h, w, dtype=torch.int64)
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    for i in range(n):
        for _ in range(int(torch.randint(1, 4, (1,), generator=gen))):
            cy, cx = int(torch.randint(0, h, (1,), generator=gen)), int(torch.randint(0, w, (1,), generator=gen))
            r = int(torch.randint(6, 21, (1,), generator=gen))
            t[i][(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1
    return t


def cpu_baseline(model_kind: str, size: int, batch: int, iters: int) -> dict:
    """Time the CPU oracle (fp32 NCHW ATen restatement of the reference) on a bounded sample."""
    sys.path.insert(0, str(ROOT))
    from oracle import unet_oracle as O
    from unet.models import AttentionUNet, UNet
    torch.manual_seed(0)
    m = AttentionUNet(1, 2) if model_kind == "attention_unet" else UNet(1, 2)
    p = O.params_from_module(m)
    g = torch.Generator().manual_seed(99)
    x = torch.rand(batch, 1, size, size, generator=g) * 2 - 1
    t = disc_targets(batch, size, size, g)
    fwd = O.attention_unet_forward if model_kind == "attention_unet" else O.unet_forward

    def one():
        for v in p.values():
            if v.grad is not None:
                v.grad = None
        loss = O.dice_bce_loss(fwd(p, x, training=True), t)
        loss.backward()

    one()  # warm-up
    t0 = time.perf_counter()
    for _ in range(iters):
        one()
    dt = time.perf_counter() - t0
    # threads: torch's intra-op pool, which follows OMP_NUM_THREADS (16 on the GPU box: the job's share of
    # the host); os.cpu_count() there reports the whole machine, and 256 threads on a 16-core share thrash
    return {"value": round(batch * iters / dt, 4), "unit": "img/s", "cores": torch.get_num_threads(),
            "cores_note": "torch.get_num_threads() = the job's CPU share (OMP_NUM_THREADS); host_cpus = os.cpu_count()",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "kind": "port",
            "sample": f"oracle/unet_oracle.py fp32 CPU, {model_kind} 1x{size}x{size}, batch {batch}, "
                      f"1 warm-up + {iters} timed fwd+DiceBCE+bwd iterations ({dt:.1f} s)"}


def _es(code: int) -> int:
    return 4 if code == 0 else 2   # UNET_F32 = 0, UNET_BF16 = 1, UNET_F16 = 2


def _hbm_bytes(name: str, a: tuple):
    """(family, algorithmic HBM bytes) of one C-ABI call: every operand read once + every output written
    once (include/unet_hip.h argument order), or None for calls that are not HBM-bound streaming kernels."""
    if name == "unet_bn_bwd_apply":             # da, y -> dy
        dt, gt, P, C = a[0], a[1], a[2], a[3]
        return name, P * C * (_es(gt) + 2 * _es(dt))
    if name == "unet_bn_bwd_reduce":            # da, y -> partial sums
        dt, gt, P, C = a[0], a[1], a[2], a[3]
        return name, P * C * (_es(gt) + _es(dt))
    if name in ("unet_bn_bwd_reduce_pool", "unet_bn_bwd_apply_pool"):
        dt, N, H, W, C, da, ph, pw = a[0], a[1], a[2], a[3], a[4], a[5], a[8], a[9]
        b = N * H * W * C * _es(dt) + (N * H * W * C * 4 if da else 0) + N * ph * pw * C * 5
        return name, b + (N * H * W * C * _es(dt) if name.endswith("apply_pool") else 0)
    if name == "unet_gate_bwd1":                # dxs, y_x, p (+dx) -> dx?, dq
        dt, P, C, dx, acc = a[0], a[1], a[2], a[12], a[13]
        return name, P * C * (4 + _es(dt)) + 8 * P + (P * C * 4 * (2 if acc else 1) if dx else 0)
    if name == "unet_gate_bwd2":
        dt, P, C = a[0], a[1], a[2]
        return name, 2 * P * C * _es(dt) + 8 * P
    if name == "unet_gate_bwd3":
        dt, P, C = a[0], a[1], a[2]
        return name, 4 * P * C * _es(dt) + 8 * P
    if name == "unet_gate_psi":
        dt, P, C = a[0], a[1], a[2]
        return name, 2 * P * C * _es(dt) + 4 * P
    if name == "unet_upsample_bwd":             # d_up (padded map) -> dx (source map)
        N, C, Hs, Ws, Hp, Wp, acc = a[0], a[1], a[2], a[3], a[8], a[9], a[14]
        return name, N * Hp * Wp * C * 4 + N * Hs * Ws * C * 4 * (2 if acc else 1)
    if name in ("unet_materialize", "unet_materialize_pool"):
        dt, src, N, H, W = a[0], a[1], a[2], a[3], a[4]
        b = N * src.H * src.W * src.C * _es(dt) + N * H * W * src.C * _es(dt)
        return name, b + (N * H * W * src.C if name.endswith("pool") else 0)
    if name == "unet_conv":
        from unet._hip.runtime import conv_kernel_name
        d = a[0]
        v = conv_kernel_name(d)
        fam = v.split("<")[0]
        if fam not in ("smallcin_fwd_kernel", "smallcin_fwd_mfma_kernel", "pw_conv_kernel"):
            return None
        P = d.N * d.H * d.W
        rd = sum(P * d.src[i].C * (4 if d.src[i].kind == 4 else _es(d.dtype)) for i in range(d.nsrc))
        if d.out_mode == 0:
            wr = P * d.Cout * _es(d.dtype)
        else:   # fp32 gradient (accumulated: read too); gated: + d(x*s) and p read
            wr = P * d.Cout * 4 * (2 if d.accum else 1) + (P * d.Cout * 4 + 4 * P if d.out_mode == 4 else 0)
        return fam + ("" if d.out_mode == 0 else "(dgrad)"), rd + wr
    return None


class HbmProbe:
    """Times the HBM-bound C-ABI calls of a step with HIP events on the launch stream (torch's current
    stream, where every call is issued) and adds up their algorithmic bytes, per kernel family."""

    def __init__(self):
        from unet._hip import lib as L
        self.L = L
        self.rec = []
        self.orig = None

    def __enter__(self):
        L, rec, orig = self.L, self.rec, self.L.call
        self.orig = orig

        def call(name, *args):
            fb = _hbm_bytes(name, args)
            if fb is None:
                return orig(name, *args)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = orig(name, *args)
            e.record()
            rec.append((fb[0], fb[1], s, e))
            return r

        L.call = call
        return self

    def __exit__(self, *exc):
        self.L.call = self.orig

    def summary(self, traffic: dict):
        torch.cuda.synchronize()
        agg = {}
        for fam, b, s, e in self.rec:
            t = agg.setdefault(fam, [0, 0.0, 0.0])
            t[0] += 1
            t[1] += b
            t[2] += s.elapsed_time(e) * 1e-3
        out = {}
        for fam, (n, b, sec) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
            gbs = b / sec / 1e9 if sec > 0 else None
            m = traffic.get(fam)
            out[fam] = {"launches": n, "algorithmic_bytes_per_launch": round(b / n),
                        "avg_us": round(sec / n * 1e6, 2), "GBs": round(gbs, 1) if gbs else None,
                        "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                        "measured_bytes_per_launch": m.get("bytes_per_launch") if isinstance(m, dict) else None}
        return out


def max_over_ranks(elapsed: float, device: torch.device) -> float:
    """The job's wall time: the slowest rank's timed region (all ranks get the same value)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed
    te = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(te, op=dist.ReduceOp.MAX)
    return float(te)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="attention_unet", choices=["attention_unet", "unet"])
    ap.add_argument("--batch", type=int, default=4, help="per-GPU batch")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--in-ch", type=int, default=1, help="input channels (C5: 3)")
    ap.add_argument("--accum", type=int, default=1, help="micro-batches per optimizer step (C5: 8; scripts/train.py:133-143)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="operand type; fp16 adds dynamic loss scaling (torch.amp.GradScaler), as C5 asks")
    ap.add_argument("--probe", default=None, help="kernel family to time live (default: conv_kernel<prec,3,64>)")
    ap.add_argument("--bucket-mb", type=float, default=25.0, help="DDP bucket_cap_mb (N>1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--no-fp32-line", action="store_true",
                    help="skip the fp32-operand (reference numerics) rate reported beside a 16-bit run at N=1")
    ap.add_argument("--no-graph-line", action="store_true",
                    help="skip the HIP-graph replay rate of the same step reported beside the eager one at N=1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # UNET_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one GPU (the driver's N>1 runs
    # use RCCL, one rank per GPU)
    backend = os.environ.get("UNET_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    # the device first: RCCL's communicator binds to the current device of the rank
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from unet._hip.runtime import probe
    from unet.models import AttentionUNet, UNet
    from unet.utils.loss import DiceBCELoss

    torch.manual_seed(0)
    model = (AttentionUNet(args.in_ch, 2) if args.model == "attention_unet" else UNet(args.in_ch, 2)).to(dev).train()
    model.hip_precision = args.precision
    net = model
    if world > 1:
        # stock torch DDP over RCCL: the HIP backward is one autograd node per reference module, so the
        # reducer all-reduces each full bucket while the remaining stages run (unet.utils.distributed)
        from unet.utils.distributed import wrap_ddp
        net = wrap_ddp(model, local if backend == "nccl" else None, bucket_cap_mb=args.bucket_mb,
                       broadcast_buffers=False)
    opt = torch.optim.AdamW(model.parameters(), lr=5e-5, weight_decay=1e-4, fused=True)
    # fp16 operands: dynamic loss scaling as torch.amp prescribes for fp16 training (SURVEY §5 mixed
    # precision); gradients are unscaled before the clip (scripts/train.py:136-141 order)
    scaler = torch.amp.GradScaler("cuda", enabled=args.precision == "fp16")
    crit = DiceBCELoss()
    gen = torch.Generator().manual_seed(1234 + rank)
    x = (torch.rand(args.batch, args.in_ch, args.size, args.size, generator=gen) * 2 - 1).to(dev)
    t = disc_targets(args.batch, args.size, args.size, gen).to(dev)
    params = list(model.parameters())

    def step():
        # grad accumulation as scripts/train.py:133-143: loss / accum per micro-batch, gradients
        # all-reduced once per optimizer step (DDP no_sync on the first accum-1 micro-batches)
        for k in range(args.accum):
            last = k == args.accum - 1
            ctx = net.no_sync() if (world > 1 and not last) else contextlib.nullcontext()
            with ctx:
                loss = crit(net(x), t)
                scaler.scale(loss / args.accum if args.accum > 1 else loss).backward()
        scaler.unscale_(opt)
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        scaler.step(opt)
        scaler.update()
        opt.zero_grad(set_to_none=True)
        return loss

    def timed(fn, steps):
        """barrier + synchronize on both sides; the slowest rank's wall time"""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return max_over_ranks(time.perf_counter() - t0, dev), out

    for _ in range(args.warmup):
        step()
    elapsed, loss = timed(step, args.steps)          # the headline: no probe events inside
    final_loss = round(float(loss.detach()), 5)
    del loss     # the last step's autograd graph (its AccumulateGrad nodes) must not outlive the step

    # the dominant kernel family, timed live in a separate pass of the same steps: every 16-bit 3x3 conv
    # launch (fwd + dgrad; the 32x32x16-MFMA conv5_kernel tiles on the large maps, their 128-output-channel
    # conv5w_kernel form (round 6) where it serves, and the 16x16x32 conv3_kernel tiles on the rest, prefix match)
    tn = {"bf16": "bf16", "fp16": "fp16"}.get(args.precision)
    family = (f"conv3_kernel<{tn},3,", f"conv5_kernel<{tn},", f"conv5w_kernel<{tn}") if tn else ("conv2_kernel<fp32,3,",)
    if args.probe:
        family = (args.probe,)
    target = "|".join(family)
    probe.enable(family)
    timed(step, max(2, min(args.steps, 10)))
    probe.disable()
    ps = probe.summary()
    # the HBM-bound kernels (BN backward passes, gate backward, upsample backward, materialised pool /
    # upsample, first conv, 1x1 convs): algorithmic bytes / HIP-event time, in a separate pass
    with HbmProbe() as hp:
        timed(step, 2)

    # SURVEY §8(d) also asks for the rate without the optimizer: the same fwd + loss + bwd (+ gradient
    # averaging) micro-steps, gradients dropped instead of clip + AdamW (reported beside `value`)
    def fwd_bwd():
        for k in range(args.accum):
            last = k == args.accum - 1
            ctx = net.no_sync() if (world > 1 and not last) else contextlib.nullcontext()
            with ctx:
                l = crit(net(x), t)
                scaler.scale(l / args.accum if args.accum > 1 else l).backward()
        opt.zero_grad(set_to_none=True)

    fwd_bwd()
    el_nb, _ = timed(fwd_bwd, args.steps)

    images = world * args.batch * args.accum * args.steps
    value = images / elapsed
    peak = MFMA_PEAK_TFLOPS[args.precision]
    achieved = ps["tflops"] or 0.0
    traffic = None
    tr = {}
    tfile = ROOT / "profiles" / "traffic.json"
    if tfile.exists():
        tr = json.loads(tfile.read_text())
        # the un-suffixed key is the AttentionUNet headline's; a UNet line (C2) has its own "@unet" key or none
        ent = tr.get(f"{target}@{args.size}x{args.in_ch}") or (
            tr.get(target) if args.model == "attention_unet" else tr.get(f"{target}@unet"))
        traffic = ent.get("bytes_per_launch") if isinstance(ent, dict) else ent
    headline = (args.size, args.in_ch, args.accum, args.model) == (512, 1, 1, "attention_unet")
    metric = METRIC if headline else (
        f"{args.size}x{args.size} {args.in_ch}-ch slices/sec fwd+bwd, {'AttentionUNet' if args.model == 'attention_unet' else 'UNet'} "
        f"bs={args.batch}/GPU x grad-accum {args.accum}, {args.precision}, 1/2/4/8 MI355X")
    fpi = FLOPS_PER_IMAGE[args.model] if (args.size, args.in_ch) == (512, 1) else (
        FLOPS_PER_IMAGE_C5 if (args.size, args.in_ch, args.model) == (1024, 3, "attention_unet") else None)
    line = {
        "metric": metric,
        "value": round(value, 3), "unit": "img/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision, "data": "synthetic (x~U(-1,1), 1-3 disc masks/img; seeded)",
        "config": {"workload": f"{args.model} {args.in_ch}x{args.size}x{args.size} train step "
                               f"(fwd+DiceBCE+bwd{' x%d accum' % args.accum if args.accum > 1 else ''}+clip+AdamW"
                               f"{'; GradScaler' if scaler.is_enabled() else ''})",
                   "model": args.model, "global_batch": world * args.batch * args.accum, "per_gpu_batch": args.batch,
                   "grad_accum": args.accum, "image": [args.in_ch, args.size, args.size],
                   "parallelism": f"dp{world}" if world > 1 else "single",
                   "grad_sync": f"torch DDP ({backend}, bucket {args.bucket_mb:g} MB)" if world > 1 else None},
        "whole_step_tflops": round(value * fpi / 1e12, 2) if fpi else None,
        "roofline": {"kernel": target, "bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_unit": "HBM bytes/launch (rocprofv3 PMC, profiles/traffic.json)",
                     "launches": ps["launches"], "avg_us": round(ps["avg_us"], 2) if ps["avg_us"] else None,
                     "flops_per_launch": round(ps["flops"] / ps["launches"]) if ps["launches"] else None,
                     "timed": "separate probe pass (HIP events on the launch stream), not the headline loop"},
        "hbm": {"peak": HBM_PEAK_GBS, "unit": "GB/s", "kernels": hp.summary(tr),
                "note": "algorithmic bytes (each operand read once, each output written once) / HIP-event time "
                        "per launch, separate pass; measured_bytes_per_launch: rocprofv3 FETCH_SIZE x2 + "
                        "WRITE_SIZE (profiles/traffic.json)"},
        "final_loss": final_loss,
        "without_optimizer": {"value": round(world * args.batch * args.accum * args.steps / el_nb, 3),
                              "ms_per_step": round(el_nb / args.steps * 1e3, 3),
                              "note": "fwd+DiceBCE+bwd (+grad averaging), no clip/AdamW"},
    }
    if scaler.is_enabled():
        line["loss_scale"] = float(scaler.get_scale())
    if world == 1 and args.accum == 1 and not scaler.is_enabled() and not args.no_graph_line:
        # the same step (fwd + DiceBCE + bwd + clip + AdamW) captured once as a HIP graph and replayed
        # (unet.utils.graphed.GraphedTrainStep): identical kernels, one host launch per step
        from unet.utils.graphed import GraphedTrainStep
        gopt = torch.optim.AdamW(model.parameters(), lr=5e-5, weight_decay=1e-4, fused=True, capturable=True)
        gs = GraphedTrainStep(model, crit, gopt, x.shape, t.shape, target_dtype=t.dtype, clip_norm=1.0)
        for _ in range(3):
            gs(x, t)
        elg, _ = timed(lambda: gs(x, t), args.steps)
        line["graphed_step"] = {"value": round(args.batch * args.steps / elg, 3),
                                "ms_per_step": round(elg / args.steps * 1e3, 3),
                                "note": "same train step replayed as one HIP graph (GraphedTrainStep)"}
        del gs, gopt
    if world == 1 and args.precision != "fp32" and not args.no_fp32_line:
        # the same step with fp32 operands (the reference's numerics; what the parity tests pin)
        model.hip_precision = "fp32"
        scaler = torch.amp.GradScaler("cuda", enabled=False)
        step()
        n32 = max(2, min(args.steps, 5))
        el32, _ = timed(step, n32)
        line["fp32_operands"] = {"value": round(args.batch * args.accum * n32 / el32, 3),
                                 "ms_per_step": round(el32 / n32 * 1e3, 3), "steps": n32}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.model, args.size, args.cpu_batch, args.cpu_iters)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
