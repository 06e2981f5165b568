"""Diagnostic (GPU): round 3's GraphedTrainStep capture path (warm-up + capture running loss.backward()) built
while the previous eager step's loss, and with it the parameters' AccumulateGrad nodes created on the default
stream, is still alive.  Round 3's bench crashed here (gpurun_out/r03w5b).  Prints how far it gets; run it as
a child process under `timeout` with PYTHONFAULTHANDLER=1 so a segfault prints the Python stack.

  python tools/repro_graphed_live_graph.py [backward|grad]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet.models import AttentionUNet  # noqa: E402
from unet.utils.loss import DiceBCELoss  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "backward"
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=16).cuda().train()
    m.hip_precision = "bf16"
    params = list(m.parameters())
    opt = torch.optim.AdamW(params, lr=1e-3, fused=True, capturable=True)
    crit = DiceBCELoss()
    x = torch.rand(2, 1, 128, 128, device="cuda") * 2 - 1
    t = (torch.rand(2, 128, 128, device="cuda") < 0.1).long()

    def body():
        loss = crit(m(x), t)
        if mode == "backward":
            loss.backward()
        else:
            for p, g in zip(params, torch.autograd.grad(loss, params, allow_unused=True)):
                p.grad = g
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        return loss.detach()

    live = crit(m(x), t)          # the eager step whose graph stays alive
    live.backward()
    opt.step()
    torch.cuda.synchronize()
    print("eager step done; loss kept alive", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            opt.zero_grad(set_to_none=True)
            body()
            print(f"side-stream warm-up {i} done", flush=True)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    opt.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    print("capturing", flush=True)
    with torch.cuda.graph(g):
        out = body()
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"replayed: loss {float(out):.6f}; live loss {float(live):.6f}", flush=True)


if __name__ == "__main__":
    main()
