"""Diagnostic: one HIP fp32 training step of the C1 model (tools/overfit_diag.py setup) with the outputs, the loss and
every parameter gradient saved to argv[1] (torch.save of a dict of CPU tensors), so two trees can be compared bit for
bit (python tools/c1_step_dump.py cmp a.pt b.pt)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import torch  # noqa: E402


def dump(path):
    import overfit_diag as D
    init, names, x, t = D.setup()
    h = D.Hip(init, x, t)
    out = h.m(h.x)
    rec = {f"out{i}": o.detach().float().cpu() for i, o in enumerate(out)}
    loss = h.crit(out, h.t)
    loss.backward()
    rec["loss"] = loss.detach().float().cpu()
    for k, p in h.m.named_parameters():
        rec["grad." + k] = p.grad.detach().float().cpu()
    for k, v in h.m.state_dict().items():
        if "running" in k:
            rec["buf." + k] = v.detach().float().cpu()
    h.opt.step()
    torch.save(rec, path)


def cmp(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    for k in A:
        d = (A[k] - B[k]).abs()
        n = int((A[k].view(torch.int32) != B[k].view(torch.int32)).sum())
        if n:
            print(f"{k:60s} differ {n}/{A[k].numel()} max|d| {float(d.max()):.3e}")
    print("compared", len(A))


if __name__ == "__main__":
    if sys.argv[1] == "cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
