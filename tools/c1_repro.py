"""C1 reproducibility probe (diagnostic): HIP fp32 member 0 of the overfit protocol (tools/overfit_diag.py), run
fresh, again in the same process, and after a 16-epoch HIP + oracle run (the test file's order); prints the
last-epoch Tumor-Dice and a digest of the per-epoch losses, so two trees / contexts can be compared bit for bit."""
import hashlib
import struct
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import torch  # noqa: E402
import overfit_diag as D  # noqa: E402


def digest(hist):
    return hashlib.sha1(b"".join(struct.pack("<dd", l, d) for l, d in hist)).hexdigest()[:16]


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    init, names, x, t = D.setup()
    for tag in ("fresh", "again"):
        h = D.run_hip(init, x, t, epochs, 64)
        print(f"{tag}: last dice {h[-1][1]:.6f} loss {h[-1][0]:.7f} digest {digest(h)} epoch16 {digest(h[:16])}", flush=True)
    D.run_hip(init, x, t, 16, 64)
    D.run_oracle(init, names, x, t, 16, torch.float32)
    h = D.run_hip(init, x, t, epochs, 64)
    print(f"after-16: last dice {h[-1][1]:.6f} loss {h[-1][0]:.7f} digest {digest(h)} epoch16 {digest(h[:16])}", flush=True)


if __name__ == "__main__":
    main()
