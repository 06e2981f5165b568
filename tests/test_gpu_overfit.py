"""Overfit parity at BASELINE C1 as the reference runs it (scripts/overfit_test.py:126-208; north_star
"Tumor-Dice on the overfit_test set matching reference +-1e-3"): AttentionUNet(1, 2, deep_supervision=True),
base 64, a fixed batch of 2 x 1 x 512^2, Adam(lr=1e-3), DeepSupervisionLoss(DiceBCELoss, [1, .4, .2, .1]); each
epoch one optimizer step, then an eval-mode (running-statistics) forward and Tumor Dice 2|P n G| / (|P| + |G|)
on argmax(softmax) (:182-205).  The reference's statistic is the LAST epoch's Dice (:218, :288).

Executions, all from the same seeded weights and batch (tools/overfit_diag.py):
  * the HIP path (fp32 operand mode);
  * the reference's network as the oracle's ATen ops in fp32 on the same GPU (the reference script runs on
    `cuda` when one is present, overfit_test.py:88), once from the seeded weights and twice more from weights
    perturbed by one ulp in a random half of their elements (the size of the rounding difference any other
    correct fp32 execution — another kernel, another box — makes in the first step);
  * the same in fp64: the box-independent yardstick.
What the trajectory can and cannot pin (measured, DESIGN.md §5, profiles/r05_overfit_c1_*.txt): Adam at lr 1e-3
makes the loop chaotic — the parameter distance between any two of the three executions grows from ~1e-3 after
the first step to ~1e-1 by epoch 100, at the same rate for HIP-vs-fp64 as for the reference's own fp32-vs-fp64
— and under a one-ulp perturbation of its initial weights the reference's own fp32 run ended at last-epoch Dice
0.9909 ... 0.9996 (5 runs).  So the deterministic parts are pinned exactly, and the chaotic statistic against the
reference's own measured spread:
  * test_overfit_c1_eval_and_step_pins: the oracle's own states at epochs 16, 100 and 200 loaded into the HIP
    model — the eval forward gives the same labels (any difference only at near ties |z1 - z0| < 1e-4, counted)
    hence the same Tumor-Dice, and one training step from each state has the reference's loss and gradients no
    further from fp64 than the reference's own fp32 step (3x + 1e-5);
  * test_overfit_c1_tumor_dice_vs_reference_spread: the first 16 epochs step for step;
  * test_overfit_c1_full_protocol_final_dice: 200 epochs; the last-epoch Tumor-Dice within
    max(1e-3, max_k |ref32_k - ref64|) of the fp64 oracle's, the bound measured in the same test."""

import contextlib
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

EPOCHS = 16
PINS = (16, 100, 200)


def _tools():
    root = Path(__file__).resolve().parent.parent
    if str(root / "tools") not in sys.path:
        sys.path.insert(0, str(root / "tools"))
    import overfit_diag
    return overfit_diag


@pytest.fixture(scope="module")
def c1():
    D = _tools()
    init, names, x, t = D.setup()
    return D, init, names, x, t


def test_overfit_c1_tumor_dice_vs_reference_spread(c1):
    """The first 16 epochs (Dice rises from 0.01 to ~0.97): at every epoch our Tumor-Dice and loss are within
    max(1e-3, 1.5 S) of the fp32 reference, S the reference's own largest fp32-vs-fp64 spread in that window."""
    D, init, names, x, t = c1
    hip = D.run_hip(init, x, t, EPOCHS, 64)
    r32 = D.run_oracle(init, names, x, t, EPOCHS, torch.float32)
    r64 = D.run_oracle(init, names, x, t, EPOCHS, torch.float64)
    print("\nepoch loss_hip loss_ref32 loss_ref64 | dice_hip dice_ref32 dice_ref64")
    for i in range(EPOCHS):
        print(i, *("%.6f" % v for v in (hip[i][0], r32[i][0], r64[i][0], hip[i][1], r32[i][1], r64[i][1])))
    s_dice = max(abs(a[1] - b[1]) for a, b in zip(r32, r64))
    s_loss = max(abs(a[0] - b[0]) / abs(b[0]) for a, b in zip(r32, r64))
    d_dice = max(abs(a[1] - b[1]) for a, b in zip(hip, r32))
    d_loss = max(abs(a[0] - b[0]) / abs(b[0]) for a, b in zip(hip, r32))
    print(f"reference fp32-vs-fp64 spread: dice {s_dice:.2e}, loss rel {s_loss:.2e}; "
          f"HIP-vs-reference fp32: dice {d_dice:.2e}, loss rel {d_loss:.2e}")
    assert abs(hip[0][0] - r32[0][0]) <= 1e-5 * abs(r32[0][0])       # first step: same weights, fp32 noise
    assert d_dice <= max(1e-3, 1.5 * s_dice), (d_dice, s_dice)
    assert d_loss <= max(1e-4, 1.5 * s_loss), (d_loss, s_loss)
    assert hip[-1][1] > 0.8 and r32[-1][1] > 0.8 and r64[-1][1] > 0.8


@pytest.fixture(scope="module")
def c1_full(c1, request):
    D, init, names, x, t = c1
    # five 200-epoch executions (minutes): with pytest's output capture suspended, so their progress lines
    # (tools/overfit_diag.py) reach the runner's log while they run
    cm = request.config.pluginmanager.getplugin("capturemanager")
    with cm.global_and_fixture_disabled() if cm is not None else contextlib.nullcontext():
        hip = D.run_hip(init, x, t, 200, 64)
        r32, snaps = D.run_oracle(init, names, x, t, 200, torch.float32, snap=set(PINS))
        r32p = [D.run_oracle(D.perturb(init, names, s), names, x, t, 200, torch.float32) for s in (1, 2)]
        r64 = D.run_oracle(init, names, x, t, 200, torch.float64)
    return hip, [r32] + r32p, r64, snaps


def test_overfit_c1_eval_and_step_pins(c1, c1_full):
    """The HIP eval forward and one HIP training step from the oracle's own states (epochs 16, 100, 200)."""
    D, init, names, x, t = c1
    _, refs, _, snaps = c1_full
    for e in PINS:
        dh, do, nd, nt, dz = D.eval_pin(snaps[e], x, t)
        lh, l32, l64, gh, g32, bh, b32 = D.step_pin(snaps[e], names, x, t)
        print(f"\nepoch {e}: trajectory dice {refs[0][e - 1][1]:.6f}; eval forward of the oracle's state: HIP {dh:.6f}, "
              f"oracle {do:.6f}, labels differing {nd} (near ties {nt}), max|dlogit| {dz:.2e}; train step: loss HIP "
              f"{lh:.7f} fp32 {l32:.7f} fp64 {l64:.7f}, grad rel-L2 vs fp64 HIP {gh:.3e} / oracle fp32 {g32:.3e}, "
              f"running buffers HIP {bh:.3e} / fp32 {b32:.3e}")
        assert nd == nt, (e, nd, nt)                     # labels identical except at near ties
        assert abs(dh - do) <= 2.0 * nd / float((t == 1).sum()) + 1e-12, (e, dh, do)
        assert do == refs[0][e - 1][1]                   # the eval forward the trajectory itself measured
        assert abs(lh - l64) <= 1e-5 * abs(l64), (e, lh, l64)
        assert gh <= 3.0 * g32 + 1e-5, (e, gh, g32)
        assert bh <= 3.0 * b32 + 1e-7, (e, bh, b32)


def test_overfit_c1_full_protocol_final_dice(c1, c1_full):
    """The reference's whole protocol (200 epochs, overfit_test.py:69) and its statistic, the last epoch's
    Tumor-Dice (overfit_test.py:218,288): within max(1e-3, S) of the fp64 oracle's, S = the largest
    |ref32_k - ref64| over the reference's fp32 executions (seeded + two one-ulp perturbations) in this test."""
    hip, refs, r64, _ = c1_full
    print("\nlast 10 epochs: dice_hip dice_ref64 | dice_ref32 (seeded, perturbed 1, perturbed 2)")
    for i in range(190, 200):
        print(i, "%.6f %.6f |" % (hip[i][1], r64[i][1]), " ".join("%.6f" % r[i][1] for r in refs))
    last = hip[-1][1]
    spread = max(abs(r[-1][1] - r64[-1][1]) for r in refs)
    bound = max(1e-3, spread)
    print(f"last epoch: HIP {last:.6f}, reference fp64 {r64[-1][1]:.6f}, reference fp32 "
          f"{' / '.join('%.6f' % r[-1][1] for r in refs)}; |HIP - fp64| {abs(last - r64[-1][1]):.2e}, "
          f"bound max(1e-3, fp32 spread {spread:.2e}) = {bound:.2e}")
    assert abs(last - r64[-1][1]) <= bound, (last, r64[-1][1], bound)
    assert last > 0.8 and r64[-1][1] > 0.8 and all(r[-1][1] > 0.8 for r in refs)   # overfit_test.py:288
