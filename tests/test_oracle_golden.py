"""Pin the CPU oracle (oracle/pntf_oracle.py) to the reference's own outputs.

The golden vectors were produced by importing yhsong0804/P-NTFields itself
(tests/golden/make_goldens.py) with the seeded weights of pntf.synth.  Tolerances: the
reference runs fp32, the oracle fp64, so agreement is at the fp32 rounding level.
"""
import numpy as np
import pytest

from golden_util import load, max_rel, rel_l2, weight_checksum, weights
from oracle import pntf_oracle as O
from pntf import synth

TOL = 1e-5   # fp64 oracle vs fp32 reference


@pytest.fixture(scope="module")
def W():
    return weights()


def test_weights_regenerate_bit_exact(W):
    for name in ("fwd_grad_d3.npz", "loss_d3.npz", "plan_gib.npz", "fwd_grad_d6.npz"):
        np.testing.assert_array_equal(weight_checksum(W), load(name)["weight_checksum"])


def test_inputs_regenerate():
    f = load("fwd_grad_d3.npz")
    np.testing.assert_array_equal(f["xp"], synth.make_pairs(1024, 3, seed=2))
    np.testing.assert_array_equal(f["B"], synth.make_B(3, seed=1))


def test_tau_and_exact_grad(W):
    f = load("fwd_grad_d3.npz")
    t, d = O.tau_grad(W, f["xp"], f["B"])
    assert rel_l2(t, f["tau"]) < TOL
    assert rel_l2(d, f["dtau"]) < TOL           # Model.gradient autograd
    assert rel_l2(d, f["dtau_fwdmode"]) < TOL   # NN.out_grad forward mode


def test_backgrad_compat_quirk(W):
    f = load("fwd_grad_d3.npz")
    t, d = O.tau_grad(W, f["xp"], f["B"], compat=True)
    assert rel_l2(t, f["tau_backgrad"]) < TOL
    assert rel_l2(d, f["dtau_backgrad"]) < TOL
    # the quirk is real: out_backgrad is not the true gradient
    assert rel_l2(f["dtau_backgrad"], f["dtau"]) > 0.1


def test_epilogues(W):
    f = load("fwd_grad_d3.npz")
    t, d = O.tau_grad(W, f["xp"], f["B"])
    tc, dc = O.tau_grad(W, f["xp"], f["B"], compat=True)
    assert rel_l2(O.path_velocity(f["xp"], tc, dc), f["gradient"]) < TOL
    assert rel_l2(O.speed(f["xp"], t, d), f["speed"]) < TOL
    assert rel_l2(O.travel_time(f["xp"], t), f["travel_time"]) < TOL


def test_env_table(W):
    g = load("fwd_grad_env_d3.npz")
    t, d = O.tau_grad(W, g["xp"], g["B_table"], g["env"])
    assert rel_l2(t, g["tau"]) < TOL and rel_l2(d, g["dtau"]) < TOL
    _, dc = O.tau_grad(W, g["xp"], g["B_table"], g["env"], compat=True)
    assert rel_l2(dc, g["dtau_backgrad"]) < TOL


def test_laplace_and_loss(W):
    f = load("loss_d3.npz")
    E, n, _ = f["pts"].shape
    xp = f["pts"].reshape(-1, 6)
    env = np.repeat(np.arange(E), n)
    tau, dtau, ltau, diff = O.eikonal_residual(W, xp, f["yobs"].reshape(-1, 2), f["B_table"],
                                               env, gamma=float(f["gamma"]))
    assert rel_l2(tau, f["tau"].reshape(-1, 1)) < TOL
    assert rel_l2(dtau, f["dtau"].reshape(-1, 6)) < TOL
    assert rel_l2(ltau, f["ltau"].reshape(-1, 6)) < 1e-4
    assert rel_l2(diff, f["diff"].reshape(-1)) < 1e-4
    assert abs(O.loss_n(diff, f["B_table"], E, n) - float(f["loss_n"])) < 1e-5


def test_gibson_planner(W):
    p = load("plan_gib.npz")
    path, steps = O.plan(W, p["starts"], p["B"], step=0.03, tol=0.06, max_iter=500,
                         compat=True)
    np.testing.assert_array_equal(steps, p["iters"])
    assert np.abs(path - p["paths"]).max() < 1e-5


def test_arm(W):
    a = load("fwd_grad_d6.npz")
    t, d = O.tau_grad(W, a["xp"], a["B"].T, dim=6)
    assert rel_l2(t, a["tau"]) < TOL and rel_l2(d, a["dtau"]) < TOL
    v = O.path_velocity(a["xp"][:16], t[:16], d[:16], dim=6)
    assert max_rel(v, a["gradient16"], 1e-3) < 1e-4


def test_arm_planner(W):
    p = load("plan_arm.npz")
    path, steps = O.plan(W, p["starts"], p["B"].T, dim=6, step=0.015, tol=0.03, max_iter=300,
                         compat=False)
    np.testing.assert_array_equal(steps, p["iters"])
    assert np.abs(path - p["paths"]).max() < 1e-5


def test_planner_cap_semantics(W):
    """iter > max_iter break => at most max_iter + 1 updates (test/gib_plan.py:83-86)."""
    xp0 = synth.make_pairs(4, 3, seed=11)
    B = synth.make_B(3, seed=1)
    path, steps = O.plan(W, xp0, B, step=1e-4, tol=1e-9, max_iter=3, compat=True)
    assert path.shape == (4, 5, 6)
    np.testing.assert_array_equal(steps, [4, 4, 4, 4])


def test_arm_laplace_and_loss_variant(W):
    f = load("loss_d6.npz")
    B = f["B"].T
    tau, dtau, ltau, diff = O.eikonal_residual_arm(W, f["pts"], f["yobs"], B, dim=6,
                                                   gamma=float(f["gamma"]))
    assert rel_l2(tau, f["tau"]) < TOL
    assert rel_l2(dtau, f["dtau"]) < TOL
    assert rel_l2(ltau, f["ltau"]) < 1e-4
    assert rel_l2(diff, f["diff"]) < 1e-4
    assert abs(diff.sum() / len(diff) - float(f["loss_n"])) < 1e-5


@pytest.mark.parametrize("name", ["fwd_grad_d3.npz", "fwd_grad_env_d3.npz", "fwd_grad_d6.npz"])
def test_torch_ref_cpu_baseline_vs_reference(W, name):
    """oracle/torch_ref.py (the op sequence bench.py times as cpu_baseline) reproduces the
    reference's NN.out + Model.gradient outputs: single B, per-pair env table, and the arm
    (dim 6, B.T).  fp32 on both sides, same torch CPU kernels: agreement at rounding level."""
    from oracle.torch_ref import TorchRef
    f = load(name)
    ref = TorchRef(W)
    if name == "fwd_grad_d6.npz":
        t, d = ref.tau_grad(f["xp"], f["B"].T)
    elif "B_table" in f.files:
        t, d = ref.tau_grad(f["xp"], f["B_table"], f["env"])
    else:
        t, d = ref.tau_grad(f["xp"], f["B"])
    assert rel_l2(t.numpy(), f["tau"].reshape(-1)) < TOL
    assert rel_l2(d.numpy(), f["dtau"]) < TOL
    if "B_table" in f.files:
        # the labelled per-pair gather form agrees too (it is only slower)
        tg, dg = ref.tau_grad_gather(f["xp"], f["B_table"], f["env"])
        assert rel_l2(tg.numpy(), f["tau"].reshape(-1)) < TOL
        assert rel_l2(dg.numpy(), f["dtau"]) < TOL


def test_torch_ref_per_env_calls_are_the_single_b_calls(W):
    """The per-env split is exactly one single-B NN.out + Model.gradient call per env:
    contiguous env blocks (the bench's layout) give bitwise the rows of those calls."""
    from oracle.torch_ref import TorchRef, env_groups
    ref = TorchRef(W)
    xp = synth.make_pairs(300, 3, seed=2)
    Bt = synth.make_B_table(3, 3)
    env = synth.make_env_ids(300, 3)
    groups = env_groups(env)
    assert [g[0] for g in groups] == [0, 1, 2]
    assert all(isinstance(g[1], slice) for g in groups)
    t, d = ref.tau_grad(xp, Bt, env)
    for e, rows in groups:
        te, de = ref.tau_grad(xp[rows], Bt[e])
        assert np.array_equal(t.numpy()[rows], te.numpy())
        assert np.array_equal(d.numpy()[rows], de.numpy())
    f = load("fwd_grad_env_d3.npz")              # interleaved ids -> gathered groups
    assert all(not isinstance(g[1], slice) for g in env_groups(f["env"]))
