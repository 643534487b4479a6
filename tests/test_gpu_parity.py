"""HIP path (libpntf.so through the C ABI / drop-in models) vs the reference goldens and
the CPU oracle.

Tolerance (BASELINE.json north_star): τ and ∇τ within 1e-4 relative (fp32) of the
reference — checked as relative L2 over the batch AND as the max abs error over the max
|value| — and, elementwise, every value within ELEM relative of the reference's, with
relative error measured against max(|ref|, ELEM_FLOOR · max|ref|): a component of ∇τ that is
off by 10 % or more fails unless it is below 1e-3 of the batch's largest component (where the
fp32 reference itself carries ~1e-4 relative noise: oracle fp64 vs reference 1.4e-4).
Planner endpoints within 1e-3 of the reference's batch-1 loop.
"""
import numpy as np
import pytest
import torch

from golden_util import fp64_of, load, max_rel, north_star_pairs, rel_l2, weights
from oracle import pntf_oracle as O
from pntf import ops, synth

pytestmark = pytest.mark.gpu

REL = 1e-4
ELEM = 1e-3
ELEM_FLOOR = 1e-2


def close(a, b, tol=REL, elem=ELEM, pairs=False, diff=False):
    """Normwise and elementwise bounds (module docstring); pairs=True adds the north star per
    pair against `b`, which is then the fp64 oracle itself (diff: the Eikonal residual,
    relative to |diff| + 4)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    l2 = rel_l2(a, b)
    scale = max(np.abs(b).max(), 1e-30)
    mx = float(np.abs(a - b).max() / scale)
    el = max_rel(a, b, ELEM_FLOOR * scale)
    assert l2 < tol and mx < tol and el < elem, \
        "rel_l2=%.3g max=%.3g elementwise=%.3g (tol %.1g, elem %.1g)" % (l2, mx, el, tol, elem)
    if pairs:
        north_star_pairs("vs fp64 oracle", a, b, b, diff=diff)


def check(got, name, key, **kw):
    """`got` against the reference golden `name`[`key`]: close() (normwise and elementwise)
    and the north star per pair — each pair within 1e-4 of the reference's fp32 value, or,
    where that value is itself >= 1e-4 from exact, within 1e-4 of the fp64 oracle on the same
    inputs (golden_util.north_star_pairs)."""
    ref = np.asarray(load(name)[key], np.float64)
    got = np.asarray(got, np.float64).reshape(ref.shape)
    close(got, ref, **kw)
    north_star_pairs("%s[%s]" % (name, key), got, ref, fp64_of(name)[key], diff=(key == "diff"))


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def W():
    return weights()


@pytest.fixture(scope="module")
def packed(W, dev):
    params = [torch.from_numpy(v).to(dev) for v in W.values()]
    return ops.pack_weights(params)


@pytest.fixture(params=["wave_tile", "split_tile", "wide_tile", "quad_tile"])
def field_schedule(request):
    """Run a field test with one wave per 16-pair tile, with split tiles (pntf_split.h), with
    one wave per 32-pair tile (pntf_wide.h) and with 4-pair quad tiles (pntf_quad.h); the
    schedule is passed per call (pntf_field_ex), no library state changes."""
    return request.param


def T(a, dev, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dtype)


def test_tau_grad_exact_vs_reference(packed, dev, field_schedule):
    f = load("fwd_grad_d3.npz")
    t, d = ops.tau_grad(packed, T(f["xp"], dev), T(f["B"], dev), dim=3, mode=ops.GRAD_EXACT, schedule=field_schedule)
    check(t.detach().cpu().numpy(), "fwd_grad_d3.npz", "tau")
    check(d.detach().cpu().numpy(), "fwd_grad_d3.npz", "dtau")
    check(d.detach().cpu().numpy(), "fwd_grad_d3.npz", "dtau_fwdmode")


def test_tau_only_kernel(packed, dev, field_schedule):
    f = load("fwd_grad_d3.npz")
    t = ops.tau(packed, T(f["xp"], dev), T(f["B"], dev), dim=3, schedule=field_schedule)
    check(t.detach().cpu().numpy(), "fwd_grad_d3.npz", "tau")


def test_backgrad_compat_vs_reference(packed, dev, field_schedule):
    f = load("fwd_grad_d3.npz")
    t, d = ops.tau_grad(packed, T(f["xp"], dev), T(f["B"], dev), dim=3,
                        mode=ops.GRAD_BACKGRAD_COMPAT, schedule=field_schedule)
    check(t.detach().cpu().numpy(), "fwd_grad_d3.npz", "tau_backgrad")
    check(d.detach().cpu().numpy(), "fwd_grad_d3.npz", "dtau_backgrad")


def test_epilogues_vs_reference(packed, dev, field_schedule):
    f = load("fwd_grad_d3.npz")
    xp, B = T(f["xp"], dev), T(f["B"], dev)
    v, _ = ops.path_velocity(packed, xp, B, dim=3, mode=ops.GRAD_BACKGRAD_COMPAT, schedule=field_schedule)
    check(v.detach().cpu().numpy(), "fwd_grad_d3.npz", "gradient")
    check(ops.speed(packed, xp, B, dim=3, schedule=field_schedule).detach().cpu().numpy(), "fwd_grad_d3.npz", "speed")
    check(ops.travel_time(packed, xp, B, dim=3, schedule=field_schedule).detach().cpu().numpy(), "fwd_grad_d3.npz", "travel_time")


def test_env_table_vs_reference(packed, dev, field_schedule):
    g = load("fwd_grad_env_d3.npz")
    xp, Bt, env = T(g["xp"], dev), T(g["B_table"], dev), T(g["env"], dev, torch.int32)
    t, d = ops.tau_grad(packed, xp, Bt, env, dim=3, schedule=field_schedule)
    check(t.detach().cpu().numpy(), "fwd_grad_env_d3.npz", "tau")
    check(d.detach().cpu().numpy(), "fwd_grad_env_d3.npz", "dtau")
    _, dc = ops.tau_grad(packed, xp, Bt, env, dim=3, mode=ops.GRAD_BACKGRAD_COMPAT, schedule=field_schedule)
    check(dc.detach().cpu().numpy(), "fwd_grad_env_d3.npz", "dtau_backgrad")


def test_arm_dim6_vs_reference(packed, dev, field_schedule):
    a = load("fwd_grad_d6.npz")
    xp, B = T(a["xp"], dev), T(a["B"].T, dev)
    t, d = ops.tau_grad(packed, xp, B, dim=6, schedule=field_schedule)
    check(t.detach().cpu().numpy(), "fwd_grad_d6.npz", "tau")
    check(d.detach().cpu().numpy(), "fwd_grad_d6.npz", "dtau")
    v, _ = ops.path_velocity(packed, xp[:16], B, dim=6, mode=ops.GRAD_EXACT, schedule=field_schedule)
    check(v.detach().cpu().numpy(), "fwd_grad_d6.npz", "gradient16")


@pytest.mark.parametrize("n", [1, 15, 16, 17, 33, 1000, 4099])
def test_ragged_batches_vs_oracle(packed, dev, W, field_schedule, n):
    xp = synth.make_pairs(n, 3, seed=100 + n)
    Bt = synth.make_B_table(3, 3, first_seed=20)
    env = synth.make_env_ids(n, 3, contiguous=False, seed=n)
    t, d = ops.tau_grad(packed, T(xp, dev), T(Bt, dev), T(env, dev, torch.int32), dim=3, schedule=field_schedule)
    to, do = O.tau_grad(W, xp, Bt, env)
    close(t.detach().cpu().numpy(), to[:, 0], pairs=True)
    close(d.detach().cpu().numpy(), do, pairs=True)


def test_empty_batch(packed, dev):
    xp = torch.zeros((0, 6), device=dev)
    t, d = ops.tau_grad(packed, xp, T(synth.make_B(3), dev), dim=3)
    assert t.shape == (0,) and d.shape == (0, 6)


def test_invalid_env_gives_nan(packed, dev, field_schedule):
    xp = synth.make_pairs(20, 3, seed=5)
    Bt = synth.make_B_table(2, 3)
    env = np.zeros(20, np.int32)
    env[3] = 7
    env[11] = -1
    t, d = ops.tau_grad(packed, T(xp, dev), T(Bt, dev), T(env, dev, torch.int32), dim=3, schedule=field_schedule)
    t, d = t.detach().cpu().numpy(), d.detach().cpu().numpy()
    assert np.isnan(t[3]) and np.isnan(t[11]) and np.isnan(d[3]).all()
    ok = np.ones(20, bool)
    ok[[3, 11]] = False
    assert np.isfinite(t[ok]).all() and np.isfinite(d[ok]).all()


@pytest.mark.parametrize("dim,fit", [(3, 13), (6, 6)])
def test_wide_env_table_in_lds_matches_global(packed, dev, dim, fit):
    """The wide kernels stage the env-B table in LDS when n_env · dim · 128 floats fit in
    WBL_FLOATS (pntf_common.h; 13 envs at dim 3, 6 at dim 6) and read it from global memory
    otherwise.  Same pairs and env ids, the table padded by one more environment so that it no
    longer fits, at the limit and one below it: τ bitwise equal; ∇τ equal to fp32 rounding (the
    LDS-table instantiation — the headline's — runs the Fourier fold on split-bf16 MFMA, the
    global-table one on fp32 MFMA: pntf_wide.h xfold, round 6), per pair within 1e-5."""
    n = 2 * 32 * 257
    xp = T(synth.make_pairs(n, dim, seed=41), dev)
    for E in (fit, fit - 1):
        Bt = synth.make_B_table(E + 1, dim, first_seed=60)
        env = T(synth.make_env_ids(n, E, contiguous=False, seed=E), dev, torch.int32)
        t_l, d_l = ops.tau_grad(packed, xp, T(Bt[:E], dev), env, dim=dim, schedule="wide_tile")
        t_g, d_g = ops.tau_grad(packed, xp, T(Bt, dev), env, dim=dim, schedule="wide_tile")
        assert torch.equal(t_l, t_g)
        dl, dg = d_l.double(), d_g.double()
        r = (dl - dg).norm(dim=1) / dg.norm(dim=1).clamp_min(1e-30)
        assert float(r.max()) < 1e-5, float(r.max())
        assert torch.isfinite(t_l).all() and torch.isfinite(d_l).all()


def test_coincident_endpoints(packed, dev, W):
    """xs == xg: τ and ∇τ are finite (the merge is symmetric), Speed = τ."""
    x = synth.make_pairs(8, 3, seed=9)
    x[:, 3:] = x[:, :3]
    B = synth.make_B(3)
    t, d = ops.tau_grad(packed, T(x, dev), T(B, dev), dim=3)
    to, do = O.tau_grad(W, x, B)
    close(t.detach().cpu().numpy(), to[:, 0], pairs=True)
    close(d.detach().cpu().numpy(), do, pairs=True)


@pytest.mark.parametrize("schedule", ["wave_tile", "split_tile", "quad_tile"])
def test_gibson_planner_vs_reference(packed, dev, schedule):
    p = load("plan_gib.npz")
    path, steps = ops.plan(packed, T(p["starts"], dev), T(p["B"], dev), dim=3, step=0.03,
                           tol=0.06, max_iter=500, mode=ops.GRAD_BACKGRAD_COMPAT,
                           schedule=schedule)
    path, steps = path.detach().cpu().numpy(), steps.detach().cpu().numpy()
    np.testing.assert_array_equal(steps, p["iters"])
    assert np.abs(path - p["paths"]).max() < 1e-3
    # endpoints
    last = p["paths"][np.arange(len(steps)), steps]
    assert np.abs(path[np.arange(len(steps)), steps] - last).max() < 1e-3


@pytest.mark.parametrize("schedule", ["wave_tile", "split_tile", "quad_tile"])
def test_arm_planner_vs_reference(packed, dev, schedule):
    p = load("plan_arm.npz")
    path, steps = ops.plan(packed, T(p["starts"], dev), T(p["B"].T, dev), dim=6, step=0.015,
                           tol=0.03, max_iter=300, mode=ops.GRAD_EXACT, schedule=schedule)
    path, steps = path.detach().cpu().numpy(), steps.detach().cpu().numpy()
    np.testing.assert_array_equal(steps, p["iters"])
    assert np.abs(path - p["paths"]).max() < 1e-3


@pytest.mark.parametrize("schedule", ["wave_tile", "split_tile", "quad_tile"])
def test_planner_batch_vs_oracle(packed, dev, schedule, W):
    q = 37
    xp0 = synth.make_box_pairs(q, 6, seed=77)
    B = synth.make_B(6, seed=12, arm=True).T.copy()
    path, steps = ops.plan(packed, T(xp0, dev), T(B, dev), dim=6, step=0.015, tol=0.03,
                           max_iter=60, mode=ops.GRAD_EXACT, schedule=schedule)
    po, so = O.plan(W, xp0, B, dim=6, step=0.015, tol=0.03, max_iter=60, compat=False)
    np.testing.assert_array_equal(steps.detach().cpu().numpy(), so)
    assert np.abs(path.detach().cpu().numpy() - po).max() < 1e-3


@pytest.mark.parametrize("dim,compat", [(3, True), (6, False)])
def test_planner_schedules_agree(packed, dev, dim, compat):
    """Split tiles (4 waves per 16 queries, several tiles per workgroup at this q) against
    one wave per tile: same iteration counts, paths equal to fp32 rounding."""
    q = 16 * 600 + 5
    xp0 = T(synth.make_box_pairs(q, dim, seed=91), dev)
    B = synth.make_B(dim, seed=12, arm=dim == 6)
    B = T(B.T.copy() if dim == 6 else B, dev)
    kw = dict(dim=dim, step=0.03 if dim == 3 else 0.015, tol=0.06 if dim == 3 else 0.03,
              max_iter=12, mode=ops.GRAD_BACKGRAD_COMPAT if compat else ops.GRAD_EXACT)
    pw, sw = ops.plan(packed, xp0, B, schedule="wave_tile", **kw)
    ps, ss = ops.plan(packed, xp0, B, schedule="split_tile", **kw)
    assert torch.equal(sw, ss)
    assert (ps - pw).abs().max().item() < 1e-4
    # quad tiles (4 queries per workgroup, ~9 tiles per workgroup at this q)
    pq, sq = ops.plan(packed, xp0, B, schedule="quad_tile", **kw)
    assert torch.equal(sw, sq)
    assert (pq - pw).abs().max().item() < 1e-4


def test_drop_in_models_api(W, dev):
    """The reference call sequence of test/gib_plan.py / Model.gradient through the
    drop-in modules."""
    from models import model_res_sigmoid_multi as md
    f = load("fwd_grad_d3.npz")
    m = md.Model(".", ".", 3, 2, device="cuda")
    m.network = md.NN("cuda", 3)
    m.network.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m.network.to(dev).float().eval()
    xp, B = T(f["xp"], dev), T(f["B"], dev)
    tau, coords = m.network.out(xp, B)
    assert tau.shape == (1024, 1)
    dtau = m.gradient(tau, coords)
    check(tau.detach().cpu().numpy(), "fwd_grad_d3.npz", "tau")
    check(dtau.detach().cpu().numpy(), "fwd_grad_d3.npz", "dtau")
    check(m.Gradient(xp.clone(), B).detach().cpu().numpy(), "fwd_grad_d3.npz", "gradient")
    m.B = B
    check(m.Speed(xp).detach().cpu().numpy(), "fwd_grad_d3.npz", "speed")
    check(m.TravelTimes(xp).detach().cpu().numpy(), "fwd_grad_d3.npz", "travel_time")
    check(m.Tau(xp).detach().cpu().numpy(), "fwd_grad_d3.npz", "tau")
    t2, d2, _ = m.network.out_backgrad(xp, B)
    check(d2.detach().cpu().numpy(), "fwd_grad_d3.npz", "dtau_backgrad")
    # weights edited in place -> repacked
    with torch.no_grad():
        m.network.generator[4].bias.add_(0.5)
    t3, _ = m.network.out(xp, B)
    assert not torch.allclose(t3, tau)


def test_arm_models_api(W, dev):
    from models import model_res_sigmoid as ma
    a = load("fwd_grad_d6.npz")
    m = ma.Model(".", ".", 6, device="cuda")
    m.B = torch.from_numpy(a["B"])
    m.network = ma.NN("cuda", 6, m.B)
    m.network.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m.network.to(dev)
    xp = T(a["xp"], dev)
    tau, coords = m.network.out(xp)
    check(m.gradient(tau, coords).detach().cpu().numpy(), "fwd_grad_d6.npz", "dtau")
    g = torch.cat([m.Gradient(xp[i:i + 1].clone()) for i in range(16)])
    check(g.detach().cpu().numpy(), "fwd_grad_d6.npz", "gradient16")


def test_large_batch_properties(packed, dev):
    """Full-size (C2: 262 144 pairs) properties: finite, τ in (0,1), tile-boundary-free
    (a permuted batch gives the permuted answer), a sampled subset matches the oracle."""
    n = 262144
    xp = synth.make_pairs(n, 3, seed=2)
    B = synth.make_B(3, seed=1)
    t, d = ops.tau_grad(packed, T(xp, dev), T(B, dev), dim=3)
    t, d = t.detach().cpu().numpy(), d.detach().cpu().numpy()
    assert np.isfinite(t).all() and np.isfinite(d).all() and (t > 0).all() and (t < 1).all()
    perm = np.random.default_rng(0).permutation(n)
    tp, dp = ops.tau_grad(packed, T(xp[perm], dev), T(B, dev), dim=3)
    np.testing.assert_array_equal(tp.detach().cpu().numpy(), t[perm])
    np.testing.assert_array_equal(dp.detach().cpu().numpy(), d[perm])
    idx = np.random.default_rng(1).choice(n, 512, replace=False)
    to, do = O.tau_grad(weights(), xp[idx], B)
    close(t[idx], to[:, 0], pairs=True)
    close(d[idx], do, pairs=True)


# ---------------------------------------------------------------- Eikonal residual (A11)
def test_out_laplace_and_loss_vs_reference(W, dev):
    """NN.out_laplace + Model.Loss on the HIP Taylor kernel vs the reference goldens
    (10 envs x 64 pairs, per-env B)."""
    from models import model_res_sigmoid_multi as md
    f = load("loss_d3.npz")
    m = md.Model(".", ".", 3, 10, device="cuda")
    m.network = md.NN("cuda", 3)
    m.network.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m.network.to(dev)
    pts, yobs, Bt = T(f["pts"], dev), T(f["yobs"], dev), T(f["B_table"], dev)
    tau, dtau, ltau, _ = m.network.out_laplace(pts, Bt)
    check(tau.detach().cpu().numpy(), "loss_d3.npz", "tau")
    check(dtau.detach().cpu().numpy(), "loss_d3.npz", "dtau")
    check(ltau.detach().cpu().numpy(), "loss_d3.npz", "ltau")
    loss, loss_n, diff = m.Loss(pts, yobs, Bt, 1.0, float(f["gamma"]))
    check(diff.detach().cpu().numpy(), "loss_d3.npz", "diff")
    assert abs(float(loss_n) - float(f["loss_n"])) < 1e-4 * abs(float(f["loss_n"]))


def test_arm_out_laplace_and_loss_vs_reference(W, dev):
    from models import model_res_sigmoid as ma
    f = load("loss_d6.npz")
    m = ma.Model(".", ".", 6, device="cuda")
    m.B = torch.from_numpy(f["B"])
    m.network = ma.NN("cuda", 6, m.B)
    m.network.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m.network.to(dev)
    pts = T(f["pts"], dev)
    tau, dtau, ltau, _ = m.network.out_laplace(pts)
    check(tau.detach().cpu().numpy(), "loss_d6.npz", "tau")
    check(dtau.detach().cpu().numpy(), "loss_d6.npz", "dtau")
    check(ltau.detach().cpu().numpy(), "loss_d6.npz", "ltau")
    _, loss_n, diff = m.Loss(pts, T(f["yobs"], dev), 1.0, float(f["gamma"]))
    check(diff.detach().cpu().numpy(), "loss_d6.npz", "diff")


@pytest.mark.parametrize("n", [1, 17, 300])
def test_residual_ragged_vs_oracle(packed, dev, W, n):
    xp = synth.make_pairs(n, 3, seed=300 + n)
    Bt = synth.make_B_table(4, 3, first_seed=30)
    env = synth.make_env_ids(n, 4, contiguous=False, seed=n)
    yobs = synth.make_speeds(n, seed=n)
    out = ops.eikonal_residual(packed, T(xp, dev), T(Bt, dev), T(env, dev, torch.int32), 3,
                               yobs=T(yobs, dev), gamma=1e-3)
    to, do, lo, dfo = O.eikonal_residual(W, xp, yobs, Bt, env, gamma=1e-3)
    close(out["tau"].detach().cpu().numpy(), to[:, 0], pairs=True)
    close(out["dtau"].detach().cpu().numpy(), do, pairs=True)
    close(out["ltau"].detach().cpu().numpy(), lo, pairs=True)
    close(out["diff"].detach().cpu().numpy(), dfo, pairs=True, diff=True)


def _elem_report(name, a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    return "%s rel_l2 %.2e max %.2e elem %.2e" % (name, rel_l2(a, b), np.abs(a - b).max() / scale,
                                                  max_rel(a, b, ELEM_FLOOR * scale))


def per_pair_rel(a, b):
    """Per-pair relative error: ‖a_p - b_p‖ / ‖b_p‖ over each pair's row (a scalar per pair
    for τ, the 2·dim vector for ∇τ, the 2·dim Laplacian row for Δτ)."""
    a = np.asarray(a, np.float64).reshape(len(a), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-30)


def north_star_per_pair(name, got, fp64, tol=1e-4):
    """The north star's 1e-4 relative bound, held for EVERY pair of the sample against the
    fp64 oracle (not only normwise over the batch)."""
    r = per_pair_rel(got, fp64)
    print("%s per-pair rel vs fp64: max %.2e (pair %d)" % (name, r.max(), int(r.argmax())))
    assert r.max() < tol, "%s: pair %d per-pair rel %.3g >= %.1g" % (name, int(r.argmax()),
                                                                      r.max(), tol)


def test_residual_grad_agrees_with_reverse_sweep(packed, dev, W):
    """C3 at full size (BASELINE config 3: 1M pairs, 10 envs, Eikonal residual included):
    a 512-pair sample of τ, ∇τ, Δτ and the residual `diff` against the fp64 oracle
    (SURVEY §8a A11), plus size-independent properties over all 1M pairs: the forward-mode ∇τ
    of the Taylor kernel equals the reverse-sweep ∇τ of the τ+∇τ kernels, τ is bit-identical
    to the 16-pair kernel's (same forward MFMA sequence), everything finite."""
    n = 1 << 20
    xp_np = synth.make_pairs(n, 3, seed=5)
    Bt_np = synth.make_B_table(10, 3)
    env_np = synth.make_env_ids(n, 10)
    y_np = synth.make_speeds(n)
    xp, Bt, env = T(xp_np, dev), T(Bt_np, dev), T(env_np, dev, torch.int32)
    out = ops.eikonal_residual(packed, xp, Bt, env, 3, yobs=T(y_np, dev), gamma=1e-3)
    for k in ("tau", "dtau", "ltau", "diff"):
        assert torch.isfinite(out[k]).all(), k
    idx = np.random.default_rng(3).choice(n, 512, replace=False)
    to, do, lo, dfo = O.eikonal_residual(W, xp_np[idx], y_np[idx], Bt_np, env_np[idx],
                                         gamma=1e-3)
    got = {k: v.detach().cpu().numpy()[idx] for k, v in out.items()}
    print("C3 1M sample vs fp64: " + "; ".join(
        _elem_report(k, got[k], r) for k, r in (("tau", to[:, 0]), ("dtau", do), ("ltau", lo),
                                                ("diff", dfo))))
    close(got["tau"], to[:, 0], pairs=True)
    close(got["dtau"], do, pairs=True)
    close(got["ltau"], lo, pairs=True)
    close(got["diff"], dfo, pairs=True, diff=True)
    # north star per pair: τ, ∇τ and the Laplacian row within 1e-4 of fp64 for every pair;
    # diff = Σ_e (Ŝ/Y + Y/Ŝ) - 4 cancels (|diff| down to ~1e-3 beside summands of ~4), so it
    # is held to 1e-4 of its summands' magnitude |diff| + 4 (fp32 itself gives 1.5e-4 of
    # |diff| on this sample: tests measure)
    north_star_per_pair("C3 tau", got["tau"], to[:, 0])
    north_star_per_pair("C3 dtau", got["dtau"], do)
    north_star_per_pair("C3 ltau", got["ltau"], lo)
    dd = np.abs(got["diff"].astype(np.float64) - dfo) / (np.abs(dfo) + 4.0)
    print("C3 diff |err|/(|diff|+4) max %.2e" % dd.max())
    assert dd.max() < 1e-4
    # componentwise (floored at 1 % of the largest component), ∇τ and Δτ: the direction passes
    # run on split-bf16 MFMA (pntf_taylor.h, round 6) and must be no worse than the fp32 op
    # sequence of out_laplace (the oracle in float32) against the same fp64 values
    _, do32, lo32 = O.laplace(W, xp_np[idx], Bt_np, env_np[idx], dim=3, dtype=np.float32)
    for k, ref64, ref32 in (("dtau", do, do32), ("ltau", lo, lo32)):
        floor = ELEM_FLOOR * np.abs(ref64).max()
        e_hip, e_ref = max_rel(got[k], ref64, floor), max_rel(ref32, ref64, floor)
        print("C3 %s componentwise vs fp64: HIP %.2e, fp32 op sequence %.2e" % (k, e_hip, e_ref))
        assert e_hip <= max(1e-4, e_ref), k
    # the 16-pair τ+∇τ kernel runs the same forward MFMA sequence: τ bit-identical
    t, d = ops.tau_grad(packed, xp, Bt, env, dim=3, schedule="wave_tile")
    assert torch.equal(out["tau"], t)
    close(out["dtau"].detach().cpu().numpy(), d.detach().cpu().numpy(), tol=1e-5)
    # the 32-pair (wide) kernel sums in another order: fp32-rounding agreement
    tw, dw = ops.tau_grad(packed, xp, Bt, env, dim=3, schedule="wide_tile")
    close(tw.detach().cpu().numpy(), t.detach().cpu().numpy(), tol=1e-6)
    close(out["dtau"].detach().cpu().numpy(), dw.detach().cpu().numpy(), tol=1e-5)


def test_headline_1m_sample_vs_fp64_oracle(packed, dev, W):
    """The bench's headline workload itself (bench.py run(): 1 048 576 pairs of seed 1000,
    10 envs, per-pair env id, exact mode, AUTO = the wide kernel): a 512-pair sample of τ and
    ∇τ against the fp64 oracle, at the north-star 1e-4 normwise and, elementwise (floored at
    1 % of the batch's largest component), τ within 1e-5 and ∇τ within 5e-4 of the fp64
    value — 20x and 2x tighter than the bound used against the fp32 goldens (measured on
    MI355X with the split-bf16 wide layers: τ 2.0e-7, ∇τ 2.0e-4 against the fp32 reference's
    own 2.0e-4; 2.8e-7 / 1.5e-4 with fp32 MFMA throughout); all outputs finite, τ in (0,1)."""
    n = 1 << 20
    xp_np = synth.make_pairs(n, 3, seed=1000)
    Bt_np = synth.make_B_table(10, 3)
    env_np = synth.make_env_ids(n, 10)
    assert ops.resolved_schedule(n) == "wide_tile"
    t, d = ops.tau_grad(packed, T(xp_np, dev), T(Bt_np, dev), T(env_np, dev, torch.int32), dim=3)
    t, d = t.detach().cpu().numpy(), d.detach().cpu().numpy()
    assert np.isfinite(t).all() and np.isfinite(d).all() and (t > 0).all() and (t < 1).all()
    idx = np.random.default_rng(4).choice(n, 512, replace=False)
    to, do = O.tau_grad(W, xp_np[idx], Bt_np, env_np[idx])
    print("headline 1M sample vs fp64: %s; %s" % (_elem_report("tau", t[idx], to[:, 0]),
                                                  _elem_report("dtau", d[idx], do)))
    close(t[idx], to[:, 0], elem=1e-5, pairs=True)
    close(d[idx], do, elem=5e-4, pairs=True)
    north_star_per_pair("headline tau", t[idx], to[:, 0])
    north_star_per_pair("headline dtau", d[idx], do)
    # componentwise (floored at 1 % of the largest |∇τ| component): no worse than the
    # reference's own fp32 op sequence (oracle/torch_ref.py, the per-env NN.out +
    # Model.gradient calls) against the same fp64 values — elementwise 1e-4 is not met by the
    # fp32 reference itself (1.66e-4 on this sample, measured in the build container)
    from oracle.torch_ref import TorchRef
    tr, dr = TorchRef(W).tau_grad(xp_np[idx], Bt_np, env_np[idx])
    floor = ELEM_FLOOR * np.abs(do).max()
    e_hip, e_ref = max_rel(d[idx], do, floor), max_rel(dr.numpy(), do, floor)
    # the same pairs through the fp32-MFMA wave-tile kernel: the wide kernel's split-bf16
    # layers against fp32 MFMA throughout
    _, dw = ops.tau_grad(packed, T(xp_np[idx], dev), T(Bt_np, dev), T(env_np[idx], dev, torch.int32),
                         dim=3, schedule="wave_tile")
    e_f32 = max_rel(dw.cpu().numpy(), do, floor)
    print("headline dtau componentwise vs fp64: HIP %.2e, fp32 reference %.2e, fp32-MFMA "
          "wave-tile kernel %.2e (HIP / reference %.3f)" % (e_hip, e_ref, e_f32, e_hip / e_ref))
    # measured headroom: 1.77e-4 against the reference's 2.02e-4 (0.876) with the
    # split-bf16 layers of round 6; held to 0.95 so that a change eating the margin fails here
    assert e_hip <= 0.95 * max(1e-4, e_ref)


def test_c4_shape_sharded_on_one_gpu(packed, dev, W):
    """BASELINE C4 at its full size on one GPU: 8 x 1 048 576 (+ 5, so the shards are uneven)
    Gibson pairs, 10 envs, per-pair env id.  Each of the 8 rank shards (pntf.dist.shard_range,
    the bench's N > 1 split) evaluated alone equals the same rows of the whole batch bit for
    bit, so the sharded job's all-gathered output is the single-batch output; a 256-pair sample
    of the whole batch against the fp64 oracle."""
    from pntf import dist
    n, ws = 8 * (1 << 20) + 5, 8
    xp_np = synth.make_pairs(n, 3, seed=2024)
    Bt_np = synth.make_B_table(10, 3)
    env_np = synth.make_env_ids(n, 10)
    xp, Bt, env = T(xp_np, dev), T(Bt_np, dev), T(env_np, dev, torch.int32)
    t, d = ops.tau_grad(packed, xp, Bt, env, dim=3)
    assert torch.isfinite(t).all() and torch.isfinite(d).all()
    for r in range(ws):
        lo, hi = dist.shard_range(n, r, ws)
        ts, dsh = ops.tau_grad(packed, xp[lo:hi].contiguous(), Bt, env[lo:hi].contiguous(), dim=3)
        assert torch.equal(ts, t[lo:hi]) and torch.equal(dsh, d[lo:hi]), r
    idx = np.random.default_rng(8).choice(n, 256, replace=False)
    to, do = O.tau_grad(W, xp_np[idx], Bt_np, env_np[idx])
    close(t.detach().cpu().numpy()[idx], to[:, 0], pairs=True)
    close(d.detach().cpu().numpy()[idx], do, pairs=True)


def test_device_sum_deterministic(dev):
    x = torch.from_numpy(np.random.default_rng(0).standard_normal(1000003).astype(np.float32)).to(dev)
    a, b = ops.device_sum(x), ops.device_sum(x)
    assert a.item() == b.item()
    assert abs(a.item() - float(x.double().sum())) < 1e-6 * float(x.abs().sum())


@pytest.mark.parametrize("schedule", ["wave_tile", "split_tile", "quad_tile"])
def test_planner_edge_cases(packed, dev, schedule, W):
    """Loop-cap semantics (at most max_iter + 1 updates, test/gib_plan.py:83-86), max_iter 0,
    queries already within tol (0 steps, constant path), an invalid env id (steps -1), a
    ragged batch of 5 — every schedule against the oracle."""
    q = 5
    xp0 = synth.make_pairs(q, 3, seed=11)
    xp0[1, 3:] = xp0[1, :3] + 0.001            # already converged: |xg - xs| < tol
    B1 = synth.make_B(3, seed=1)
    Bt = np.stack([B1, synth.make_B(3, seed=2)])
    env = np.array([0, 1, 0, 7, 1], np.int32)   # env 7 does not exist
    for max_iter in (3, 0):
        path, steps = ops.plan(packed, T(xp0, dev), T(Bt, dev), T(env, dev, torch.int32), dim=3,
                               step=1e-4, tol=0.06, max_iter=max_iter,
                               mode=ops.GRAD_BACKGRAD_COMPAT, schedule=schedule)
        path, steps = path.detach().cpu().numpy(), steps.detach().cpu().numpy()
        assert path.shape == (q, max_iter + 2, 6)
        assert steps[3] == -1
        assert steps[1] == 0 and np.all(path[1] == xp0[1])
        for i in (0, 2, 4):
            po, so = O.plan(W, xp0[i:i + 1], Bt[env[i]], step=1e-4, tol=0.06,
                            max_iter=max_iter, compat=True)
            assert steps[i] == so[0] == max_iter + 1
            assert np.abs(path[i] - po[0]).max() < 1e-5


@pytest.mark.parametrize("golden", ["plan_gib.npz", "plan_arm.npz"])
def test_single_query_planner_vs_reference(packed, dev, golden):
    """The reference plans one query at a time (test/gib_plan.py, test/arm_plan.py: Q = 1).
    A single-query call runs plan_quad_solo_kernel (VALU layers for the one pair): every
    golden query planned alone gives the reference's iteration count and path within 1e-3."""
    p = load(golden)
    gib = golden == "plan_gib.npz"
    B = T(p["B"] if gib else p["B"].T, dev)
    kw = (dict(dim=3, step=0.03, tol=0.06, max_iter=500, mode=ops.GRAD_BACKGRAD_COMPAT) if gib
          else dict(dim=6, step=0.015, tol=0.03, max_iter=300, mode=ops.GRAD_EXACT))
    for i in range(len(p["iters"])):
        path, steps = ops.plan(packed, T(p["starts"][i:i + 1], dev), B, **kw)
        assert int(steps.cpu()[0]) == int(p["iters"][i]), i
        assert np.abs(path.detach().cpu().numpy()[0] - p["paths"][i]).max() < 1e-3, i


@pytest.mark.parametrize("dim,q", [(3, 37), (6, 200)])
def test_solo_layers_bitwise_equal_mfma_layers(packed, dev, dim, q):
    """The planner's two quad layer forms give identical bits: AUTO runs batches of at most
    one query per CU on the SOLO (VALU) layers, QUAD_TILE on the 4x4x1 MFMA layers; same
    fma chains, same cross-lane sum order (pntf_quad.h qlayer).  This is what lets the C5 tail
    hand-off move a query from one form to the other mid-plan without changing its path."""
    xp0 = T(synth.make_box_pairs(q, dim, seed=55 + q), dev)
    B = synth.make_B(dim, seed=12, arm=dim == 6)
    B = T(B.T.copy() if dim == 6 else B, dev)
    kw = dict(dim=dim, step=0.03 if dim == 3 else 0.015, tol=0.06 if dim == 3 else 0.03,
              max_iter=40, mode=ops.GRAD_BACKGRAD_COMPAT if dim == 3 else ops.GRAD_EXACT)
    ps, ss = ops.plan(packed, xp0, B, schedule="auto", **kw)
    pq, sq = ops.plan(packed, xp0, B, schedule="quad_tile", **kw)
    assert torch.equal(ss, sq)
    assert torch.equal(ps, pq), float((ps - pq).abs().max())


def test_c5_tail_handoff_bitwise_and_taken(packed, dev):
    """C5 (1024 arm queries, <= 199 steps): AUTO lets the 4-query MFMA tiles hand the last
    <= CUs active queries to a SOLO launch (pntf_plan_ex); QUAD_TILE keeps them on the tiles.
    Same bits either way, and the hand-off really happened (the workspace's hand-off count,
    pntf_common.h PlanArgs::tail, is non-zero)."""
    q = 1024
    Ba = T(synth.make_B(6, seed=12, arm=True).T.copy(), dev)
    xq = T(synth.make_box_pairs(q, 6, seed=3), dev)
    kw = dict(dim=6, step=0.015, tol=0.03, max_iter=199, mode=ops.GRAD_EXACT)
    pa, sa = ops.plan(packed, xq, Ba, schedule="auto", **kw)
    tail = ops._workspace(dev, q)[:8].view(torch.int32).detach().cpu().numpy()
    pq, sq = ops.plan(packed, xq, Ba, schedule="quad_tile", **kw)
    assert torch.equal(sa, sq)
    assert torch.equal(pa, pq), float((pa - pq).abs().max())
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    assert 0 < tail[1] <= cus, tail.tolist()          # handed-off queries
    assert tail[0] >= q - cus, tail.tolist()          # the done count that triggered it


def test_net_handle_matches_packed_blob(packed, dev, W):
    """The handle form of the C ABI (pntf_net_create / _update / _packed / _destroy) packs the
    same weights as pntf_pack_weights: pntf_tau_grad on the handle's buffer is bitwise the
    caller-owned blob's, and _update repacks after a weight change."""
    import ctypes
    from pntf import _lib
    lib = _lib.load()
    V = ctypes.c_void_p
    params = [torch.from_numpy(v).to(dev) for v in W.values()]
    arr = (V * 30)(*[p.data_ptr() for p in params])
    s = V(torch.cuda.current_stream(dev).cuda_stream)
    n = 333
    xp = T(synth.make_pairs(n, 3, seed=7), dev)
    B = T(synth.make_B(3), dev)
    ws = torch.empty(int(lib.pntf_workspace_bytes(n)), dtype=torch.uint8, device=dev)

    def run(packed_ptr):
        t = torch.empty(n, device=dev)
        d = torch.empty((n, 6), device=dev)
        st = lib.pntf_tau_grad(V(packed_ptr), 3, V(xp.data_ptr()), n, V(B.data_ptr()), None, 1,
                               0, V(t.data_ptr()), V(d.data_ptr()), V(ws.data_ptr()),
                               ws.numel(), s)
        assert st == 0, lib.pntf_last_error()
        return t, d
    h = lib.pntf_net_create(arr, 30, s)
    assert h, lib.pntf_last_error()
    try:
        t0, d0 = run(packed.data_ptr())
        t1, d1 = run(lib.pntf_net_packed(h))
        assert torch.equal(t0, t1) and torch.equal(d0, d1)
        params[5].mul_(1.5)                      # encoder.2.bias changes: repack both ways
        assert lib.pntf_net_update(h, arr, 30, s) == 0
        t2, d2 = run(lib.pntf_net_packed(h))
        blob = ops.pack_weights(params)
        t3, d3 = run(blob.data_ptr())
        assert torch.equal(t2, t3) and torch.equal(d2, d3) and not torch.equal(t2, t0)
    finally:
        torch.cuda.synchronize()
        lib.pntf_net_destroy(h)
    assert not lib.pntf_net_create(None, 30, s) and b"null" in lib.pntf_last_error()


def test_hip_graph_capture_through_the_abi(packed, dev, W):
    """The C ABI is stream-ordered: pntf_tau_grad and pntf_eikonal_residual
    launched through ctypes on torch's capture stream are recorded into a torch.cuda.CUDAGraph
    (hipStreamBeginCapture / EndCapture) and every replay, on new inputs copied into the static
    buffers, is bitwise the eager call on the same inputs.  (Round 5's capture segfault in
    hipStreamEndCapture: DESIGN.md §7 item 7.)"""
    import ctypes
    from pntf import _lib
    lib = _lib.load()
    V = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
    n, E = 40000, 10
    Bt = T(synth.make_B_table(E, 3), dev)
    ws = torch.empty(int(lib.pntf_workspace_bytes(n)), dtype=torch.uint8, device=dev)

    def inputs(seed):
        return (T(synth.make_pairs(n, 3, seed=seed), dev),
                T(synth.make_env_ids(n, E, contiguous=False, seed=seed), dev, torch.int32),
                T(synth.make_speeds(n, seed=seed), dev))

    def outputs():
        return [torch.empty(n, device=dev), torch.empty((n, 6), device=dev),
                torch.empty(n, device=dev), torch.empty((n, 6), device=dev),
                torch.empty((n, 6), device=dev), torch.empty(n, device=dev)]

    def launch(x, e, y, o):
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        st = lib.pntf_tau_grad(V(packed), 3, V(x), n, V(Bt), V(e), E, 0, V(o[0]), V(o[1]),
                               V(ws), ws.numel(), s)
        assert st == 0, lib.pntf_last_error()
        st = lib.pntf_eikonal_residual(V(packed), 3, V(x), V(y), n, V(Bt), V(e), E,
                                       ctypes.c_float(1e-3), V(o[2]), V(o[3]), V(o[4]),
                                       V(o[5]), V(ws), ws.numel(), s)
        assert st == 0, lib.pntf_last_error()

    xs, es, ys = [t.clone() for t in inputs(11)]
    go = outputs()
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        launch(xs, es, ys, go)                   # warm-up on the side stream
    torch.cuda.current_stream(dev).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        launch(xs, es, ys, go)
    for seed in (12, 13):
        x, e, y = inputs(seed)
        xs.copy_(x), es.copy_(e), ys.copy_(y)
        g.replay()
        ref = outputs()
        launch(x, e, y, ref)
        torch.cuda.synchronize()
        for a, b in zip(go, ref):
            assert torch.equal(a, b)
    # and the replayed τ+∇τ is the one the ops wrapper gives (same kernel, same inputs)
    t, d = ops.tau_grad(packed, x, Bt, e, dim=3)
    assert torch.equal(t, go[0]) and torch.equal(d, go[1])
