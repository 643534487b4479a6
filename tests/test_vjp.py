"""Autograd through the drop-in's other differentiable outputs.

The reference's `NN.out_laplace` (models/model_res_sigmoid_multi.py:710-848), `NN.out_grad`
(:303-400), `NN.out_backgrad` (:402-647) and `Model.gradient(..., create_graph=True)`
(:890-896) are plain torch graphs: a loss written on any of their outputs trains every weight
and differentiates to `coords`.  tests/golden/make_out_grad_goldens.py --stage vjp recorded
the reference's `.grad` (digests: tests/golden_util.py grad_digest) and coords' gradient for
a seeded weighted sum of each method's outputs, at init and at the reference-trained W2
weights, for both models (arm: models/model_res_sigmoid.py:300-826).
  * CPU: the fp64 oracle's `taylor_vjp` reproduces every fixture;
  * GPU: the drop-in's `.backward()` through the HIP Taylor tape (pntf/train.py field_vjp)
    gives the same `.grad` and coords gradient.
Tolerances: outputs per pair 1e-4 relative (north star); gradients max-abs / max|ref| over the
stored rows and the sketch's relative-L2 estimate below GRAD_TOL (the training gradients'
bound, tests/test_train.py).
"""
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, digest_error, load, rel_l2
from oracle import pntf_oracle as O
from pntf import synth

CASES = [("init", 3), ("w2", 3), ("init", 6), ("w2", 6)]
METHODS = ["laplace", "laplace_sum", "grad", "backgrad", "gradient2"]
GRAD_TOL = 2e-4
ORACLE_TOL = 5e-5            # the reference itself is fp32 (W2 training grads: 5e-5, test_train.py)


def _weights(tag, dim):
    if tag == "init":
        return synth.make_weights(0)
    sd = torch.load(os.path.join(GOLDEN, "ckpt_w2_d%d.pt" % dim), map_location="cpu",
                    weights_only=True)["model_state_dict"]
    return {k: v.numpy().astype(np.float32) for k, v in sd.items()}


def _upstream(f, meth, dim):
    """(g_tau, g_dtau, g_ltau) of the fixture's loss for `meth`."""
    wt, wd = f["w/wt"], f["w/wd"]
    if meth == "laplace":
        return wt, wd, f["w/wl"]
    if meth == "laplace_sum":
        return wt, wd, np.repeat(f["w/wl_sum"], dim, axis=1)
    return wt, wd, None


def _oracle_args(f, meth, dim):
    """(B, env, compat) the oracle needs for the fixture's call of `meth`."""
    if dim == 6:
        return f["B"].T, None, False                      # arm: out_backgrad is exact (:300-511)
    E, n = int(f["E"]), f["xp"].shape[0]
    if meth.startswith("laplace"):
        return f["Btab"], np.repeat(np.arange(E), n // E).astype(np.int32), False
    return f["Btab"][0], None, meth == "backgrad"


def _fixture_grads(f, meth):
    out = {}
    for k in synth.state_dict_keys():
        pre = "%s/g/%s/" % (meth, k)
        if pre + "none" in f.files:
            out[k] = None
        else:
            out[k] = {kk[len(pre):]: f[kk] for kk in f.files if kk.startswith(pre)}
    return out


def check_grads(f, meth, grads, tol):
    """Every trained parameter's gradient against the fixture digest; encoder1.0 gets none."""
    worst = 0.0
    for k, ref in _fixture_grads(f, meth).items():
        if ref is None:
            assert grads.get(k) is None, k
            continue
        assert grads.get(k) is not None, k
        e_rows, e_sk = digest_error(k, grads[k], ref)
        assert e_rows < tol and e_sk < tol, (meth, k, e_rows, e_sk)
        worst = max(worst, e_rows, e_sk)
    return worst


def per_pair(a, b):
    """Largest per-pair relative error ||a_p - b_p|| / ||b_p|| (rows of 2-D arrays)."""
    a = np.asarray(a, np.float64).reshape(len(b), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    return float(np.max(np.linalg.norm(a - b, axis=1) /
                        np.maximum(np.linalg.norm(b, axis=1), 1e-30)))


@pytest.mark.parametrize("tag,dim", CASES)
@pytest.mark.parametrize("meth", METHODS)
def test_oracle_vjp_vs_reference(tag, dim, meth):
    f = load("vjp_%s_d%d.npz" % (tag, dim))
    B, env, compat = _oracle_args(f, meth, dim)
    gt, gd, gl = _upstream(f, meth, dim)
    (t, d, lt), g, dx = O.taylor_vjp(_weights(tag, dim), f["xp"], B, env, dim, gt, gd, gl,
                                     compat=compat)
    assert per_pair(t, f[meth + "/tau"]) < 1e-5
    assert rel_l2(d, f[meth + "/dtau"]) < 1e-5
    if meth.startswith("laplace"):
        assert rel_l2(lt, f[meth + "/ltau"]) < 1e-5
    assert rel_l2(dx, f[meth + "/dcoords"]) < ORACLE_TOL, meth
    check_grads(f, meth, {k: g.get(k) for k in synth.state_dict_keys()}, ORACLE_TOL)


def test_oracle_vjp_value_only_is_tau_weight_grad():
    """With only g_tau the Taylor adjoint is NN.out's value-tape adjoint (tau_weight_grad)."""
    W = synth.make_weights(0)
    xp = synth.make_pairs(33, 3, seed=5)
    B = synth.make_B(3)
    wt = np.linspace(-1, 1, 33)
    _, g, dx = O.taylor_vjp(W, xp, B, None, 3, wt, None, None)
    _, g0, dx0 = O.tau_weight_grad(W, xp, B, wt, dim=3)
    assert rel_l2(dx, dx0) < 1e-12
    for k in g0:
        assert rel_l2(g[k], g0[k]) < 1e-12, k


# ------------------------------------------------------------------------------ GPU
def _drop_in(tag, dim, dev, f):
    """The drop-in net and Model at the fixture's weights, and the method calls the golden
    script made on the reference (make_out_grad_goldens.py record_vjp)."""
    W = {k: torch.from_numpy(v) for k, v in _weights(tag, dim).items()}
    if dim == 3:
        from models import model_res_sigmoid_multi as md
        net = md.NN(dev, 3)
        model = md.Model(".", ".", 3, 2, device=dev)
        Bt = torch.from_numpy(f["Btab"]).to(dev)
        B0 = Bt[0]
        calls = {"laplace": lambda x: net.out_laplace(x, Bt),
                 "grad": lambda x: net.out_grad(x, B0),
                 "backgrad": lambda x: net.out_backgrad(x, B0),
                 "out": lambda x: net.out(x, B0)}
    else:
        from models import model_res_sigmoid as ma
        net = ma.NN(dev, 6, torch.from_numpy(f["B"]))
        model = ma.Model(".", ".", 6, device=dev)
        calls = {"laplace": lambda x: net.out_laplace(x), "grad": lambda x: net.out_grad(x),
                 "backgrad": lambda x: net.out_backgrad(x), "out": lambda x: net.out(x)}
    net.load_state_dict(W, strict=True)
    net.to(dev)
    model.network = net
    return net, model, calls


def run_method(net, model, calls, f, meth, dim, dev):
    """The fixture's loss for `meth` through the drop-in, backward; returns (tau, dtau, ltau,
    dcoords) as numpy."""
    xp = torch.from_numpy(f["xp"]).to(dev)
    n = xp.shape[0]
    E = int(f["E"])
    wt = torch.from_numpy(f["w/wt"]).to(dev)
    wd = torch.from_numpy(f["w/wd"]).to(dev)
    net.zero_grad(set_to_none=True)
    x = xp.clone().requires_grad_(True)
    lt = None
    if meth.startswith("laplace"):
        wl = (torch.from_numpy(f["w/wl"]) if meth == "laplace"
              else torch.from_numpy(np.repeat(f["w/wl_sum"], dim, axis=1))).to(dev)
        tau, dtau, ltau, X = calls["laplace"](x.view(E, n // E, 2 * dim) if E else x)
        tau, dtau, ltau = tau.reshape(n), dtau.reshape(n, 2 * dim), ltau.reshape(n, 2 * dim)
        loss = (wt * tau).sum() + (wd * dtau).sum() + (wl * ltau).sum()
        leaf = X if X.is_leaf else x
        lt = ltau.detach().cpu().numpy()
    elif meth == "gradient2":
        tau, leaf = calls["out"](xp)
        dtau = model.gradient(tau, leaf)
        tau = tau.reshape(n)
        loss = (wt * tau).sum() + (wd * dtau).sum()
    else:
        tau, dtau, _ = calls[meth](x)
        tau = tau.reshape(n)
        loss = (wt * tau).sum() + (wd * dtau).sum()
        leaf = x
    loss.backward()
    dc = leaf.grad.detach().cpu().numpy() if leaf.grad is not None else None
    return tau.detach().cpu().numpy(), dtau.detach().cpu().numpy(), lt, dc


@pytest.mark.gpu
@pytest.mark.parametrize("tag,dim", CASES)
@pytest.mark.parametrize("meth", METHODS)
def test_drop_in_vjp_vs_reference(tag, dim, meth):
    """`.backward()` of a weighted sum of out_laplace / out_grad / out_backgrad / create_graph
    Model.gradient outputs fills every weight's `.grad` and coords' gradient as the
    reference's autograd does (fixtures from the reference itself)."""
    dev = torch.device("cuda:0")
    f = load("vjp_%s_d%d.npz" % (tag, dim))
    net, model, calls = _drop_in(tag, dim, dev, f)
    t, d, lt, dc = run_method(net, model, calls, f, meth, dim, dev)
    # outputs: per pair against the fp64 oracle at the north star's 1e-4
    B, env, compat = _oracle_args(f, meth, dim)
    (to, do, lo), go, dxo = O.taylor_vjp(_weights(tag, dim), f["xp"], B, env, dim,
                                         *_upstream(f, meth, dim), compat=compat)
    assert per_pair(t, to) < 1e-4 and per_pair(d, do) < 1e-4, meth
    if lt is not None:
        assert per_pair(lt, lo) < 1e-4
    assert dc is not None, "coords received no gradient"
    e_dc = float(np.abs(dc - f[meth + "/dcoords"]).max() / np.abs(f[meth + "/dcoords"]).max())
    assert e_dc < GRAD_TOL, (meth, e_dc)
    grads = {k: (p.grad.detach().cpu().numpy() if p.grad is not None else None)
             for k, p in net.named_parameters()}
    worst = check_grads(f, meth, grads, GRAD_TOL)
    print("%s %s d%d: coords %.2e, worst param %.2e" % (meth, tag, dim, e_dc, worst))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 37])
@pytest.mark.parametrize("nle", ["none", "sum", "dir"])
def test_field_vjp_ragged_env_table_vs_oracle(n, nle):
    """field_vjp on ragged batches with a per-pair env table (random env ids) against the fp64
    oracle: all three second-derivative layouts (none / per-endpoint sums / per direction)."""
    from pntf import train
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    xp = synth.make_pairs(n, 3, seed=60 + n)
    Bt = synth.make_B_table(3, 3)
    env = synth.make_env_ids(n, 3, contiguous=False, seed=n)
    rng = np.random.Generator(np.random.PCG64(n))
    gt = rng.uniform(-1, 1, n)
    gd = rng.uniform(-1, 1, (n, 6))
    gl = None if nle == "none" else rng.uniform(-1, 1, (n, 6))
    if nle == "sum":
        gl = np.repeat(gl[:, [0, 3]], 3, axis=1)
    _, go, dxo = O.taylor_vjp(W, xp, Bt, env, 3, gt, gd, gl)
    p = {k: torch.from_numpy(v).to(dev) for k, v in W.items() if not k.startswith("encoder1.0")}
    grads = {k: torch.empty_like(v) for k, v in p.items()}
    cuda = lambda a: None if a is None else torch.from_numpy(np.asarray(a, np.float32)).to(dev)  # noqa
    glap = {"none": None, "sum": cuda(None if gl is None else gl[:, [0, 3]]), "dir": cuda(gl)}[nle]
    k = {"none": 0, "sum": 1, "dir": 3}[nle]
    gx = train.field_vjp(p, cuda(xp), cuda(Bt), torch.from_numpy(env).to(dev), 3, k, False,
                         cuda(gt), cuda(gd), glap, grads, True)
    assert float(np.abs(gx.detach().cpu().numpy() - dxo).max() / np.abs(dxo).max()) < GRAD_TOL
    for key, g in grads.items():
        r = go[key]
        # the head bias gradient is one sum over the pairs of ±-weighted terms and can cancel
        # to far below its terms: it is held relative to the head weight gradient's scale
        scale = np.abs(go["generator.4.weight"]).max() if r.size == 1 else np.abs(r).max()
        assert float(np.abs(g.detach().cpu().numpy() - r).max() / scale) < GRAD_TOL, key


@pytest.mark.gpu
def test_frozen_layers_get_no_grad_and_others_match():
    """with encoder layers frozen (requires_grad False) a backward through NN.out
    and through out_laplace works, leaves the frozen parameters without .grad and gives the
    trainable ones the same gradient as the unfrozen net."""
    from models import model_res_sigmoid_multi as md
    dev = torch.device("cuda:0")
    W = {k: torch.from_numpy(v) for k, v in synth.make_weights(0).items()}
    xp = torch.from_numpy(synth.make_pairs(50, 3, seed=70)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(2, 3)).to(dev)

    def grads(frozen):
        net = md.NN(dev, 3)
        net.load_state_dict(W, strict=True)
        net.to(dev)
        for name in frozen:
            getattr(net, name.split(".")[0])[int(name.split(".")[1])].requires_grad_(False)
        tau, _ = net.out(xp, Bt[0])
        t2, d2, l2, _ = net.out_laplace(xp.view(2, 25, 6), Bt)
        (tau.sum() + d2.sum() + l2.pow(2).sum()).backward()
        return {k: (None if p.grad is None else p.grad.clone()) for k, p in net.named_parameters()}

    ref = grads([])
    fr = grads(["encoder.0", "encoder.1"])
    for k, g in fr.items():
        if k.startswith(("encoder.0.", "encoder.1.", "encoder1.0.")):
            assert g is None, k
        else:
            assert torch.allclose(g, ref[k], rtol=1e-5, atol=1e-7), k


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["Speed", "Tau", "TravelTimes", "Gradient"])
def test_epilogue_outputs_differentiable_vs_oracle(which):
    """Model.Speed / Tau / TravelTimes / Gradient (models/model_res_sigmoid_multi.py:1173-1248)
    are torch graphs of NN.out / out_grad / out_backgrad in the reference, so a loss on them
    trains the weights.  With autograd recording and trainable weights the drop-in composes
    them from its differentiable outputs (pntf.net compose_*): the values equal
    the fused epilogue kernels' (no-grad path) to fp32 rounding, and the weight gradients of a
    seeded weighted sum match the fp64 oracle (the composition's upstream gradient through
    oracle.taylor_vjp) within GRAD_TOL of each tensor's largest gradient.  B's gradient still
    raises."""
    from models import model_res_sigmoid_multi as md
    from pntf import net as pnet
    from pntf.ops import PntfError
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()})
    net.to(dev)
    m = md.Model(".", ".", 3, 2, device=dev)
    m.network = net
    B = synth.make_B(3)
    m.B = torch.from_numpy(B).to(dev)
    n = 64
    xp = synth.make_pairs(n, 3, seed=71)
    x = torch.from_numpy(xp).to(dev)
    fn = {"Speed": m.Speed, "Tau": m.Tau, "TravelTimes": m.TravelTimes,
          "Gradient": lambda v: m.Gradient(v, m.B)}[which]
    out = fn(x)
    with torch.no_grad():
        fused = fn(x)
    assert out.grad_fn is not None and fused.grad_fn is None
    np.testing.assert_allclose(out.detach().cpu().numpy(), fused.cpu().numpy(), rtol=2e-5,
                               atol=1e-6)
    wt = np.random.default_rng(5).standard_normal(tuple(out.shape))
    net.zero_grad()
    (out * torch.from_numpy(wt).to(dev, out.dtype)).sum().backward()
    # the oracle: τ, ∇τ in fp64 (out_backgrad's quirk for Gradient), the composition's upstream
    # gradient by torch autograd in fp64 on the CPU, then the Taylor adjoint
    compat = which == "Gradient"
    (tau64, dtau64, _), _, _ = O.taylor_vjp(W, xp, B, dim=3, compat=compat, want_x=False)
    t = torch.from_numpy(tau64).requires_grad_(True)
    d = torch.from_numpy(dtau64).requires_grad_(True)
    X = torch.from_numpy(xp.astype(np.float64))
    comp = {"Speed": lambda: pnet.compose_speed(t, d, X, 3), "Tau": lambda: t,
            "TravelTimes": lambda: pnet.compose_travel_time(t, X, 3),
            "Gradient": lambda: pnet.compose_velocity(t, d, X, 3)}[which]()
    (comp * torch.from_numpy(wt).reshape(comp.shape)).sum().backward()
    gd = None if d.grad is None else d.grad.numpy()
    _, g64, _ = O.taylor_vjp(W, xp, B, dim=3, g_tau=t.grad.numpy().reshape(-1), g_dtau=gd,
                             compat=compat, want_x=False)
    for k, p in net.named_parameters():
        if k.startswith("encoder1.0"):
            assert p.grad is None, k
            continue
        got, ref = p.grad.detach().cpu().numpy(), g64[k]
        err = float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))
        assert err < GRAD_TOL, (which, k, err)
    Bg = m.B.clone().requires_grad_(True)
    _, dd, _ = net.out_grad(x, Bg)
    with pytest.raises(PntfError):
        dd.sum().backward()


@pytest.mark.gpu
def test_fused_bwd_multi_round_matches_two_kernel():
    """the fused input-gradient kernel (pntf_tt_linear_bwd; AUTO took it for layers
    of >= 100 000 points until the split-bf16 GEMMs made the pair faster at every batch, round
    5; PNTF_TT_BWD=1 still selects it) at a size where every workgroup strides over several 32-point blocks
    (8 192 pairs: 16 384 encoder points = 512 blocks per column group over <= 256
    workgroups) agrees with the GEMM + act pair on the loss gradients."""
    from pntf import train
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    n = 8192
    p = {k: torch.from_numpy(v).to(dev) for k, v in W.items() if not k.startswith("encoder1.0")}
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=72)).to(dev)
    yobs = torch.from_numpy(synth.make_speeds(n, seed=73)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(2, 3)).to(dev)
    env = torch.from_numpy(synth.make_env_ids(n, 2)).to(dev)
    out = {}
    saved = train._LINEAR_BWD
    try:
        for mode in (0, 1):
            train._LINEAR_BWD = mode
            grads = {k: torch.empty_like(v) for k, v in p.items()}
            diff = train.loss_grad(p, xp, yobs, Bt, env, 3, 1e-3, 1.0 / n, False, grads)
            out[mode] = (diff, grads)
    finally:
        train._LINEAR_BWD = saved
    assert torch.allclose(out[0][0], out[1][0])
    for k in p:
        a, b = out[0][1][k], out[1][1][k]
        assert float((a - b).abs().max() / b.abs().max()) < 1e-4, k


@pytest.mark.gpu
def test_arm_speed2_vs_oracle():
    """Arm Model.Speed2 (models/model_res_sigmoid.py:1218-1245: the speed at the goal with the
    viscosity term from out_laplace) against the fp64 oracle's Taylor mode, per pair 1e-4."""
    from golden_util import north_star_pairs
    from models import model_res_sigmoid as ma
    dev = torch.device("cuda:0")
    W = _weights("w2", 6)
    sd = torch.load(os.path.join(GOLDEN, "ckpt_w2_d6.pt"), map_location="cpu",
                    weights_only=True)
    m = ma.Model(".", ".", 6, device=dev)
    m.load(os.path.join(GOLDEN, "ckpt_w2_d6.pt"))
    xp = synth.make_box_pairs(100, 6, seed=80)
    gamma = 1e-3
    v = m.Speed2(torch.from_numpy(xp).to(dev), gamma).detach().cpu().numpy()
    t, d, lt = O.laplace(W, xp, sd["B_state_dict"].numpy().T, dim=6)
    D = xp[:, 6:] - xp[:, :6]
    T0 = (D * D).sum(1)
    t = t[:, 0]
    S = T0 * (d[:, 6:] ** 2).sum(1) - 2 * t * (d[:, 6:] * D).sum(1) + t * t
    ref = 1.0 / (np.sqrt(S) / (t * t) + gamma * lt[:, 6:].sum(1))
    north_star_pairs("arm Speed2", v, ref, ref)
