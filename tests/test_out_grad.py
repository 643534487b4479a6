"""Weight gradients through the drop-in `NN.out`.

The reference's τ is nn.Linear + autograd (models/model_res_sigmoid_multi.py:215-259, arm
models/model_res_sigmoid.py:212-256), so a loss written on `net.out(x, B)[0]` trains every
parameter.  tests/golden/make_out_grad_goldens.py recorded the reference's `.grad` after
`(net.out(xp, B)[0][:, 0] * wt).sum().backward()` at the seeded init weights and at the
reference-trained W2 checkpoints, for both models.
  * CPU: the fp64 oracle's `tau_weight_grad` reproduces those gradients;
  * GPU: the drop-in `NN.out` gives the same `.grad` through the HIP value-only tape
    (pntf/train.py tau_weight_grad), leaves encoder1.0 without a gradient as the reference
    does, and `Model.gradient(τ, coords)` (the planner / ∇τ path) never runs the tape.
Tolerance: max-abs error / max |reference| per parameter tensor below 2e-4 (the training
gradients' bound, tests/test_train.py GRAD_TOL; fp32 GEMMs over up to 2n rows).
"""
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, load, north_star_pairs, rel_l2
from oracle import pntf_oracle as O
from pntf import synth

CASES = [("init", 3), ("w2", 3), ("init", 6), ("w2", 6)]
GRAD_TOL = 2e-4


def _weights(tag, dim):
    if tag == "init":
        return synth.make_weights(0)
    sd = torch.load(os.path.join(GOLDEN, "ckpt_w2_d%d.pt" % dim), map_location="cpu",
                    weights_only=True)["model_state_dict"]
    return {k: v.numpy().astype(np.float32) for k, v in sd.items()}


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("tag,dim", CASES)
def test_oracle_tau_weight_grad_vs_reference(tag, dim):
    f = load("out_grad_%s_d%d.npz" % (tag, dim))
    B = f["B"] if dim == 3 else f["B"].T
    t, g, dc = O.tau_weight_grad(_weights(tag, dim), f["xp"], B, f["wt"], dim=dim)
    assert np.abs(t - f["tau"]).max() < 1e-6
    assert rel_l2(dc, f["dcoords"]) < 1e-5
    for k in synth.state_dict_keys():
        if k.startswith("encoder1.0."):
            assert f["grad/" + k].size == 0 and k not in g
        else:
            assert rel_l2(g[k], f["grad/" + k]) < 1e-5, k


def _net(tag, dim, dev, f):
    if dim == 3:
        from models import model_res_sigmoid_multi as md
        net = md.NN(dev, 3)
        call = lambda x: net.out(x, torch.from_numpy(f["B"]).to(dev))  # noqa: E731
    else:
        from models import model_res_sigmoid as ma
        net = ma.NN(dev, 6, torch.from_numpy(f["B"]))
        call = lambda x: net.out(x)  # noqa: E731
    net.load_state_dict({k: torch.from_numpy(v) for k, v in _weights(tag, dim).items()},
                        strict=True)
    net.to(dev)
    return net, call


@pytest.mark.gpu
@pytest.mark.parametrize("tag,dim", CASES)
def test_out_weight_grads_vs_reference(tag, dim):
    dev = torch.device("cuda:0")
    f = load("out_grad_%s_d%d.npz" % (tag, dim))
    net, call = _net(tag, dim, dev, f)
    tau, coords = call(torch.from_numpy(f["xp"]).to(dev))
    (tau[:, 0] * torch.from_numpy(f["wt"]).to(dev)).sum().backward()
    assert np.abs(tau.detach().cpu().numpy()[:, 0] - f["tau"]).max() < 1e-5
    B = f["B"] if dim == 3 else f["B"].T
    north_star_pairs("out_grad_%s_d%d tau" % (tag, dim), tau.detach().cpu().numpy()[:, 0],
                     f["tau"], O.forward(_weights(tag, dim), f["xp"], B, dim=dim)[:, 0])
    assert _rel(coords.grad.detach().cpu().numpy(), f["dcoords"]) < GRAD_TOL
    for k, p in net.named_parameters():
        if k.startswith("encoder1.0."):
            assert p.grad is None, k            # never used (:160, :227): no gradient
        else:
            assert p.grad is not None, k
            assert _rel(p.grad.detach().cpu().numpy(), f["grad/" + k]) < GRAD_TOL, k


@pytest.mark.gpu
def test_out_weight_grads_accumulate_and_ragged():
    """Two backward passes accumulate (.grad += as autograd does); ragged batch sizes (1, 33,
    77) and a per-env B table match the fp64 oracle."""
    from models import model_res_sigmoid_multi as md
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    net.to(dev)
    Bt = synth.make_B_table(3, 3)
    for n in (1, 33, 77):
        net.zero_grad(set_to_none=True)
        xp = synth.make_pairs(n, 3, seed=40 + n)
        env = synth.make_env_ids(n, 3, contiguous=False, seed=n)
        wt = np.linspace(-1.0, 1.0, n).astype(np.float32)
        _, g, _ = O.tau_weight_grad(W, xp, Bt, wt, env=env, dim=3)
        for rep in range(2):
            tau, _ = net.out(torch.from_numpy(xp).to(dev), torch.from_numpy(Bt).to(dev),
                             torch.from_numpy(env).to(dev))
            (tau[:, 0] * torch.from_numpy(wt).to(dev)).sum().backward()
        for k, p in net.named_parameters():
            if k in g:
                assert _rel(p.grad.detach().cpu().numpy(), 2.0 * g[k]) < GRAD_TOL, (n, k)


@pytest.mark.gpu
def test_model_gradient_does_not_run_the_tape(monkeypatch):
    """Model.gradient(τ, coords) = autograd.grad(τ, coords): the weight-gradient node is not on
    the path to coords, so the value tape never runs (the planner/∇τ path costs the same)."""
    from models import model_res_sigmoid_multi as md
    from pntf import train
    calls = []
    real = train.tau_weight_grad
    monkeypatch.setattr(train, "tau_weight_grad", lambda *a, **k: calls.append(1) or real(*a, **k))
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    net.to(dev)
    model = md.Model(".", ".", 3, 2, device=dev)
    model.network = net
    xp = torch.from_numpy(synth.make_pairs(64, 3, seed=5)).to(dev)
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev)
    tau, coords = net.out(xp, B)
    d = model.gradient(tau, coords)
    assert calls == [] and all(p.grad is None for p in net.parameters())
    _, d_ref = O.tau_grad(W, xp.detach().cpu().numpy(), B.detach().cpu().numpy())
    assert rel_l2(d.detach().cpu().numpy(), d_ref) < 1e-4
    with torch.no_grad():                      # no graph: no weight term at all
        t2, _ = net.out(xp, B)
    assert not t2.requires_grad
