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
