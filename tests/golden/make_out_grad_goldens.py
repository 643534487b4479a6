"""Golden weight gradients of `NN.out` from the REFERENCE (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_out_grad_goldens.py [--ref /root/reference]

The reference's τ is plain `nn.Linear` + autograd (models/model_res_sigmoid_multi.py:215-259,
arm models/model_res_sigmoid.py:212-256), so a user loss on `NN.out` differentiates into all
trained parameters.  This records, for the seeded init weights (`pntf.synth`) and for the
reference-trained W2 checkpoints (`ckpt_w2_d3.pt`, `ckpt_w2_d6.pt`, loaded through the
reference's own `Model.load`):

    tau, coords = net.out(xp, B)            # arm: net.out(xp)
    (tau[:, 0] * wt).sum().backward()       # per-pair weights wt exercise the incoming gradient

and stores τ, every parameter's `.grad` (encoder1.0 gets none: it is never used, :160, :227)
and coords' gradient.  Only inputs and outputs are written.

`--stage vjp` (round 5) records, at the same weights, the reference's autograd through its
other differentiable outputs, each with seeded per-element weights:

    laplace      tau, dtau, ltau, X = net.out_laplace(coords, B)      (:710-848)
                 (wt·tau + wd·dtau + wl·ltau).sum().backward()
    laplace_sum  the same with wl constant over each endpoint's dim entries (a loss on the
                 per-endpoint Laplacian, as Model.Loss :919-920 uses it)
    grad         tau, dtau, _ = net.out_grad(coords, B); (wt·tau + wd·dtau).sum()  (:303-400)
    backgrad     the same through net.out_backgrad (:402-647, encoder[0] quirk :435-438;
                 arm :300-511)
    gradient2    tau, X = net.out(x, B); dtau = Model.gradient(tau, X) (create_graph=True,
                 :890-896); (wt·tau + wd·dtau).sum()

into vjp_{init,w2}_d{3,6}.npz: the outputs, coords' gradient, and per parameter a digest of
its `.grad` (the bias / head gradients whole; per weight matrix seeded rows and a 16-vector
sketch: tests/golden_util.py grad_digest) so the fixtures stay ~100 KB each.
"""
import argparse
import os
import pickle
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "p-ntfields_amd"))
from pntf import synth  # noqa: E402


def load_reference(ref):
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.modules.setdefault("pickle5", pickle)
    sys.path.insert(0, ref)
    from models import model_res_sigmoid_multi as md
    from models import model_res_sigmoid as ma
    return md, ma


def record(net, xp, wt, call):
    import torch
    net.zero_grad(set_to_none=True)
    tau, coords = call(torch.tensor(xp))
    (tau[:, 0] * torch.tensor(wt)).sum().backward()
    out = {"tau": tau.detach().numpy()[:, 0], "xp": xp, "wt": wt}
    # coords is a fresh leaf inside NN.out (:217); its grad is autograd's ∇τ·wt
    out["dcoords"] = coords.grad.numpy() if coords.grad is not None else np.zeros_like(xp)
    for k, p in net.named_parameters():
        out["grad/" + k] = p.grad.numpy().copy() if p.grad is not None else np.zeros(0, np.float32)
    return out


def _digest_into(out, prefix, net):
    from golden_util import grad_digest
    for k, p in net.named_parameters():
        if p.grad is None:
            out[prefix + "g/" + k + "/none"] = np.zeros(0, np.float32)
            continue
        for kk, v in grad_digest(k, p.grad.numpy()).items():
            out[prefix + "g/" + k + "/" + kk] = np.asarray(v)


def record_vjp(net, model, xp, E, dim, wts, calls):
    """Every method of the module docstring's --stage vjp list at the current weights."""
    import torch
    out = {"xp": xp, "E": np.int32(E)}
    for k, v in wts.items():
        out["w/" + k] = v
    n = xp.shape[0]
    wt, wd, wl = (torch.tensor(wts[k]) for k in ("wt", "wd", "wl"))
    wls = torch.tensor(np.repeat(wts["wl_sum"], dim, axis=1))
    for meth in ("laplace", "laplace_sum", "grad", "backgrad", "gradient2"):
        net.zero_grad(set_to_none=True)
        x = torch.tensor(xp).requires_grad_(True)
        if meth.startswith("laplace"):
            xin = x.view(E, n // E, 2 * dim) if E else x
            tau, dtau, ltau, X = calls["laplace"](xin)
            tau, dtau, ltau = tau.reshape(n), dtau.reshape(n, 2 * dim), ltau.reshape(n, 2 * dim)
            loss = (wt * tau).sum() + (wd * dtau).sum() + \
                ((wl if meth == "laplace" else wls) * ltau).sum()
            out[meth + "/ltau"] = ltau.detach().numpy()
            # the arm's out_laplace detaches coords and returns a fresh leaf (:678): its
            # gradient lands there; the multi model's returns the caller's coords (:848)
            leaf = X if X.is_leaf else x
        elif meth == "gradient2":
            tau, leaf = calls["out"](x.detach())
            dtau = model.gradient(tau, leaf)
            tau = tau.reshape(n)
            loss = (wt * tau).sum() + (wd * dtau).sum()
        else:
            tau, dtau, _ = calls[meth](x)
            tau = tau.reshape(n)
            loss = (wt * tau).sum() + (wd * dtau.reshape(n, 2 * dim)).sum()
            leaf = x
        loss.backward()
        out[meth + "/tau"] = tau.detach().numpy()
        out[meth + "/dtau"] = dtau.detach().reshape(n, 2 * dim).numpy()
        out[meth + "/dcoords"] = (leaf.grad.numpy() if leaf.grad is not None
                                  else np.zeros_like(xp))
        _digest_into(out, meth + "/", net)
    return out


def main_vjp(args):
    import torch
    sys.path.insert(0, os.path.dirname(HERE))            # tests/ (golden_util)
    md, ma = load_reference(args.ref)
    versions = np.array([torch.__version__, np.__version__])
    W = {k: torch.tensor(v) for k, v in synth.make_weights(0).items()}
    rng = np.random.Generator(np.random.PCG64(51))

    def weights(n, dim):
        return {"wt": rng.uniform(-1, 1, n).astype(np.float32),
                "wd": rng.uniform(-1, 1, (n, 2 * dim)).astype(np.float32),
                "wl": rng.uniform(-1, 1, (n, 2 * dim)).astype(np.float32),
                "wl_sum": rng.uniform(-1, 1, (n, 2)).astype(np.float32)}

    # ---- Gibson multi model, dim 3: out_laplace over E = 2 environments (per-env B table);
    # out_grad / out_backgrad / out take the first environment's single B, as the reference's
    # scripts call them (test/gib_plan.py)
    E, ne = 2, 40
    xp3 = synth.make_pairs(E * ne, 3, seed=52)
    Bt = torch.tensor(synth.make_B_table(E, 3, first_seed=53))
    w3 = weights(E * ne, 3)
    for tag, ckpt in (("init", None), ("w2", os.path.join(HERE, "ckpt_w2_d3.pt"))):
        m = md.Model(".", ".", 3, 2, device="cpu")
        if ckpt is None:
            m.network = md.NN("cpu", 3)
            m.network.load_state_dict(W, strict=True)
        else:
            m.load(ckpt)
        net = m.network.float()
        B0 = Bt[0]
        calls = {"laplace": lambda x: net.out_laplace(x, Bt),
                 "grad": lambda x: net.out_grad(x, B0),
                 "backgrad": lambda x: net.out_backgrad(x, B0),
                 "out": lambda x: net.out(x, B0)}
        res = record_vjp(net, m, xp3, E, 3, w3, calls)
        np.savez_compressed(os.path.join(args.out, "vjp_%s_d3.npz" % tag), Btab=Bt.numpy(),
                            versions=versions, **res)

    # ---- UR5 arm model, dim 6 (B held in the net)
    n6 = 64
    xp6 = synth.make_box_pairs(n6, 6, seed=54)
    w6 = weights(n6, 6)
    Ba = torch.tensor(synth.make_B(6, seed=12, arm=True))
    for tag, ckpt in (("init", None), ("w2", os.path.join(HERE, "ckpt_w2_d6.pt"))):
        m = ma.Model(".", ".", 6, device="cpu")
        if ckpt is None:
            m.network = ma.NN("cpu", 6, Ba)
            m.network.load_state_dict(W, strict=True)
            B = Ba
        else:
            m.load(ckpt)
            B = m.B
        net = m.network.float()
        calls = {"laplace": lambda x: net.out_laplace(x), "grad": lambda x: net.out_grad(x),
                 "backgrad": lambda x: net.out_backgrad(x), "out": lambda x: net.out(x)}
        res = record_vjp(net, m, xp6, 0, 6, w6, calls)
        np.savez_compressed(os.path.join(args.out, "vjp_%s_d6.npz" % tag),
                            B=np.asarray(B.detach().numpy(), np.float32), versions=versions,
                            **res)
    print("wrote vjp_{init,w2}_d{3,6}.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--stage", choices=["out", "vjp"], default="out")
    args = ap.parse_args()
    if args.stage == "vjp":
        return main_vjp(args)
    import torch
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    md, ma = load_reference(args.ref)
    versions = np.array([torch.__version__, np.__version__])
    W = {k: torch.tensor(v) for k, v in synth.make_weights(0).items()}
    rng = np.random.Generator(np.random.PCG64(31))

    # ---- Gibson multi model, dim 3
    n3 = 300
    xp3 = synth.make_pairs(n3, 3, seed=32)
    wt3 = rng.uniform(-1.0, 1.0, size=n3).astype(np.float32)
    B3 = torch.tensor(synth.make_B(3, seed=1))
    for tag, ckpt in (("init", None), ("w2", os.path.join(HERE, "ckpt_w2_d3.pt"))):
        m = md.Model(".", ".", 3, 2, device="cpu")
        if ckpt is None:
            m.network = md.NN("cpu", 3)
            m.network.load_state_dict(W, strict=True)
        else:
            m.load(ckpt)
        net = m.network.float()
        res = record(net, xp3, wt3, lambda x: net.out(x, B3))
        np.savez_compressed(os.path.join(args.out, "out_grad_%s_d3.npz" % tag), B=B3.numpy(),
                            versions=versions, **res)

    # ---- UR5 arm model, dim 6 (B held in the net, models/model_res_sigmoid.py:139)
    n6 = 200
    xp6 = synth.make_box_pairs(n6, 6, seed=33)
    wt6 = rng.uniform(-1.0, 1.0, size=n6).astype(np.float32)
    Ba = torch.tensor(synth.make_B(6, seed=12, arm=True))
    for tag, ckpt in (("init", None), ("w2", os.path.join(HERE, "ckpt_w2_d6.pt"))):
        m = ma.Model(".", ".", 6, device="cpu")
        if ckpt is None:
            m.network = ma.NN("cpu", 6, Ba)
            m.network.load_state_dict(W, strict=True)
            B = Ba
        else:
            m.load(ckpt)
            B = m.B
        net = m.network.float()
        res = record(net, xp6, wt6, lambda x: net.out(x))
        np.savez_compressed(os.path.join(args.out, "out_grad_%s_d6.npz" % tag),
                            B=np.asarray(B.detach().numpy(), np.float32), versions=versions,
                            **res)
    print("wrote out_grad_{init,w2}_d{3,6}.npz")


if __name__ == "__main__":
    main()
