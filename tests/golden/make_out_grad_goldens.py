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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
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
