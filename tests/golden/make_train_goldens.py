"""Generate the training-step golden vectors by running the REFERENCE (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_goldens.py [--ref /root/reference]

One inner training step of `Model.train` is `loss, loss_n, diff = self.Loss(points, speed, B,
beta, gamma); loss.backward(); optimizer.step(); optimizer.zero_grad()` with
`torch.optim.AdamW(network.parameters(), lr=1e-3, weight_decay=0.1)`
(models/model_res_sigmoid_multi.py:959-961, 1040-1052; arm: models/model_res_sigmoid.py:954-956,
1062-1075).  This script imports the reference modules (same loader as make_goldens.py), loads
the seeded synthetic weights, and records for each model family:
  * the per-parameter weight gradients of loss.backward() (encoder1.0 has none: the reference
    creates it but never uses it, so AdamW skips it);
  * a few parameters after two AdamW steps on the same batch (checks the moment state).
Only inputs and outputs (data) are written.
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_goldens import load_reference, to_t, weight_checksum  # noqa: E402
from make_goldens import synth  # noqa: E402


# parameters whose post-AdamW values are recorded (the whole set would triple the fixture):
# first and last layers, a generator block, and the unused encoder1.0 (must stay untouched)
AFTER_KEYS = ("encoder.0.weight", "encoder.0.bias", "encoder1.0.weight", "encoder1.0.bias",
              "generator1.1.weight", "generator.4.weight", "generator.4.bias")


def _step_record(model, net, loss_fn, keys):
    import torch
    opt = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    loss, loss_n, diff = loss_fn()
    loss.backward()
    grads = {}
    for k, p in net.named_parameters():
        if p.grad is not None:
            grads[k] = p.grad.detach().numpy().copy()
    opt.step()
    opt.zero_grad()
    loss2, _, _ = loss_fn()
    loss2.backward()
    opt.step()
    opt.zero_grad()
    after = {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}
    out = {"loss_n": np.float64(loss_n.item()), "diff": diff.detach().numpy(),
           "loss2": np.float64(loss2.item())}
    for k in keys:
        if k in grads:
            out["grad:" + k] = grads[k]
        if k in AFTER_KEYS:
            out["after2:" + k] = after[k]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    import torch
    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    md, ma = load_reference(args.ref)
    versions = np.array([torch.__version__, np.__version__])
    W = synth.make_weights(0)
    keys = list(W.keys())
    csum = weight_checksum(W)

    # ---- Gibson multi-env: E=2 environments (Batch Size 2, :1010-1036), beta=1, gamma=1e-3
    net = md.NN("cpu", 3)
    net.load_state_dict({k: to_t(v) for k, v in W.items()}, strict=True)
    net.float()
    model = md.Model(".", ".", 3, 2, device="cpu")
    model.network = net
    E, npe = 2, 48
    Bt = synth.make_B_table(E, 3, first_seed=21)
    pts = synth.make_pairs(E * npe, 3, seed=22).reshape(E, npe, 6)
    yobs = synth.make_speeds(E * npe, seed=23).reshape(E, npe, 2)
    beta, gamma = 1.0, 1e-3

    def loss_d3():
        x = to_t(pts).requires_grad_()        # batch_points.requires_grad_() (:1042)
        return model.Loss(x, to_t(yobs), to_t(Bt), beta, gamma)

    rec = _step_record(model, net, loss_d3, keys)
    np.savez_compressed(os.path.join(args.out, "train_d3.npz"), pts=pts, yobs=yobs, B_table=Bt,
                        beta=np.float64(beta), gamma=np.float64(gamma), weight_checksum=csum,
                        versions=versions, **rec)

    # ---- arm (dim 6): B (128, 6) inside the net, loss_n = sum(diff)/N
    Ba = synth.make_B(6, seed=24, arm=True)
    anet = ma.NN("cpu", 6, to_t(Ba))
    anet.load_state_dict({k: to_t(v) for k, v in W.items()}, strict=True)
    anet.float()
    amodel = ma.Model(".", ".", 6, device="cpu")
    amodel.network = anet
    na = 64
    pts_a = synth.make_box_pairs(na, 6, seed=25)
    yobs_a = synth.make_speeds(na, seed=26)

    def loss_d6():
        x = to_t(pts_a).requires_grad_()
        return amodel.Loss(x, to_t(yobs_a), beta, gamma)

    rec = _step_record(amodel, anet, loss_d6, keys)
    np.savez_compressed(os.path.join(args.out, "train_d6.npz"), pts=pts_a, yobs=yobs_a, B=Ba,
                        beta=np.float64(beta), gamma=np.float64(gamma), weight_checksum=csum,
                        versions=versions, **rec)
    print("training goldens written to", args.out)


if __name__ == "__main__":
    main()
