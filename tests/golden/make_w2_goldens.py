"""Trained-weight (W2) goldens and reference-written checkpoints (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_w2_goldens.py [--ref /root/reference]
        [--steps 400] [--stage all|train|goldens|c5]

SURVEY.md §8c F5 / VERDICT r01 items 2 and 7.  The random-init goldens (make_goldens.py)
leave softplus mostly unsaturated and plans short (22-25 steps).  This script, importing the
reference the same way as make_goldens.py:

1. train: starts from the seeded weights (pntf.synth, seed 0) and runs `--steps` reference
   training steps — `loss = Model.Loss(...)`, `loss.backward()`, `torch.optim.AdamW(lr 1e-3,
   wd 0.1).step()` (models/model_res_sigmoid_multi.py:959-961, 1070-1080; arm
   models/model_res_sigmoid.py:954-956, 1065-1075) — on an analytic speed field: the speed
   of a point is clip(d/margin, 0.1, 1), d = distance to a few seeded spheres
   (dataprocessing/speed_sampling_gpu.py:418-419 maps obstacle distance to speed the same
   way).  It then saves each model with the REFERENCE's own `Model.save` (multi :1143-1152,
   arm :1139-1148) into tests/golden/ckpt_w2_{d3,d6}.pt.  To keep the fixtures small the
   saved `optimizer_state_dict` is that of a fresh AdamW over the trained network (the
   reference's `load` never reads it).
2. goldens: reloads those files through the REFERENCE's own `Model.load` (the arm one restores
   `B_state_dict`) and records outputs at the trained weights: τ/∇τ/out_grad/out_backgrad/
   Gradient/Speed/TravelTimes, out_laplace + Loss, and batch-1 planner loops
   (test/gib_plan.py:74-86, test/arm_plan.py:140-152) on long queries.
3. c5: the C5 workload (1024 arm queries, synth.make_box_pairs(1024, 6, seed=3), step 0.015,
   tol 0.03) as 1024 independent batch-1 reference loops capped at 199 steps (the bench's
   max_iter): iteration counts, final states and the first 16 full paths.
4. train_grads: at the same reloaded checkpoints, the reference's training step on batches of
   the trained field — every parameter's `loss.backward()` gradient and selected parameters
   after two AdamW steps (train_w2_d{3,6}.npz; make_train_goldens.py's recorder).

Only inputs and outputs (data) and the reference-written checkpoints are stored.
"""
import argparse
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_goldens import load_reference, to_t, weight_checksum  # noqa: E402
from make_goldens import synth  # noqa: E402


# ------------------------------------------------------------------ analytic speed fields
def sphere_field(dim, k, seed, margin):
    rng = np.random.Generator(np.random.PCG64(seed))
    c = rng.uniform(-0.35, 0.35, size=(k, dim))
    r = rng.uniform(0.05, 0.15, size=(k,))

    def speed(x):
        d = np.linalg.norm(x[:, None, :] - c[None], axis=-1) - r[None]
        return np.clip(np.maximum(d.min(1), 0.0) / margin, 0.1, 1.0).astype(np.float32)
    return speed


def field_speeds(xp, speed, dim):
    return np.stack([speed(xp[:, :dim]), speed(xp[:, dim:])], 1).astype(np.float32)


def planner_loop(grad_fn, x0, dim, step, tol, cap):
    """Batch-1 reference loop (test/gib_plan.py:74-86, test/arm_plan.py:140-152)."""
    import torch
    XP = to_t(x0[None])
    pts = [XP.detach().clone()]
    dis = torch.norm(XP[:, dim:] - XP[:, :dim])
    it = 0
    while dis > tol:
        g = grad_fn(XP.clone())
        XP = (XP + step * g).detach()
        dis = torch.norm(XP[:, dim:] - XP[:, :dim])
        pts.append(XP.clone())
        it += 1
        if it > cap:
            break
    return torch.cat(pts).numpy(), it


def pack_paths(runs, cap, width):
    paths = np.zeros((len(runs), cap + 2, width), np.float32)
    iters = np.zeros(len(runs), np.int32)
    for q, (arr, it) in enumerate(runs):
        paths[q, :arr.shape[0]] = arr
        paths[q, arr.shape[0]:] = arr[-1]
        iters[q] = it
    return paths, iters


def saturation(W, xp, B, dim):
    """Fraction of encoder/generator pre-activations y with 10y > 20 (torch Softplus's
    identity branch) at these weights — reported so the fixture documents what it covers."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import pntf_oracle as O
    return float(O.softplus_saturation(W, xp.astype(np.float64), B.astype(np.float64), dim))


# ------------------------------------------------------------------ stage 1: training
def train_multi(md, steps, out, log):
    import torch
    W0 = synth.make_weights(0)
    net = md.NN("cpu", 3)
    net.load_state_dict({k: to_t(v) for k, v in W0.items()}, strict=True)
    net.float()
    model = md.Model(out, ".", 3, 2, device="cpu")
    model.network = net
    opt = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    E, n = 2, 4000
    Bt = synth.make_B_table(E, 3, first_seed=41)
    fields = [sphere_field(3, 6, 51 + e, 1.0) for e in range(E)]
    for s in range(steps):
        xp = synth.make_pairs(E * n, 3, seed=1000 + s).reshape(E, n, 6)
        y = np.stack([field_speeds(xp[e], fields[e], 3) for e in range(E)])
        x = to_t(xp).requires_grad_()
        loss, loss_n, _ = model.Loss(x, to_t(y), to_t(Bt), 1.0, 1e-3)
        loss.backward()
        opt.step()
        opt.zero_grad()
        if s % 25 == 0 or s == steps - 1:
            log("multi step %d loss_n %.5f" % (s, loss_n.item()))
    model.B = to_t(Bt[0])
    model.optimizer = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    model.total_train_loss = [loss.detach()]
    model.save(epoch=steps, val_loss=float(loss_n.item()))
    src = [f for f in os.listdir(out) if f.startswith("Model_Epoch_%05d" % steps)][0]
    os.replace(os.path.join(out, src), os.path.join(out, "ckpt_w2_d3.pt"))


def train_arm(ma, steps, out, log):
    import torch
    W0 = synth.make_weights(0)
    Ba = synth.make_B(6, seed=61, arm=True)               # (128, 6)
    net = ma.NN("cpu", 6, to_t(Ba))
    net.load_state_dict({k: to_t(v) for k, v in W0.items()}, strict=True)
    net.float()
    model = ma.Model(out, ".", 6, device="cpu")
    model.network = net
    opt = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    field = sphere_field(6, 8, 62, 1.5)
    n = 4000
    for s in range(steps):
        xp = synth.make_box_pairs(n, 6, seed=2000 + s)
        y = field_speeds(xp, field, 6)
        x = to_t(xp).requires_grad_()
        loss, loss_n, _ = model.Loss(x, to_t(y), 1.0, 1e-3)
        loss.backward()
        opt.step()
        opt.zero_grad()
        if s % 25 == 0 or s == steps - 1:
            log("arm step %d loss_n %.5f" % (s, loss_n.item()))
    model.B = to_t(Ba)
    model.optimizer = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    model.total_train_loss = [loss.detach()]
    model.save(epoch=steps, val_loss=float(loss_n.item()))
    src = [f for f in os.listdir(out) if f.startswith("Model_Epoch_%05d" % steps)][0]
    os.replace(os.path.join(out, src), os.path.join(out, "ckpt_w2_d6.pt"))


# ------------------------------------------------------------------ stage 2: goldens
def state_np(net):
    return {k: v.detach().numpy().astype(np.float32) for k, v in net.state_dict().items()}


def goldens_multi(md, out, log):
    import torch
    model = md.Model(out, ".", 3, 2, device="cpu")
    model.load(os.path.join(out, "ckpt_w2_d3.pt"))           # the reference's own loader
    net = model.network
    W = state_np(net)
    csum = weight_checksum(W)
    Bt = synth.make_B_table(2, 3, first_seed=41)
    B = Bt[0]
    model.B = to_t(B)
    n = 1024
    xp = synth.make_pairs(n, 3, seed=71)
    tau, coords = net.out(to_t(xp), to_t(B))
    dtau = model.gradient(tau, coords)
    _, dtau_fwd, _ = net.out_grad(to_t(xp), to_t(B))
    tau_bg, dtau_bg, _ = net.out_backgrad(to_t(xp), to_t(B))
    sat = saturation(W, xp, B, 3)
    np.savez_compressed(
        os.path.join(out, "fwd_grad_w2_d3.npz"), xp=xp, B=B, tau=tau.detach().numpy(),
        dtau=dtau.detach().numpy(), dtau_fwdmode=dtau_fwd.detach().numpy(),
        tau_backgrad=tau_bg.detach().numpy(), dtau_backgrad=dtau_bg.detach().numpy(),
        gradient=model.Gradient(to_t(xp), to_t(B)).detach().numpy(),
        speed=model.Speed(to_t(xp)).detach().numpy(),
        travel_time=model.TravelTimes(to_t(xp)).detach().numpy(),
        softplus_saturation=np.float64(sat), weight_checksum=csum)
    log("multi W2: softplus saturation %.4f, tau range %.3f..%.3f" % (
        sat, float(tau.min()), float(tau.max())))
    E, npe = 2, 64
    fields = [sphere_field(3, 6, 51 + e, 1.0) for e in range(E)]
    pts = synth.make_pairs(E * npe, 3, seed=72).reshape(E, npe, 6)
    yobs = np.stack([field_speeds(pts[e], fields[e], 3) for e in range(E)])
    tl, dl, ll, _ = net.out_laplace(to_t(pts), to_t(Bt))
    _, loss_n, diff = model.Loss(to_t(pts), to_t(yobs), to_t(Bt), 1.0, 1e-3)
    np.savez_compressed(
        os.path.join(out, "loss_w2_d3.npz"), pts=pts, yobs=yobs, B_table=Bt,
        gamma=np.float64(1e-3), tau=tl.detach().numpy(), dtau=dl.detach().numpy(),
        ltau=ll.detach().numpy(), diff=diff.detach().numpy(),
        loss_n=np.float64(loss_n.item()), weight_checksum=csum)
    # planner: the demo query plus long corner-to-corner queries (test/gib_plan.py:51-97)
    demo = np.array([[-6, -7, -6, 2, 7, -2.5]], np.float32) / 20.0
    rng = np.random.Generator(np.random.PCG64(73))
    cs = rng.uniform(-0.45, -0.2, size=(15, 3)) * rng.choice([-1, 1], size=(15, 3))
    starts = np.concatenate([demo, np.concatenate([cs, -cs + rng.uniform(-0.05, 0.05, (15, 3))],
                                                  1)]).astype(np.float32)
    cap = 500
    runs = [planner_loop(lambda x: model.Gradient(x, to_t(B)), starts[q], 3, 0.03, 0.06, cap)
            for q in range(starts.shape[0])]
    paths, iters = pack_paths(runs, cap, 6)
    log("multi W2 plans: iters %s" % iters.tolist())
    np.savez_compressed(os.path.join(out, "plan_gib_w2.npz"), starts=starts, B=B, paths=paths,
                        iters=iters, step=np.float64(0.03), tol=np.float64(0.06),
                        max_iter=np.int32(cap), weight_checksum=csum)


def arm_model(ma, out):
    model = ma.Model(out, ".", 6, device="cpu")
    model.load(os.path.join(out, "ckpt_w2_d6.pt"))           # restores B_state_dict
    return model


def goldens_arm(ma, out, log):
    import torch
    model = arm_model(ma, out)
    net = model.network
    W = state_np(net)
    csum = weight_checksum(W)
    Ba = model.B.detach().numpy().astype(np.float32)          # (128, 6)
    na = 256
    xpa = synth.make_box_pairs(na, 6, seed=81)
    tau, coords = net.out(to_t(xpa))
    dtau = model.gradient(tau, coords)
    grad16 = np.concatenate([model.Gradient(to_t(xpa[i:i + 1])).detach().numpy()
                             for i in range(16)])
    sat = saturation(W, xpa, Ba.T, 6)
    np.savez_compressed(os.path.join(out, "fwd_grad_w2_d6.npz"), xp=xpa, B=Ba,
                        tau=tau.detach().numpy(), dtau=dtau.detach().numpy(),
                        gradient16=grad16, softplus_saturation=np.float64(sat),
                        weight_checksum=csum)
    log("arm W2: softplus saturation %.4f" % sat)
    field = sphere_field(6, 8, 62, 1.5)
    nl = 64
    pts = synth.make_box_pairs(nl, 6, seed=82)
    yobs = field_speeds(pts, field, 6)
    tl, dl, ll, _ = net.out_laplace(to_t(pts))
    _, lna, dfa = model.Loss(to_t(pts), to_t(yobs), 1.0, 1e-3)
    np.savez_compressed(os.path.join(out, "loss_w2_d6.npz"), pts=pts, yobs=yobs, B=Ba,
                        gamma=np.float64(1e-3), tau=tl.detach().numpy(),
                        dtau=dl.detach().numpy(), ltau=ll.detach().numpy(),
                        diff=dfa.detach().numpy(), loss_n=np.float64(lna.item()),
                        weight_checksum=csum)
    rng = np.random.Generator(np.random.PCG64(83))
    cs = rng.uniform(-0.5, -0.25, size=(8, 6)) * rng.choice([-1, 1], size=(8, 6))
    starts = np.concatenate([cs, -cs], 1).astype(np.float32)
    cap = 300
    runs = [planner_loop(model.Gradient, starts[q], 6, 0.015, 0.03, cap)
            for q in range(starts.shape[0])]
    paths, iters = pack_paths(runs, cap, 12)
    log("arm W2 plans: iters %s" % iters.tolist())
    np.savez_compressed(os.path.join(out, "plan_arm_w2.npz"), starts=starts, B=Ba, paths=paths,
                        iters=iters, step=np.float64(0.015), tol=np.float64(0.03),
                        max_iter=np.int32(cap), weight_checksum=csum)


def goldens_c5(ma, out, log, q=1024, cap=199, keep=16):
    model = arm_model(ma, out)
    csum = weight_checksum(state_np(model.network))
    xq = synth.make_box_pairs(q, 6, seed=3)
    final = np.zeros((q, 12), np.float32)
    iters = np.zeros(q, np.int32)
    full = []
    t0 = time.time()
    for i in range(q):
        arr, it = planner_loop(model.Gradient, xq[i], 6, 0.015, 0.03, cap)
        final[i], iters[i] = arr[-1], it
        if i < keep:
            full.append((arr, it))
        if i % 128 == 0:
            log("c5 query %d/%d (%.0f s)" % (i, q, time.time() - t0))
    paths, _ = pack_paths(full, cap, 12)
    log("c5 W2: mean %.1f max %d steps, %d capped" % (iters.mean(), iters.max(),
                                                     int((iters > cap).sum())))
    np.savez_compressed(os.path.join(out, "plan_c5_w2.npz"), xq=xq, final=final, iters=iters,
                        paths16=paths, step=np.float64(0.015), tol=np.float64(0.03),
                        max_iter=np.int32(cap), weight_checksum=csum)


def goldens_train(md, ma, out, log):
    """The reference's training step at the trained weights:
    `loss.backward()` gradients of every parameter and selected parameters after two
    torch.optim.AdamW steps (models/model_res_sigmoid_multi.py:1070-1080; arm
    models/model_res_sigmoid.py:1065-1075), on batches of the analytic field the weights were
    trained on, so the saturated-softplus regime of the Taylor adjoint is exercised."""
    from make_train_goldens import _step_record
    import torch
    model = md.Model(out, ".", 3, 2, device="cpu")
    model.load(os.path.join(out, "ckpt_w2_d3.pt"))
    net = model.network
    net.train()
    W = state_np(net)
    keys = list(W.keys())
    E, npe = 2, 96
    Bt = synth.make_B_table(E, 3, first_seed=41)
    fields = [sphere_field(3, 6, 51 + e, 1.0) for e in range(E)]
    pts = synth.make_pairs(E * npe, 3, seed=91).reshape(E, npe, 6)
    yobs = np.stack([field_speeds(pts[e], fields[e], 3) for e in range(E)])
    sat = saturation(W, pts.reshape(-1, 6), Bt[0], 3)

    def loss_d3():
        x = to_t(pts).requires_grad_()
        return model.Loss(x, to_t(yobs), to_t(Bt), 1.0, 1e-3)
    rec = _step_record(model, net, loss_d3, keys)
    np.savez_compressed(os.path.join(out, "train_w2_d3.npz"), pts=pts, yobs=yobs, B_table=Bt,
                        beta=np.float64(1.0), gamma=np.float64(1e-3),
                        weight_checksum=weight_checksum(W), softplus_saturation=np.float64(sat),
                        versions=np.array([torch.__version__, np.__version__]), **rec)
    log("train W2 d3: loss_n %.5f, saturation %.4f" % (float(rec["loss_n"]), sat))
    amodel = arm_model(ma, out)
    anet = amodel.network
    anet.train()
    Wa = state_np(anet)
    Ba = amodel.B.detach().numpy().astype(np.float32)
    field = sphere_field(6, 8, 62, 1.5)
    na = 128
    pts_a = synth.make_box_pairs(na, 6, seed=92)
    yobs_a = field_speeds(pts_a, field, 6)
    sat = saturation(Wa, pts_a, Ba.T, 6)

    def loss_d6():
        x = to_t(pts_a).requires_grad_()
        return amodel.Loss(x, to_t(yobs_a), 1.0, 1e-3)
    rec = _step_record(amodel, anet, loss_d6, list(Wa.keys()))
    np.savez_compressed(os.path.join(out, "train_w2_d6.npz"), pts=pts_a, yobs=yobs_a, B=Ba,
                        beta=np.float64(1.0), gamma=np.float64(1e-3),
                        weight_checksum=weight_checksum(Wa), softplus_saturation=np.float64(sat),
                        versions=np.array([torch.__version__, np.__version__]), **rec)
    log("train W2 d6: loss_n %.5f, saturation %.4f" % (float(rec["loss_n"]), sat))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--steps", type=int, default=400)   # the committed checkpoints: epoch 400
    ap.add_argument("--stage", default="all",
                    choices=["all", "train", "goldens", "c5", "train_grads"])
    args = ap.parse_args()
    import torch
    torch.manual_seed(0)
    random.seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    md, ma = load_reference(args.ref)
    t0 = time.time()

    def log(msg):
        print("[%6.0f s] %s" % (time.time() - t0, msg), flush=True)
    if args.stage in ("all", "train"):
        train_multi(md, args.steps, args.out, log)
        train_arm(ma, args.steps, args.out, log)
    if args.stage in ("all", "goldens"):
        goldens_multi(md, args.out, log)
        goldens_arm(ma, args.out, log)
    if args.stage in ("all", "c5"):
        goldens_c5(ma, args.out, log)
    if args.stage in ("all", "train_grads"):
        goldens_train(md, ma, args.out, log)
    log("done")


if __name__ == "__main__":
    main()
