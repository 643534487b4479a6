"""Generate golden vectors by running the REFERENCE implementation (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py [--ref /root/reference]

Imports yhsong0804/P-NTFields' own `models/model_res_sigmoid_multi.py` and
`models/model_res_sigmoid.py` from the read-only reference checkout (with `pickle5`
aliased to `pickle`; it is only used by `Model.train`, model_res_sigmoid_multi.py:25,990),
loads the seeded synthetic weights of `pntf.synth` with `load_state_dict(strict=True)`,
and records the reference's outputs.  Inputs are regenerated from the same seeds at test
time; each fixture also stores its inputs (small) and a weight checksum so a drift in the
generator is caught.  The planner goldens run the reference loop bodies of
`test/gib_plan.py:74-86` / `test/arm_plan.py:140-152` with batch 1, one query at a time
(those scripts import igl/open3d at top level and cannot be imported here).

Only outputs and inputs (data) are written; nothing from the reference source is copied.
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


def weight_checksum(w):
    return np.array([float(np.sum(np.abs(v.astype(np.float64)))) for v in w.values()])


def load_reference(ref):
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.modules.setdefault("pickle5", pickle)
    sys.path.insert(0, ref)
    import torch  # noqa: F401
    from models import model_res_sigmoid_multi as md
    from models import model_res_sigmoid as ma
    return md, ma


def to_t(a):
    import torch
    return torch.tensor(np.asarray(a), dtype=torch.float32)


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
    sd = {k: to_t(v) for k, v in W.items()}
    csum = weight_checksum(W)

    # ---------------------------------------------------------------- F1 Gibson tau/grad
    net = md.NN("cpu", 3)
    net.load_state_dict(sd, strict=True)
    net.float().eval()
    model = md.Model(".", ".", 3, 2, device="cpu")
    model.network = net
    B = synth.make_B(3, seed=1)
    model.B = to_t(B)
    n = 1024
    xp = synth.make_pairs(n, 3, seed=2)
    tau, coords = net.out(to_t(xp), to_t(B))
    dtau = model.gradient(tau, coords)
    _, dtau_fwd, _ = net.out_grad(to_t(xp), to_t(B))
    tau_bg, dtau_bg, _ = net.out_backgrad(to_t(xp), to_t(B))
    grad_vel = model.Gradient(to_t(xp), to_t(B))
    spd = model.Speed(to_t(xp))
    tt = model.TravelTimes(to_t(xp))
    np.savez_compressed(
        os.path.join(args.out, "fwd_grad_d3.npz"),
        xp=xp, B=B, tau=tau.detach().numpy(), dtau=dtau.detach().numpy(),
        dtau_fwdmode=dtau_fwd.detach().numpy(), tau_backgrad=tau_bg.detach().numpy(),
        dtau_backgrad=dtau_bg.detach().numpy(), gradient=grad_vel.detach().numpy(),
        speed=spd.detach().numpy(), travel_time=tt.detach().numpy(),
        weight_checksum=csum, versions=versions)

    # ---------------------------------------------------------------- F1b per-env B table
    n_env, n_per = 4, 128
    Bt = synth.make_B_table(n_env, 3, first_seed=1)
    xpe = synth.make_pairs(n_env * n_per, 3, seed=7)
    env = synth.make_env_ids(n_env * n_per, n_env, contiguous=False, seed=8)
    tau_e = np.zeros((n_env * n_per, 1), np.float32)
    dtau_e = np.zeros((n_env * n_per, 6), np.float32)
    dtau_bg_e = np.zeros((n_env * n_per, 6), np.float32)
    for e in range(n_env):
        idx = np.nonzero(env == e)[0]
        t, c = net.out(to_t(xpe[idx]), to_t(Bt[e]))
        g = model.gradient(t, c)
        _, gb, _ = net.out_backgrad(to_t(xpe[idx]), to_t(Bt[e]))
        tau_e[idx] = t.detach().numpy()
        dtau_e[idx] = g.detach().numpy()
        dtau_bg_e[idx] = gb.detach().numpy()
    np.savez_compressed(
        os.path.join(args.out, "fwd_grad_env_d3.npz"), xp=xpe, B_table=Bt, env=env,
        tau=tau_e, dtau=dtau_e, dtau_backgrad=dtau_bg_e, weight_checksum=csum,
        versions=versions)

    # ---------------------------------------------------------------- F2 Eikonal residual
    E, npe = 10, 64
    BtL = synth.make_B_table(E, 3, first_seed=1)
    pts = synth.make_pairs(E * npe, 3, seed=9).reshape(E, npe, 6)
    yobs = synth.make_speeds(E * npe, seed=10).reshape(E, npe, 2)
    gamma = 1e-3
    tau_l, dtau_l, ltau_l, _ = net.out_laplace(to_t(pts), to_t(BtL))
    loss, loss_n, diff = model.Loss(to_t(pts), to_t(yobs), to_t(BtL), 1.0, gamma)
    np.savez_compressed(
        os.path.join(args.out, "loss_d3.npz"), pts=pts, yobs=yobs, B_table=BtL,
        gamma=np.float64(gamma), tau=tau_l.detach().numpy(), dtau=dtau_l.detach().numpy(),
        ltau=ltau_l.detach().numpy(), diff=diff.detach().numpy(),
        loss_n=np.float64(loss_n.item()), weight_checksum=csum, versions=versions)

    # ---------------------------------------------------------------- F3 Gibson planner
    demo = np.array([[-6, -7, -6, 2, 7, -2.5]], np.float32) / 20.0   # test/gib_plan.py:53-58
    starts = np.concatenate([demo, synth.make_pairs(15, 3, seed=11)]).astype(np.float32)
    cap = 500
    paths = np.zeros((starts.shape[0], cap + 2, 6), np.float32)
    iters = np.zeros(starts.shape[0], np.int32)
    Bg = to_t(B)
    for qi in range(starts.shape[0]):
        XP = to_t(starts[qi:qi + 1])
        pts_q = [XP.detach().clone()]
        dis = torch.norm(XP[:, 3:6] - XP[:, 0:3])
        it = 0
        while dis > 0.06:
            g = model.Gradient(XP.clone(), Bg)
            XP = (XP + 0.03 * g).detach()
            dis = torch.norm(XP[:, 3:6] - XP[:, 0:3])
            pts_q.append(XP.clone())
            it += 1
            if it > cap:
                break
        arr = torch.cat(pts_q).numpy()
        paths[qi, :arr.shape[0]] = arr
        paths[qi, arr.shape[0]:] = arr[-1]
        iters[qi] = it
    np.savez_compressed(os.path.join(args.out, "plan_gib.npz"), starts=starts, B=B,
                        paths=paths, iters=iters, step=np.float64(0.03), tol=np.float64(0.06),
                        max_iter=np.int32(cap), weight_checksum=csum, versions=versions)

    # ---------------------------------------------------------------- F4 arm (dim 6)
    Ba = synth.make_B(6, seed=12, arm=True)                 # (128, 6)
    anet = ma.NN("cpu", 6, to_t(Ba))
    anet.load_state_dict(sd, strict=True)
    anet.float().eval()
    amodel = ma.Model(".", ".", 6, device="cpu")
    amodel.network = anet
    amodel.B = to_t(Ba)
    na = 256
    xpa = synth.make_box_pairs(na, 6, seed=13)
    tau_a, coords_a = anet.out(to_t(xpa))
    dtau_a = amodel.gradient(tau_a, coords_a)
    grad_a = np.concatenate([amodel.Gradient(to_t(xpa[i:i + 1])).detach().numpy()
                             for i in range(16)])
    np.savez_compressed(os.path.join(args.out, "fwd_grad_d6.npz"), xp=xpa, B=Ba,
                        tau=tau_a.detach().numpy(), dtau=dtau_a.detach().numpy(),
                        gradient16=grad_a, weight_checksum=csum, versions=versions)

    # F5: arm Taylor mode + the arm loss variant (models/model_res_sigmoid.py:676-935)
    nl = 64
    pts_a = synth.make_box_pairs(nl, 6, seed=15)
    yobs_a = synth.make_speeds(nl, seed=16)
    tl, dl, ll, _ = anet.out_laplace(to_t(pts_a))
    la, lna, dfa = amodel.Loss(to_t(pts_a), to_t(yobs_a), 1.0, 1e-3)
    np.savez_compressed(os.path.join(args.out, "loss_d6.npz"), pts=pts_a, yobs=yobs_a, B=Ba,
                        gamma=np.float64(1e-3), tau=tl.detach().numpy(),
                        dtau=dl.detach().numpy(), ltau=ll.detach().numpy(),
                        diff=dfa.detach().numpy(), loss_n=np.float64(lna.item()),
                        weight_checksum=csum, versions=versions)

    base = np.array([[0, -0.5 * np.pi, 0.0, -0.5 * np.pi, 0.0, 0.0] * 2], np.float32)
    demo_a = np.array([[-2.2, 0.4, 1.1, 0.5, -0.5, 0.9, -1.3, 0.4, 1.1, 0.5, -0.5, 0.0]],
                      np.float32)                            # test/arm_plan.py:115-128
    demo_a = ((to_t(demo_a) + to_t(base)) / (np.pi / 0.5)).numpy()
    starts_a = np.concatenate([demo_a, synth.make_box_pairs(7, 6, seed=14)]).astype(np.float32)
    cap_a = 300
    paths_a = np.zeros((starts_a.shape[0], cap_a + 2, 12), np.float32)
    iters_a = np.zeros(starts_a.shape[0], np.int32)
    for qi in range(starts_a.shape[0]):
        XP = to_t(starts_a[qi:qi + 1])
        pts_q = [XP.detach().clone()]
        dis = torch.norm(XP[:, 6:] - XP[:, :6])
        it = 0
        while dis > 0.03:
            g = amodel.Gradient(XP.clone())
            XP = (XP + 0.015 * g).detach()
            dis = torch.norm(XP[:, 6:] - XP[:, :6])
            pts_q.append(XP.clone())
            it += 1
            if it > cap_a:
                break
        arr = torch.cat(pts_q).numpy()
        paths_a[qi, :arr.shape[0]] = arr
        paths_a[qi, arr.shape[0]:] = arr[-1]
        iters_a[qi] = it
    np.savez_compressed(os.path.join(args.out, "plan_arm.npz"), starts=starts_a, B=Ba,
                        paths=paths_a, iters=iters_a, step=np.float64(0.015),
                        tol=np.float64(0.03), max_iter=np.int32(cap_a),
                        weight_checksum=csum, versions=versions)
    print("goldens written to", args.out)


if __name__ == "__main__":
    main()
