"""fp32-MFMA (PNTF_GEMM_PANEL 2) vs split-bf16 (3) panel GEMMs on the training shapes, then
the whole training step (Loss + backward + AdamW, 2 x n pairs) under each mode, alternating.
Diagnostics only.      python tests/diag/x6_probe.py [n] [rounds]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))
from pntf import _lib, synth, train  # noqa: E402
from pntf.train import AdamW  # noqa: E402
from models import model_res_sigmoid_multi as md  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2

# (rows, N, K, tb, beta): generator fwd / input grad (9 planes x 2n... the tape's R*m rows)
shapes = [(9 * 2 * n, 256, 256, True, 0.0), (9 * 2 * n, 256, 256, False, 1.0),
          (5 * 4 * n, 128, 128, True, 0.0), (5 * 4 * n, 128, 128, False, 1.0),
          (5 * 4 * n, 128, 256, True, 0.0), (9 * 2 * n, 256, 128, True, 0.0)]
g = torch.Generator(device="cpu").manual_seed(1)
for M, N, K, tb, beta in shapes:
    A = torch.randn(M, K, generator=g).to(dev)
    B = torch.randn((N, K) if tb else (K, N), generator=g).to(dev)
    C = torch.randn(M, N, generator=g).to(dev)
    res = {}
    for rep in range(2):
        for mode in (2, 3, 7):
            lib.pntf_tt_set_panel_mode(mode)
            for _ in range(3):
                train.gemm(C, A, B, False, tb, beta)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                train.gemm(C, A, B, False, tb, beta)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / 20 * 1e3)
    fl = 2.0 * M * N * K
    print("gemm M=%7d N=%d K=%d %s: fp32-mfma %s us, x6 %s us, x6 V3 %s us  (%.0f / %.0f / %.0f TFLOP/s)" % (
        M, N, K, "fwd" if tb else "bwd", ["%.1f" % v for v in res[2]],
        ["%.1f" % v for v in res[3]], ["%.1f" % v for v in res[7]], fl / min(res[2]) / 1e6,
        fl / min(res[3]) / 1e6, fl / min(res[7]) / 1e6), flush=True)
    del A, B, C

# weight gradients gYᵀ·X (wgrad kernels: mode 1 fp32 MFMA, 2 split bf16)
for rows, M, N in [(9 * 2 * n, 256, 256), (5 * 4 * n, 128, 128), (5 * 4 * n, 128, 256),
                   (9 * 2 * n, 128, 256)]:
    G = torch.randn(rows, M, generator=g).to(dev)
    X = torch.randn(rows, N, generator=g).to(dev)
    W = torch.empty(M, N, device=dev)
    res = {}
    for rep in range(2):
        for mode in (1, 2):
            lib.pntf_tt_set_wgrad_mode(mode)
            for _ in range(3):
                train.weight_grad(G, X, W)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                train.weight_grad(G, X, W)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / 20 * 1e3)
    ref = (G.double().t() @ X.double())
    lib.pntf_tt_set_wgrad_mode(1)
    train.weight_grad(G, X, W)
    e1_ = float(((W.double() - ref).abs() / (G.double().abs().t() @ X.double().abs())).max())
    lib.pntf_tt_set_wgrad_mode(2)
    train.weight_grad(G, X, W)
    e2_ = float(((W.double() - ref).abs() / (G.double().abs().t() @ X.double().abs())).max())
    fl = 2.0 * rows * M * N
    print("wgrad rows=%7d %dx%d: fp32-mfma %s us, x6 %s us  (%.0f / %.0f TFLOP/s)  max rel err %.3g / %.3g" % (
        rows, M, N, ["%.1f" % v for v in res[1]], ["%.1f" % v for v in res[2]],
        fl / min(res[1]) / 1e6, fl / min(res[2]) / 1e6, e1_, e2_), flush=True)
    del G, X, W

net = md.NN(dev, 3)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_weights(0).items()})
net.to(dev)
m = md.Model(".", ".", 3, 2, device=dev)
m.network = net
opt = AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
E = 2
pts = torch.from_numpy(synth.make_pairs(E * n, 3, seed=77).reshape(E, n, 6)).to(dev)
yo = torch.from_numpy(synth.make_speeds(E * n, seed=78).reshape(E, n, 2)).to(dev)
Bt = torch.from_numpy(synth.make_B_table(E, 3, first_seed=21)).to(dev)


def step():
    loss, _, _ = m.Loss(pts, yo, Bt, 1.0, 1e-3)
    loss.backward()
    opt.step()
    opt.zero_grad()
    return loss


for r in range(rounds):
    for mode in (2, 3):
        lib.pntf_tt_set_panel_mode(mode)
        lib.pntf_tt_set_wgrad_mode(mode - 1)
        for _ in range(8):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            loss = step()
        torch.cuda.synchronize()
        print("train step 2x%d panel mode %d (wgrad %d): %.3f ms (loss %.6g)" % (
            n, mode, mode - 1, (time.perf_counter() - t0) / 30 * 1e3, float(loss.detach())), flush=True)
