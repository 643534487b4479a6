"""Training-step accuracy of the GEMM kernels against the fp64 oracle on the reference's
training fixtures: for each (panel, wgrad) mode pair, the step-1 weight gradients (max error
relative to each parameter's max |g|, sign disagreements with fp64 among elements with
|g| > 1e-7·max) and the loss after two AdamW steps (vs the fp64 trajectory and the
reference's fp32 loss2).  Diagnostics only.   python tests/diag/x6_train_acc.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "p-ntfields_amd")):
    sys.path.insert(0, p)
import test_train as T  # noqa: E402
from oracle import pntf_oracle as O  # noqa: E402
from pntf import _lib  # noqa: E402
from pntf.train import AdamW  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
for name, dim in T.CASES:
    W = T._case_weights(name)
    f, c = T._golden_case(name)
    B = c["B"][0] if c["env"] is None else c["B"]
    P = {k: v.astype(np.float64).copy() for k, v in W.items()}
    m = {k: np.zeros_like(v) for k, v in P.items()}
    v = {k: np.zeros_like(x) for k, x in P.items()}
    beta = float(f["beta"])
    g64 = None
    for step in (1, 2):
        diff, g = O.eikonal_loss_grad(P, c["xp"], c["yobs"], B, c["env"], dim, float(f["gamma"]),
                                      c["scale"], c["arm"])
        if step == 1:
            g64 = {k: x.copy() for k, x in g.items()}
        else:
            if c["arm"]:
                loss2_64 = beta * float(np.sum(diff)) / diff.size
            else:
                E = int(c["env"].max()) + 1
                loss2_64 = beta * O.loss_n(diff, f["B_table"], E, diff.size // E)
        for k in g:
            O.adamw_step(P[k], g[k], m[k], v[k], step)
    print("%s: loss2 fp64 %.9f, reference fp32 %.3g off" % (name, loss2_64, float(f["loss2"]) - loss2_64))
    for pm, wm in ((2, 1), (3, 2), (7, 2), (6, 2)):
        lib.pntf_tt_set_panel_mode(pm)
        lib.pntf_tt_set_wgrad_mode(wm)
        model, net = T._nets(dim, W, dev, f["B"] if dim == 6 else None)
        opt = AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
        worst, flips, loss2, wk = 0.0, 0, None, ""

        for step in range(2):
            loss, _, _ = T._loss(model, f, dim, dev)
            if step == 1:
                loss2 = loss.item()
            loss.backward()
            if step == 0:
                for k, p in net.named_parameters():
                    if p.grad is None:
                        continue
                    a = p.grad.detach().cpu().double().numpy()
                    b = g64[k]
                    sc = max(np.abs(b).max(), 1e-30)
                    e = float(np.abs(a - b).max() / sc)
                    if e > worst:
                        worst, wk = e, k
                    big = np.abs(b) > 1e-7 * sc
                    flips += int(np.sum(np.sign(a[big]) != np.sign(b[big])))
            opt.step()
            opt.zero_grad()
        print("  panel %d wgrad %d: step-1 grad max rel err %.3g (%s), sign flips %d, loss2 - fp64 %.3g"
              % (pm, wm, worst, wk, flips, loss2 - loss2_64), flush=True)
