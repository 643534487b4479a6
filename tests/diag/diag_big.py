"""Diagnostic: full-chip ∇τ repeatability and oracle agreement at 262k pairs."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np, torch
from pntf import ops, synth
from oracle import pntf_oracle as O
dev = torch.device("cuda:0")
W = synth.make_weights(0)
packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
n = 262144
xp = synth.make_pairs(n, 3, seed=2); B = synth.make_B(3, seed=1)
xt = torch.from_numpy(xp).to(dev); Bt = torch.from_numpy(B).to(dev)
ref = None
for r in range(4):
    t, d = ops.tau_grad(packed, xt, Bt, dim=3)
    d = d.cpu().numpy()
    if ref is None:
        ref = d
        idx = np.arange(0, n, 97)
        to, do = O.tau_grad(W, xp[idx], B)
        bad = np.abs(d[idx] - do).max(1) > 1e-4 * np.abs(do).max()
        print("run0 vs oracle: bad", bad.sum(), "of", len(idx), flush=True)
    else:
        print("run", r, "mismatch vs run0:", int((d != ref).any(1).sum()), flush=True)
