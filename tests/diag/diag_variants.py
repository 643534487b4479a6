"""Diagnostic: ∇τ errors at 262k pairs for launch-bound / occupancy variants (tests/diag/libdiag.so)."""
import ctypes, sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np, torch
from pntf import ops, synth
from oracle import pntf_oracle as O
dev = torch.device("cuda:0")
W = synth.make_weights(0)
packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
lib = ctypes.CDLL(os.path.join(ROOT, "tests", "diag", "libdiag.so"))
n = 262144
xp = synth.make_pairs(n, 3, seed=2); B = synth.make_B(3, seed=1)
idx = np.arange(0, n, 97)
to, do = O.tau_grad(W, xp[idx], B)
xt = torch.from_numpy(xp).to(dev); Bt = torch.from_numpy(B).to(dev).unsqueeze(0).contiguous()
slot = 192 * 256 * 4
ws = torch.empty(4096 * slot, dtype=torch.uint8, device=dev)
V = lambda x: ctypes.c_void_p(x.data_ptr())
lib.diag_tau_grad.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
for variant, grid in [(0, 256), (0, 512), (1, 256), (1, 512), (2, 256), (2, 128)]:
    t = torch.empty(n, device=dev); d = torch.empty(n, 6, device=dev)
    st = lib.diag_tau_grad(variant, grid, V(packed), V(xt), n, V(Bt), V(t), V(d), V(ws))
    torch.cuda.synchronize()
    dn = d.cpu().numpy()
    bad = np.abs(dn[idx] - do).max(1) > 1e-4 * np.abs(do).max()
    print("variant", variant, "grid", grid, "st", st, "bad", bad.sum(), "of", len(idx), "lanes", np.bincount(idx[bad] % 16, minlength=16), flush=True)
