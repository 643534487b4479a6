"""Diagnostic: ∇τ correctness vs tiles-per-wave (workspace-limited grid)."""
import ctypes, sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np, torch
from pntf import ops, synth, _lib
from oracle import pntf_oracle as O
dev = torch.device("cuda:0")
W = synth.make_weights(0)
packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
lib = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
xp = synth.make_pairs(n, 3, seed=2); B = synth.make_B(3, seed=1)
to, do = O.tau_grad(W, xp, B, dtype=np.float64)
xt = torch.from_numpy(xp).to(dev); Bt = torch.from_numpy(B).to(dev).unsqueeze(0).contiguous()
slot = 192 * 256 * 4
for wgs in [1, 2, 8, 64, 512]:
    ws = torch.empty(wgs * 4 * slot, dtype=torch.uint8, device=dev)
    t = torch.empty(n, device=dev); d = torch.empty(n, 6, device=dev)
    st = lib.pntf_tau_grad(ctypes.c_void_p(packed.data_ptr()), 3, ctypes.c_void_p(xt.data_ptr()), n, ctypes.c_void_p(Bt.data_ptr()), None, 1, 0, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    dn = d.cpu().numpy()
    bad = np.abs(dn - do).max(1) > 1e-4 * np.abs(do).max()
    tiles = np.arange(n) // 16
    print("wgs", wgs, "status", st, "bad pairs", bad.sum(), "of", n, "bad tiles", np.unique(tiles[bad])[:10], "tau err", np.abs(t.cpu().numpy() - to[:, 0]).max(), flush=True)
