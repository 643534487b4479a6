"""Diagnostic: ∇τ errors vs grid size at 262k pairs (1 vs 2 workgroups per CU)."""
import ctypes, sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np, torch
from pntf import ops, synth, _lib
from oracle import pntf_oracle as O
dev = torch.device("cuda:0")
print(torch.cuda.get_device_properties(0), flush=True)
W = synth.make_weights(0)
packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
lib = _lib.load()
n = 262144
xp = synth.make_pairs(n, 3, seed=2); B = synth.make_B(3, seed=1)
idx = np.arange(0, n, 97)
to, do = O.tau_grad(W, xp[idx], B)
xt = torch.from_numpy(xp).to(dev); Bt = torch.from_numpy(B).to(dev).unsqueeze(0).contiguous()
slot = 192 * 256 * 4
print("workspace_bytes(n)/slot/4 =", lib.pntf_workspace_bytes(n) / slot / 4, flush=True)
def run(wgs, kind="grad"):
    ws = torch.empty(wgs * 4 * slot, dtype=torch.uint8, device=dev)
    t = torch.empty(n, device=dev); d = torch.empty(n, 6, device=dev)
    V = lambda x: ctypes.c_void_p(x.data_ptr())
    st = lib.pntf_tau_grad(V(packed), 3, V(xt), n, V(Bt), None, 1, 0, V(t), V(d), V(ws), ws.numel(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return d.cpu().numpy()
for wgs in [128, 256, 384, 512, 256, 512]:
    d = run(wgs)
    bad = np.abs(d[idx] - do).max(1) > 1e-4 * np.abs(do).max()
    bi = idx[bad]
    print("wgs", wgs, "bad", bad.sum(), "of", len(idx), "lanes", np.bincount(bi % 16, minlength=16), "tile%8", np.bincount((bi // 16) % 8, minlength=8), flush=True)
