"""Split-tile τ+∇τ variants (tests/diag/libperf_<name>.so built with -DPERF_SPLIT) against the
library's wave-tile kernel on the same pairs: max relative ∇τ error by pair lane (lane & 15).
Diagnostics only."""
import ctypes, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "p-ntfields_amd"))
from pntf import ops, synth


def main(names):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    n = 4096
    xp = torch.from_numpy(synth.make_pairs(n, 3)).to(dev).contiguous()
    B = torch.from_numpy(synth.make_B(3)).to(dev).contiguous()
    t0, d0 = ops.tau_grad(packed, xp, B, dim=3, schedule="wave_tile")
    t0, d0 = t0.cpu().numpy(), d0.cpu().numpy()
    stream = torch.cuda.current_stream().cuda_stream
    V = lambda t: ctypes.c_void_p(t.data_ptr())
    for name in names:
        lib = ctypes.CDLL(os.path.join(HERE, "libperf_%s.so" % name))
        lib.perf_tau_grad.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
            [ctypes.c_void_p] * 4 + [ctypes.c_void_p]
        split = lib.perf_split_width()
        per = 4 if split < 0 else 16          # pairs per workgroup tile
        split = abs(split)
        grid = n // per
        ws = torch.empty(256 * split * 96 * 1024 * 4, dtype=torch.uint8, device=dev)
        t = torch.empty(n, device=dev)
        d = torch.empty(n, 6, device=dev)
        assert lib.perf_tau_grad(grid, V(packed), V(xp), n, V(B), V(t), V(d), V(ws),
                                 ctypes.c_void_p(stream)) == 0
        torch.cuda.synchronize()
        t1, d1 = t.cpu().numpy(), d.cpu().numpy()
        e = np.abs(d1 - d0) / np.abs(d0).max()
        times = {}
        for m in (4, 16, 1024):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            g = (m + per - 1) // per
            for r in range(3):
                lib.perf_tau_grad(g, V(packed), V(xp), m, V(B), V(t), V(d), V(ws),
                                  ctypes.c_void_p(stream))
            ev[0].record()
            for r in range(50):
                lib.perf_tau_grad(g, V(packed), V(xp), m, V(B), V(t), V(d), V(ws),
                                  ctypes.c_void_p(stream))
            ev[1].record()
            torch.cuda.synchronize()
            times[m] = round(ev[0].elapsed_time(ev[1]) / 50 * 1e3, 1)
        print("%-10s us/call %s" % (name, times))
        print("%-10s split %d tau %.2g dtau %.2g by lane %s" % (
            name, split, np.abs(t1 - t0).max(), e.max(),
            np.round(e.reshape(-1, 16, 6).max((0, 2)), 3).tolist()), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
