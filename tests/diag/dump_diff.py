"""Diagnostic: run two -DPNTF_DEBUG_DUMP perf variants (tests/diag/libperf_<a>.so, _<b>.so)
on the same 1M-pair batch and report, per dump point, where their intermediate tiles differ
(lanes and magnitude) — locates the first point at which a miscompiled variant diverges.

    python tests/diag/dump_diff.py d1 d2
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402

NAMES = {0: "E0 sg", 16: "E0 sp", 32: "fold B (Y)", 48: "fold acc", 56: "reduced ds/dg"}


def main(a, b):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    n = 1 << 20
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000)).to(dev)
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev).unsqueeze(0).contiguous()
    t_ref, d_ref = ops.tau_grad(packed, xp, B[0], dim=3)
    grid = torch.cuda.get_device_properties(0).multi_processor_count
    ws = torch.empty(grid * 8 * 192 * 256 * 4, dtype=torch.uint8, device=dev)
    V = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    stream = torch.cuda.current_stream().cuda_stream
    dumps = {}
    for name in (a, b):
        lib = ctypes.CDLL(os.path.join(ROOT, "tests", "diag", "libperf_%s.so" % name))
        lib.perf_tau_grad.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
            [ctypes.c_void_p] * 4 + [ctypes.c_void_p]
        dbg = torch.zeros(grid * 4 * 64 * 256, device=dev)
        assert lib.perf_set_dbg(V(dbg)) == 0
        t = torch.empty(n, device=dev)
        d = torch.empty(n, 6, device=dev)
        assert lib.perf_tau_grad(grid, V(packed), V(xp), n, V(B), V(t), V(d), V(ws), stream) == 0
        torch.cuda.synchronize()
        err = float(((d - d_ref).norm() / d_ref.norm()).item())
        print("%s: dtau rel err vs shipped %.2e" % (name, err), flush=True)
        dumps[name] = dbg.cpu().numpy().reshape(grid * 4, 64, 64, 4)   # wave, idx, lane, s
    da, db = dumps[a], dumps[b]
    for idx in list(range(0, 64)):
        x, y = da[:, idx], db[:, idx]
        if not np.any(x) and not np.any(y):
            continue
        diff = np.abs(x - y)
        scale = np.abs(y).max() + 1e-30
        bad = diff.max(axis=(0, 2)) > 1e-5 * scale      # per lane
        label = max(k for k in NAMES if k <= idx)
        print("idx %2d (%s+%d): max|diff| %.3e (scale %.3e); bad lanes %s" % (
            idx, NAMES[label], idx - label, diff.max(), scale, np.nonzero(bad)[0].tolist()),
            flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
