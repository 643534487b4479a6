"""Diagnostic: per-phase cycle counts of the τ+∇τ kernel (dim 3, exact) from s_memtime stamps
(libperf_stamps.so, built with -DPNTF_DEBUG_STAMPS by build_perf.sh), against the ideal
MFMA-issue cycles of each phase (32 cycles per v_mfma_f32_16x16x4_f32).

    python tests/diag/stamps.py [name]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402

# (from stamp, to stamp, name, MFMAs)
PHASES = [(0, 1, "fwd E0+fourier", 1024), (1, 2, "fwd enc0a", 512), (2, 3, "fwd enc0b", 512),
          (3, 4, "fwd enc1a", 512), (4, 5, "fwd enc1b", 512), (5, 6, "fwd E3", 512),
          (6, 7, "merge", 0), (7, 13, "fwd gen x6", 6144),
          (13, 14, "fwd G3", 512), (14, 15, "head", 0), (15, 16, "drain", 0), (16, 17, "bwd head", 0),
          (17, 18, "bwd G3T", 512), (18, 24, "bwd gen x6", 6144),
          (24, 25, "bwd merge", 0), (25, 26, "bwd E3T", 512), (26, 27, "bwd enc1b", 512),
          (27, 28, "bwd enc1a", 512), (28, 29, "bwd enc0b", 512), (29, 30, "bwd enc0a", 512),
          (30, 31, "fold E0T", 1024)]


def main(name):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    n = 1 << 20
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000)).to(dev)
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev).unsqueeze(0).contiguous()
    grid = torch.cuda.get_device_properties(0).multi_processor_count
    ws = torch.empty(grid * 8 * 192 * 256 * 4, dtype=torch.uint8, device=dev)
    st = torch.zeros(grid * 4 * 64, dtype=torch.int64, device=dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "diag", "libperf_%s.so" % name))
    V = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    assert lib.perf_set_stamps(V(st)) == 0
    t = torch.empty(n, device=dev)
    d = torch.empty(n, 6, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    lib.perf_tau_grad.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
        [ctypes.c_void_p] * 4 + [ctypes.c_void_p]
    for _ in range(2):
        assert lib.perf_tau_grad(grid, V(packed), V(xp), n, V(B), V(t), V(d), V(ws), stream) == 0
    torch.cuda.synchronize()
    s = st.cpu().numpy().reshape(grid * 4, 64).astype(np.float64)
    tot_ideal = tot_med = 0.0
    print("%-16s %9s %9s %7s" % ("phase", "cycles", "ideal", "eff"))
    for a, b, nm, mf in PHASES:
        dc = np.median(s[:, b] - s[:, a])
        ideal = mf * 32
        tot_ideal += ideal
        tot_med += dc
        print("%-16s %9.0f %9d %6.1f%%" % (nm, dc, ideal, 100 * ideal / dc if dc else 0))
    print("%-16s %9.0f %9.0f %6.1f%%" % ("TOTAL 0->31", tot_med, tot_ideal, 100 * tot_ideal / tot_med))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "stamps")
