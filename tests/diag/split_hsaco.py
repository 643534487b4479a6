"""Split-tile τ+∇τ code objects (tests/diag/hsaco_<name>.hsaco from build_asm.sh, built with
-DPERF_SPLIT [-DPNTF_SPLIT=8]) against the library's wave-tile kernel on the same pairs:
max relative ∇τ error by pair lane.  Diagnostics only:
    python tests/diag/split_hsaco.py <split> <name> ..."""
import ctypes, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "p-ntfields_amd"))
from perf_variants import FieldArgs, hip_runtime  # noqa: E402
from pntf import ops, synth  # noqa: E402


def main(split, names):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    n = 4096
    xp = torch.from_numpy(synth.make_pairs(n, 3)).to(dev).contiguous()
    B = torch.from_numpy(synth.make_B(3)).to(dev).contiguous()
    t0, d0 = ops.tau_grad(packed, xp, B, dim=3, schedule="wave_tile")
    d0 = d0.cpu().numpy()
    hip = hip_runtime()
    hip.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint] * 7 + \
        [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    for name in names:
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipModuleLoad(ctypes.byref(mod), os.path.join(
            HERE, "hsaco_%s.hsaco" % name).encode()) == 0, name
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod,
                                        b"_ZN4pntf18field_split_kernelILi3ELi1EEEvNS_9FieldArgsE") == 0
        grid = n // 16
        ws = torch.empty(grid * split * 96 * 1024 * 4, dtype=torch.uint8, device=dev)
        t = torch.empty(n, device=dev)
        d = torch.empty(n, 6, device=dev)
        a = FieldArgs(packed.data_ptr(), xp.data_ptr(), B.data_ptr(), None, n, 1, 0, t.data_ptr(),
                      d.data_ptr(), ws.data_ptr())
        params = (ctypes.c_void_p * 1)(ctypes.cast(ctypes.pointer(a), ctypes.c_void_p))
        assert hip.hipModuleLaunchKernel(fn, grid, 1, 1, 64 * split, 1, 1, 0,
                                         ctypes.c_void_p(stream), params, None) == 0
        torch.cuda.synchronize()
        e = np.abs(d.cpu().numpy() - d0) / np.abs(d0).max()
        print("%-10s split %d dtau %.2g by lane %s" % (
            name, split, e.max(), np.round(e.reshape(-1, 16, 6).max((0, 2)), 3).tolist()),
            flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2:])
