"""Diagnostic: time perf variants of the τ+∇τ kernel (tests/diag/libperf_<name>.so, built by
build_perf.sh) at 1M pairs against the shipped kernel, and check each variant's output against
the shipped kernel's (same math, so agreement is at the fp32 rounding level).

    python tests/diag/perf_variants.py base f3 f4 ...
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402

FLOP_PER_PAIR = 2_621_440


class FieldArgs(ctypes.Structure):
    _fields_ = [("P", ctypes.c_void_p), ("xp", ctypes.c_void_p), ("Btab", ctypes.c_void_p),
                ("env", ctypes.c_void_p), ("n", ctypes.c_int64), ("n_env", ctypes.c_int32),
                ("compat", ctypes.c_int32), ("out0", ctypes.c_void_p), ("out1", ctypes.c_void_p),
                ("ws", ctypes.c_void_p)]


def hip_runtime():
    """The libamdhip64 torch already loaded (same context)."""
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


def hsaco_launcher(path):
    hip = hip_runtime()
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), path.encode()) == 0, path
    name = b"_ZN4pntf12field_kernelILi3ELi1EEEvNS_9FieldArgsE"
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, name) == 0
    hip.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint] * 7 + \
        [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]

    def launch(grid, P, xp, n, B, t, d, ws, stream):
        a = FieldArgs(P.value, xp.value, B.value, None, n, 1, 0, t.value, d.value, ws.value)
        params = (ctypes.c_void_p * 1)(ctypes.cast(ctypes.pointer(a), ctypes.c_void_p))
        return hip.hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(stream),
                                         params, None)
    return launch


def main(names):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    n = 1 << 20
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000)).to(dev)
    if os.environ.get("PERF_DATA") == "same":   # every pair the same: lanes carry equal values
        xp = xp[:1].expand(n, -1).contiguous()
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev).unsqueeze(0).contiguous()
    t_ref, d_ref = ops.tau_grad(packed, xp, B[0], dim=3)
    torch.cuda.synchronize()
    grid = torch.cuda.get_device_properties(0).multi_processor_count
    slot = 96 * 1024 * 4            # the larger (wide) slot
    ws = torch.empty(grid * 4 * slot, dtype=torch.uint8, device=dev)
    V = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    stream = torch.cuda.current_stream().cuda_stream
    for name in names:
        if name.startswith("hsaco:"):
            fn = hsaco_launcher(os.path.join(ROOT, "tests", "diag", "hsaco_%s.hsaco" % name[6:]))
            P = packed
        else:
            lib = ctypes.CDLL(os.path.join(ROOT, "tests", "diag", "libperf_%s.so" % name))
            fn = lib.perf_tau_grad
            fn.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
                [ctypes.c_void_p] * 4 + [ctypes.c_void_p]
            P = packed
            if hasattr(lib, "perf_packed_total"):
                lib.perf_packed_total.restype = ctypes.c_longlong
                total = lib.perf_packed_total()
                if total > int(0.6 * packed.numel()):   # x6 build: its own split-bf16 order
                    P = torch.zeros(max(total, packed.numel()), dtype=torch.float32, device=dev)
                    P[:packed.numel()] = packed
                    assert lib.perf_pack_x6(ctypes.c_void_p(P.data_ptr()),
                                            ctypes.c_void_p(stream)) == 0
        t = torch.empty(n, device=dev)
        d = torch.empty(n, 6, device=dev)

        def run():
            assert fn(grid, V(P), V(xp), n, V(B), V(t), V(d), V(ws), stream) == 0
        run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        a.record()
        for _ in range(reps):
            run()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        err = float(((d - d_ref).norm() / d_ref.norm()).item())
        terr = float(((t - t_ref).norm() / t_ref.norm()).item())
        dmax = float((d - d_ref).abs().max().item())
        print("%-10s %8.3f ms  %6.2f Mpairs/s  %6.1f TF/s  dtau rel %.2e  tau rel %.2e  "
              "dtau max abs %.1e" % (name, ms, n / ms / 1e3, FLOP_PER_PAIR * n / ms / 1e9, err,
                                     terr, dmax), flush=True)
        if err > 1e-5:
            bad = ((d - d_ref).abs().max(1).values > 1e-4 * d_ref.abs().max()).cpu().numpy()
            idx = np.nonzero(bad)[0]
            print("    bad pairs %d; by column (pair %% 16) %s; first %s" % (
                bad.sum(), np.bincount(idx % 16, minlength=16).tolist(), idx[:8].tolist()),
                flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
