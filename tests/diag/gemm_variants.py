"""Time builds of csrc/pntf_gemm.hip (tests/diag/libgemm_<name>.so, built by hand with other
-DPNTF_GEMM_* values) on the training step's GEMM shapes.  Diagnostics only."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
FIRST = {}   # outputs of the first build named, to report each later build's bitwise difference


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main(names, pairs=20000, check=True):
    dev = torch.device("cuda:0")
    V = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)   # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    shapes = (("gen", 13 * pairs, 256, 256), ("enc", 14 * pairs, 128, 128),
              ("enc0", 14 * pairs, 256, 128))
    torch.manual_seed(0)
    for name in names:
        # "<lib>@<mode>": libgemm_<lib>.so with pntf_tt_set_panel_mode(<mode>)
        lname, _, mode = name.partition("@")
        lib = ctypes.CDLL(os.path.join(HERE, "libgemm_%s.so" % lname))
        if mode:
            lib.pntf_tt_set_panel_mode.argtypes = [ctypes.c_int]
            lib.pntf_tt_set_panel_mode(int(mode))
        lib.pntf_tt_gemm_work_floats.restype = ctypes.c_size_t
        lib.pntf_tt_gemm_work_floats.argtypes = [ctypes.c_int64] * 3
        lib.pntf_tt_gemm.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_int64] * 3 + \
            [ctypes.c_void_p, ctypes.c_int64] * 3 + [ctypes.c_float, ctypes.c_void_p,
                                                     ctypes.c_size_t, ctypes.c_void_p]
        res = {}
        for tag, rows, K, N in shapes:
            X = torch.randn(rows, K, device=dev)
            G = torch.randn(rows, N, device=dev)
            W = torch.randn(N, K, device=dev)
            Y = torch.empty(rows, N, device=dev)
            GX = torch.empty(rows, K, device=dev)
            GW = torch.empty(N, K, device=dev)
            fl = 2.0 * rows * K * N / 1e9

            def run(C, A, B, ta, tb, M, Nn, Kk):
                nw = lib.pntf_tt_gemm_work_floats(M, Nn, Kk)
                work = torch.empty(max(nw, 1), device=dev)
                return lambda: lib.pntf_tt_gemm(ta, tb, M, Nn, Kk, V(A), A.shape[1], V(B),
                                                B.shape[1], V(C), C.shape[1], 0.0, V(work), nw, s)
            f = run(Y, X, W, 0, 1, rows, N, K)
            res[tag + "_fwd"] = round(fl / timeit(f), 1)
            ref = X @ W.t()
            f()
            torch.cuda.synchronize()
            assert not check or (Y - ref).abs().max().item() < 1e-3 * ref.abs().max().item()
            f = run(GX, G, W, 0, 0, rows, K, N)
            res[tag + "_bwdx"] = round(fl / timeit(f), 1)
            ref = G @ W
            f()
            torch.cuda.synchronize()
            assert not check or (GX - ref).abs().max().item() < 1e-3 * ref.abs().max().item()
            res[tag + "_bwdw"] = round(fl / timeit(run(GW, G, X, 1, 0, N, K, rows)), 1)
            torch.cuda.synchronize()
            for t, o in (("fwd", Y), ("bwdx", GX), ("bwdw", GW)):
                k = tag + "_" + t
                if k not in FIRST:
                    FIRST[k] = o.clone()
                else:
                    res[k + "_maxdiff_vs_first"] = (o - FIRST[k]).abs().max().item()
        print(name, res, flush=True)


if __name__ == "__main__":
    # names starting with "abl" are ablation builds (wrong results: no check)
    for nm in sys.argv[1:]:
        main([nm], check=not nm.startswith("abl"))
