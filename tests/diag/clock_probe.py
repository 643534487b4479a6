"""In-kernel effective clock of the headline wide kernel, the C5 quad planner and the training
GEMMs (MI355X_MICROARCH.md 'DVFS give-back' item 6): diagnostic builds with -DPNTF_CLOCK_STAMP
(csrc/pntf_stamp.h) record Δs_memtime / Δs_memrealtime per workgroup; each kernel runs back to
back for ~2 s on random-data inputs first, then the last launch's stamps are read and the
median over workgroups is reported as GHz, beside that launch's wall time.  No profiler is
attached.  Build (CPU):

    bash tests/diag/build_perf.sh "wstamp=-DPERF_WIDE -DPNTF_PF_STEPS=2 -DPERF_WBL=1 -DPNTF_CLOCK_STAMP" \
        "qstamp=-DPERF_QUAD -DPNTF_CLOCK_STAMP"
    bash tests/diag/build_gemm.sh "stamp=-DPNTF_CLOCK_STAMP"
    python tests/diag/clock_probe.py
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402

V = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731


def clocks(lib, nblocks):
    buf = (ctypes.c_ulonglong * (2 * 8192))()
    assert lib.pntf_diag_clock_stamps(buf, 8192) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)[:nblocks].astype(np.float64)
    a = a[a[:, 1] > 0]
    ghz = a[:, 0] / a[:, 1] * 0.1             # memrealtime ticks at 100 MHz
    return {"ghz_median": float(np.median(ghz)), "ghz_min": float(ghz.min()),
            "ghz_max": float(ghz.max()), "workgroups": int(len(ghz)),
            "wg_lifetime_us_median": float(np.median(a[:, 1]) / 100.0)}


def soak(fn, seconds=2.0):
    t0 = time.time()
    n = 0
    while time.time() - t0 < seconds:
        fn()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b)


def main(only=None, wlib="libperf_wstamp.so"):
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    out = {}
    # ---- headline wide kernel (1M pairs)
    lib = ctypes.CDLL(os.path.join(HERE, wlib))
    n = 1 << 20
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000)).to(dev)
    if os.environ.get("PERF_DATA") == "same":   # every pair the same: lanes carry equal values
        xp = xp[:1].expand(n, -1).contiguous()
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev).unsqueeze(0).contiguous()
    t, d = torch.empty(n, device=dev), torch.empty(n, 6, device=dev)
    ws = torch.empty(cus * 4 * 96 * 1024 * 4, dtype=torch.uint8, device=dev)
    lib.perf_tau_grad.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
        [ctypes.c_void_p] * 5
    ms = soak(lambda: lib.perf_tau_grad(cus, V(packed), V(xp), n, V(B), V(t), V(d), V(ws),
                                        stream))
    out["wide_tau_grad_1M"] = dict(clocks(lib, cus), launch_ms=ms)
    print(json.dumps({"wide_tau_grad_1M": out["wide_tau_grad_1M"], "lib": wlib}), flush=True)
    if only == "wide":
        return
    # ---- C5 planner, quad MFMA tiles only (no tail hand-off)
    lib = ctypes.CDLL(os.path.join(HERE, "libperf_qstamp.so"))
    q = 1024
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev).contiguous()
    xq = torch.from_numpy(synth.make_box_pairs(q, 6, seed=3)).to(dev)
    path = torch.empty((q, 201, 12), device=dev)
    steps = torch.empty(q, dtype=torch.int32, device=dev)
    lib.perf_plan6.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_float, ctypes.c_float,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p]
    ms = soak(lambda: lib.perf_plan6(min(cus, q // 4), cus, V(packed), V(xq), q, V(Ba), 0.015,
                                     0.03, 199, V(path), V(steps), None, stream))
    out["c5_quad_planner"] = dict(clocks(lib, min(cus, q // 4)), launch_ms=ms,
                                  max_steps=int(steps.max().item()))
    print(json.dumps({"c5_quad_planner": out["c5_quad_planner"]}), flush=True)
    # ---- training GEMMs at the reference batch (2 x 10 000 pairs: 9 generator planes)
    lib = ctypes.CDLL(os.path.join(HERE, "libgemm_stamp.so"))
    lib.pntf_tt_gemm_work_floats.restype = ctypes.c_size_t
    lib.pntf_tt_gemm_work_floats.argtypes = [ctypes.c_int64] * 3
    lib.pntf_tt_gemm.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_int64] * 3 + \
        [ctypes.c_void_p, ctypes.c_int64] * 3 + [ctypes.c_float, ctypes.c_void_p,
                                                 ctypes.c_size_t, ctypes.c_void_p]
    rows, K, N = 9 * 20000, 256, 256
    X = torch.randn(rows, K, device=dev)
    G = torch.randn(rows, N, device=dev)
    Wt = torch.randn(N, K, device=dev)
    Y = torch.empty(rows, N, device=dev)
    GW = torch.empty(N, K, device=dev)
    # the split-bf16 kernels (the default modes) and the fp32-MFMA ones
    lib.pntf_tt_set_panel_mode.argtypes = [ctypes.c_int]
    lib.pntf_tt_set_wgrad_mode.argtypes = [ctypes.c_int]
    for tag, mode, (ta, tb, M, Nn, Kk, A, lda, Bm, ldb, C, ldc) in (
            ("gemm_forward_gen_x6", 3, (0, 1, rows, N, K, X, K, Wt, K, Y, N)),
            ("gemm_wgrad_gen_x6", 2, (1, 0, N, K, rows, G, N, X, K, GW, K)),
            ("gemm_forward_gen_panel_lds_fp32", 2, (0, 1, rows, N, K, X, K, Wt, K, Y, N)),
            ("gemm_wgrad_gen_fp32", 1, (1, 0, N, K, rows, G, N, X, K, GW, K))):
        if ta:
            lib.pntf_tt_set_wgrad_mode(mode)
        else:
            lib.pntf_tt_set_panel_mode(mode)
        nw = lib.pntf_tt_gemm_work_floats(M, Nn, Kk)
        work = torch.empty(max(nw, 1), device=dev)
        ms = soak(lambda: lib.pntf_tt_gemm(ta, tb, M, Nn, Kk, V(A), lda, V(Bm), ldb, V(C), ldc,
                                           0.0, V(work), nw, stream))
        flop = 2.0 * M * Nn * Kk
        out[tag] = dict(clocks(lib, 1024), launch_ms=ms, tflops=flop / ms / 1e9)
        print(json.dumps({tag: out[tag]}), flush=True)


if __name__ == "__main__":
    # python tests/diag/clock_probe.py [wide [libperf_<name>.so]]: the headline leg only
    main(*sys.argv[1:])
