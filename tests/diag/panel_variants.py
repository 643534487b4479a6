"""Panel-GEMM ablations (csrc/pntf_gemm.hip, PNTF_PANEL_DIAG / PNTF_PANEL_PF): each variant is
a standalone build of pntf_gemm.hip (tests/diag/panel/*.so, made by `build` here on the CPU
container) timed on the training shapes through its own pntf_tt_gemm (run on the GPU box:
python tests/diag/panel_variants.py run)."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "panel")
VARIANTS = {"base": [], "pf1": ["-DPNTF_PANEL_PF=1"], "nonext": ["-DPNTF_PANEL_DIAG=1"],
            "nonext_nofrag": ["-DPNTF_PANEL_DIAG=5"], "nofrag": ["-DPNTF_PANEL_DIAG=4"],
            "wps2_pf1": ["-DPNTF_PANEL_WPS=2", "-DPNTF_PANEL_PF=1"],
            "wps2_pf3": ["-DPNTF_PANEL_WPS=2"]}


def build():
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(8) as ex:
        list(ex.map(lambda kv: build_one(*kv), VARIANTS.items()))


def build_one(name, defs):
    if True:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
               "-I" + os.path.join(REPO, "include"), "-Xclang", "-target-feature", "-Xclang",
               "-packed-fp32-ops"] + defs + [os.path.join(REPO, "p-ntfields_amd/csrc/pntf_gemm.hip"),
                                             "-o", os.path.join(OUT, name + ".so")]
        subprocess.check_call(cmd)
        print("built", name)


def run():
    import torch
    dev = torch.device("cuda:0")
    pairs = 20000
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    res = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(OUT, name + ".so"))
        lib.pntf_tt_gemm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_float, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_void_p]
        r = {}
        for tag, rows, K, N in (("gen", 13 * pairs, 256, 256), ("enc", 14 * pairs, 128, 128)):
            X = torch.randn(rows, K, device=dev)
            W = torch.randn(N, K, device=dev)
            Y = torch.empty(rows, N, device=dev)
            work = torch.empty(K * N, device=dev)
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            f = lambda: lib.pntf_tt_gemm(0, 1, rows, N, K, V(X), K, V(W), K, V(Y), N, 0.0,  # noqa
                                         V(work), K * N, s)
            f()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                f()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 20
            r[tag] = round(2.0 * rows * K * N / ms / 1e9, 1)
        res[name] = r
        print(name, r, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else run()
