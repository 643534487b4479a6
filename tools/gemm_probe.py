"""Time the fp32 library GEMM shapes of the training step's Taylor tape (pntf/train.py) in
their possible operand layouts, to pick the fastest (run on the GPU box)."""
import json
import sys

import torch


def SHAPES(pairs):
    """(tag, rows, K, N) of the dim-3 tape (pntf/train.py): R = 5 planes over the 2·pairs
    encoder points, R = 9 over the pairs after the merge."""
    return (("gen", 9 * pairs, 256, 256), ("enc", 5 * 2 * pairs, 128, 128),
            ("enc0", 5 * 2 * pairs, 256, 128), ("g3", 9 * pairs, 256, 128))


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


def main():
    dev = torch.device("cuda:0")
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    out = {}
    for tag, rows, K, N in SHAPES(pairs):
        X = torch.randn(rows, K, device=dev)
        G = torch.randn(rows, N, device=dev)
        W = torch.randn(N, K, device=dev)
        Wt = W.t().contiguous()
        Y = torch.empty(rows, N, device=dev)
        GX = torch.empty(rows, K, device=dev)
        GW = torch.empty(N, K, device=dev)
        GWt = torch.empty(K, N, device=dev)
        fl = 2.0 * rows * K * N / 1e9
        r = {}
        r["fwd_X@W.t()"] = fl / timeit(lambda: torch.mm(X, W.t(), out=Y))
        r["fwd_X@Wt"] = fl / timeit(lambda: torch.mm(X, Wt, out=Y))
        r["bwdx_G@W"] = fl / timeit(lambda: torch.mm(G, W, out=GX))
        r["bwdx_G@Wt.t()"] = fl / timeit(lambda: torch.mm(G, Wt.t(), out=GX))
        r["bwdw_G.t()@X"] = fl / timeit(lambda: torch.mm(G.t(), X, out=GW))
        r["bwdw_X.t()@G"] = fl / timeit(lambda: torch.mm(X.t(), G, out=GWt))
        out[tag] = {k: round(v, 1) for k, v in r.items()}   # TFLOP/s (GFLOP per ms)
    print(json.dumps(out, indent=1))




def split_probe(pairs=20000):
    """Split-K weight-gradient GEMM (pntf/train.py weight_grad) vs the single GEMM."""
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/p-ntfields_amd")
    from pntf.train import weight_grad
    dev = torch.device("cuda:0")
    out = {}
    for tag, rows, K, N in SHAPES(pairs):
        X = torch.randn(rows, K, device=dev)
        G = torch.randn(rows, N, device=dev)
        GW = torch.empty(N, K, device=dev)
        ref = torch.mm(G.t().double(), X.double()).float()
        weight_grad(G, X, GW)
        err = ((GW - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * rows * K * N / 1e9
        out[tag] = {"splitK_TFLOPs": round(fl / timeit(lambda: weight_grad(G, X, GW)), 1),
                    "rel_err": err}
    print(json.dumps(out, indent=1))


def mfma_probe(pairs=20000):
    """The library's own MFMA GEMM (pntf.train.gemm, csrc/pntf_gemm.hip) on the same shapes,
    TFLOP/s, beside the torch (hipBLASLt) GEMM of the same layout."""
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/p-ntfields_amd")
    from pntf.train import gemm
    dev = torch.device("cuda:0")
    out = {}
    for tag, rows, K, N in SHAPES(pairs):
        X = torch.randn(rows, K, device=dev)
        G = torch.randn(rows, N, device=dev)
        W = torch.randn(N, K, device=dev)
        Y = torch.empty(rows, N, device=dev)
        GX = torch.empty(rows, K, device=dev)
        GW = torch.empty(N, K, device=dev)
        fl = 2.0 * rows * K * N / 1e9
        r = {"fwd": fl / timeit(lambda: gemm(Y, X, W, False, True)),
             "fwd_torch": fl / timeit(lambda: torch.mm(X, W.t(), out=Y)),
             "bwdx": fl / timeit(lambda: gemm(GX, G, W, False, False)),
             "bwdx_torch": fl / timeit(lambda: torch.mm(G, W, out=GX)),
             "bwdx_acc": fl / timeit(lambda: gemm(GX, G, W, False, False, 1.0)),
             "bwdw": fl / timeit(lambda: gemm(GW, G, X, True, False)),
             "bwdw_torch": fl / timeit(lambda: torch.mm(G.t(), X, out=GW))}
        gemm(Y, X, W, False, True)
        ref = X.double() @ W.double().t()
        r["fwd_err"] = ((Y.double() - ref).abs().max() / ref.abs().max()).item()
        GX.copy_(X if K == X.shape[1] else GX)
        C0 = GX.clone()
        gemm(GX, G, W, False, False, 1.0)
        ref = C0.double() + G.double() @ W.double()
        r["bwdx_acc_err"] = ((GX.double() - ref).abs().max() / ref.abs().max()).item()
        out[tag] = {k: (round(v, 1) if v > 1e-3 else v) for k, v in r.items()}
    print(json.dumps(out, indent=1))


def one_probe(pairs=20000, reps=5):
    """The generator forward shape alone on the library GEMM (for PMC passes)."""
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/p-ntfields_amd")
    from pntf.train import gemm
    dev = torch.device("cuda:0")
    _, rows, K, N = SHAPES(pairs)[0]
    X = torch.randn(rows, K, device=dev)
    W = torch.randn(N, K, device=dev)
    Y = torch.empty(rows, N, device=dev)
    fl = 2.0 * rows * K * N / 1e9
    print(json.dumps({"gen_fwd_TFLOPs": fl / timeit(lambda: gemm(Y, X, W, False, True), reps)}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "one":
        one_probe(int(sys.argv[1]))
    elif len(sys.argv) > 2 and sys.argv[2] == "mfma":
        mfma_probe(int(sys.argv[1]))
    else:
        main()
        split_probe(int(sys.argv[1]) if len(sys.argv) > 1 else 20000)
