"""Training step (Loss + loss.backward() + AdamW, bench.py train_extras) under each schedule of
the forward Linear + act (pntf_tt_linear_act: 0 AUTO, 1 fused one-wave-per-block, 2 GEMM +
act kernel, 3 fused four-waves-per-block), with and without the fused input gradient + act
adjoint (pntf_tt_linear_bwd), at the reference batch 2 x 10 000 and 2 x 100 000.

    python tools/train_sched_probe.py [reps [bwd]]   (bwd: only the input-gradient kernels)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import torch  # noqa: E402

from pntf import synth, train  # noqa: E402


def main(reps=10, only_bwd=False):
    from models import model_res_sigmoid_multi as md
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    net.to(dev)
    model = md.Model(".", ".", 3, 2, device=dev)
    model.network = net
    opt = train.AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    for E, n in ((2, 10000), (2, 100000)):
        pts = torch.from_numpy(synth.make_pairs(E * n, 3, seed=77).reshape(E, n, 6)).to(dev)
        yobs = torch.from_numpy(synth.make_speeds(E * n, seed=78).reshape(E, n, 2)).to(dev)
        Bt = torch.from_numpy(synth.make_B_table(E, 3, first_seed=21)).to(dev)

        def step():
            loss, _, _ = model.Loss(pts, yobs, Bt, 1.0, 1e-3)
            loss.backward()
            opt.step()
            opt.zero_grad()
        defaults = (train._LINEAR_ACT, train._LINEAR_BWD)
        runs = ((defaults + (1,)), (0, 0, 1), (2, 0, 1), (1, 0, 1), (3, 0, 1), (3, 1, 1),
                (2, 1, 1), (defaults + (1,)))
        if only_bwd:   # the fused input gradient + act adjoint: pair / split-bf16 / fp32 MFMA
            runs = ((2, 0, 1), (2, 1, 1), (2, 1, 0), (2, 0, 1), (2, 1, 1), (2, 1, 0))
        lib = train._lib.load()
        for sched, bwd, bmode in runs:
            train._LINEAR_ACT = sched
            train._LINEAR_BWD = bwd
            lib.pntf_tt_set_bwd_mode(bmode)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / reps * 1e3
            print("train step %dx%d  linear_act schedule %d, fused bwd %s (bwd kernel %s): "
                  "%.3f ms" % (E, n, sched, "auto" if bwd is None else bwd,
                               "x6" if bmode else "fp32", ms), flush=True)
        train._LINEAR_ACT, train._LINEAR_BWD = defaults
        lib.pntf_tt_set_bwd_mode(1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10, len(sys.argv) > 2 and sys.argv[2] == "bwd")
