"""Training step (Model.Loss -> loss.backward() -> AdamW) eager vs replayed from a HIP graph
(torch.cuda.CUDAGraph capture of Loss + backward; AdamW eager), at 2 x n pairs:

    python tools/train_graph_probe.py [n] [reps]

Prints one JSON line: eager and graph ms per step and the max relative difference of the
weight gradients between the two (the graph replays the same kernels on the same buffers)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))

import torch  # noqa: E402


def main():
    from models import model_res_sigmoid_multi as md
    from pntf import synth
    from pntf.train import AdamW
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    W = synth.make_weights(0)
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    net.to(dev)
    model = md.Model(".", ".", 3, 2, device=dev)
    model.network = net
    opt = AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    E = 2
    pts = torch.from_numpy(synth.make_pairs(E * n, 3, seed=77).reshape(E, n, 6)).to(dev)
    yobs = torch.from_numpy(synth.make_speeds(E * n, seed=78).reshape(E, n, 2)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(E, 3, first_seed=21)).to(dev)

    def fwd_bwd():
        loss, _, _ = model.Loss(pts, yobs, Bt, 1.0, 1e-3)
        loss.backward()

    def eager():
        fwd_bwd()
        opt.step()
        opt.zero_grad()

    def timeit(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    ms_eager = timeit(eager)
    # eager reference gradients at the current weights
    opt.zero_grad()
    fwd_bwd()
    ref = {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None}
    opt.zero_grad()
    # capture Loss + backward (warm-up on a side stream, as torch.cuda.graphs documents)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            fwd_bwd()
    torch.cuda.current_stream().wait_stream(s)
    opt.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fwd_bwd()
    g.replay()
    torch.cuda.synchronize()
    err = max(float((p.grad - ref[k]).abs().max() / ref[k].abs().max())
              for k, p in net.named_parameters() if k in ref)

    def graphed():
        g.replay()
        opt.step()

    ms_graph = timeit(graphed)
    print(json.dumps({"pairs": E * n, "eager_ms": ms_eager, "graph_ms": ms_graph,
                      "grad_max_rel_diff_graph_vs_eager": err}), flush=True)


if __name__ == "__main__":
    main()
