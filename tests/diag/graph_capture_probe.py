"""Diagnostic: which HIP-graph captures of the library's stream-ordered
entry points work, and what made round 5's `GraphedLoss` capture segfault in
`hipStreamEndCapture` inside the GPU test suite while the same capture ran in a fresh process
(tools/train_graph_probe.py).

    python tests/diag/graph_capture_probe.py <mode>

modes (each in its own process; run the ones expected to crash last):
  abi                 capture pntf_tau_grad + pntf_eikonal_residual (ops.tau_grad /
                      ops.eikonal_residual) into a torch.cuda.CUDAGraph, replay on new inputs,
                      compare bitwise with eager calls
  loss                capture Model.Loss + loss.backward() (the Taylor tape: ~150 launches incl.
                      hipMemsetAsync nodes) and replay, compare with eager
  profiler_then_abi   a torch.profiler CUDA-activity session first (as
                      tests/test_train.py::test_training_uses_no_vendor_gemm runs one earlier
                      in the same pytest process), then mode abi
  profiler_then_loss  the same, then mode loss
  eager_then_loss     round 5's test_graphed_loss_matches_eager sequence: an eager Loss + backward
                      on the default stream whose `loss` stays referenced (its autograd graph,
                      AccumulateGrad nodes included, is kept alive), then the capture of mode loss
  eager_freed_then_loss  the same eager step, its outputs dropped before the capture
Prints one line per mode: "<mode> OK ..." or raises.
"""
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402


def capture(fn):
    """Warm up on a side stream, then capture fn() into a CUDAGraph; returns (graph, outputs)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def mode_abi(dev):
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    n = 40000
    Bt = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)

    def inputs(seed):
        return (torch.from_numpy(synth.make_pairs(n, 3, seed=seed)).to(dev),
                torch.from_numpy(synth.make_env_ids(n, 10, contiguous=False, seed=seed)).to(dev, torch.int32),
                torch.from_numpy(synth.make_speeds(n, seed=seed)).to(dev))
    xs, es, ys = [t.clone() for t in inputs(11)]

    def fn():
        t, d = ops.tau_grad(packed, xs, Bt, es, dim=3)
        r = ops.eikonal_residual(packed, xs, Bt, es, 3, yobs=ys, gamma=1e-3)
        return t, d, r
    g, (t, d, r) = capture(fn)
    for seed in (12, 13):
        x, e, y = inputs(seed)
        xs.copy_(x), es.copy_(e), ys.copy_(y)
        g.replay()
        torch.cuda.synchronize()
        t0, d0 = ops.tau_grad(packed, x, Bt, e, dim=3)
        r0 = ops.eikonal_residual(packed, x, Bt, e, 3, yobs=y, gamma=1e-3)
        assert torch.equal(t, t0) and torch.equal(d, d0)
        for k in r0:
            assert torch.equal(r[k], r0[k]), k
    return "tau_grad (%s) + eikonal_residual, %d pairs: replays bitwise equal" % (
        ops.resolved_schedule(n), n)


def mode_loss(dev, eager_first=False):
    from models import model_res_sigmoid_multi as md
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_weights(0).items()})
    net.to(dev)
    model = md.Model(".", ".", 3, 2, device=dev)
    model.network = net
    E, n = 2, 3000
    Bt = torch.from_numpy(synth.make_B_table(E, 3, first_seed=5)).to(dev)
    pts = torch.from_numpy(synth.make_pairs(E * n, 3, seed=90).reshape(E, n, 6)).to(dev)
    yo = torch.from_numpy(synth.make_speeds(E * n, seed=91).reshape(E, n, 2)).to(dev)
    params = [p for p in net.parameters() if p.requires_grad]
    keep = None
    if eager_first:   # as round 5's test: the eager step's loss is still referenced at capture
        keep = model.Loss(pts, yo, Bt, 1.0, 1e-3)
        keep[0].backward()
        if eager_first == "freed":
            keep = None

    def fn():
        for p in params:
            p.grad = None
        out = model.Loss(pts, yo, Bt, 1.0, 1e-3)
        out[0].backward()
        return out
    g, out = capture(fn)
    params = [p for p in params if p.grad is not None]   # encoder1.0 is never used (:227)
    grads = [p.grad for p in params]
    g.replay()
    torch.cuda.synchronize()
    got = [x.clone() for x in grads]
    for p in params:
        p.grad = None
    loss, _, _ = model.Loss(pts, yo, Bt, 1.0, 1e-3)
    loss.backward()
    for p, x in zip(params, got):
        if p.grad is not None:
            assert torch.equal(p.grad, x)
    return "Loss + backward (2 x %d pairs): replay bitwise equal to eager" % n


def profiler_session(dev):
    from torch.profiler import ProfilerActivity, profile
    x = torch.randn(1 << 20, device=dev)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        (x * 2).sum().item()
        torch.cuda.synchronize()
    return len(prof.key_averages())


def main(mode):
    faulthandler.enable()   # a crash names the Python frame it happened in
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    pre = ""
    if mode.startswith("profiler_then_"):
        pre = "after a profiler session (%d events); " % profiler_session(dev)
        mode = mode[len("profiler_then_"):]
    msg = {"abi": mode_abi, "loss": mode_loss,
           "eager_then_loss": lambda d: mode_loss(d, eager_first=True),
           "eager_freed_then_loss": lambda d: mode_loss(d, eager_first="freed")}[mode](dev)
    print("%s OK: %s%s" % (sys.argv[1], pre, msg), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
