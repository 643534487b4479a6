"""C5 planner (1024 arm queries, <= 199 steps, per-query freeze, tail hand-off as pntf_plan_ex
AUTO) on quad-kernel builds of tests/diag/libperf_<name>.so (build_perf.sh -DPERF_QUAD ...),
against the shipped library's plan (ops.plan): wall time per plan, and whether the paths and
step counts are bitwise those of the shipped kernels.  Diagnostics only.

    python tests/diag/c5_variants.py q16 q24 ...
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "p-ntfields_amd"))
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main(names):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    q = 1024
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev).contiguous()
    xq = torch.from_numpy(synth.make_box_pairs(q, 6, seed=3)).to(dev)
    res = {}

    def ref():
        res["r"] = ops.plan(packed, xq, Ba, dim=6, step=0.015, tol=0.03, max_iter=199,
                            mode=ops.GRAD_EXACT)
    ms = timed(ref)
    p0, s0 = res["r"]
    print("shipped     %.3f ms  max steps %d" % (ms, int(s0.max())), flush=True)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    stream = torch.cuda.current_stream().cuda_stream
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for name in names:
        lib = ctypes.CDLL(os.path.join(HERE, "libperf_%s.so" % name))
        fn = lib.perf_plan6
        fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_float, ctypes.c_float,
                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_void_p]
        path = torch.empty_like(p0)
        steps = torch.empty_like(s0)
        tail = torch.zeros(2 + 2 * q, dtype=torch.int32, device=dev)

        def run():
            tail[:2].zero_()
            assert fn(min(cus, q // 4), cus, V(packed), V(xq), q, V(Ba), 0.015, 0.03, 199,
                      V(path), V(steps), V(tail), ctypes.c_void_p(stream)) == 0
        ms = timed(run)
        same = torch.equal(path, p0) and torch.equal(steps, s0)
        ok = torch.isfinite(path) & torch.isfinite(p0)
        print("%-10s  %.3f ms  handoffs %d  bitwise equal to shipped: %s  max steps %d  "
              "steps equal %d/%d  max |dpath| %.3g" % (
                  name, ms, int(tail[1].item()), same, int(steps.max()),
                  int((steps == s0).sum()), q, float((path - p0)[ok].abs().max())), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
