"""Planner step time at Q = 1 (test/gib_plan.py's batch), 16 and 256 queries, as bench.py's
extras measure it; run once with PNTF_QSOLO=0 to time the MFMA quad layers instead of the
one-query-per-CU SOLO layers."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from pntf import ops, synth  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    out = {"solo": os.environ.get("PNTF_QSOLO", "1")}
    for dim, B, kw in ((3, synth.make_B(3, seed=1), dict(step=0.03, mode=ops.GRAD_BACKGRAD_COMPAT)),
                       (6, synth.make_B(6, seed=12, arm=True).T.copy(),
                        dict(step=0.015, mode=ops.GRAD_EXACT))):
        x1 = torch.from_numpy(synth.make_pairs(1, dim, seed=21)).to(dev)
        Bt = torch.from_numpy(B).to(dev)
        res = {}

        def run1():
            res["p"] = ops.plan(packed, x1, Bt, dim=dim, tol=1e-9, max_iter=99, **kw)
        out["q1_ms_per_step_d%d" % dim] = bench._timeit(run1, reps=5) / 100.0
        for q in (16, 256):
            xq = torch.from_numpy(synth.make_pairs(q, dim, seed=22)).to(dev)

            def runq():
                res["p"] = ops.plan(packed, xq, Bt, dim=dim, tol=1e-9, max_iter=99, **kw)
            out["q%d_ms_per_step_d%d" % (q, dim)] = bench._timeit(runq, reps=5) / 100.0
    # C5: 1024 arm queries, <= 199 steps, per-query freeze (bench.py's extra)
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev)
    xq = torch.from_numpy(synth.make_box_pairs(1024, 6, seed=3)).to(dev)
    res = {}

    def c5():
        res["p"] = ops.plan(packed, xq, Ba, dim=6, step=0.015, tol=0.03, max_iter=199,
                            mode=ops.GRAD_EXACT)
    out["c5_ms"] = bench._timeit(c5, reps=5)
    out["c5_max_steps"] = int(res["p"][1].max())
    print(json.dumps(out), flush=True)
