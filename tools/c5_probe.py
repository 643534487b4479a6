"""The C5 workload alone (1024 arm queries, <= 199 steps, per-query freeze; bench.py's
extra), for rocprofv3 stats / PMC passes on the planner kernel:

    python tools/c5_probe.py [reps] [schedule]
"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    sched = sys.argv[2] if len(sys.argv) > 2 else "auto"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev)
    xq = torch.from_numpy(synth.make_box_pairs(1024, 6, seed=3)).to(dev)
    res = {}

    def c5():
        res["p"] = ops.plan(packed, xq, Ba, dim=6, step=0.015, tol=0.03, max_iter=199,
                            mode=ops.GRAD_EXACT, schedule=sched)
    ms = bench._timeit(c5, reps=reps, warm=5)
    st = res["p"][1]
    # active queries per step and the step at which at most one query per CU is left (the
    # tail hand-off point of the AUTO schedule)
    import numpy as np
    sc = st.cpu().numpy()
    active = [int((sc > s).sum()) for s in range(int(sc.max()) + 1)]
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    handoff = next((s for s, a in enumerate(active) if a <= cus), None)
    print(json.dumps({"active_per_step": active[::5], "handoff_step": handoff,
                      "steps_hist": np.bincount(sc // 10).tolist()}), flush=True)
    print(json.dumps({"c5_ms": ms, "schedule": sched, "mean_steps": float(st.float().mean()),
                      "max_steps": int(st.max()), "query_steps": int(st.sum()),
                      "us_per_step": 1e3 * ms / int(st.max())}), flush=True)
