#!/usr/bin/env python
"""Headline benchmark: (start, goal) τ+∇τ evaluations per second, Gibson 3D, 1M pairs per
GPU (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One step = the fused HIP τ+∇τ kernel (exact reverse mode, = Model.gradient(NN.out)) over the
rank's resident batch of synthetic Gibson-shaped pairs (10 environments, per-pair env id),
followed for N > 1 by the RCCL all-gather of every rank's τ+∇τ rows (the multi-GPU exchange
the north star names).  Weak scaling: every rank holds --pairs pairs.  Rank 0 prints one
JSON line; `value` = all ranks' pairs / max-over-ranks wall time of the K timed steps.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "p-ntfields_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

from pntf import dist, ops, synth  # noqa: E402

FLOP_PER_PAIR = 2_621_440          # 2 x (40*128^2 fwd + 40*128^2 bwd) GEMM MACs
BYTES_PER_PAIR = 52                # 24 B in + 4 B tau + 24 B dtau (algorithmic HBM bytes)
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: Peak FP32 (matrix)
METRIC = "(start,goal) tau+grad-tau evals/sec at batch=1M, Gibson 3D"
UNIT = "pairs/s"


def cpu_baseline(seconds, n_chunk=4096):
    """The fp32 numpy oracle (a restatement of the reference CPU path) on a bounded sample."""
    from oracle import pntf_oracle as O
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    W = synth.make_weights(0)
    xp = synth.make_pairs(n_chunk, 3, seed=2)
    Bt = synth.make_B_table(10, 3)
    env = synth.make_env_ids(n_chunk, 10)
    O.tau_grad(W, xp[:256], Bt, env[:256], dtype=np.float32)      # warm-up
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.tau_grad(W, xp, Bt, env, dtype=np.float32)
        done += n_chunk
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": UNIT, "cores": cores, "kind": "port",
            "sample": "%d pairs (%d-pair chunks, 10 envs) of the same synthetic workload, "
                      "oracle/pntf_oracle.tau_grad in fp32 numpy, %.1f s" % (done, n_chunk, el)}


def load_pmc(path, pairs):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/), scaled to
    this launch's pair count; None when absent."""
    try:
        with open(path) as fh:
            j = json.load(fh)
        return float(j["hbm_bytes_per_pair"]) * pairs
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=1 << 20, help="pairs per GPU")
    ap.add_argument("--envs", type=int, default=10)
    ap.add_argument("--mode", choices=["exact", "compat"], default="exact")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_tau_grad.json"))
    args = ap.parse_args()

    rank, ws = dist.init()
    _, _, local = dist.world()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    mode = ops.GRAD_EXACT if args.mode == "exact" else ops.GRAD_BACKGRAD_COMPAT

    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    n = args.pairs
    n_total = n * ws
    lo, hi = rank * n, (rank + 1) * n
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000 + rank)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(args.envs, 3)).to(dev)
    env = torch.from_numpy(synth.make_env_ids(n_total, args.envs)[lo:hi].copy()).to(dev)
    gather = ws > 1 and not args.no_gather

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        t, d = ops.tau_grad(packed, xp, Bt, env, dim=3, mode=mode)
        if ev is not None:
            ev[1].record()
        if gather:
            dist.all_gather_rows(torch.cat([t.unsqueeze(1), d], 1), n_total)
        return t

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if ws > 1:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if ws > 1:
        tdist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        el = float(tt.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    value = n_total * args.steps / el
    achieved = FLOP_PER_PAIR * n / (kern_ms * 1e-3) / 1e12
    traffic = load_pmc(args.pmc, n)

    extra = {}
    if rank == 0 and ws == 1 and not args.no_extra:
        extra = extras(packed, dev)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "gibson_multi_env_tau_grad (C3/C4 shape: %d pairs/GPU, %d "
                                   "envs, per-pair env id, dim 3)" % (n, args.envs),
                       "pairs_per_gpu": n, "global_batch": n_total, "envs": args.envs,
                       "grad_mode": args.mode, "allgather_outputs": gather,
                       "parallelism": "dp%d" % ws},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                         "traffic": traffic, "kernel": "field_kernel<3,K_TAU_GRAD>",
                         "kernel_ms": kern_ms, "flop_per_pair": FLOP_PER_PAIR,
                         "algorithmic_bytes_per_pair": BYTES_PER_PAIR},
            "cpu_baseline": cpu,
        }
        if extra:
            line["extra"] = extra
        print(json.dumps(line), flush=True)
    if ws > 1:
        tdist.barrier()
        tdist.destroy_process_group()


def extras(packed, dev):
    """Secondary configs measured after the headline (not part of `value`)."""
    out = {}

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    # C2: 262 144 pairs, single env
    n2 = 262144
    xp = torch.from_numpy(synth.make_pairs(n2, 3, seed=2)).to(dev)
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev)
    ms = timeit(lambda: ops.tau_grad(packed, xp, B, dim=3))
    out["c2_tau_grad_262144_pairs_per_s"] = n2 / (ms * 1e-3)
    ms = timeit(lambda: ops.tau(packed, xp, B, dim=3))
    out["c2_tau_only_262144_pairs_per_s"] = n2 / (ms * 1e-3)
    ms = timeit(lambda: ops.path_velocity(packed, xp, B, dim=3))
    out["c2_path_velocity_262144_pairs_per_s"] = n2 / (ms * 1e-3)
    # C1 shape on the GPU (4096 pairs, latency-bound): split tiles vs one wave per tile
    x1 = torch.from_numpy(synth.make_pairs(4096, 3, seed=2)).to(dev)
    for sched in ("auto", "wave_tile"):
        ops.set_field_schedule(sched)
        out["c1_tau_grad_4096_us_" + sched] = 1e3 * timeit(
            lambda: ops.tau_grad(packed, x1, B, dim=3), reps=20)
    ops.set_field_schedule("auto")
    # C3: Eikonal residual (Taylor mode + Model.Loss residual), 10 envs
    n3 = 1 << 20
    x3 = torch.from_numpy(synth.make_pairs(n3, 3, seed=5)).to(dev)
    B3 = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
    e3 = torch.from_numpy(synth.make_env_ids(n3, 10)).to(dev)
    y3 = torch.from_numpy(synth.make_speeds(n3)).to(dev)
    ms = timeit(lambda: ops.eikonal_residual(packed, x3, B3, e3, 3, yobs=y3, gamma=1e-3),
                reps=3)
    out["c3_eikonal_residual_1M_pairs_per_s"] = n3 / (ms * 1e-3)
    out["c3_eikonal_residual_TFLOPs"] = 14_286_848 * n3 / (ms * 1e-3) / 1e12
    # C5: UR5 arm, 1024 queries, <= 200 steps, per-query freeze
    q = 1024
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev)
    xq = torch.from_numpy(synth.make_box_pairs(q, 6, seed=3)).to(dev)
    res = {}

    def run_plan(schedule):
        res["p"] = ops.plan(packed, xq, Ba, dim=6, step=0.015, tol=0.03, max_iter=199,
                            mode=ops.GRAD_EXACT, schedule=schedule)
    ms = timeit(lambda: run_plan("auto"), reps=2)
    steps = res["p"][1].cpu().numpy()
    out["c5_arm_plan_1024q_ms"] = ms
    out["c5_arm_plan_query_steps_per_s"] = float(steps.sum()) / (ms * 1e-3)
    out["c5_arm_plan_mean_steps"] = float(steps.mean())
    out["c5_arm_plan_max_steps"] = int(steps.max())
    out["c5_arm_plan_1024q_wave_tile_ms"] = timeit(lambda: run_plan("wave_tile"), reps=2)
    # batch-1 Gibson planner (test/gib_plan.py runs Q = 1): device time per loop step
    x1 = torch.from_numpy(synth.make_pairs(1, 3, seed=21)).to(dev)
    B1 = torch.from_numpy(synth.make_B(3, seed=1)).to(dev)
    for sched in ("auto", "wave_tile"):
        def run1():
            res["p1"] = ops.plan(packed, x1, B1, dim=3, step=0.03, tol=1e-9, max_iter=99,
                                 mode=ops.GRAD_BACKGRAD_COMPAT, schedule=sched)
        ms = timeit(run1, reps=2)
        out["gib_plan_q1_ms_per_step_" + sched] = ms / 100.0
    out.update(train_extras(dev))
    out.update(mesh_extras(dev))
    return out


def mesh_extras(dev, n=1 << 20, t=20000, reps=3):
    """Speed-sample generator distance query (dataprocessing/speed_sampling_gpu.py:325-336):
    n sampled points against a t-triangle synthetic obstacle mesh (Gibson meshes are
    10^3..10^5 triangles).  VALU-bound; reported as point-triangle tests per second."""
    g = torch.Generator(device="cpu").manual_seed(9)
    tris = ((torch.rand(t, 1, 3, generator=g) - 0.5) * 0.8
            + torch.randn(t, 3, 3, generator=g) * 0.02).to(dev)
    pts = (torch.rand(n, 3, generator=g) - 0.5).to(dev)
    ops.point_mesh_distance(pts, tris)
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        ops.point_mesh_distance(pts, tris)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    return {"mesh_distance_1M_pts_20k_tris_ms": ms,
            "mesh_distance_point_tri_tests_per_s": n * t / (ms * 1e-3)}


TRAIN_FLOP_PER_PAIR = 3 * 14_286_848   # Taylor forward + 2x for the adjoint (GEMM MACs x 2)


def train_extras(dev, sizes=((2, 10000), (2, 100000)), reps=5):
    """Model.train inner step (model_res_sigmoid_multi.py:1040-1052) on the HIP Taylor tape:
    Loss forward + loss.backward() + AdamW step.  (2, 10000) is the reference's batch
    (Batch Size 2 environments x inner_batch 10000 pairs, :1010-1036)."""
    from models import model_res_sigmoid_multi as md
    from pntf.train import AdamW
    out = {}
    W = synth.make_weights(0)
    net = md.NN(dev, 3)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    net.to(dev)
    model = md.Model(".", ".", 3, 2, device=dev)
    model.network = net
    opt = AdamW(net.parameters(), lr=1e-3, weight_decay=0.1)
    for E, n in sizes:
        pts = torch.from_numpy(synth.make_pairs(E * n, 3, seed=77).reshape(E, n, 6)).to(dev)
        yobs = torch.from_numpy(synth.make_speeds(E * n, seed=78).reshape(E, n, 2)).to(dev)
        Bt = torch.from_numpy(synth.make_B_table(E, 3, first_seed=21)).to(dev)

        def step():
            loss, _, _ = model.Loss(pts, yobs, Bt, 1.0, 1e-3)
            loss.backward()
            opt.step()
            opt.zero_grad()
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        tag = "train_step_%dx%d" % (E, n)
        out[tag + "_ms"] = ms
        out[tag + "_pairs_per_s"] = E * n / (ms * 1e-3)
        out[tag + "_TFLOPs"] = TRAIN_FLOP_PER_PAIR * E * n / (ms * 1e-3) / 1e12
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--train-only":
        torch.cuda.set_device(0)
        print(json.dumps(train_extras(torch.device("cuda", 0))), flush=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--mesh-only":
        torch.cuda.set_device(0)
        print(json.dumps(mesh_extras(torch.device("cuda", 0))), flush=True)
        sys.exit(0)
    main()
