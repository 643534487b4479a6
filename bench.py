#!/usr/bin/env python
"""Headline benchmark: (start, goal) τ+∇τ evaluations per second, Gibson 3D, 1M pairs per
GPU (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--total-pairs T]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` without a torch.distributed environment starts N rank processes itself
(pntf/launch.py: one fresh interpreter per GPU, before anything touches the GPU); under
torchrun the ranks come from the environment and WORLD_SIZE must equal N.

One step = the fused HIP τ+∇τ kernel (exact reverse mode, = Model.gradient(NN.out); at this
size AUTO picks the 32-pair wide kernel, pntf_wide.h) over the rank's resident batch of
synthetic Gibson-shaped pairs (10 environments, per-pair env id),
followed for N > 1 by the RCCL all-gather of every rank's τ+∇τ rows (the multi-GPU exchange
the north star names).  Weak scaling by default (--pairs per rank); --total-pairs T splits a
fixed total over the ranks instead (strong scaling).  Rank 0 prints one JSON line; `value` =
all ranks' pairs / max-over-ranks wall time of the K timed steps.

After the timed steps every rank launches the kernel alone `--roofline-launches` times with
a HIP event pair around each launch (on the stream it runs on): `roofline.achieved` is the
algorithmic FLOP of one launch over the mean event-timed duration.  The CPU baseline (rank 0,
N = 1) runs last, after every GPU leg.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "p-ntfields_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

from pntf import dist, launch  # noqa: E402

FLOP_PER_PAIR = 2_621_440          # 2 x (40*128^2 fwd + 40*128^2 bwd) GEMM MACs
BYTES_PER_PAIR = 52                # 24 B in + 4 B tau + 24 B dtau (algorithmic HBM bytes)
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: Peak FP32 (matrix)
# v_mfma_f32_32x32x16_bf16: 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md
# "Peak BF16 ~2.5 PF dense")
BF16_MFMA_PEAK_TFLOPS = 2516.6
# The headline kernel's arithmetic ("split-bf16 wide layers"): 95 % of the
# algorithmic FLOP (every layer but encoder[0]'s transpose, the Fourier fold: 2 x 256 x 128 of
# the 40 x 128^2 MACs of the reverse sweep) run as six bf16 products per fp32 product, the
# rest on fp32 MFMA, so its MFMA roof is the harmonic mix
X6_FLOP_SHARE = 0.95
HEADLINE_PEAK_TFLOPS = 1.0 / (X6_FLOP_SHARE / (BF16_MFMA_PEAK_TFLOPS / 6)
                              + (1.0 - X6_FLOP_SHARE) / FP32_MFMA_PEAK_TFLOPS)
HEADLINE_ARITHMETIC = ("fp32 in/out and accumulation; 95 % of the FLOP as split-bf16 MFMA "
                       "(3-term operands, 6 products, fp32-exact products), the Fourier fold "
                       "on fp32 MFMA")
METRIC = "(start,goal) tau+grad-tau evals/sec at batch=1M, Gibson 3D"
UNIT = "pairs/s"
# per-CU weight-stream ceiling of the planner: 4.33 MB per step per CU read by the quad
# workgroup's 8 waves, 8-16 x 1 KiB loads in flight per wave (tests/diag/stream_probe2.hip on
# MI355X: 131 GB/s with one workgroup, 132-134 with one on every CU; 103 with 4 waves;
# DESIGN.md §3)
C5_STREAM_GBPS_PER_CU = 131.0
HEADLINE_UNIT = "wide_d3_k1"       # build unit of wide_field_kernel<3, K_TAU_GRAD> (pntf/build.py)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=1 << 20, help="pairs per GPU (weak scaling)")
    ap.add_argument("--total-pairs", type=int, default=0,
                    help="fixed total split over the GPUs (strong scaling)")
    ap.add_argument("--envs", type=int, default=10)
    ap.add_argument("--mode", choices=["exact", "compat"], default="exact")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--force-gather", action="store_true",
                    help="build the RCCL group and run the all-gather even at N = 1 (a "
                         "one-rank collective: measures the exchange path on one GPU)")
    ap.add_argument("--roofline-launches", type=int, default=100)
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_tau_grad.json"))
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU/gloo rehearsal of the launcher, sharding, all-gather and "
                         "max-over-ranks timing; no kernel runs and no metric is reported")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------ helpers
def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(sizes=(4096, 262144), reps=5):
    """The reference's CPU call pattern (oracle/torch_ref.py: one NN.out(coords, B) +
    Model.gradient autograd call per environment with that environment's (3, 128) B,
    models/model_res_sigmoid_multi.py:186-190, 215-259, 890-896; pinned to the reference by
    tests/test_oracle_golden.py::test_torch_ref_cpu_baseline_vs_reference) on the same
    synthetic workload, as SURVEY.md §8(d) specifies: all host threads
    (torch.set_num_threads), one warm-up call, then the median of `reps` timed calls at each
    batch size.  `value` is the rate at the largest size."""
    from oracle.torch_ref import TorchRef
    from pntf import synth
    threads = int(os.environ.get("OMP_NUM_THREADS", 0) or os.cpu_count() or 1)
    torch.set_num_threads(threads)
    ref = TorchRef(synth.make_weights(0))
    Bt = synth.make_B_table(10, 3)
    per_size, total = {}, 0.0
    for n in sizes:
        xp = synth.make_pairs(n, 3, seed=2)
        env = synth.make_env_ids(n, 10)
        ref.tau_grad(xp, Bt, env)                                     # warm-up
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ref.tau_grad(xp, Bt, env)
            ts.append(time.perf_counter() - t0)
        total += sum(ts)
        med = float(np.median(ts))
        per_size[str(n)] = {"pairs_per_s": n / med, "median_s": med,
                            "min_s": float(min(ts)), "max_s": float(max(ts)), "reps": reps}
    big = str(max(sizes))
    return {"value": per_size[big]["pairs_per_s"], "unit": UNIT,
            "cores": torch.get_num_threads(), "kind": "port", "cpu_model": cpu_model(),
            "pairs_per_s_per_core": per_size[big]["pairs_per_s"] / torch.get_num_threads(),
            "sizes": per_size,
            "sample": "median of %d reps after one warm-up at N = %s pairs (10 envs, per-pair "
                      "env id; `value` at N = %s) of the same synthetic workload through "
                      "oracle/torch_ref.py (the reference's torch CPU call pattern: one NN.out(coords, "
                      "B) + Model.gradient autograd call, create_graph=True, per environment "
                      "with its own (3,128) B), fp32, %.1f s timed"
                      % (reps, " and ".join(str(s) for s in sizes), big, total)}


def pmc_traffic(path, pairs, unit_hash):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/), scaled to
    this launch's pair count — only if it was collected from the kernel build that is loaded
    now (same unit hash); otherwise (None, reason)."""
    try:
        with open(path) as fh:
            j = json.load(fh)
    except (OSError, ValueError) as e:
        return None, "no PMC summary (%s)" % e
    if j.get("unit_hash") != unit_hash:
        return None, ("PMC summary %s was collected from build %s, loaded kernel is %s"
                      % (os.path.basename(path), j.get("unit_hash"), unit_hash))
    return float(j["hbm_bytes_per_pair"]) * pairs, "PMC %s (unit %s)" % (
        os.path.basename(path), unit_hash)


def timed(step, steps, warmup, ws, sync, dev_for_max):
    """Warm-up, then exactly `steps` steps bracketed by barrier + sync; max over ranks."""
    for _ in range(warmup):
        step()
    sync()
    if ws > 1:
        tdist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if ws > 1:
        tdist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev_for_max)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        el = float(tt.item())
    return el


def rank_share(args, rank, ws):
    """(pairs on this rank, pairs over all ranks, scaling)."""
    if args.total_pairs > 0:
        lo, hi = dist.shard_range(args.total_pairs, rank, ws)
        return hi - lo, args.total_pairs, "strong"
    return args.pairs, args.pairs * ws, "weak"


# ------------------------------------------------------------------------------ rehearsal
def rehearse(args):
    """Launcher rehearsal on CPU (gloo): the same rank layout, shard sizes, all-gather and
    max-over-ranks timing as the GPU run, with a rank-tagged row block standing in for the
    kernel output (nothing is computed, no metric is reported)."""
    rank, ws = dist.init("gloo")
    n, n_total, scaling = rank_share(args, rank, ws)
    lo = dist.shard_range(n_total, rank, ws)[0] if scaling == "strong" else rank * n
    rows = torch.arange(lo, lo + n, dtype=torch.float64).unsqueeze(1).repeat(1, 7)
    rows[:, 1] = rank
    res = {}

    def step():
        res["g"] = dist.all_gather_rows(rows, n_total)

    el = timed(step, args.steps, args.warmup, ws, lambda: None, "cpu")
    g = res["g"]
    ok = bool(g.shape == (n_total, 7) and torch.equal(
        g[:, 0], torch.arange(n_total, dtype=torch.float64)))
    # C5-style planner paths, uneven query shards (q not a multiple of ws)
    q = 37
    ql, qh = dist.shard_range(q, rank, ws)
    paths = torch.full((qh - ql, 5, 12), float(rank), dtype=torch.float32)
    paths[:, 0, 0] = torch.arange(ql, qh, dtype=torch.float32)
    gp = dist.all_gather_rows(paths, q)
    ok = ok and bool(torch.equal(gp[:, 0, 0], torch.arange(q, dtype=torch.float32)))
    if rank == 0:
        print(json.dumps({"rehearsal": True, "n_gpus": ws, "world_size": tdist.get_world_size()
                          if ws > 1 else 1, "steps": args.steps, "warmup": args.warmup,
                          "scaling": scaling, "pairs_per_rank0": n, "global_batch": n_total,
                          "gather_ok": ok, "max_over_ranks_s": el,
                          "config": {"parallelism": "dp%d" % ws}}), flush=True)
    if ws > 1:
        tdist.barrier()
        tdist.destroy_process_group()
    return 0 if ok else 1


# ------------------------------------------------------------------------------ GPU run
def run(args):
    from pntf import _lib, ops, synth
    rank, ws, local = dist.world()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init("nccl", device=dev, force=args.force_gather)
    if ws > 1 and tdist.get_world_size() != args.gpus:
        raise RuntimeError("RCCL world size %d != --gpus %d" % (tdist.get_world_size(),
                                                                  args.gpus))
    mode = ops.GRAD_EXACT if args.mode == "exact" else ops.GRAD_BACKGRAD_COMPAT

    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    n, n_total, scaling = rank_share(args, rank, ws)
    lo = dist.shard_range(n_total, rank, ws)[0] if scaling == "strong" else rank * n
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000 + rank)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(args.envs, 3)).to(dev)
    env_all = synth.make_env_ids(n_total, args.envs)
    env = torch.from_numpy(env_all[lo:lo + n].copy()).to(dev)
    gather = (ws > 1 or args.force_gather) and not args.no_gather
    res = {}

    def kernel():
        return ops.tau_grad(packed, xp, Bt, env, dim=3, mode=mode)

    def rows(t, d):
        return torch.cat([t.unsqueeze(1), d], 1)

    def step():
        t, d = kernel()
        if gather:
            res["g"] = dist.all_gather_rows(rows(t, d), n_total, force=args.force_gather)

    el = timed(step, args.steps, args.warmup, ws, torch.cuda.synchronize, dev)
    value = n_total * args.steps / el

    # roofline: per-launch HIP events on the launch stream (torch's current stream, which
    # ops.* hands to the C ABI), kernel alone
    stream = torch.cuda.current_stream(dev)
    R = max(args.roofline_launches, args.steps)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(R)]
    for a, b in evs:
        a.record(stream)
        kernel()
        b.record(stream)
    torch.cuda.synchronize()
    kms = np.array([a.elapsed_time(b) for a, b in evs])
    kern_ms = float(kms.mean())
    achieved = FLOP_PER_PAIR * n / (kern_ms * 1e-3) / 1e12
    unit_hash = _lib.build_info().get(HEADLINE_UNIT)
    traffic, traffic_src = pmc_traffic(args.pmc, n, unit_hash)
    split = None
    if gather:
        # the exchange alone (same row block, same stream), so a scaling run separates
        # per-rank compute from the xGMI all-gather; every rank's numbers go to rank 0
        blk = rows(*kernel())
        dist.all_gather_rows(blk, n_total, force=args.force_gather)
        torch.cuda.synchronize()
        gevs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(R)]
        for a, b in gevs:
            a.record(stream)
            dist.all_gather_rows(blk, n_total, force=args.force_gather)
            b.record(stream)
        torch.cuda.synchronize()
        ag_ms = float(np.mean([a.elapsed_time(b) for a, b in gevs]))
        mine = torch.tensor([kern_ms, ag_ms], dtype=torch.float64, device=dev)
        every = [torch.zeros_like(mine) for _ in range(tdist.get_world_size())]
        tdist.all_gather(every, mine)
        every = torch.stack(every).cpu().numpy()
        split = {"kernel_ms_per_rank": every[:, 0].tolist(),
                 "allgather_ms_per_rank": every[:, 1].tolist(),
                 "allgather_bytes_per_rank": int(blk.numel() * blk.element_size()),
                 "rccl_world_size": tdist.get_world_size()}

    extra = {}
    if not args.no_extra:
        if ws == 1:
            extra = extras(packed, dev)
        else:
            extra = sharded_extras(packed, dev, rank, ws)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        cpu = cpu_baseline(reps=args.cpu_reps)        # last: after every GPU leg

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "gibson_multi_env_tau_grad (C3/C4 shape: %d pairs/GPU, %d "
                                   "envs, per-pair env id, dim 3)" % (n, args.envs),
                       "pairs_per_gpu": n, "global_batch": n_total, "envs": args.envs,
                       "grad_mode": args.mode, "allgather_outputs": gather,
                       "parallelism": "dp%d" % ws,
                       "rccl_world_size": tdist.get_world_size() if tdist.is_initialized()
                       else 1},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": HEADLINE_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / HEADLINE_PEAK_TFLOPS,
                         "arithmetic": HEADLINE_ARITHMETIC,
                         "peak_fp32_mfma": FP32_MFMA_PEAK_TFLOPS,
                         "achieved_over_fp32_mfma_peak": achieved / FP32_MFMA_PEAK_TFLOPS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "wide_field_kernel<3,K_TAU_GRAD>", "unit_hash": unit_hash,
                         "kernel_ms": kern_ms, "kernel_ms_min": float(kms.min()),
                         "kernel_ms_max": float(kms.max()), "launches_timed": R,
                         "flop_per_pair": FLOP_PER_PAIR,
                         "algorithmic_bytes_per_pair": BYTES_PER_PAIR},
            "cpu_baseline": cpu,
        }
        if split:
            line["exchange"] = split
        if extra:
            line["extra"] = extra
        print(json.dumps(line), flush=True)
    if tdist.is_initialized():
        tdist.barrier()
        tdist.destroy_process_group()
    return 0


def _timeit(fn, reps=5, warm=1, stats=False):
    """Time `reps` back-to-back calls after `warm` untimed ones, one HIP event pair per call on
    the launch stream.  Returns the mean (ms), or with `stats` {"mean", "median", "min", "max",
    "reps", "warm"}.  After any idle gap the GPU's clocks ramp back over ~5 launches
    (profiles/r04_c2_launches.txt: 6.3 -> 5.2 ms for the 262 144-pair kernel), so every leg
    warms up with >= 5 calls and reports the median and the minimum as well."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = np.array([a.elapsed_time(b) for a, b in evs])
    if not stats:
        return float(ts.mean())
    return {"mean": float(ts.mean()), "median": float(np.median(ts)), "min": float(ts.min()),
            "max": float(ts.max()), "reps": reps, "warm": warm}


def shard_gather_plans(plan_local, xq_all, rank, ws):
    """The sharded planner exchange of SURVEY.md §8e: rank `rank` of `ws` plans its contiguous
    shard_range of the queries with plan_local(xq_shard) -> (path (q_r, T, 2dim), steps
    (q_r,)) and every rank receives all paths and step counts in query order (the all-gather
    of dist.all_gather_rows; uneven shards padded inside it).  bench.py's sharded C5 extra
    and the 8-rank CPU rehearsal (tests/test_dist.py) both go through here."""
    q = xq_all.shape[0]
    lo, hi = dist.shard_range(q, rank, ws)
    path, steps = plan_local(xq_all[lo:hi])
    return dist.all_gather_rows(path, q), dist.all_gather_rows(steps, q)


def sharded_extras(packed, dev, rank, ws, q=1024):
    """N > 1: the C5 arm planner with its 1024 queries sharded over the ranks, then the RCCL
    all-gather of every rank's paths (the planner-path exchange of SURVEY.md §8e); the wall
    time of both, and per rank the planner kernel alone and the all-gather alone."""
    from pntf import ops, synth
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev)
    xq_all = synth.make_box_pairs(q, 6, seed=3)
    lo, hi = dist.shard_range(q, rank, ws)
    xq = torch.from_numpy(xq_all[lo:hi].copy()).to(dev)
    res = {}

    def plan():
        res["local"] = ops.plan(packed, xq, Ba, dim=6, step=0.015, tol=0.03, max_iter=199,
                                mode=ops.GRAD_EXACT)

    def gather():
        path, steps = res["local"]
        res["paths"] = dist.all_gather_rows(path, q)
        res["steps"] = dist.all_gather_rows(steps, q)

    def run():
        res["paths"], res["steps"] = shard_gather_plans(
            lambda x: ops.plan(packed, torch.from_numpy(x.copy()).to(dev), Ba, dim=6,
                               step=0.015, tol=0.03, max_iter=199, mode=ops.GRAD_EXACT),
            xq_all, rank, ws)

    el = timed(run, 3, 1, ws, torch.cuda.synchronize, dev)
    mine = torch.tensor([_timeit(plan, reps=10, warm=5, stats=True)["median"],
                         _timeit(gather, reps=10, warm=2, stats=True)["median"]],
                        dtype=torch.float64, device=dev)
    every = [torch.zeros_like(mine) for _ in range(ws)]
    tdist.all_gather(every, mine)
    every = torch.stack(every).cpu().numpy()
    return {"c5_arm_plan_1024q_sharded_allgather_ms": el / 3 * 1e3,
            "c5_plan_kernel_ms_per_rank": every[:, 0].tolist(),
            "c5_path_allgather_ms_per_rank": every[:, 1].tolist(),
            "c5_arm_plan_mean_steps": float(res["steps"].float().mean().item())}


def extras(packed, dev):
    """Secondary configs measured after the headline (not part of `value`)."""
    from pntf import ops, synth
    out = {}
    timeit = _timeit
    # C2: 262 144 pairs, single env
    n2 = 262144
    xp = torch.from_numpy(synth.make_pairs(n2, 3, seed=2)).to(dev)
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev)
    ms = timeit(lambda: ops.tau_grad(packed, xp, B, dim=3), reps=20, warm=8)
    out["c2_tau_grad_262144_pairs_per_s"] = n2 / (ms * 1e-3)
    ms = timeit(lambda: ops.tau(packed, xp, B, dim=3), reps=20, warm=8)
    out["c2_tau_only_262144_pairs_per_s"] = n2 / (ms * 1e-3)
    ms = timeit(lambda: ops.path_velocity(packed, xp, B, dim=3), reps=20, warm=8)
    out["c2_path_velocity_262144_pairs_per_s"] = n2 / (ms * 1e-3)
    # the headline batch on the 16-pair kernel (pntf_field.h), for comparison with the wide one
    n1 = 1 << 20
    xh = torch.from_numpy(synth.make_pairs(n1, 3, seed=1000)).to(dev)
    Bh = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
    eh = torch.from_numpy(synth.make_env_ids(n1, 10)).to(dev)
    out["headline_1M_wave_tile_kernel_ms"] = timeit(
        lambda: ops.tau_grad(packed, xh, Bh, eh, dim=3, schedule="wave_tile"), reps=3, warm=3)
    del xh, eh
    # C1 shape on the GPU (4096 pairs, latency-bound): split tiles vs one wave per tile
    x1 = torch.from_numpy(synth.make_pairs(4096, 3, seed=2)).to(dev)
    for sched in ("auto", "wave_tile"):
        out["c1_tau_grad_4096_us_" + sched] = 1e3 * timeit(
            lambda: ops.tau_grad(packed, x1, B, dim=3, schedule=sched), reps=20)
    # C3: Eikonal residual (Taylor mode + Model.Loss residual), 10 envs
    n3 = 1 << 20
    x3 = torch.from_numpy(synth.make_pairs(n3, 3, seed=5)).to(dev)
    B3 = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
    e3 = torch.from_numpy(synth.make_env_ids(n3, 10)).to(dev)
    y3 = torch.from_numpy(synth.make_speeds(n3)).to(dev)
    st = timeit(lambda: ops.eikonal_residual(packed, x3, B3, e3, 3, yobs=y3, gamma=1e-3),
                reps=10, warm=5, stats=True)
    ms = st["median"]
    out["c3_eikonal_residual_1M_ms"] = st
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
    st = timeit(lambda: run_plan("auto"), reps=10, warm=5, stats=True)
    ms = st["median"]
    steps = res["p"][1].cpu().numpy()
    out["c5_arm_plan_1024q_ms"] = ms                   # median of 10 after 5 warm-up plans
    out["c5_arm_plan_1024q_ms_min"] = st["min"]
    out["c5_arm_plan_1024q_ms_stats"] = st
    out["c5_arm_plan_query_steps_per_s"] = float(steps.sum()) / (ms * 1e-3)
    out["c5_arm_plan_mean_steps"] = float(steps.mean())
    out["c5_arm_plan_max_steps"] = int(steps.max())
    out["c5_arm_plan_handoffs"] = ops.plan_handoff_counts(dev)[1]   # 0 = no tail hand-off
    out["c5_arm_plan_1024q_wave_tile_ms"] = timeit(lambda: run_plan("wave_tile"), reps=5,
                                                   warm=2, stats=True)["median"]
    out["c5_arm_plan_1024q_split_tile_ms"] = timeit(lambda: run_plan("split_tile"), reps=10,
                                                    warm=5, stats=True)["median"]
    # the quad planner's C5 step time and its roofline: a step streams both weight directions
    # (4.33 MB) through each tile's CU; the measured per-CU stream floor is ~33 us with the
    # tile's 8 waves loading (tests/diag/stream_probe2.hip), the 4x4x1 MFMA work ~17 us at the
    # fp32 MFMA peak
    out["c5_arm_plan_us_per_step"] = 1e3 * ms / max(int(steps.max()), 1)
    # the roofline that binds this kernel is the per-CU weight stream, not the MFMA: every
    # step of the critical path streams the CU's 4224 fragments of 1 KiB (both weight
    # directions, 8 waves x 528, pntf_quad.h) from L2/MALL; its ceiling is the measured per-CU
    # stream rate (tests/diag/stream_probe2.hip), not a datasheet number
    step_bytes = 4 * 1056 * 1024
    achieved = step_bytes / (out["c5_arm_plan_us_per_step"] * 1e-6) / 1e9
    out["c5_arm_plan_roofline"] = {
        "bound": "per-CU L2/MALL weight stream", "unit": "GB/s per CU",
        "bytes_per_step": step_bytes, "achieved": achieved, "peak": C5_STREAM_GBPS_PER_CU,
        "peak_source": "measured 8-wave stream floor (tests/diag/stream_probe2.hip)",
        "frac": achieved / C5_STREAM_GBPS_PER_CU}
    # batch-1 Gibson planner (test/gib_plan.py runs Q = 1): device time per loop step
    x1 = torch.from_numpy(synth.make_pairs(1, 3, seed=21)).to(dev)
    B1 = torch.from_numpy(synth.make_B(3, seed=1)).to(dev)
    for sched in ("auto", "split_tile", "wave_tile"):
        def run1():
            res["p1"] = ops.plan(packed, x1, B1, dim=3, step=0.03, tol=1e-9, max_iter=99,
                                 mode=ops.GRAD_BACKGRAD_COMPAT, schedule=sched)
        st = timeit(run1, reps=10, warm=5, stats=True)
        out["gib_plan_q1_ms_per_step_" + sched] = st["median"] / 100.0
        out["gib_plan_q1_ms_per_step_min_" + sched] = st["min"] / 100.0
    out.update(train_extras(dev))
    out.update(mesh_extras(dev))
    return out


def mesh_extras(dev, n=1 << 20, t=20000, reps=3):
    """Speed-sample generator distance query (dataprocessing/speed_sampling_gpu.py:325-336):
    n sampled points against a t-triangle synthetic obstacle mesh (Gibson meshes are
    10^3..10^5 triangles).  VALU-bound; reported as point-triangle tests per second."""
    from pntf import ops
    g = torch.Generator(device="cpu").manual_seed(9)
    tris = ((torch.rand(t, 1, 3, generator=g) - 0.5) * 0.8
            + torch.randn(t, 3, 3, generator=g) * 0.02).to(dev)
    pts = (torch.rand(n, 3, generator=g) - 0.5).to(dev)
    ms = _timeit(lambda: ops.point_mesh_distance(pts, tris), reps=reps)
    return {"mesh_distance_1M_pts_20k_tris_ms": ms,
            "mesh_distance_point_tri_tests_per_s": n * t / (ms * 1e-3)}


# Taylor forward + 2x for the adjoint (GEMM MACs x 2), per pair and training step:
#  * the reference's NN.out_laplace graph (one second-derivative row per direction):
#    3 x 2 x 436·128² = 3 x 14 286 848 FLOP — the count the "reference-equivalent" rate uses;
#  * what the tape executes (pntf_train.hip: the second-derivative rows summed per endpoint,
#    5 / 9 rows per encoder point / pair instead of 7 / 13 for dim 3): 3 x 2 x 4 980 736.
TRAIN_FLOP_PER_PAIR = 3 * 14_286_848
TRAIN_FLOP_EXECUTED_PER_PAIR = 3 * 2 * (2 * 5 * 114_688 + 9 * 425_984)


def train_extras(dev, sizes=((2, 10000), (2, 100000)), reps=20, warm=5):
    """Model.train inner step (model_res_sigmoid_multi.py:1040-1052) on the HIP Taylor tape:
    Loss forward + loss.backward() + AdamW step, as Model.train runs it.  (2, 10000) is the
    reference's batch (Batch Size 2 environments x inner_batch 10000 pairs, :1010-1036).  `warm` untimed
    steps first: after the host syncs of the legs before it the GPU clock ramps back over the
    first few launches, which one warm-up step does not cover."""
    from models import model_res_sigmoid_multi as md
    from pntf import synth
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

        def eager():
            loss, _, _ = model.Loss(pts, yobs, Bt, 1.0, 1e-3)
            loss.backward()
            opt.step()
            opt.zero_grad()

        def per_step(fn):
            for _ in range(warm):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3
        tag = "train_step_%dx%d" % (E, n)
        ms = per_step(eager)
        out[tag + "_ms"] = ms
        out[tag + "_pairs_per_s"] = E * n / (ms * 1e-3)
        out[tag + "_TFLOPs_reference_equivalent"] = TRAIN_FLOP_PER_PAIR * E * n / (ms * 1e-3) / 1e12
        out[tag + "_TFLOPs_executed"] = TRAIN_FLOP_EXECUTED_PER_PAIR * E * n / (ms * 1e-3) / 1e12
    # the GEMM arithmetic of the step: fp32 operands and results, each
    # product as six bf16 MFMA products of three-term operand splits (fp32-level error against
    # fp64: tests/test_train.py::test_x6_gemm_vs_fp64, profiles/r05_x6_accuracy.txt)
    from pntf import _lib
    out["train_gemm_arithmetic"] = (
        "fp32 in/out, split-bf16 MFMA (3-term operands, 6 products, per-order accumulators)"
        if _lib.load().pntf_tt_set_panel_mode(-1) == 3 else "fp32 MFMA")
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if argv and argv[0] in ("--train-only", "--mesh-only"):
        torch.cuda.set_device(0)
        fn = train_extras if argv[0] == "--train-only" else mesh_extras
        print(json.dumps(fn(torch.device("cuda", 0))), flush=True)
        return 0
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one fresh process per GPU; this parent never initialises HIP
        return launch.spawn(args.gpus, [os.path.abspath(__file__)] + list(argv))
    ws = int(os.environ.get("WORLD_SIZE", 1))
    if ws != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, ws), file=sys.stderr)
        return 2
    return rehearse(args) if args.rehearse else run(args)


if __name__ == "__main__":
    sys.exit(main())
