"""The RCCL path on hardware at world size 1.

bench.py's N > 1 run builds an `nccl` (= RCCL on ROCm) process group bound to the rank's
device and all-gathers every rank's τ+∇τ rows and planner paths (pntf/dist.py).  A one-GPU
box cannot run N > 1, so this test builds the same group at world size 1 (dist.init(...,
force=True), device_id as in bench.py) and sends a τ+∇τ row block and a C5-style planner path
block through all_gather_into_tensor (all_gather_rows(force=True)): the rows must come back
bit-identical, from a real RCCL collective (not the world-size-1 shortcut).  It also times the
collective against the kernel that produced the rows (reported, not asserted)."""
import json
import os

import numpy as np
import pytest
import torch


@pytest.mark.gpu
def test_rccl_world1_allgather():
    import torch.distributed as tdist
    from pntf import dist, ops, synth
    from test_dist import _free_port
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    env = {k: os.environ.get(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                          "MASTER_PORT")}
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(_free_port()))
    try:
        assert dist.init("nccl", device=dev, force=True) == (0, 1)
        assert tdist.get_backend() == "nccl" and tdist.get_world_size() == 1
        W = synth.make_weights(0)
        packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
        n = 1 << 16
        xp = torch.from_numpy(synth.make_pairs(n, 3, seed=5)).to(dev)
        Bt = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
        e = torch.from_numpy(synth.make_env_ids(n, 10)).to(dev)
        t, d = ops.tau_grad(packed, xp, Bt, e, dim=3)
        rows = torch.cat([t.unsqueeze(1), d], 1)
        full = dist.all_gather_rows(rows, n, force=True)
        assert full.data_ptr() != rows.data_ptr() and torch.equal(full, rows)
        Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev)
        xq = torch.from_numpy(synth.make_box_pairs(37, 6, seed=3)).to(dev)
        path, steps = ops.plan(packed, xq, Ba, dim=6, step=0.015, tol=0.03, max_iter=40,
                               mode=ops.GRAD_EXACT)
        gp = dist.all_gather_rows(path, 37, force=True)
        gs = dist.all_gather_rows(steps, 37, force=True)
        assert torch.equal(gp, path) and torch.equal(gs, steps)
        # single-rank RCCL overhead against the kernel that made the rows (1M-pair rows: the
        # bench's per-rank block, 28 B/pair)
        big = torch.zeros((1 << 20, 7), device=dev)
        evs = []
        for fn in (lambda: dist.all_gather_rows(big, 1 << 20, force=True),
                   lambda: ops.tau_grad(packed, xp, Bt, e, dim=3)):
            fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                fn()
            b.record()
            torch.cuda.synchronize()
            evs.append(a.elapsed_time(b) / 10)
        print(json.dumps({"rccl_ws1_allgather_1M_rows_ms": evs[0],
                          "tau_grad_65536_pairs_ms": evs[1]}))
    finally:
        if tdist.is_initialized():
            tdist.destroy_process_group()
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _gpu_worker(rank, world, port, n, q):
    """One rank of the sharded path on the box's single GPU: its contiguous shard through the
    HIP kernels (the same entry points bench.py's ranks call), then the all-gather of the
    per-rank rows (gloo over host copies: two RCCL ranks cannot share one device)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as tdist
    from pntf import dist, ops, synth
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    assert dist.init("gloo") == (rank, world)
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=5)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
    e = torch.from_numpy(synth.make_env_ids(n, 10)).to(dev)
    lo, hi = dist.shard_range(n, rank, world)
    # one schedule for the shards and the whole batch: per-pair results are then bitwise equal
    t, d = ops.tau_grad(packed, xp[lo:hi], Bt, e[lo:hi], dim=3, schedule="wide_tile")
    full = dist.all_gather_rows(torch.cat([t.unsqueeze(1), d], 1).cpu(), n)
    tf, df = ops.tau_grad(packed, xp, Bt, e, dim=3, schedule="wide_tile")
    assert torch.equal(full, torch.cat([tf.unsqueeze(1), df], 1).cpu())
    # planner queries sharded the same way (uneven shards)
    Ba = torch.from_numpy(synth.make_B(6, seed=12, arm=True).T.copy()).to(dev)
    xq = torch.from_numpy(synth.make_box_pairs(q, 6, seed=3)).to(dev)
    lo, hi = dist.shard_range(q, rank, world)
    kw = dict(dim=6, step=0.015, tol=0.03, max_iter=40, mode=ops.GRAD_EXACT,
              schedule="quad_tile")
    path, steps = ops.plan(packed, xq[lo:hi], Ba, **kw)
    gp = dist.all_gather_rows(path.cpu(), q)
    gs = dist.all_gather_rows(steps.cpu(), q)
    pf, sf = ops.plan(packed, xq, Ba, **kw)
    assert torch.equal(gs, sf.cpu()) and torch.equal(gp, pf.cpu())
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_share_gpu_sharded_path():
    """bench.py's N > 1 data path (contiguous shards, per-rank HIP kernels, all-gather of the
    per-rank rows) with two rank processes on the one GPU: the gathered τ+∇τ rows and planner
    paths equal the single-process results bitwise."""
    import torch.multiprocessing as mp
    from test_dist import _free_port
    mp.start_processes(_gpu_worker, args=(2, _free_port(), 5001, 37), nprocs=2, join=True,
                       start_method="spawn")
