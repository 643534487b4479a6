"""Multi-process sharding path on CPU (gloo, world_size 2): each rank evaluates its
contiguous shard (here with the oracle standing in for the HIP kernel, which needs a GPU)
and the RCCL/gloo all-gather of per-rank rows reassembles the full batch in order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from pntf import dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as tdist
    from oracle import pntf_oracle as O
    from pntf import synth
    r, ws = dist.init("gloo")
    assert (r, ws) == (rank, world)
    W = synth.make_weights(0)
    xp = synth.make_pairs(n, 3, seed=2)
    B = synth.make_B(3)
    lo, hi = dist.shard_range(n, rank, world)
    t, d = O.tau_grad(W, xp[lo:hi], B, dtype=np.float32)
    local = torch.from_numpy(np.concatenate([t, d], 1).astype(np.float32))
    full = dist.all_gather_rows(local, n)
    tf, df = O.tau_grad(W, xp, B, dtype=np.float32)
    np.testing.assert_allclose(full.numpy(), np.concatenate([tf, df], 1), rtol=1e-5, atol=1e-6)
    # planner paths gathered the same way (q queries, uneven shards)
    xq = synth.make_pairs(q, 3, seed=11)
    lo, hi = dist.shard_range(q, rank, world)
    p, s = O.plan(W, xq[lo:hi], B, max_iter=20, dtype=np.float32)
    paths = dist.all_gather_rows(torch.from_numpy(p.astype(np.float32)), q)
    pf, sf = O.plan(W, xq, B, max_iter=20, dtype=np.float32)
    np.testing.assert_allclose(paths.numpy(), pf, rtol=1e-5, atol=1e-6)
    tdist.barrier()
    tdist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1048577):
        for w in (1, 2, 3, 8):
            ranges = [dist.shard_range(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [h - l for l, h in ranges]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("n,q", [(100, 5), (64, 4)])
def test_gloo_world2_gather(n, q):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, n, q), nprocs=2, join=True, start_method="spawn")


def _worker_ws1(_rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as tdist
    assert dist.init("gloo") == (0, 1) and not tdist.is_initialized()
    assert dist.init("gloo", force=True) == (0, 1) and tdist.get_world_size() == 1
    local = torch.arange(21, dtype=torch.float32).reshape(7, 3)
    assert dist.all_gather_rows(local, 7) is local               # no collective by default
    full = dist.all_gather_rows(local, 7, force=True)            # the collective, one rank
    assert full is not local and torch.equal(full, local)
    tdist.destroy_process_group()


def test_gloo_world1_forced_collective():
    """`force` runs the real collective at world size 1 (the path the GPU test
    test_rccl.py::test_rccl_world1_allgather drives over RCCL)."""
    mp.start_processes(_worker_ws1, args=(_free_port(),), nprocs=1, join=True,
                       start_method="spawn")


def _worker_c5(rank, world, port, q, max_iter):
    """One rank of the sharded C5 exchange (bench.py shard_gather_plans) with the fp32 oracle
    planner standing in for the HIP kernel; rank 0 checks the gathered paths and step counts
    against the unsharded plan, query by query."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as tdist
    import bench
    from oracle import pntf_oracle as O
    from pntf import synth
    torch.set_num_threads(1)
    dist.init("gloo")
    W = synth.make_weights(0)
    Ba = synth.make_B(6, seed=12, arm=True).T
    xq = synth.make_box_pairs(q, 6, seed=3)

    def plan_local(x):
        p, s = O.plan(W, x, Ba, dim=6, step=0.015, tol=0.03, max_iter=max_iter, compat=False,
                      dtype=np.float32)
        return torch.from_numpy(p.astype(np.float32)), torch.from_numpy(s.astype(np.int32))
    paths, steps = bench.shard_gather_plans(plan_local, xq, rank, world)
    assert paths.shape == (q, max_iter + 2, 12) and steps.shape == (q,)
    if rank == 0:
        pf, sf = plan_local(xq)
        assert torch.equal(steps, sf)
        # each shard is planned alone, so only the fp32 summation order of the batch differs
        assert float((paths - pf).abs().max()) < 1e-5
        assert torch.equal(paths[:, 0], torch.from_numpy(xq))        # query order kept
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("q", [1024, 1027])
def test_gloo_world8_c5_sharded_gather(q):
    """The deployment size: 8 ranks, the C5 1024 queries (128 per rank) and an uneven 1027
    (129 on ranks 0-2, 128 on the rest), gathered in query order (bench.py
    sharded_extras).  4 planner steps keep the oracle's CPU time small."""
    port = _free_port()
    mp.start_processes(_worker_c5, args=(8, port, q, 4), nprocs=8, join=True,
                       start_method="spawn")
