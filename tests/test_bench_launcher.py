"""bench.py's multi-GPU plumbing on CPU: `--gpus N` without a torch.distributed environment
starts N rank processes itself (pntf/launch.py), each rank joins the process group (gloo
here, RCCL on the GPU box), shards the pairs (weak: --pairs per rank; strong: --total-pairs
split), all-gathers the per-rank rows and takes the max-over-ranks time.  `--rehearse` runs
exactly that orchestration with rank-tagged rows in place of the kernel output."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=ROOT)
    return r


def _line(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout          # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [2, 4, 8])
def test_launcher_weak_scaling(gpus):
    j = _line(_run(["--gpus", str(gpus), "--rehearse", "--steps", "3", "--warmup", "1",
                    "--pairs", "1000"]))
    assert j["n_gpus"] == gpus and j["world_size"] == gpus
    assert j["config"]["parallelism"] == "dp%d" % gpus
    assert j["scaling"] == "weak" and j["global_batch"] == 1000 * gpus
    assert j["gather_ok"] and j["steps"] == 3


@pytest.mark.parametrize("gpus,total,rank0", [(3, 1001, 334), (8, 1027, 129),
                                              (8, 1 << 23, 1 << 20)])
def test_launcher_strong_scaling_uneven(gpus, total, rank0):
    """--total-pairs split over the ranks, including the deployment size of 8 (the C4 8M
    workload, 8 x 1M pairs, and an uneven 1027)."""
    j = _line(_run(["--gpus", str(gpus), "--rehearse", "--steps", "2", "--warmup", "0",
                    "--total-pairs", str(total)]))
    assert j["scaling"] == "strong" and j["global_batch"] == total
    assert j["n_gpus"] == gpus and j["world_size"] == gpus
    assert j["pairs_per_rank0"] == rank0 and j["gather_ok"]


def test_single_rank_rehearsal():
    j = _line(_run(["--rehearse", "--steps", "2", "--warmup", "1", "--pairs", "64"]))
    assert j["n_gpus"] == 1 and j["gather_ok"]


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--rehearse"], env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_failed_rank_fails_the_job():
    """A rank that dies makes the launcher exit non-zero instead of hanging the others."""
    sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))
    from pntf import launch
    code = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "sys.exit(3) if r == 1 else time.sleep(60)\n")
    rc = launch.spawn(2, ["-c", code], timeout=30)
    assert rc == 3
