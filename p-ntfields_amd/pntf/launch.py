"""One-process-per-GPU launcher: what `torchrun --nproc-per-node N` does, for
`bench.py --gpus N` started without a torch.distributed environment.

The parent never touches the GPU (it imports nothing from HIP and makes no device call): it
picks a free 127.0.0.1 port, starts N fresh child interpreters running the same script with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, relays rank 0's stdout and
every rank's stderr, and returns the first non-zero exit status (0 when all ranks succeed).
If one rank fails, the others are terminated (by the PIDs it started, never by pattern) so
a collective cannot leave them waiting forever.
"""
import os
import socket
import subprocess
import sys
import threading
import time


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _pump(src, dst, prefix=""):
    for line in iter(src.readline, b""):
        dst.write((prefix + line.decode(errors="replace")) if prefix else
                  line.decode(errors="replace"))
        dst.flush()
    src.close()


def spawn(nproc, argv, extra_env=None, timeout=None):
    """Run `sys.executable argv` as `nproc` ranks; return the job's exit status."""
    port = free_port()
    procs, pumps = [], []
    for rank in range(nproc):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable] + list(argv), env=env,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        procs.append(p)
        out = sys.stdout if rank == 0 else sys.stderr
        for src, dst, pre in ((p.stdout, out, "" if rank == 0 else "[rank %d] " % rank),
                              (p.stderr, sys.stderr, "[rank %d] " % rank)):
            t = threading.Thread(target=_pump, args=(src, dst, pre), daemon=True)
            t.start()
            pumps.append(t)
    t0 = time.monotonic()
    status = 0
    live = set(range(nproc))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for o in live:                      # a failed rank strands the collective
                    procs[o].terminate()
        if timeout is not None and time.monotonic() - t0 > timeout and live:
            for o in live:
                procs[o].kill()
            status = status or 124
        time.sleep(0.05)
    for t in pumps:
        t.join(timeout=5)
    return status
