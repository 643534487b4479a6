"""Torch-facing wrappers of the libpntf C ABI (device tensors in, device tensors out).

Every call is stream-ordered on torch's current HIP stream of the input's device; torch's
caching allocator owns all buffers (outputs and the scratch workspace).  Inputs must be
HIP (``cuda``) tensors: there is deliberately no CPU path.

The scratch workspace is cached per (device, stream): two streams of one device never share
a slot set, so concurrent calls on different streams cannot overwrite each other's saved σ
tiles.  The kernel schedule is an argument of every call (pntf_field_ex); nothing here
mutates process-wide library state.
"""
import collections
import ctypes

import torch

from . import _lib
from ._lib import GRAD_BACKGRAD_COMPAT, GRAD_EXACT, PntfError, check

__all__ = ["GRAD_EXACT", "GRAD_BACKGRAD_COMPAT", "PntfError", "pack_weights", "tau",
           "tau_grad", "path_velocity", "speed", "travel_time", "plan", "eikonal_residual",
           "device_sum", "packed_floats", "workspace_bytes", "point_mesh_distance"]

class StreamScratch:
    """Grow-only device scratch per (device, stream), least-recently-used first out.

    A buffer is recorded on the stream it serves, so the caching allocator keeps its memory
    alive until that stream's queued work is done even after the entry is dropped or
    replaced.  At most `cap` streams keep a buffer: a caller that cycles through short-lived
    streams does not pin one buffer per dead stream, and a recycled stream handle at worst
    reuses a live buffer of the right size."""

    def __init__(self, dtype, cap=8):
        self.dtype, self.cap = dtype, cap
        self.entries = collections.OrderedDict()

    def get(self, device, numel):
        stream = torch.cuda.current_stream(device)
        key = (device.index, stream.cuda_stream)
        buf = self.entries.pop(key, None)
        if buf is None or buf.numel() < numel:
            buf = torch.empty(max(int(numel), 1), dtype=self.dtype, device=device)
            if not torch.cuda.is_current_stream_capturing():
                buf.record_stream(stream)     # (a graph's pool keeps its buffers alive)
        self.entries[key] = buf
        while len(self.entries) > self.cap:
            self.entries.popitem(last=False)
        return buf


_ws_cache = StreamScratch(torch.uint8)


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_device(t, name):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise PntfError("%s must be a HIP device tensor (got %s); the P-NTFields MI355X path "
                        "has no CPU fallback" % (name, getattr(t, "device", type(t))))


def packed_floats():
    return int(_lib.load().pntf_packed_floats())


def workspace_bytes(n):
    return int(_lib.load().pntf_workspace_bytes(int(n)))


def _workspace(device, n):
    """Scratch buffer per (device, stream) for the saved σ10 tiles of the reverse sweep
    (StreamScratch: grow-only, LRU over streams)."""
    return _ws_cache.get(device, workspace_bytes(n))


def pack_weights(params, out=None):
    """Pack the 30 state-dict tensors (reference order, see synth.state_dict_keys) into the
    MFMA fragment blob consumed by every kernel (pntf_pack_weights)."""
    lib = _lib.load()
    params = list(params)
    if len(params) != 30:
        raise PntfError("expected the 30 state-dict tensors of NN, got %d" % len(params))
    dev = params[0].device
    ts = []
    for i, p in enumerate(params):
        _require_device(p, "param[%d]" % i)
        ts.append(p.detach().to(torch.float32).contiguous())
    if out is None:
        out = torch.empty(packed_floats(), dtype=torch.float32, device=dev)
    arr = (ctypes.c_void_p * 30)(*[t.data_ptr() for t in ts])
    check(lib.pntf_pack_weights(arr, 30, _vp(out), _stream(dev)), "pntf_pack_weights")
    return out


def _prep(xp, Btab, env, dim):
    _require_device(xp, "xp")
    if dim not in (3, 6):
        raise PntfError("dim must be 3 or 6")
    if xp.dim() != 2 or xp.shape[1] != 2 * dim:
        raise PntfError("xp must be (n, %d), got %s" % (2 * dim, tuple(xp.shape)))
    xp = xp.detach().to(torch.float32).contiguous()
    _require_device(Btab, "B")
    Bt = Btab.detach().to(device=xp.device, dtype=torch.float32)
    if Bt.dim() == 2:
        Bt = Bt.unsqueeze(0)
    if Bt.dim() != 3 or Bt.shape[1] != dim or Bt.shape[2] != 128:
        raise PntfError("B must be (dim, 128) or (n_env, dim, 128), got %s" % (tuple(Btab.shape),))
    Bt = Bt.contiguous()
    if env is not None:
        _require_device(env, "env")
        if env.numel() != xp.shape[0]:
            raise PntfError("env must hold one id per pair")
        env = env.detach().to(torch.int32).contiguous()
    return xp, Bt, env


SCHEDULES = {"auto": 0, "wave_tile": 1, "split_tile": 2, "wide_tile": 3, "quad_tile": 4}
FIELD_TAU, FIELD_TAU_GRAD, FIELD_VELOCITY, FIELD_SPEED, FIELD_TRAVEL = range(5)


def resolved_schedule(n, schedule="auto"):
    """Name of the kernel family a field call of n pairs runs (pntf_field_schedule_for)."""
    r = int(_lib.load().pntf_field_schedule_for(int(n), _sched(schedule)))
    if r < 0:
        raise PntfError("bad batch size or schedule")
    return {v: k for k, v in SCHEDULES.items()}[r]


def _sched(schedule):
    if schedule not in SCHEDULES:
        raise PntfError("unknown schedule %r (one of %s)" % (schedule, sorted(SCHEDULES)))
    return SCHEDULES[schedule]


def _field(kind, packed, xp, Bt, env, dim, mode, out0, out1, ws, schedule, what):
    n = xp.shape[0]
    check(_lib.load().pntf_field_ex(kind, _vp(packed), dim, _vp(xp), n, _vp(Bt), _vp(env),
                                    Bt.shape[0], mode, _vp(out0), _vp(out1), _vp(ws),
                                    ws.numel() if ws is not None else 0, _sched(schedule),
                                    _stream(xp.device)), what)


def tau(packed, xp, Btab, env=None, dim=3, schedule="auto"):
    """τ (n,) — NN.out (model_res_sigmoid_multi.py:215-259)."""
    xp, Bt, env = _prep(xp, Btab, env, dim)
    out = torch.empty(xp.shape[0], dtype=torch.float32, device=xp.device)
    _field(FIELD_TAU, packed, xp, Bt, env, dim, 0, out, None, None, schedule, "pntf_tau")
    return out


def tau_grad(packed, xp, Btab, env=None, dim=3, mode=GRAD_EXACT, schedule="auto"):
    """τ (n,) and ∇τ (n, 2dim): Model.gradient(NN.out) (EXACT) or NN.out_backgrad (COMPAT)."""
    xp, Bt, env = _prep(xp, Btab, env, dim)
    n = xp.shape[0]
    t = torch.empty(n, dtype=torch.float32, device=xp.device)
    d = torch.empty((n, 2 * dim), dtype=torch.float32, device=xp.device)
    _field(FIELD_TAU_GRAD, packed, xp, Bt, env, dim, mode, t, d, _workspace(xp.device, n),
           schedule, "pntf_tau_grad")
    return t, d


def path_velocity(packed, xp, Btab, env=None, dim=3, mode=GRAD_BACKGRAD_COMPAT,
                  schedule="auto"):
    """[v_start | v_goal] (n, 2dim) and τ (n,) — Model.Gradient (:1218-1248)."""
    xp, Bt, env = _prep(xp, Btab, env, dim)
    n = xp.shape[0]
    v = torch.empty((n, 2 * dim), dtype=torch.float32, device=xp.device)
    t = torch.empty(n, dtype=torch.float32, device=xp.device)
    _field(FIELD_VELOCITY, packed, xp, Bt, env, dim, mode, v, t, _workspace(xp.device, n),
           schedule, "pntf_path_velocity")
    return v, t


def speed(packed, xp, Btab, env=None, dim=3, schedule="auto"):
    """Speed at the goal (n,) — Model.Speed (:1195-1216)."""
    xp, Bt, env = _prep(xp, Btab, env, dim)
    n = xp.shape[0]
    s = torch.empty(n, dtype=torch.float32, device=xp.device)
    _field(FIELD_SPEED, packed, xp, Bt, env, dim, GRAD_EXACT, s, None,
           _workspace(xp.device, n), schedule, "pntf_speed")
    return s


def travel_time(packed, xp, Btab, env=None, dim=3, schedule="auto"):
    """|x_g - x_s| / τ (n,) — Model.TravelTimes (:1173-1186)."""
    xp, Bt, env = _prep(xp, Btab, env, dim)
    tt = torch.empty(xp.shape[0], dtype=torch.float32, device=xp.device)
    _field(FIELD_TRAVEL, packed, xp, Bt, env, dim, 0, tt, None, None, schedule,
           "pntf_travel_time")
    return tt


def plan(packed, xp0, Btab, env=None, dim=3, step=0.03, tol=0.06, max_iter=500,
         mode=GRAD_BACKGRAD_COMPAT, schedule="auto"):
    """Batched bidirectional planner (test/gib_plan.py:74-86; arm: test/arm_plan.py:140-152).

    Returns path (q, max_iter + 2, 2dim) — row 0 the start, frozen rows repeating the final
    state — and steps (q,) int32 (updates taken per query).  `schedule` picks the kernel
    (include/pntf.h pntf_plan_ex): "wave_tile" (one wave per 16 queries), "split_tile" (four
    waves share 16 queries: lower latency per step) or "auto"."""
    sched = _sched(schedule)
    lib = _lib.load()
    xp0, Bt, env = _prep(xp0, Btab, env, dim)
    q = xp0.shape[0]
    path = torch.empty((q, max_iter + 2, 2 * dim), dtype=torch.float32, device=xp0.device)
    steps = torch.empty(q, dtype=torch.int32, device=xp0.device)
    ws = _workspace(xp0.device, q)
    check(lib.pntf_plan_ex(_vp(packed), dim, _vp(xp0), q, _vp(Bt), _vp(env), Bt.shape[0],
                           mode, float(step), float(tol), int(max_iter), _vp(path), _vp(steps),
                           _vp(ws), ws.numel(), sched, _stream(xp0.device)),
          "pntf_plan_ex")
    return path, steps


def plan_handoff_counts(device):
    """(queries the 4-query tiles counted done, queries handed to the SOLO launch) of the last
    AUTO quad-tile plan on the current stream (pntf_plan_ex's tail counters at the start of
    the workspace, pntf_quad.h "Tail hand-off").  A query that runs to max_iter without
    converging is never counted done, so when more than CUs queries of a batch never converge
    the hand-off does not fire (results are unaffected; the plan just keeps its MFMA tiles):
    a zero second count shows that."""
    ws = _ws_cache.get(device, 8)
    c = ws[:8].view(torch.int32).cpu()
    return int(c[0]), int(c[1])


def eikonal_residual(packed, xp, Btab, env=None, dim=3, yobs=None, gamma=1e-3, want=("tau",
                     "dtau", "ltau", "diff")):
    """Taylor-mode τ, ∇τ, diagonal ∇²τ and the per-pair Eikonal residual of Model.Loss
    (NN.out_laplace :710-848, Loss :914-946).  Returns a dict of the requested outputs."""
    lib = _lib.load()
    xp, Bt, env = _prep(xp, Btab, env, dim)
    n = xp.shape[0]
    dv = xp.device
    out = {}
    if "tau" in want:
        out["tau"] = torch.empty(n, dtype=torch.float32, device=dv)
    if "dtau" in want:
        out["dtau"] = torch.empty((n, 2 * dim), dtype=torch.float32, device=dv)
    if "ltau" in want:
        out["ltau"] = torch.empty((n, 2 * dim), dtype=torch.float32, device=dv)
    yo = None
    if "diff" in want:
        if yobs is None:
            raise PntfError("the residual needs yobs (n, 2)")
        _require_device(yobs, "yobs")
        yo = yobs.detach().to(torch.float32).reshape(n, 2).contiguous()
        out["diff"] = torch.empty(n, dtype=torch.float32, device=dv)
    ws = _workspace(dv, n)
    check(lib.pntf_eikonal_residual(_vp(packed), dim, _vp(xp), _vp(yo), n, _vp(Bt), _vp(env),
                                    Bt.shape[0], float(gamma), _vp(out.get("tau")),
                                    _vp(out.get("dtau")), _vp(out.get("ltau")),
                                    _vp(out.get("diff")), _vp(ws), ws.numel(), _stream(dv)),
          "pntf_eikonal_residual")
    return out


def device_sum(x):
    """Deterministic fp64 sum of a float32 device tensor (pntf_sum); returns a 0-d float64
    device tensor."""
    lib = _lib.load()
    _require_device(x, "x")
    x = x.detach().to(torch.float32).contiguous().reshape(-1)
    out = torch.empty((), dtype=torch.float64, device=x.device)
    check(lib.pntf_sum(_vp(x), x.numel(), _vp(out), _stream(x.device)), "pntf_sum")
    return out


def _spread10(x):
    x = (x | (x << 16)) & 0x030000FF
    x = (x | (x << 8)) & 0x0300F00F
    x = (x | (x << 4)) & 0x030C30C3
    return (x | (x << 2)) & 0x09249249


def morton_order(pts):
    """Permutation putting pts (n, 3) in 30-bit Morton (Z-curve) order, on the device."""
    lo = pts.min(0).values
    span = (pts.max(0).values - lo).clamp_min(1e-30)
    q = ((pts - lo) / span * 1023.0).long().clamp_(0, 1023)
    code = _spread10(q[:, 0]) | (_spread10(q[:, 1]) << 1) | (_spread10(q[:, 2]) << 2)
    return torch.argsort(code)


def point_mesh_distance(pts, tris, chunks=0, order=None):
    """Unsigned distance (n,) from pts (n, 3) to the triangle mesh tris (t, 3, 3) on the HIP
    kernel (pntf_point_mesh_distance) — what point_obstacle_distance returns
    (dataprocessing/speed_sampling_gpu.py:325-336: bvh_distance_queries, then sqrt).
    `chunks` = 0 picks the triangle split automatically; every value gives the same bits.
    `order` (default: n >= 4096) queries the points in Morton order, so each workgroup's
    points are compact and the kernel's exact tile culling skips far triangles; results are
    scattered back, bit-identical to the unordered query."""
    _require_device(pts, "pts")
    _require_device(tris, "tris")
    if pts.dim() != 2 or pts.shape[1] != 3:
        raise PntfError("pts must be (n, 3), got %s" % (tuple(pts.shape),))
    tris = tris.reshape(-1, 3, 3) if tris.dim() == 4 and tris.shape[0] == 1 else tris
    if tris.dim() != 3 or tuple(tris.shape[1:]) != (3, 3):
        raise PntfError("tris must be (t, 3, 3) or (1, t, 3, 3), got %s" % (tuple(tris.shape),))
    if pts.device != tris.device:
        raise PntfError("pts and tris must be on the same device")
    pts = pts.detach().to(torch.float32).contiguous()
    tris = tris.detach().to(torch.float32).contiguous()
    out = torch.empty(pts.shape[0], dtype=torch.float32, device=pts.device)
    if pts.shape[0] == 0:
        return out
    if order is None:
        order = pts.shape[0] >= 4096
    perm = morton_order(pts) if order else None
    q = pts[perm].contiguous() if order else pts
    res = torch.empty_like(out) if order else out
    check(_lib.load().pntf_point_mesh_distance(_vp(q), q.shape[0], _vp(tris), tris.shape[0],
                                                _vp(res), int(chunks), _stream(pts.device)),
          "pntf_point_mesh_distance")
    if order:
        out[perm] = res
    return out
