"""Training step on MI355X: the weight gradient of the Eikonal residual loss and AdamW.

Reference: one inner step of `Model.train` is
    loss, loss_n, diff = self.Loss(points, speed, B, beta, gamma)   # :1040-1046
    loss.backward(); optimizer.step(); optimizer.zero_grad()        # :1048-1052
with `torch.optim.AdamW(lr=1e-3, weight_decay=0.1)` (:959-961) — models/model_res_sigmoid_multi.py
(arm: models/model_res_sigmoid.py:954-956, 1062-1075).  The reference differentiates its
Taylor-mode graph `NN.out_laplace` (:710-848) with autograd; here the adjoint is explicit:

  forward  Φ planes (tt_fourier) → per Linear: one fp32 GEMM over all R·M Taylor rows
           (pntf_tt_gemm, csrc/pntf_gemm.hip) + a fused bias/residual/act_laplace kernel (tt_act_fwd) that
           keeps the pre-activation as the tape → merge (tt_merge_fwd) → generator → generator[3]
  head     generator[4] + actout_laplace + Model.Loss forward and backward in one kernel
           (tt_head_loss): diff per pair and d(Σdiff)/d(generator[3] output)
  backward per Linear, reversed: fused act_laplace adjoint + bias gradient (tt_act_bwd), the
           weight gradient gW = gYᵀ·X as ONE GEMM over all R·M rows, the input gradient gY·W
           (+ the residual branch, accumulated in place by the GEMM) → merge adjoint
           (tt_merge_bwd)

Layout: a Taylor tensor of M points and width W is (R, M, W) fp32, R = 1 + ndir + nl planes
[value | ∂ (ndir) | Σ diagonal ∂² (nl)], (ndir, nl) = (dim, 1) in the encoder and (2·dim, 2)
after the merge: the loss needs each endpoint's Laplacian only (Model.Loss :919-920), and the
reference's per-direction second-derivative rows enter every layer linearly, so the tape
carries their per-endpoint sums (R = 5 / 9 instead of 7 / 13 rows per point for dim 3).
The GEMMs are the library's own fp32 MFMA kernels (pntf_tt_gemm: v_mfma_f32_32x32x2_f32,
128 x 128 LDS tiles, deterministic split-K for the weight gradients); every elementwise stage
is a HIP kernel of libpntf.so (csrc/pntf_train.hip).  There is no CPU path and no vendor GEMM.
"""
import ctypes
import os

import torch

from . import _lib, ops
from ._lib import PntfError, check

H = 128
# Schedule of the forward Linear + act (pntf_tt_linear_act): 2 (default) the LDS panel GEMM
# (with bias and residual in its epilogue on residual layers) + the act pass; 0 the library's
# AUTO, 1 / 3 the fused kernels (one / four waves per 32-point block).  PNTF_TT_FUSED sets it
# (to compare; profiles/r04_train_sched*.txt).
_LINEAR_ACT = int(os.environ.get("PNTF_TT_FUSED", "2"))
# Input gradient + the previous layer's act adjoint in one kernel (pntf_tt_linear_bwd, fp32
# MFMA): 1, or pntf_tt_gemm then pntf_tt_act_bwd: 0; unset (None): the fused kernel for layers
# of at least _BWD_FUSED_MIN_POINTS points.  With the fp32-MFMA GEMMs the fused kernel won at
# large batches (2 x 100 000 pairs 64.9 -> 63.3 ms); since the split-bf16 GEMMs (round 5) the
# pair wins everywhere (2 x 100 000: 57.6 vs 59.6 ms, 2 x 10 000: 6.09 vs 6.65;
# profiles/r05_train_sched.txt), so AUTO never takes it.  PNTF_TT_BWD sets it.
_LINEAR_BWD = (int(os.environ["PNTF_TT_BWD"]) if os.environ.get("PNTF_TT_BWD", "") != ""
               else None)
_BWD_FUSED_MIN_POINTS = None
_BLOCK_HEADS = ("encoder.1", "encoder.2", "generator.0", "generator.1", "generator.2")


def trained_keys():
    """State-dict keys that receive gradients (encoder1.0 is created at :160 but never used,
    so the reference's AdamW skips it)."""
    from .synth import state_dict_keys
    return [k for k in state_dict_keys() if not k.startswith("encoder1.0.")]


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_partial_cache = ops.StreamScratch(torch.float32)


def _partial(device):
    """Reduction scratch per (device, stream): calls on different streams never share it."""
    return _partial_cache.get(device, int(_lib.load().pntf_tt_partial_floats()))


_work_cache = ops.StreamScratch(torch.float32)


def _work(device, floats):
    """Split-K partial sums of pntf_tt_gemm per (device, stream), grown on demand."""
    return _work_cache.get(device, floats)


def gemm(C, A, B, ta, tb, beta=0.0):
    """C (M, N) = beta·C + op(A) · op(B) on the library's MFMA GEMM (pntf_tt_gemm):
    op(A) = A (M, K) or, ta, A (K, M) transposed; op(B) = B (K, N) or, tb, B (N, K)
    transposed.  All fp32 contiguous 2-D device tensors."""
    lib = _lib.load()
    M, N = C.shape
    K = A.shape[0] if ta else A.shape[1]
    if (B.shape[1] if tb else B.shape[0]) != K or (A.shape[1] if ta else A.shape[0]) != M or \
            (B.shape[0] if tb else B.shape[1]) != N:
        raise PntfError("gemm shape mismatch")
    nw = int(lib.pntf_tt_gemm_work_floats(M, N, K))
    work = _work(C.device, nw) if nw else None
    st = lib.pntf_tt_gemm(int(ta), int(tb), M, N, K, _vp(A), A.shape[1], _vp(B), B.shape[1],
                          _vp(C), C.shape[1], float(beta), _vp(work), nw,
                          _stream(C.device))
    if st != 0:
        raise PntfError("pntf_tt_gemm: " + lib.pntf_tt_gemm_last_error().decode())


class _Tape:
    """Forward tape of one loss evaluation: (name, input planes, pre-activation planes, act,
    has_residual) per Linear, in execution order.  `nle` second-derivative rows per endpoint:
    1 (the per-endpoint sums of the Eikonal loss), dim (one per direction: a general loss on
    out_laplace's ∇²τ) or 0 (first derivatives only: a loss on ∇τ).  `fused` allows the fused
    input-gradient kernel (pntf_tt_linear_bwd), which takes the Loss / value layouts only."""

    def __init__(self, params, dim, device, nle=1, fused=True):
        self.p = params
        self.dim = dim
        self.dev = device
        self.s = _stream(device)
        self.lib = _lib.load()
        self.ops = []
        self.nle = nle
        self.fused = fused

    def planes(self, R):
        """(ndir, nl) of a Taylor tensor with R planes: (dim, nle) in the encoder, (2dim, 2nle)
        after the merge (pntf_train.hip); (0, 0) for the value-only tape of NN.out."""
        if R == 1:
            return (0, 0)
        if R == 1 + self.dim + self.nle:
            return (self.dim, self.nle)
        return (2 * self.dim, 2 * self.nle)

    def lin(self, x3, name, act=True, res=None):
        W, b = self.p[name + ".weight"], self.p[name + ".bias"]
        R, M, K = x3.shape
        N = W.shape[0]
        ndir, nl = self.planes(R)
        y = torch.empty((R, M, N), dtype=torch.float32, device=self.dev)
        h = torch.empty_like(y) if act else None
        # GEMM + bias + residual + act_laplace (pntf_tt_linear_act: one fused kernel, or the
        # GEMM and the act kernel where the fused one would not balance)
        work = _work(self.dev, int(self.lib.pntf_tt_gemm_work_floats(R * M, N, K)))
        st = self.lib.pntf_tt_linear_act(ndir, nl, _vp(x3), M, K, _vp(W), N, _vp(b), _vp(res),
                                         _vp(y), _vp(h), int(act),
                                         _LINEAR_ACT if self.fused else 2, _vp(work),
                                         work.numel(), self.s)
        if st != 0:
            raise PntfError("pntf_tt_linear_act: %s | %s" % (
                self.lib.pntf_tt_gemm_last_error().decode(),
                self.lib.pntf_tt_last_error().decode()))
        self.ops.append((name, x3, y, int(act), res is not None))
        return h if act else y


def weight_grad(g2, x2, out):
    """out (N, K) = g2ᵀ (N, rows) · x2 (rows, K).  The reduction runs over every Taylor row of
    every point (rows = R·M, 10⁵-10⁶) into a tiny 128/256-square output, so pntf_tt_gemm
    splits the rows over ~2 workgroups per CU and sums the partials in a fixed order."""
    gemm(out, g2, x2, ta=True, tb=False)


def loss_grad(params, xp, yobs, Btab, env, dim, gamma, scale, arm, grads):
    """diff (n,) of Model.Loss and, into `grads` (key -> tensor shaped like the parameter),
    the gradient of scale·Σ diff w.r.t. every trained parameter.

    params: state-dict key -> fp32 contiguous device tensor; xp (n, 2dim); yobs (n, 2);
    Btab (n_env, dim, 128); env (n,) int32 or None."""
    dev = xp.device
    lib = _lib.load()
    n = xp.shape[0]
    if n == 0:
        for g in grads.values():
            g.zero_()
        return torch.empty(0, dtype=torch.float32, device=dev)
    tape = _Tape(params, dim, dev)
    s = tape.s
    Re, Rg = 2 + dim, 3 + 2 * dim        # summed second-derivative planes (pntf_train.hip)
    phi = torch.empty((Re, 2 * n, 2 * H), dtype=torch.float32, device=dev)
    n_env = Btab.shape[0]
    check(lib.pntf_tt_fourier(dim, _vp(xp), n, _vp(Btab), _vp(env), n_env, _vp(phi), s),
          "pntf_tt_fourier")
    h = tape.lin(phi, "encoder.0")
    for i in (1, 2):
        a = tape.lin(h, "encoder.%d" % i)
        h = tape.lin(a, "encoder1.%d" % i, res=h)
    z = tape.lin(h, "encoder.3", act=False)
    u = torch.empty((Rg, n, 2 * H), dtype=torch.float32, device=dev)
    check(lib.pntf_tt_merge_fwd(dim, _vp(z), n, _vp(u), s), "pntf_tt_merge_fwd")
    for i in (0, 1, 2):
        a = tape.lin(u, "generator.%d" % i)
        u = tape.lin(a, "generator1.%d" % i, res=u)
    v = tape.lin(u, "generator.3")
    diff = torch.empty(n, dtype=torch.float32, device=dev)
    g = torch.empty_like(v)
    part = _partial(dev)
    check(lib.pntf_tt_head_loss(dim, int(arm), _vp(v), _vp(params["generator.4.weight"]),
                                _vp(params["generator.4.bias"]), _vp(xp), _vp(yobs), n,
                                float(gamma), float(scale), _vp(diff), _vp(g),
                                _vp(grads["generator.4.weight"]), _vp(grads["generator.4.bias"]),
                                _vp(part), s), "pntf_tt_head_loss")
    def merge_bwd(g):
        gz = torch.empty((Re, 2 * n, H), dtype=torch.float32, device=dev)
        check(lib.pntf_tt_merge_bwd(dim, _vp(z), _vp(g), n, _vp(gz), s), "pntf_tt_merge_bwd")
        return gz
    _adjoint(tape, g, grads, part, merge_bwd)
    return diff


def _adjoint(tape, g, grads, part, merge_bwd, want_input=False):
    """Walk the tape back from g = dL/d(generator[3] output planes): per Linear the act adjoint
    (+ bias gradient), the weight gradient and the input gradient; merge_bwd(g) at the merge.
    With _LINEAR_BWD the input gradient of a Linear and the act adjoint of the layer before it
    run as one kernel (pntf_tt_linear_bwd) wherever that layer's output feeds this one directly
    (not across the merge).  want_input: returns dL/dΦ, the Fourier planes' gradient (one more
    GEMM through encoder[0]); otherwise None."""
    lib, s, dev, params = tape.lib, tape.s, tape.dev, tape.p
    pending = []
    order = list(reversed(tape.ops))
    fused_in = False          # this layer's act adjoint already ran in the previous kernel
    for idx, (name, x3, y, act, has_res) in enumerate(order):
        R, M, K = x3.shape
        N = y.shape[2]
        ndir, nl = tape.planes(R)
        if not fused_in:
            check(lib.pntf_tt_act_bwd(ndir, nl, _vp(y), _vp(g), M, N, int(act),
                                      _vp(grads[name + ".bias"]), 0, _vp(part), s),
                  "pntf_tt_act_bwd")
        g2 = g.view(R * M, N)
        weight_grad(g2, x3.view(R * M, K), grads[name + ".weight"])
        if name == "encoder.0":
            if not want_input:
                return None
            gphi = torch.empty((R, M, K), dtype=torch.float32, device=dev)
            gemm(gphi.view(R * M, K), g2, params[name + ".weight"], ta=False, tb=False)
            return gphi
        if has_res:
            pending.append(g)
        W = params[name + ".weight"]
        prev = order[idx + 1]
        res = pending.pop() if name in _BLOCK_HEADS else None
        if _LINEAR_BWD is None:
            use_bwd = tape.fused and _BWD_FUSED_MIN_POINTS is not None and \
                M >= _BWD_FUSED_MIN_POINTS
        else:
            use_bwd = tape.fused and bool(_LINEAR_BWD)
        fused_in = use_bwd and name != "generator.0" and prev[3]
        if fused_in:
            # gx = act_bwd_prev(g·W (+ res)): in place into the residual branch's buffer
            gx = res if res is not None else torch.empty((R, M, K), dtype=torch.float32,
                                                         device=dev)
            work = _work(dev, int(lib.pntf_tt_linear_bwd_work_floats(N, K)))
            st = lib.pntf_tt_linear_bwd(ndir, nl, _vp(g), M, N, _vp(W), K, _vp(prev[2]),
                                        _vp(res), _vp(gx), _vp(grads[prev[0] + ".bias"]),
                                        _vp(work), work.numel(), s)
            if st != 0:
                raise PntfError("pntf_tt_linear_bwd: " + lib.pntf_tt_gemm_last_error().decode())
        elif res is not None:
            # the block input also fed the residual add: accumulate into that branch's
            # gradient in place (beta = 1, no copy); it is not read again
            gx = res
            gemm(gx.view(R * M, K), g2, W, ta=False, tb=False, beta=1.0)
        else:
            gx = torch.empty((R, M, K), dtype=torch.float32, device=dev)
            gemm(gx.view(R * M, K), g2, W, ta=False, tb=False)
        g = gx
        if name == "generator.0":
            g = merge_bwd(g)


def tau_weight_grad(params, xp, Btab, env, dim, gtau, grads):
    """Into `grads` (key -> tensor shaped like the parameter): the gradient of Σ_p gtau_p·τ_p
    w.r.t. every trained parameter, τ = NN.out(xp, B) (models/model_res_sigmoid_multi.py:
    215-259; arm models/model_res_sigmoid.py:212-256) — what the reference's autograd leaves
    in `.grad` after a backward through NN.out.  The value-only tape (R = 1): Fourier value
    plane, per Linear one GEMM + the fused bias/residual/softplus kernel, the value merge,
    the τ head with dL/dτ, then the same adjoint sweep as the Eikonal loss.  Returns τ (n,)."""
    dev = xp.device
    lib = _lib.load()
    n = xp.shape[0]
    tau = torch.empty(n, dtype=torch.float32, device=dev)
    if n == 0:
        for g in grads.values():
            g.zero_()
        return tau
    tape = _Tape(params, dim, dev)
    s = tape.s
    phi = torch.empty((1, 2 * n, 2 * H), dtype=torch.float32, device=dev)
    check(lib.pntf_tt_fourier_value(dim, _vp(xp), n, _vp(Btab), _vp(env), Btab.shape[0],
                                    _vp(phi), s), "pntf_tt_fourier_value")
    h = tape.lin(phi, "encoder.0")
    for i in (1, 2):
        a = tape.lin(h, "encoder.%d" % i)
        h = tape.lin(a, "encoder1.%d" % i, res=h)
    z = tape.lin(h, "encoder.3", act=False)
    u = torch.empty((1, n, 2 * H), dtype=torch.float32, device=dev)
    check(lib.pntf_tt_merge_value_fwd(_vp(z), n, _vp(u), s), "pntf_tt_merge_value_fwd")
    for i in (0, 1, 2):
        a = tape.lin(u, "generator.%d" % i)
        u = tape.lin(a, "generator1.%d" % i, res=u)
    v = tape.lin(u, "generator.3")
    g = torch.empty_like(v)
    part = _partial(dev)
    gtau = gtau.detach().to(device=dev, dtype=torch.float32).contiguous()
    check(lib.pntf_tt_head_tau(_vp(v), _vp(params["generator.4.weight"]),
                               _vp(params["generator.4.bias"]), n, _vp(gtau), _vp(tau), _vp(g),
                               _vp(grads["generator.4.weight"]), _vp(grads["generator.4.bias"]),
                               _vp(part), s), "pntf_tt_head_tau")

    def merge_bwd(gu):
        gz = torch.empty((1, 2 * n, H), dtype=torch.float32, device=dev)
        check(lib.pntf_tt_merge_value_bwd(_vp(z), _vp(gu), n, _vp(gz), s),
              "pntf_tt_merge_value_bwd")
        return gz
    _adjoint(tape, g, grads, part, merge_bwd)
    return tau


def field_vjp(params, xp, Btab, env, dim, nle, quirk, gtau, gdtau, glap, grads, want_x):
    """The backward of Σ_p (gtau_p·τ_p + gdtau_p·∇τ_p + glap_p·Δ_p) through the Taylor graph of
    NN.out_laplace (models/model_res_sigmoid_multi.py:710-848), NN.out_grad (:303-400),
    NN.out_backgrad (quirk: encoder[0]'s derivative row scaled by σ(10·softplus(y)),
    :435-438) or Model.gradient's ∇τ (:890-896): what the reference's autograd leaves in
    every trained parameter's `.grad` (written into `grads`, key -> tensor shaped like the
    parameter) and, with want_x, returns as coords' gradient (n, 2dim).

    nle second-derivative rows per endpoint: 0 (a loss on τ and ∇τ only), 1 (glap (n, 2) on
    each endpoint's Laplacian Σ_d ∂²τ/∂x_d², the rows the Eikonal loss uses) or dim (glap
    (n, 2dim) on the diagonal ∇²τ).  gtau (n,), gdtau (n, 2dim), glap: device tensors or None
    (zero).  Tape: the Fourier planes (pntf_tt_fourier_ex), per Linear one GEMM + the fused
    bias/residual/act kernel, the merge (pntf_tt_merge_fwd_ex), generator[4] + actout_laplace
    with the upstream gradient (pntf_tt_head_vjp), the adjoint sweep of the training step, and
    the Fourier adjoint for the coordinates (pntf_tt_fourier_bwd).  Returns gx or None."""
    dev = xp.device
    lib = _lib.load()
    n = xp.shape[0]
    if nle not in (0, 1, dim) or (quirk and nle):
        raise PntfError("field_vjp: nle must be 0, 1 or dim (0 with the out_backgrad quirk)")
    if n == 0:
        for g in grads.values():
            g.zero_()
        return torch.empty((0, 2 * dim), dtype=torch.float32, device=dev) if want_x else None
    tape = _Tape(params, dim, dev, nle=nle, fused=False)
    s = tape.s
    Re, Rg = 1 + dim + nle, 1 + 2 * dim + 2 * nle
    n_env = Btab.shape[0]
    phi = torch.empty((Re, 2 * n, 2 * H), dtype=torch.float32, device=dev)
    check(lib.pntf_tt_fourier_ex(dim, dim, nle, _vp(xp), n, _vp(Btab), _vp(env), n_env, _vp(phi),
                                 s), "pntf_tt_fourier_ex")
    h = tape.lin(phi, "encoder.0", act=2 if quirk else 1)
    for i in (1, 2):
        a = tape.lin(h, "encoder.%d" % i)
        h = tape.lin(a, "encoder1.%d" % i, res=h)
    z = tape.lin(h, "encoder.3", act=False)
    u = torch.empty((Rg, n, 2 * H), dtype=torch.float32, device=dev)
    check(lib.pntf_tt_merge_fwd_ex(dim, nle, _vp(z), n, _vp(u), s), "pntf_tt_merge_fwd_ex")
    for i in (0, 1, 2):
        a = tape.lin(u, "generator.%d" % i)
        u = tape.lin(a, "generator1.%d" % i, res=u)
    v = tape.lin(u, "generator.3")
    g = torch.empty_like(v)
    part = _partial(dev)

    def dev32(t):
        return None if t is None else t.detach().to(device=dev, dtype=torch.float32).contiguous()
    gtau, gdtau, glap = dev32(gtau), dev32(gdtau), dev32(glap)
    check(lib.pntf_tt_head_vjp(dim, nle, _vp(v), _vp(params["generator.4.weight"]),
                               _vp(params["generator.4.bias"]), n, _vp(gtau), _vp(gdtau),
                               _vp(glap), None, None, None, _vp(g),
                               _vp(grads["generator.4.weight"]), _vp(grads["generator.4.bias"]),
                               _vp(part), s), "pntf_tt_head_vjp")

    def merge_bwd(gu):
        gz = torch.empty((Re, 2 * n, H), dtype=torch.float32, device=dev)
        check(lib.pntf_tt_merge_bwd_ex(dim, nle, _vp(z), _vp(gu), n, _vp(gz), s),
              "pntf_tt_merge_bwd_ex")
        return gz
    gphi = _adjoint(tape, g, grads, part, merge_bwd, want_input=want_x)
    if not want_x:
        return None
    gx = torch.empty((n, 2 * dim), dtype=torch.float32, device=dev)
    check(lib.pntf_tt_fourier_bwd(dim, dim, nle, _vp(gphi), _vp(xp), n, _vp(Btab), _vp(env),
                                  n_env, _vp(gx), s), "pntf_tt_fourier_bwd")
    return gx


def module_params(module):
    """The trained parameters of an NN module as {key: fp32 contiguous device tensor}."""
    sd = module.state_dict(keep_vars=True)
    out = {}
    for k in trained_keys():
        p = sd[k]
        ops._require_device(p, k)
        if p.dtype != torch.float32 or not p.is_contiguous():
            raise PntfError("parameter %s must be fp32 contiguous" % k)
        out[k] = p.detach()
    return out


class EikonalLossFunction(torch.autograd.Function):
    """Σdiff·scale of Model.Loss with a HIP backward to the weights.  The adjoint sweep runs
    inside forward (its head kernel fuses the loss backward), the weight gradients wait in
    ctx until autograd asks for them.  Inputs (points, speeds, B) get no gradient: the
    reference never reads theirs."""

    @staticmethod
    def forward(ctx, xp, yobs, Btab, env, dim, gamma, scale, arm, keys, *params):
        p = {k: t.detach() for k, t in zip(keys, params)}
        # all weight gradients in one flat buffer (views at 256-byte aligned offsets), so that
        # backward scales them by the incoming gradient in one launch instead of one per tensor
        offs, n = [], 0
        for k in keys:
            offs.append(n)
            n += (p[k].numel() + 63) // 64 * 64
        flat = torch.empty(n, dtype=torch.float32, device=xp.device)
        grads = {k: flat[o:o + p[k].numel()].view(p[k].shape) for k, o in zip(keys, offs)}
        diff = loss_grad(p, xp, yobs, Btab, env, dim, gamma, scale, arm, grads)
        ctx.flat, ctx.offs = flat, offs
        ctx.shapes = [p[k].shape for k in keys]
        ctx.mark_non_differentiable(diff)
        total = ops.device_sum(diff).float() * scale
        return total, diff

    @staticmethod
    def backward(ctx, g_total, g_diff):
        flat = ctx.flat * g_total
        ctx.flat = None
        gs = [flat[o:o + sh.numel()].view(sh) for o, sh in zip(ctx.offs, ctx.shapes)]
        return (None,) * 9 + tuple(gs)


def eikonal_loss(module, xp, yobs, Btab, env, dim, gamma, scale, arm=False):
    """(scale·Σdiff (0-d, differentiable w.r.t. the module's parameters), diff (n,))."""
    ops._require_device(xp, "points")
    xp = xp.detach().to(torch.float32).contiguous()
    yobs = yobs.detach().to(device=xp.device, dtype=torch.float32).contiguous()
    Btab = Btab.detach().to(device=xp.device, dtype=torch.float32).contiguous()
    if env is not None:
        env = env.to(device=xp.device, dtype=torch.int32).contiguous()
    if xp.dim() != 2 or xp.shape[1] != 2 * dim or yobs.shape != (xp.shape[0], 2):
        raise PntfError("points must be (n, %d) and speeds (n, 2)" % (2 * dim))
    if Btab.dim() != 3 or Btab.shape[1:] != (dim, H):
        raise PntfError("B table must be (n_env, %d, 128)" % dim)
    p = module_params(module)
    keys = list(p.keys())
    sd = module.state_dict(keep_vars=True)
    return EikonalLossFunction.apply(xp, yobs, Btab, env, dim, float(gamma), float(scale),
                                     bool(arm), keys, *[sd[k] for k in keys])


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (the reference's optimizer, :959-961) with the update as one
    fused HIP launch per param group (pntf_adamw_multi: every tensor of the group whose step
    counts agree; pntf_adamw per tensor otherwise).  Parameters without a gradient are skipped,
    exactly as torch does (encoder1.0).  state_dict()/load_state_dict() work as in torch, so
    the reference's rollback of (network, optimizer) states (:1093-1101) is unchanged."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            hyper = (float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                     float(group["weight_decay"]))
            todo = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                ops._require_device(p, "param")
                if not p.is_contiguous():
                    raise PntfError("AdamW: parameters must be contiguous")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                todo.append((p, p.grad.contiguous(), st, int(st["step"].item())))
            if not todo:
                continue
            steps = {t[3] for t in todo}
            same_dev = len({t[0].device for t in todo}) == 1
            if len(steps) == 1 and same_dev:
                # one launch per 64 tensors (the model's 28 trained tensors: one)
                for c0 in range(0, len(todo), 64):
                    chunk = todo[c0:c0 + 64]
                    k = len(chunk)
                    arr = lambda xs: (ctypes.c_void_p * k)(*xs)  # noqa: E731
                    check(lib.pntf_adamw_multi(
                        k, arr([_vp(t[0]) for t in chunk]), arr([_vp(t[1]) for t in chunk]),
                        arr([_vp(t[2]["exp_avg"]) for t in chunk]),
                        arr([_vp(t[2]["exp_avg_sq"]) for t in chunk]),
                        (ctypes.c_int64 * k)(*[t[0].numel() for t in chunk]), *hyper,
                        chunk[0][3], _stream(chunk[0][0].device)), "pntf_adamw_multi")
            else:
                for p, g, st, step in todo:
                    check(lib.pntf_adamw(_vp(p), _vp(g), _vp(st["exp_avg"]),
                                         _vp(st["exp_avg_sq"]), p.numel(), *hyper, step,
                                         _stream(p.device)), "pntf_adamw")
            for t in todo:
                # the kernel wrote through a raw pointer: tell torch (and PackedCache)
                torch.autograd.graph.increment_version(t[0])
        return loss

