"""Shared pieces of the drop-in `NN` modules: layer table, packed-weight cache, autograd op.

The module keeps the reference's `torch.nn.Linear` parameters (so reference checkpoints
load with `load_state_dict(strict=True)`), and hands the kernels a packed fragment blob
(pntf_pack_weights) that is rebuilt whenever a parameter is moved or modified.
"""
import math

import torch
from torch.autograd.function import once_differentiable

from . import ops
from .synth import state_dict_keys

H = 128


def build_layers(module, in_features=2 * H):
    """The reference layer table (models/model_res_sigmoid_multi.py:155-175)."""
    Linear = torch.nn.Linear
    module.nl1 = 3
    module.nl2 = 3
    module.encoder = torch.nn.ModuleList()
    module.encoder1 = torch.nn.ModuleList()
    module.encoder.append(Linear(in_features, H))
    module.encoder1.append(Linear(in_features, H))   # created but never used by NN.out (:227)
    for _ in range(module.nl1 - 1):
        module.encoder.append(Linear(H, H))
        module.encoder1.append(Linear(H, H))
    module.encoder.append(Linear(H, H))
    module.generator = torch.nn.ModuleList()
    module.generator1 = torch.nn.ModuleList()
    for _ in range(module.nl2):
        module.generator.append(Linear(2 * H, 2 * H))
        module.generator1.append(Linear(2 * H, 2 * H))
    module.generator.append(Linear(2 * H, H))
    module.generator.append(Linear(H, 1))


def init_weights(m):
    """NN.init_weights (model_res_sigmoid_multi.py:177-183): U(±2/sqrt(fan_in))."""
    if type(m) == torch.nn.Linear:
        stdv = (1.0 / math.sqrt(m.weight.size(1)) / 1.0) * 2
        m.weight.data.uniform_(-stdv, stdv)
        m.bias.data.uniform_(-stdv, stdv)


class PackedCache:
    """Packed weights for the module's current parameters, repacked on any change
    (device move, in-place update, load_state_dict)."""

    def __init__(self):
        self._key = None
        self._packed = None

    def get(self, module):
        sd = module.state_dict(keep_vars=True)
        keys = list(sd.keys())
        if keys != state_dict_keys():
            raise ops.PntfError("unexpected NN state-dict layout: %s" % keys)
        params = list(sd.values())
        key = tuple((p.device, p.data_ptr(), p._version, p.dtype) for p in params)
        if key != self._key:
            self._packed = ops.pack_weights(params)
            self._key = key
        return self._packed


def _trained(module):
    """(keys, tensors) of the module's trained parameters (every key but encoder1.0, which the
    reference creates at :160 and never uses), validated once per parameter version: fp32,
    contiguous, on a HIP device."""
    from . import train
    sd = module.state_dict(keep_vars=True)
    keys = train.trained_keys()
    ps = [sd[k] for k in keys]
    stamp = tuple((p.data_ptr(), p._version, p.dtype, p.device) for p in ps)
    if getattr(module, "_pntf_trained_stamp", None) != stamp:
        for k, p in zip(keys, ps):
            ops._require_device(p, k)
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ops.PntfError("parameter %s must be fp32 contiguous" % k)
        module._pntf_trained_stamp = stamp
    return keys, ps


def _param_grads(ctx, keys, params, first):
    """Scratch gradient tensors for every trained parameter (the tape writes all of them) and
    the tuple autograd expects: a tensor where input `first + i` needs a gradient, else None
    (a frozen layer's gradient is computed and dropped, as autograd would)."""
    grads = {k: torch.empty_like(p) for k, p in zip(keys, params)}
    out = tuple(grads[k] if ctx.needs_input_grad[first + i] else None
                for i, k in enumerate(keys))
    return grads, out


def _no_b_grad(ctx, idx):
    if ctx.needs_input_grad[idx]:
        raise ops.PntfError("the HIP path has no gradient with respect to the Fourier matrix B "
                            "(the reference scripts pass it as data); detach B")


class TauFunction(torch.autograd.Function):
    """τ = NN.out(coords); d τ / d coords by the fused HIP reverse sweep.

    When coords needs a gradient the forward launches the fused τ+∇τ kernel once and keeps
    ∇τ, so `Model.gradient(tau, coords)` (model_res_sigmoid_multi.py:890-896) costs no second
    launch.  With `create_graph=True` the ∇τ it returns is itself differentiable (GradTauFunction:
    its backward runs the first-order Taylor tape to every weight and to coords), as the
    reference's double-backward through nn.Linear + autograd is.  The weights are inputs only
    for that link: their first-order gradient comes from TauWeightFunction."""

    @staticmethod
    def forward(ctx, coords, B, env, packed, dim, keys, *params):
        ctx.dim, ctx.keys, ctx.np = dim, keys, len(params)
        if ctx.needs_input_grad[0]:
            t, d = ops.tau_grad(packed, coords, B, env, dim, ops.GRAD_EXACT)
            ctx.save_for_backward(d, coords, B, env, *params)
        else:
            t = ops.tau(packed, coords, B, env, dim)
        return t.unsqueeze(1)

    @staticmethod
    def backward(ctx, grad_tau):
        none = (None,) * (5 + ctx.np)
        if not ctx.needs_input_grad[0]:
            return (None,) + none
        d, coords, B, env, *params = ctx.saved_tensors
        if torch.is_grad_enabled():            # create_graph: ∇τ enters a graph of its own
            d = GradTauFunction.apply(coords, B, env, ctx.dim, ctx.keys, d, *params)
        return (grad_tau * d,) + none


class GradTauFunction(torch.autograd.Function):
    """∇τ (n, 2dim) of NN.out as a function of coords and the weights (the value of
    Model.gradient(τ, coords, create_graph=True), :890-896); forward returns the fused kernel's
    ∇τ, backward the exact first-order Taylor adjoint (pntf/train.py field_vjp, nle = 0)."""

    @staticmethod
    def forward(ctx, coords, B, env, dim, keys, d, *params):
        ctx.save_for_backward(coords, B, env, *params)
        ctx.dim, ctx.keys = dim, keys
        return d.clone()

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        from . import train
        coords, B, env, *params = ctx.saved_tensors
        _no_b_grad(ctx, 1)
        grads, gp = _param_grads(ctx, ctx.keys, params, 6)
        Btab = B if B.dim() == 3 else B.unsqueeze(0)
        gx = train.field_vjp(dict(zip(ctx.keys, params)), coords.detach().contiguous(),
                             Btab.detach().contiguous(), env, ctx.dim, 0, False, None, g, None,
                             grads, ctx.needs_input_grad[0])
        return (gx, None, None, None, None, None) + gp


class TaylorFunction(torch.autograd.Function):
    """The outputs of NN.out_grad / NN.out_backgrad (order 1: τ (n,), ∇τ (n, 2dim)) or
    NN.out_laplace (order 2: + diagonal ∇²τ (n, 2dim)) as functions of coords and the
    weights, as the reference's plain torch graphs are (models/model_res_sigmoid_multi.py:
    303-400, 402-647, 710-848).  Forward: the fused HIP kernels (ops.tau_grad,
    ops.eikonal_residual).  Backward: the HIP Taylor tape with the incoming gradients
    (pntf/train.py field_vjp): only first-derivative rows when ∇²τ gets no gradient, the
    per-endpoint Laplacian rows when its gradient is constant over each endpoint's dims (a
    loss on Σ_d ∂²τ/∂x_d², as Model.Loss :919-920), one row per direction otherwise."""

    @staticmethod
    def forward(ctx, coords, B, env, dim, order, quirk, packed, keys, *params):
        if order == 2:
            out = ops.eikonal_residual(packed, coords, B, env, dim, want=("tau", "dtau", "ltau"))
            res = (out["tau"], out["dtau"], out["ltau"])
        else:
            res = ops.tau_grad(packed, coords, B, env, dim,
                               ops.GRAD_BACKGRAD_COMPAT if quirk else ops.GRAD_EXACT)
        ctx.save_for_backward(coords, B, env, *params)
        ctx.dim, ctx.quirk, ctx.keys = dim, quirk, keys
        if hasattr(ctx, "set_materialize_grads"):
            ctx.set_materialize_grads(False)         # an unused output's gradient stays None
        return res

    @staticmethod
    @once_differentiable
    def backward(ctx, g_tau, g_dtau, g_ltau=None):
        from . import train
        coords, B, env, *params = ctx.saved_tensors
        _no_b_grad(ctx, 1)
        dim, n = ctx.dim, coords.shape[0]
        if g_tau is None and g_dtau is None and g_ltau is None:
            return (None,) * (8 + len(params))
        nle, glap = 0, None
        if g_ltau is not None:
            gl3 = g_ltau.reshape(n, 2, dim)
            if bool((gl3 == gl3[:, :, :1]).all()):        # one value per endpoint: summed rows
                nle, glap = 1, gl3[:, :, 0].contiguous()
            else:
                nle, glap = dim, g_ltau
        grads, gp = _param_grads(ctx, ctx.keys, params, 8)
        Btab = B if B.dim() == 3 else B.unsqueeze(0)
        gx = train.field_vjp(dict(zip(ctx.keys, params)), coords.detach().contiguous(),
                             Btab.detach().contiguous(), env, dim, nle, ctx.quirk, g_tau,
                             g_dtau, glap, grads, ctx.needs_input_grad[0])
        return (gx,) + (None,) * 7 + gp


def taylor_outputs(module, coords, B, env, dim, order, quirk):
    """(τ (n,), ∇τ (n,2dim)[, ∇²τ (n,2dim)]) of NN.out_grad / out_backgrad (order 1) or
    NN.out_laplace (order 2) on the fused kernels; differentiable (TaylorFunction) when
    autograd records and coords or any parameter requires grad."""
    packed = module.packed()
    keys, ps = _trained(module)
    if torch.is_grad_enabled() and (coords.requires_grad or B.requires_grad or
                                    any(p.requires_grad for p in ps)):
        if env is not None:
            env = env.to(device=coords.device, dtype=torch.int32).contiguous()
        return TaylorFunction.apply(coords, B, env, dim, order, quirk, packed, keys, *ps)
    with torch.no_grad():
        return TaylorFunction.forward(_NoCtx(), coords, B, env, dim, order, quirk, packed, keys,
                                      *ps)


class _NoCtx:
    """Stand-in ctx for a forward that records nothing."""

    def save_for_backward(self, *a):
        pass


class TauWeightFunction(torch.autograd.Function):
    """The weight-gradient half of NN.out: a zero-valued term added to τ whose backward gives
    every trained parameter the gradient of Σ gτ·τ, as the reference's nn.Linear + autograd
    graph does (models/model_res_sigmoid_multi.py:215-259).  Forward computes nothing (τ
    itself comes from TauFunction's fused kernel); backward runs the value-only Taylor tape
    forward and its adjoint on the HIP GEMMs (pntf/train.py tau_weight_grad).  A backward
    that asks only for coords (Model.gradient = autograd.grad(τ, coords)) never reaches this
    node, so the planner / ∇τ path launches nothing for it.  Frozen parameters (requires_grad
    False) are still read by the tape and get no gradient."""

    @staticmethod
    def forward(ctx, coords, B, env, dim, keys, *params):
        ctx.save_for_backward(coords, B, env, *params)
        ctx.dim, ctx.keys = dim, keys
        return torch.zeros((coords.shape[0], 1), dtype=torch.float32, device=coords.device)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        from . import train
        coords, B, env, *params = ctx.saved_tensors
        grads, gp = _param_grads(ctx, ctx.keys, params, 5)
        Btab = B if B.dim() == 3 else B.unsqueeze(0)
        train.tau_weight_grad(dict(zip(ctx.keys, params)), coords, Btab.contiguous(), env,
                              ctx.dim, g.reshape(-1), grads)
        return (None,) * 5 + gp


def weight_term(module, coords, B, env, dim):
    """τ's weight-gradient term for NN.out (TauWeightFunction) when autograd records a graph
    and any parameter requires grad; None otherwise."""
    if not torch.is_grad_enabled():
        return None
    keys, ps = _trained(module)
    if not any(p.requires_grad for p in ps):
        return None
    if env is not None:
        env = env.to(device=coords.device, dtype=torch.int32).contiguous()
    x = coords.detach().to(torch.float32).contiguous()
    return TauWeightFunction.apply(x, B.detach().contiguous(), env, dim, keys, *ps)


def out_tau(module, coords, B, env, dim):
    """NN.out's τ (N, 1) (models/model_res_sigmoid_multi.py:215-259): the fused kernel through
    TauFunction (coords gradient, and ∇τ differentiable under create_graph) plus the
    weight-gradient term."""
    if env is not None:
        env = env.to(device=coords.device, dtype=torch.int32).contiguous()
    keys, ps = _trained(module)
    tau = TauFunction.apply(coords, B, env, module.packed(), dim, keys, *ps)
    wt = weight_term(module, coords, B, env, dim)
    return tau if wt is None else tau + wt


def records_weights(module):
    """True when autograd records a graph and a parameter of `module` requires grad: the
    drop-in Model epilogues (Speed / Tau / TravelTimes / Gradient) then compose their output
    from the differentiable NN.out / out_grad / out_backgrad, as the reference's torch graphs
    do (models/model_res_sigmoid_multi.py:1173-1248), instead of the fused epilogue kernels."""
    return torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters())


def compose_travel_time(tau, Xp, dim):
    """Model.TravelTimes (:1173-1186): sqrt(|x_g - x_s|²) / τ."""
    D = Xp[:, dim:] - Xp[:, :dim]
    return torch.sqrt(torch.einsum("ij,ij->i", D, D)) / tau[:, 0]


def compose_speed(tau, dtau, Xp, dim):
    """Model.Speed (:1195-1216): τ² / sqrt(T0 |∇_g τ|² - 2 τ ∇_g τ·D + τ²)."""
    D = Xp[:, dim:] - Xp[:, :dim]
    T0 = torch.einsum("ij,ij->i", D, D)
    DT1 = dtau[:, dim:]
    T3 = tau[:, 0] ** 2
    S = T0 * torch.einsum("ij,ij->i", DT1, DT1) - 2 * tau[:, 0] * torch.einsum("ij,ij->i", DT1, D) + T3
    return T3 / torch.sqrt(S)


def compose_velocity(tau, dtau, Xp, dim):
    """Model.Gradient (:1218-1248): [v_start | v_goal], each row normalised by its own norm
    (the arm reference's whole-tensor norm only defines a batch of one)."""
    D = Xp[:, dim:] - Xp[:, :dim]
    T0 = torch.sqrt(torch.einsum("ij,ij->i", D, D))
    T3 = tau[:, 0] ** 2
    out = []
    for V0, V1 in ((-D, dtau[:, :dim]), (D, dtau[:, dim:])):
        Y = -(1 / (T0 * tau[:, 0]).unsqueeze(1) * V0 - (T0 / T3).unsqueeze(1) * V1)
        S = torch.norm(Y, p=2, dim=1).unsqueeze(1)
        out.append(1 / S ** 2 * Y)
    return torch.cat(out, dim=1)
