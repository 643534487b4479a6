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


class TauFunction(torch.autograd.Function):
    """τ = NN.out(coords); d τ / d coords by the fused HIP reverse sweep.

    When coords needs a gradient the forward launches the fused τ+∇τ kernel once and keeps
    ∇τ, so `Model.gradient(tau, coords)` (model_res_sigmoid_multi.py:890-896) costs no second
    launch.  The backward is first-order only (double backward is not on the hot path)."""

    @staticmethod
    def forward(ctx, coords, B, env, packed, dim):
        if ctx.needs_input_grad[0]:
            t, d = ops.tau_grad(packed, coords, B, env, dim, ops.GRAD_EXACT)
            ctx.save_for_backward(d)
        else:
            t = ops.tau(packed, coords, B, env, dim)
        return t.unsqueeze(1)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_tau):
        (d,) = ctx.saved_tensors
        return grad_tau * d, None, None, None, None


class TauWeightFunction(torch.autograd.Function):
    """The weight-gradient half of NN.out: a zero-valued term added to τ whose backward gives
    every trained parameter the gradient of Σ gτ·τ, as the reference's nn.Linear + autograd
    graph does (models/model_res_sigmoid_multi.py:215-259).  Forward computes nothing (τ
    itself comes from TauFunction's fused kernel); backward runs the value-only Taylor tape
    forward and its adjoint on the HIP GEMMs (pntf/train.py tau_weight_grad).  A backward
    that asks only for coords (Model.gradient = autograd.grad(τ, coords)) never reaches this
    node, so the planner / ∇τ path pays nothing for it."""

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
        p = dict(zip(ctx.keys, params))
        grads = {k: torch.empty_like(v) for k, v in p.items()}
        Btab = B if B.dim() == 3 else B.unsqueeze(0)
        train.tau_weight_grad(p, coords, Btab.contiguous(), env, ctx.dim,
                              g.reshape(-1), grads)
        return (None,) * 5 + tuple(grads[k] for k in ctx.keys)


def weight_term(module, coords, B, env, dim):
    """τ's weight-gradient term for NN.out (TauWeightFunction) when autograd records a graph
    and any parameter requires grad; None otherwise."""
    if not torch.is_grad_enabled():
        return None
    from . import train
    sd = module.state_dict(keep_vars=True)
    keys = [k for k in train.trained_keys() if sd[k].requires_grad]
    if not keys:
        return None
    for k in keys:
        ops._require_device(sd[k], k)
        if sd[k].dtype != torch.float32 or not sd[k].is_contiguous():
            raise ops.PntfError("parameter %s must be fp32 contiguous" % k)
    if env is not None:
        env = env.to(device=coords.device, dtype=torch.int32).contiguous()
    x = coords.detach().to(torch.float32).contiguous()
    return TauWeightFunction.apply(x, B.detach().contiguous(), env, dim, keys,
                                   *[sd[k] for k in keys])
