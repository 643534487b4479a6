"""PyTorch-CPU restatement of the reference τ+∇τ op sequence — TEST INFRASTRUCTURE ONLY.

The reference evaluates τ with `NN.out` (models/model_res_sigmoid_multi.py:215-259): torch
`nn.Linear` layers, `nn.Softplus(beta=10)` activations, a `logsumexp` start/goal merge and a
`sigmoid(0.1·)` head, and gets ∇τ from `Model.gradient` (:890-896), i.e. one
`torch.autograd.grad(τ, coords)`.  This module re-expresses that same op sequence with the
same torch CPU kernels (MKL GEMMs, autograd engine), so it costs what the reference's own
CPU path costs.  `bench.py` times it as `cpu_baseline` (kind "port": the reference itself
cannot travel to the GPU box); `tests/test_oracle_golden.py` pins it to the goldens the
reference produced.  Nothing in the product path imports it.
"""
import math

import torch
import torch.nn.functional as F

_SOFTPLUS_BETA = 10.0       # nn.Softplus(beta=10), default threshold 20 (:138-140)


class TorchRef:
    """The reference network's forward + autograd gradient, on CPU torch tensors.

    `params`: state-dict key -> array (SURVEY.md §8a A2 keys); `Btab`: (dim, 128) or
    (n_env, dim, 128); `env`: per-pair env id (n,) or None."""

    def __init__(self, params, dtype=torch.float32):
        self.p = {k: torch.as_tensor(v).to(dtype) for k, v in params.items()}
        self.dtype = dtype

    def _lin(self, x, name):
        return F.linear(x, self.p[name + ".weight"], self.p[name + ".bias"])

    def _act(self, x):
        return F.softplus(x, beta=_SOFTPLUS_BETA)

    def out(self, coords, Btab, env=None):
        """τ (n, 1) — NN.out (:215-259).  coords (n, 2*dim) must require grad."""
        n, two_dim = coords.shape
        dim = two_dim // 2
        x = torch.vstack((coords[:, :dim], coords[:, dim:]))                    # :219-224
        B = torch.as_tensor(Btab).to(self.dtype)
        if B.dim() == 3:                                                          # per-env B
            e = torch.as_tensor(env).long()
            w = (2.0 * math.pi) * B[torch.cat((e, e))]                          # (2n, dim, 128)
            q = torch.einsum("nd,ndf->nf", x, w)
        else:
            q = x @ ((2.0 * math.pi) * B)                                        # :186-190
        h = self._act(self._lin(torch.cat((torch.sin(q), torch.cos(q)), 1), "encoder.0"))
        for i in (1, 2):                                                          # :228-232
            h = self._act(self._lin(self._act(self._lin(h, "encoder.%d" % i)),
                                    "encoder1.%d" % i) + h)
        z = self._lin(h, "encoder.3")                                            # :234
        zs, zg = z[:n], z[n:]
        st = torch.stack((zs, zg), 2)
        zmax = torch.logsumexp(_SOFTPLUS_BETA * st, 2) / _SOFTPLUS_BETA           # :236-244
        zmin = -torch.logsumexp(-_SOFTPLUS_BETA * st, 2) / _SOFTPLUS_BETA
        u = torch.cat((zmax, zmin), 1)
        for i in range(3):                                                        # :246-249
            u = self._act(self._lin(self._act(self._lin(u, "generator.%d" % i)),
                                    "generator1.%d" % i) + u)
        v = self._act(self._lin(u, "generator.3"))                               # :251-252
        return torch.sigmoid(0.1 * self._lin(v, "generator.4"))                  # :254-255

    def tau_grad(self, xp, Btab, env=None, create_graph=True):
        """(τ (n,), ∇τ (n, 2*dim)) — NN.out + Model.gradient (:890-896), whose default
        create_graph=True also records the backward graph (part of the reference's cost)."""
        coords = torch.as_tensor(xp).to(self.dtype).clone().requires_grad_(True)
        tau = self.out(coords, Btab, env)
        (dtau,) = torch.autograd.grad(tau, coords, torch.ones_like(tau), retain_graph=True,
                                      create_graph=create_graph)
        return tau.detach()[:, 0], dtau.detach()
