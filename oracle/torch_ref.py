"""PyTorch-CPU restatement of the reference τ+∇τ call pattern — TEST INFRASTRUCTURE ONLY.

The reference evaluates τ with `NN.out(coords, B)` (models/model_res_sigmoid_multi.py:215-259)
for ONE Fourier matrix B (dim, 128) per call: `input_mapping` is `x @ 2πB` (:186-190), then
torch `nn.Linear` layers, `nn.Softplus(beta=10)` activations, a `logsumexp` start/goal merge
and a `sigmoid(0.1·)` head.  ∇τ comes from `Model.gradient` (:890-896), one
`torch.autograd.grad(τ, coords, create_graph=True)`.  A multi-environment batch is, in the
reference, one such call per environment (each environment has its own `B.npy`,
`models/data_multi.py:17-32`; `test/gib_plan.py:47-48` loads one B and plans with it).

`TorchRef.tau_grad` reproduces exactly that: a batch with a per-pair env id is split into
one `NN.out` + `Model.gradient` call per environment, each with that environment's single
(dim, 128) B (contiguous env blocks are plain slices, otherwise the env's rows are gathered
and the results scattered back).  Same torch CPU kernels (MKL GEMMs, autograd engine), so it
costs what the reference's own CPU path costs.  `bench.py` times it as `cpu_baseline` (kind
"port": the reference itself cannot travel to the GPU box); `tests/test_oracle_golden.py`
pins it to the goldens the reference produced.  Nothing in the product path imports it.

`TorchRef.tau_grad_gather` keeps the per-PAIR form (`B[env]` gathered to (2n, dim, 128) and
contracted with einsum in ONE call).  It is NOT the reference's call pattern — it materialises
2n·dim·128 floats and is ~5× slower on CPU — and is kept only as a labelled cross-check.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

_SOFTPLUS_BETA = 10.0       # nn.Softplus(beta=10), default threshold 20 (:138-140)


def env_groups(env, n_env=None):
    """[(e, rows)] for every env id present, rows = a slice when the env's pairs are one
    contiguous block (the bench's C3 layout), else an index tensor."""
    e = np.asarray(env).astype(np.int64).reshape(-1)
    out = []
    for v in np.unique(e):
        idx = np.flatnonzero(e == v)
        if idx.size and idx[-1] - idx[0] + 1 == idx.size:
            out.append((int(v), slice(int(idx[0]), int(idx[-1]) + 1)))
        else:
            out.append((int(v), torch.from_numpy(idx)))
    return out


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

    def _trunk(self, q, n):
        """Fourier features q (2n, 128) -> τ (n, 1): :226-255."""
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

    def out(self, coords, B):
        """τ (n, 1) — NN.out(coords, B) (:215-259) for ONE B (dim, 128)."""
        n, two_dim = coords.shape
        dim = two_dim // 2
        x = torch.vstack((coords[:, :dim], coords[:, dim:]))                    # :219-224
        q = x @ ((2.0 * math.pi) * torch.as_tensor(B).to(self.dtype))            # :186-190
        return self._trunk(q, n)

    def _one_call(self, xp, B, create_graph):
        """NN.out + Model.gradient (:890-896) for one B; default create_graph=True also
        records the backward graph (part of the reference's cost)."""
        coords = xp.clone().requires_grad_(True)
        tau = self.out(coords, B)
        (dtau,) = torch.autograd.grad(tau, coords, torch.ones_like(tau), retain_graph=True,
                                      create_graph=create_graph)
        return tau.detach()[:, 0], dtau.detach()

    def tau_grad(self, xp, Btab, env=None, create_graph=True):
        """(τ (n,), ∇τ (n, 2*dim)) — the reference's call pattern: one NN.out +
        Model.gradient call per environment with that environment's B."""
        xp = torch.as_tensor(xp).to(self.dtype)
        B = torch.as_tensor(Btab).to(self.dtype)
        if B.dim() == 2:
            return self._one_call(xp, B, create_graph)
        if env is None:
            raise ValueError("a (n_env, dim, 128) B table needs per-pair env ids")
        n = xp.shape[0]
        tau = torch.empty(n, dtype=self.dtype)
        dtau = torch.empty_like(xp)
        for e, rows in env_groups(env):
            t, d = self._one_call(xp[rows], B[e], create_graph)
            tau[rows] = t
            dtau[rows] = d
        return tau, dtau

    def tau_grad_gather(self, xp, Btab, env, create_graph=True):
        """Per-PAIR B gather in one call (NOT the reference's pattern; see module doc)."""
        coords = torch.as_tensor(xp).to(self.dtype).clone().requires_grad_(True)
        n, two_dim = coords.shape
        dim = two_dim // 2
        x = torch.vstack((coords[:, :dim], coords[:, dim:]))
        e = torch.as_tensor(np.asarray(env)).long()
        w = (2.0 * math.pi) * torch.as_tensor(Btab).to(self.dtype)[torch.cat((e, e))]
        tau = self._trunk(torch.einsum("nd,ndf->nf", x, w), n)
        (dtau,) = torch.autograd.grad(tau, coords, torch.ones_like(tau), retain_graph=True,
                                      create_graph=create_graph)
        return tau.detach()[:, 0], dtau.detach()
