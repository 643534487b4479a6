"""Drop-in replacement of yhsong0804/P-NTFields `models/model_res_sigmoid.py` (single-env
model used by the UR5 arm, dim = 6) on the MI355X HIP kernels.

Differences from the multi-env module follow the reference: B (128, dim) lives in the net
as `self.B = B.T` (:139) and is restored by `Model.load` from `B_state_dict` (:1155);
`Model.Gradient` uses the exact autograd ∇τ (:1247-1282).  The reference's whole-tensor
`torch.norm` in `Gradient` (:1268, :1278) only defines a batch of one; for a batch this
module normalises per row, which is the batch-of-one result applied to every query.
"""
import numpy as np
import torch

from pntf import ops
from pntf import train as _train
from pntf.net import PackedCache, TauFunction, build_layers
from pntf.net import init_weights as _init_weights

from .model_res_sigmoid_multi import (DDSigmoid_out, DSigmoid, DSigmoid_out, Sigmoid,  # noqa
                                      Sigmoid_out, sigmoid, sigmoid_out)


class NN(torch.nn.Module):
    """models/model_res_sigmoid.py:128-181 (+ out :212-256)."""

    def __init__(self, device, dim, B):
        super().__init__()
        self.dim = dim
        B = torch.as_tensor(B)
        self.B = B.T.to(device)
        input_size = B.shape[0]
        self.scale = 10
        self.act = torch.nn.Softplus(beta=self.scale)
        self.dact = Sigmoid()
        self.ddact = DSigmoid()
        self.actout = Sigmoid_out()
        self.dactout = DSigmoid_out()
        self.ddactout = DDSigmoid_out()
        build_layers(self, in_features=2 * input_size)
        self._pack = PackedCache()

    def init_weights(self, m):
        _init_weights(m)

    def packed(self):
        return self._pack.get(self)

    def _B(self, device):
        return self.B.to(device=device, dtype=torch.float32)

    def input_mapping(self, x):
        w = 2.0 * np.pi * self.B
        x_proj = x @ w
        return torch.cat([torch.sin(x_proj), torch.cos(x_proj)], dim=-1)

    def out(self, coords):
        coords = coords.clone().detach().requires_grad_(True)
        tau = TauFunction.apply(coords, self._B(coords.device), None, self.packed(), self.dim)
        return tau, coords

    def out_grad(self, coords):
        t, d = ops.tau_grad(self.packed(), coords, self._B(coords.device), None, self.dim,
                            ops.GRAD_EXACT)
        return t.unsqueeze(1), d, coords

    def out_laplace(self, coords):
        """Taylor mode (models/model_res_sigmoid.py:676-826): coords (N, 2dim) ->
        (τ (N,1), ∇τ (N,2dim), diagonal ∇²τ (N,2dim), coords)."""
        out = ops.eikonal_residual(self.packed(), coords, self._B(coords.device), None,
                                   self.dim, want=("tau", "dtau", "ltau"))
        return out["tau"].unsqueeze(1), out["dtau"], out["ltau"], coords

    def forward(self, coords):
        coords = coords.clone().detach().requires_grad_(True)
        return self.out(coords)


class Model:
    """models/model_res_sigmoid.py:829-1329, inference part."""

    def __init__(self, ModelPath, DataPath, dim, device="cpu"):
        self.Params = {"ModelPath": ModelPath, "DataPath": DataPath, "Device": device,
                       "Pytorch Amp (bool)": False,
                       "Network": {"Normlisation": "OffsetMinMax"}}
        self.dim = dim
        self.total_train_loss = []
        self.total_val_loss = []

    def gradient(self, y, x, create_graph=True):
        grad_y = torch.ones_like(y)
        return torch.autograd.grad(y, x, grad_y, only_inputs=True, retain_graph=True,
                                   create_graph=create_graph)[0]

    def Loss(self, points, Yobs, beta, gamma):
        """The arm variant of the residual (models/model_res_sigmoid.py:869-935: square-root
        speeds, viscosity on 1/Ypred).  Training (grad enabled, trainable weights): the HIP
        Taylor-tape adjoint (pntf/train.py), `loss.backward()` fills the weights' .grad.
        Otherwise τ, ∇τ and ∇²τ come from the fused HIP Taylor kernel and the few
        elementwise epilogue ops run as device tensor ops (values only)."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.network.parameters()):
            Bt = self.network._B(points.device).reshape(1, self.dim, -1)
            total, diff = _train.eikonal_loss(self.network, points, Yobs, Bt, None, self.dim,
                                              gamma, 1.0 / points.shape[0], arm=True)
            return beta * total, total, diff
        tau, dtau, ltau, Xp = self.network.out_laplace(points)
        d = self.dim
        D = Xp[:, d:] - Xp[:, :d]
        T0 = (D * D).sum(1)
        lap0, lap1 = ltau[:, :d].sum(-1), ltau[:, d:].sum(-1)
        DT0, DT1 = dtau[:, :d], dtau[:, d:]
        t = tau[:, 0]
        T3 = t * t
        S0 = T0 * (DT0 * DT0).sum(1) + 2 * t * (DT0 * D).sum(1) + T3
        S1 = T0 * (DT1 * DT1).sum(1) - 2 * t * (DT1 * D).sum(1) + T3
        yp0 = torch.sqrt(1 / (torch.sqrt(S0) / T3 + gamma * lap0))
        yp1 = torch.sqrt(1 / (torch.sqrt(S1) / T3 + gamma * lap1))
        y0, y1 = torch.sqrt(Yobs[:, 0]), torch.sqrt(Yobs[:, 1])
        diff = yp0 / y0 + y0 / yp0 + yp1 / y1 + y1 / yp1 - 4
        loss_n = ops.device_sum(diff).float() / Yobs.shape[0]
        return beta * loss_n, loss_n, diff

    def train(self):
        raise NotImplementedError("training is outside the HIP hot path of this round")

    def save(self, epoch="", val_loss=""):
        opt = getattr(self, "optimizer", None)
        torch.save({"epoch": epoch, "model_state_dict": self.network.state_dict(),
                    "optimizer_state_dict": opt.state_dict() if opt is not None else {},
                    "B_state_dict": self.B, "train_loss": self.total_train_loss,
                    "val_loss": self.total_val_loss},
                   "{}/Model_Epoch_{}_ValLoss_{:.6e}.pt".format(
                       self.Params["ModelPath"], str(epoch).zfill(5), val_loss))

    def load(self, filepath):
        """:1150-1162 — weights and B."""
        checkpoint = torch.load(filepath, map_location=torch.device(self.Params["Device"]),
                                weights_only=True)
        self.B = checkpoint["B_state_dict"]
        self.network = NN(self.Params["Device"], self.dim, self.B)
        self.network.load_state_dict(checkpoint["model_state_dict"], strict=True)
        self.network.to(torch.device(self.Params["Device"]))
        self.network.float()
        self.network.eval()

    def _dev(self):
        return torch.device(self.Params["Device"])

    def TravelTimes(self, Xp):
        Xp = Xp.to(self._dev())
        return ops.travel_time(self.network.packed(), Xp, self.network._B(Xp.device), None,
                               self.dim)

    def Tau(self, Xp):
        Xp = Xp.to(self._dev())
        return ops.tau(self.network.packed(), Xp, self.network._B(Xp.device), None,
                       self.dim).unsqueeze(1)

    def Speed(self, Xp):
        Xp = Xp.to(self._dev())
        return ops.speed(self.network.packed(), Xp, self.network._B(Xp.device), None, self.dim)

    def Gradient(self, Xp):
        """Path velocity from the exact ∇τ (autograd in the reference, :1247-1282)."""
        Xp = Xp.to(self._dev())
        v, _ = ops.path_velocity(self.network.packed(), Xp, self.network._B(Xp.device), None,
                                 self.dim, ops.GRAD_EXACT)
        return v

    def Plan(self, XP, step=0.015, tol=0.03, max_iter=300):
        """Batched test/arm_plan.py:140-152 loop on device (exact ∇τ, per-query freeze)."""
        XP = XP.to(self._dev())
        return ops.plan(self.network.packed(), XP, self.network._B(XP.device), None, self.dim,
                        step, tol, max_iter, ops.GRAD_EXACT)
