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
from pntf.net import (PackedCache, build_layers, compose_speed, compose_travel_time,
                      compose_velocity, out_tau, records_weights, taylor_outputs)
from pntf.net import init_weights as _init_weights

from .model_res_sigmoid_multi import (DDSigmoid_out, DSigmoid, DSigmoid_out, Sigmoid,  # noqa
                                      Sigmoid_out, sigmoid, sigmoid_out)


class FastTensorDataLoader:
    """models/model_res_sigmoid.py:30-73: batches of rows of same-length tensors, reshuffled
    (torch.randperm on the tensors' device) every time an iterator is created."""

    def __init__(self, *tensors, batch_size=32, shuffle=False):
        assert all(t.shape[0] == tensors[0].shape[0] for t in tensors)
        self.tensors = tensors
        self.dataset_len = self.tensors[0].shape[0]
        self.batch_size = batch_size
        self.shuffle = shuffle
        n_batches, remainder = divmod(self.dataset_len, self.batch_size)
        self.n_batches = n_batches + (1 if remainder > 0 else 0)

    def __iter__(self):
        if self.shuffle:
            r = torch.randperm(self.dataset_len, device=self.tensors[0].device)
            self.tensors = [t[r] for t in self.tensors]
        self.i = 0
        return self

    def __next__(self):
        if self.i >= self.dataset_len:
            raise StopIteration
        batch = tuple(t[self.i:self.i + self.batch_size] for t in self.tensors)
        self.i += self.batch_size
        return batch

    def __len__(self):
        return self.n_batches


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
        return out_tau(self, coords, self._B(coords.device), None, self.dim), coords

    def out_grad(self, coords):
        """(τ (N,1), ∇τ (N,2dim), coords) (:513-613); differentiable w.r.t. coords and every
        weight when autograd records."""
        t, d = taylor_outputs(self, coords, self._B(coords.device), None, self.dim, 1, False)
        return t.unsqueeze(1), d, coords

    def out_backgrad(self, coords):
        """:300-511.  Unlike the multi model's, the arm's out_backgrad carries the exact
        forward-mode ∇τ (its derivative rows use σ(10y) at every layer, :330-333); the shape
        probes it prints (:502-507) are not repeated."""
        t, d = taylor_outputs(self, coords, self._B(coords.device), None, self.dim, 1, False)
        return t.unsqueeze(1), d, coords

    def out_laplace(self, coords):
        """Taylor mode (models/model_res_sigmoid.py:676-826): coords (N, 2dim) ->
        (τ (N,1), ∇τ (N,2dim), diagonal ∇²τ (N,2dim), coords), coords a fresh grad leaf (:678)
        that receives the gradient of a loss on the outputs (as do the weights)."""
        coords = coords.clone().detach().requires_grad_(True)
        t, d, l = taylor_outputs(self, coords, self._B(coords.device), None, self.dim, 2, False)
        return t.unsqueeze(1), d, l, coords

    def forward(self, coords):
        coords = coords.clone().detach().requires_grad_(True)
        return self.out(coords)


class Model:
    """models/model_res_sigmoid.py:829-1329."""

    def __init__(self, ModelPath, DataPath, dim, device="cpu"):
        self.Params = {"ModelPath": ModelPath, "DataPath": DataPath, "Device": device,
                       "Pytorch Amp (bool)": False,
                       "Network": {"Normlisation": "OffsetMinMax"}}
        self.Params["Training"] = {
            "Number of sample points": 2e5, "Batch Size": 10000, "Validation Percentage": 10,
            "Number of Epochs": 10000, "Resampling Bounds": [0.1, 0.9],
            "Print Every * Epoch": 1, "Save Every * Epoch": 100, "Learning Rate": 1e-3,
            "Random Distance Sampling": True, "Use Scheduler (bool)": False}
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
        """Model.train (models/model_res_sigmoid.py:938-1137) over the data_mlp dataset:
        B = 0.5·N(0,1) of shape (128, dim) (:942), AdamW(lr 1e-3, wd 0.1), the progressive
        speed blend α, the per-epoch lr clip, up to 6 shuffled batches of `Batch Size` rows
        per epoch (FastTensorDataLoader), the epoch mean divided by len(dataloader) as the
        reference does, and the rollback to one of the last 5 (network, optimizer) states
        when the epoch's mean residual grows by 1.2x or more.  Every inner step is
        Loss → loss.backward() → optimizer.step() on the HIP Taylor tape (pntf/train.py);
        the dataset is moved to the device once.  Plots and checkpoints as the reference."""
        import copy
        import random
        import time

        from . import data_mlp as db
        P = self.Params
        dev = torch.device(P["Device"])
        ops._require_device(torch.empty(0, device=dev), "Model.train device")   # no CPU path
        self.B = 0.5 * torch.normal(0, 1, size=(128, self.dim))
        self.network = NN(P["Device"], self.dim, self.B)
        self.network.apply(self.network.init_weights)
        self.network.to(dev)
        self.optimizer = _train.AdamW(self.network.parameters(),
                                      lr=P["Training"]["Learning Rate"], weight_decay=0.1)
        if P["Training"]["Use Scheduler (bool)"]:
            self.scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer)
        self.dataset = db.Database(P["DataPath"])
        self.dataset.send_device(dev)
        dataloader = FastTensorDataLoader(self.dataset.data,
                                          batch_size=int(P["Training"]["Batch Size"]),
                                          shuffle=True)
        beta, prev_diff, current_diff = 1.0, 1.0, 1.0
        step = -2000.0 / 4000.0
        current_state = copy.deepcopy(self.network.state_dict())
        current_optimizer = copy.deepcopy(self.optimizer.state_dict())
        prev_state_queue, prev_optimizer_queue = [], []
        for epoch in range(1, P["Training"]["Number of Epochs"] + 1):
            alpha = min(max(0.5, 0.5 + 0.5 * step), 1.05)
            step += 1.0 / 4000 / (int(epoch / 4000) + 1.0)
            gamma = 0.001
            prev_state_queue.append(current_state)
            prev_optimizer_queue.append(current_optimizer)
            if len(prev_state_queue) > 5:
                prev_state_queue.pop(0)
                prev_optimizer_queue.pop(0)
            current_state = copy.deepcopy(self.network.state_dict())
            current_optimizer = copy.deepcopy(self.optimizer.state_dict())
            self.optimizer.param_groups[0]["lr"] = float(
                np.clip(1e-3 * (1 - (epoch - 8000) / 1000.0), a_min=5e-4, a_max=1e-3))
            prev_diff = current_diff
            t0 = time.time()
            while True:
                total_train_loss = 0
                total_diff = 0
                for i, data in enumerate(dataloader, 0):
                    if i > 5:
                        break
                    data = data[0]
                    points = data[:, :2 * self.dim].contiguous()
                    speed = (alpha * data[:, 2 * self.dim:] + 1 - alpha).contiguous()
                    loss_value, loss_n, _ = self.Loss(points, speed, beta, gamma)
                    loss_value.backward()
                    self.optimizer.step()
                    self.optimizer.zero_grad()
                    total_train_loss += loss_value.detach()
                    total_diff += loss_n.detach()
                total_train_loss /= len(dataloader)
                total_diff /= len(dataloader)
                current_diff = total_diff
                diff_ratio = current_diff / prev_diff
                if 0 < diff_ratio < 1.2:
                    break
                with torch.no_grad():
                    r = random.randint(0, len(prev_state_queue) - 1)
                    self.network.load_state_dict(prev_state_queue[r], strict=True)
                    self.optimizer.load_state_dict(prev_optimizer_queue[r])
                print("RepeatEpoch = {} -- Loss = {:.4e} -- Alpha = {:.4e}".format(
                    epoch, float(total_diff), alpha))
            self.total_train_loss.append(total_train_loss)
            beta = 1.0 / float(total_diff)
            if P["Training"]["Use Scheduler (bool)"]:
                self.scheduler.step(total_train_loss)
            if epoch % P["Training"]["Print Every * Epoch"] == 0:
                print("Epoch = {} -- Loss = {:.4e} -- Alpha = {:.4e} -- {:.3f} s".format(
                    epoch, float(total_diff), alpha, time.time() - t0))
            if (epoch % P["Training"]["Save Every * Epoch"] == 0 or
                    epoch == P["Training"]["Number of Epochs"] or epoch == 1):
                with torch.no_grad():
                    if P["Training"].get("Plot (bool)", True):
                        self.plot(epoch, float(total_diff), alpha)
                    self.save(epoch=epoch, val_loss=float(total_diff))

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

    # fused kernels, or (autograd recording, trainable weights) composed from the
    # differentiable NN.out / out_grad as the reference's torch graphs
    def TravelTimes(self, Xp):
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            return compose_travel_time(self.network.out(Xp)[0], Xp, self.dim)
        return ops.travel_time(self.network.packed(), Xp, self.network._B(Xp.device), None,
                               self.dim)

    def Tau(self, Xp):
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            return self.network.out(Xp)[0]
        return ops.tau(self.network.packed(), Xp, self.network._B(Xp.device), None,
                       self.dim).unsqueeze(1)

    def Speed(self, Xp):
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            tau, dtau, _ = self.network.out_grad(Xp)
            return compose_speed(tau, dtau, Xp, self.dim)
        return ops.speed(self.network.packed(), Xp, self.network._B(Xp.device), None, self.dim)

    def Speed2(self, Xp, gamma):
        """Speed at the goal with the viscosity term (:1218-1245): 1 / (sqrt(S)/τ² + γ Δ_gτ)
        from out_laplace's τ, ∇τ and the goal's Laplacian Σ_d ∂²τ/∂x_goal_d²."""
        Xp = Xp.to(self._dev())
        tau, dtau, ltau, _ = self.network.out_laplace(Xp)
        d = self.dim
        lap1 = ltau[:, d:].sum(-1)
        D = Xp[:, d:] - Xp[:, :d]
        T0 = (D * D).sum(1)
        DT1 = dtau[:, d:]
        t = tau[:, 0]
        S = T0 * (DT1 * DT1).sum(1) - 2 * t * (DT1 * D).sum(1) + t * t
        return 1 / (torch.sqrt(S) / (t * t) + gamma * lap1)

    def Gradient(self, Xp):
        """Path velocity from the exact ∇τ (autograd in the reference, :1247-1282)."""
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            tau, dtau, _ = self.network.out_grad(Xp)
            return compose_velocity(tau, dtau, Xp, self.dim)
        v, _ = ops.path_velocity(self.network.packed(), Xp, self.network._B(Xp.device), None,
                                 self.dim, ops.GRAD_EXACT)
        return v

    def Plan(self, XP, step=0.015, tol=0.03, max_iter=300):
        """Batched test/arm_plan.py:140-152 loop on device (exact ∇τ, per-query freeze)."""
        XP = XP.to(self._dev())
        return ops.plan(self.network.packed(), XP, self.network._B(XP.device), None, self.dim,
                        step, tol, max_iter, ops.GRAD_EXACT)

    def field_grid(self, limit=2.0):
        """The 80x80 evaluation grid of Model.plot (:1284-1311): start fixed at the reference's
        joint configuration Xsrc/(π/0.5), goal swept over [-limit, limit)^2 in the first two
        joints (after the scaling); TravelTimes, Speed and Tau on the HIP kernels.  Returns
        numpy (X, Y, TT, V, TAU)."""
        spacing = limit / 40.0
        X, Y = np.meshgrid(np.arange(-limit, limit, spacing), np.arange(-limit, limit, spacing))
        Xsrc = [-1.3, 0.4 - 0.5 * np.pi, 1.1, 0.5 - 0.5 * np.pi, -0.5, 0.7]
        XP = np.zeros((X.size, 2 * self.dim))
        XP[:, :self.dim] = Xsrc
        XP[:, self.dim:] = Xsrc
        XP = XP / (np.pi / 0.5)
        XP[:, self.dim + 0] = X.ravel()
        XP[:, self.dim + 1] = Y.ravel()
        XP = torch.from_numpy(XP.astype(np.float32)).to(self._dev())
        with torch.no_grad():          # plotting values: nothing to differentiate
            tt = self.TravelTimes(XP)
            ss = self.Speed(XP)
            tau = self.Tau(XP)
            return (X, Y, tt.cpu().numpy().reshape(X.shape), ss.cpu().numpy().reshape(X.shape),
                    tau.cpu().numpy().reshape(X.shape))

    def plot(self, epoch, total_train_loss, alpha):
        """Model.plot (:1284-1329): speed and τ maps with travel-time contours, saved as
        <ModelPath>/plots<epoch>_<alpha>_<loss>_0.jpg and tauplots...; values from field_grid."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        X, Y, TT, V, TAU = self.field_grid()
        tag = str(epoch) + "_" + str(alpha) + "_" + str(round(total_train_loss, 4)) + "_0.jpg"
        for prefix, field in (("/plots", V), ("/tauplots", TAU)):
            fig = plt.figure()
            ax = fig.add_subplot(111)
            quad = ax.pcolormesh(X, Y, field, vmin=0, vmax=1)
            ax.contour(X, Y, TT, np.arange(0, 3, 0.05), cmap="bone", linewidths=0.5)
            plt.colorbar(quad, ax=ax, pad=0.1, label="Predicted Velocity")
            plt.savefig(self.Params["ModelPath"] + prefix + tag, bbox_inches="tight")
            plt.close(fig)
