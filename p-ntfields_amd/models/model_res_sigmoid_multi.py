"""Drop-in replacement of yhsong0804/P-NTFields `models/model_res_sigmoid_multi.py`
(multi-environment Gibson model) whose hot path runs on MI355X HIP kernels.

Scripts bind the reference by module path (`from models import model_res_sigmoid_multi as
md`, test/gib_plan.py:4, train/train_gib_multi.py:3); putting `p-ntfields_amd/` first on
`sys.path` swaps this module in.  Class names, constructor signatures, method names,
return shapes and state-dict keys are the reference's:

    NN(device, dim)                              :131-175
      .out(coords, B) -> (tau (N,1), coords)     :215-259   fused HIP forward (+ ∇τ if needed;
                                                            weight grads by the HIP value tape)
      .out_grad(coords, B) -> (tau, dtau, coords):303-400   exact ∇τ (HIP reverse sweep)
      .out_backgrad(coords, B) -> (...)          :402-647   HIP reverse sweep, quirk kept
      .forward(coords, B)                        :850-854
    Model(ModelPath, DataPath, dim, length, device)          :857-888
      .gradient(y, x)  .Gradient(Xp, B)  .Speed/.Tau/.TravelTimes(Xp)  .load  .save

      .out_laplace(coords, B) -> (tau, dtau, ltau, coords)  :710-848 Taylor mode (HIP)
    Model.Loss(points, Yobs, B, beta, gamma)  :897-951 Eikonal residual (HIP), values only

    Model.train()                              :953-1141 HIP Taylor-tape backward + AdamW

    Model.field_grid() / .plot(...)            :1250-1293 80x80 Speed/Tau/TravelTimes grid

Compute needs HIP device tensors; there is no CPU path (PntfError otherwise).
"""
import numpy as np
import torch

from pntf import ops
from pntf import train as _train
from pntf.net import (PackedCache, build_layers, compose_speed, compose_travel_time,
                      compose_velocity, out_tau, records_weights, taylor_outputs)
from pntf.net import init_weights as _init_weights


# ---------------------------------------------------------------- activations (:76-127)
def sigmoid(input):
    return torch.sigmoid(10 * input)


def sigmoid_out(input):
    return torch.sigmoid(0.1 * input)


class Sigmoid(torch.nn.Module):
    def forward(self, input):
        return sigmoid(input)


class DSigmoid(torch.nn.Module):
    def forward(self, input):
        return 10 * sigmoid(input) * (1 - sigmoid(input))


class Sigmoid_out(torch.nn.Module):
    def forward(self, input):
        return sigmoid_out(input)


class DSigmoid_out(torch.nn.Module):
    def forward(self, input):
        return 0.1 * sigmoid_out(input) * (1 - sigmoid_out(input))


class DDSigmoid_out(torch.nn.Module):
    def forward(self, input):
        s = sigmoid_out(input)
        return 0.01 * s * (1 - s) * (1 - 2 * s)


def _as_table(B, device):
    """Reference B (dim,128) [or a per-env (E,dim,128) table] as a float32 device tensor."""
    if not isinstance(B, torch.Tensor):
        B = torch.as_tensor(np.asarray(B), dtype=torch.float32)
    return B.to(device=device, dtype=torch.float32)


def _env_ids(E, n, device):
    """env id of every flattened (E, n) pair."""
    return torch.arange(E, device=device, dtype=torch.int32).repeat_interleave(n)


class NN(torch.nn.Module):
    """The sigmoid-residual MLP (model_res_sigmoid_multi.py:129-854)."""

    def __init__(self, device, dim):
        super().__init__()
        self.dim = dim
        self.input_size = 128
        self.scale = 10
        self.act = torch.nn.Softplus(beta=self.scale)
        self.dact = Sigmoid()
        self.ddact = DSigmoid()
        self.actout = Sigmoid_out()
        self.dactout = DSigmoid_out()
        self.ddactout = DDSigmoid_out()
        build_layers(self)
        self._pack = PackedCache()

    def init_weights(self, m):
        _init_weights(m)

    def packed(self):
        return self._pack.get(self)

    def input_mapping(self, x, B):
        """Fourier features [sin 2πxB, cos 2πxB] (:186-190); a helper, not on the HIP path."""
        w = 2.0 * np.pi * B
        x_proj = x @ w
        return torch.cat([torch.sin(x_proj), torch.cos(x_proj)], dim=-1)

    def out(self, coords, B, env=None):
        """τ (N,1) and the fresh grad-leaf coords (:215-259).  `env` (N,) int picks rows of a
        per-env B table (E,dim,128); the reference passes a single (dim,128) B.  τ is
        differentiable w.r.t. coords (the fused reverse sweep; ∇τ itself differentiable under
        create_graph) and every weight (the HIP value tape), as the reference's graph is."""
        coords = coords.clone().detach().requires_grad_(True)
        return out_tau(self, coords, _as_table(B, coords.device), env, self.dim), coords

    def out_grad(self, coords, B, env=None):
        """(τ (N,1), ∇τ (N,2dim), coords) — forward-mode Jacobian in the reference (:303-400);
        the same values come from the exact HIP reverse sweep.  Differentiable w.r.t. coords
        and every weight (first-order Taylor tape) when autograd records."""
        t, d = taylor_outputs(self, coords, _as_table(B, coords.device), env, self.dim, 1, False)
        return t.unsqueeze(1), d, coords

    def out_backgrad(self, coords, B, env=None):
        """(τ, dτ, coords) of the reference's manual reverse mode (:402-647), including its
        encoder[0] derivative quirk (:435-438) that test/gib_plan.py plans with; differentiable
        like out_grad (the tape carries the quirk)."""
        t, d = taylor_outputs(self, coords, _as_table(B, coords.device), env, self.dim, 1, True)
        return t.unsqueeze(1), d, coords

    def out_laplace(self, coords, B):
        """Taylor mode (:710-848): coords (E, n, 2dim), B (E, dim, 128) per env ->
        (τ (E,n,1), ∇τ (E,n,2dim), diagonal ∇²τ (E,n,2dim), coords).  Differentiable w.r.t.
        coords and every weight (the HIP Taylor tape with the incoming gradients)."""
        E, n, _ = coords.shape
        t, d, l = taylor_outputs(self, coords.reshape(E * n, -1), _as_table(B, coords.device),
                                 _env_ids(E, n, coords.device), self.dim, 2, False)
        return t.view(E, n, 1), d.view(E, n, -1), l.view(E, n, -1), coords

    def forward(self, coords, B, env=None):
        coords = coords.clone().detach().requires_grad_(True)
        return self.out(coords, B, env)


class Model:
    """Model facade (model_res_sigmoid_multi.py:857-1293), inference part."""

    def __init__(self, ModelPath, DataPath, dim, length, device="cpu"):
        self.Params = {}
        self.Params["ModelPath"] = ModelPath
        self.Params["DataPath"] = DataPath
        self.dim = dim
        self.len = length
        self.Params["Device"] = device
        self.Params["Pytorch Amp (bool)"] = False
        self.Params["Network"] = {"Normlisation": "OffsetMinMax"}
        self.Params["Training"] = {
            "Number of sample points": 2e5, "Batch Size": 2, "Validation Percentage": 10,
            "Number of Epochs": 10000, "Resampling Bounds": [0.1, 0.9],
            "Print Every * Epoch": 1, "Save Every * Epoch": 100, "Learning Rate": 1e-3,
            "Random Distance Sampling": True, "Use Scheduler (bool)": False}
        self.total_train_loss = []
        self.total_val_loss = []

    def gradient(self, y, x, create_graph=True):
        """autograd ∇ (:890-896); through TauFunction it returns the HIP reverse sweep."""
        grad_y = torch.ones_like(y)
        return torch.autograd.grad(y, x, grad_y, only_inputs=True, retain_graph=True,
                                   create_graph=create_graph)[0]

    def Loss(self, points, Yobs, B, beta, gamma):
        """Eikonal residual loss (:897-951): points (E,n,2dim), Yobs (E,n,2), B (E,dim,128).
        Returns (loss, loss_n, diff (E,n)).  With grad enabled and trainable weights (the
        training step, :1040-1048) `loss.backward()` fills the weights' .grad through the HIP
        Taylor-tape adjoint (pntf/train.py); otherwise the fused residual kernel evaluates
        the values only."""
        E, n, _ = points.shape
        dev = points.device
        Bt = _as_table(B, dev)
        reg = 0.01 * ops.device_sum(Bt * Bt).float() / E / n
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.network.parameters()):
            total, diff = _train.eikonal_loss(self.network, points.reshape(E * n, -1),
                                              Yobs.reshape(E * n, 2), Bt,
                                              _env_ids(E, n, dev), self.dim, gamma,
                                              1.0 / (E * n))
            loss_n = total + reg
            return beta * loss_n, loss_n, diff.view(E, n)
        out = ops.eikonal_residual(self.network.packed(), points.reshape(E * n, -1), Bt,
                                  _env_ids(E, n, dev), self.dim,
                                  yobs=Yobs.reshape(E * n, 2), gamma=gamma, want=("diff",))
        diff = out["diff"].view(E, n)
        loss_n = (ops.device_sum(diff) / E / n).float() + reg
        return beta * loss_n, loss_n, diff

    def train(self):
        """Model.train (:953-1141): AdamW(lr 1e-3, wd 0.1) over the environment dataset
        (data_multi.Database, 2 environments per batch), the progressive speed blend α, the
        per-epoch lr clip, up to 6 inner steps of `inner_batch` (10000) shuffled pairs per
        environment batch, and the rollback to one of the last 5 (network, optimizer) states
        when the epoch's mean residual grows by 1.2x or more.  Every inner step is
        Loss → loss.backward() → optimizer.step() on the HIP Taylor tape (pntf/train.py).
        At save time it writes the same plots (`plot`, HIP field grid) and checkpoint."""
        import copy
        import random
        import time

        from . import data_multi as db
        P = self.Params
        dev = torch.device(P["Device"])
        ops._require_device(torch.empty(0, device=dev), "Model.train device")   # no CPU path
        self.network = NN(P["Device"], self.dim)
        self.network.apply(self.network.init_weights)
        self.network.to(dev)
        self.optimizer = _train.AdamW(self.network.parameters(),
                                      lr=P["Training"]["Learning Rate"], weight_decay=0.1)
        if P["Training"]["Use Scheduler (bool)"]:
            self.scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer)
        self.dataset = db.Database(P["DataPath"], dev, self.len)
        dataloader = torch.utils.data.DataLoader(
            self.dataset, batch_size=int(P["Training"]["Batch Size"]), num_workers=1,
            shuffle=True)
        beta, prev_diff, current_diff = 1.0, 1.0, 1.0
        step = -2000.0 / 4000.0
        current_state = copy.deepcopy(self.network.state_dict())
        current_optimizer = copy.deepcopy(self.optimizer.state_dict())
        prev_state_queue, prev_optimizer_queue = [], []
        inner_batch = int(P["Training"].get("Inner Batch", 10000))
        inner_rows = self.dataset[0][0].shape[0]
        inner_size = max(1, int(inner_rows / inner_batch))
        for epoch in range(1, P["Training"]["Number of Epochs"] + 1):
            alpha = min(max(0.5, 0.5 + 0.5 * step), 1.07)
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
                for data, B, _ in dataloader:
                    data = data.to(dev)
                    B = B.to(dev)
                    points = data[:, :, :2 * self.dim]
                    speed = alpha * data[:, :, 2 * self.dim:] + 1 - alpha
                    idx0 = torch.randperm(inner_rows, device=dev)
                    idx1 = torch.randperm(inner_rows, device=dev)
                    E = points.shape[0]
                    idx = [idx0, idx1] + [torch.randperm(inner_rows, device=dev)
                                          for _ in range(E - 2)]
                    points_sh = torch.stack([points[e, idx[e]] for e in range(E)])
                    speed_sh = torch.stack([speed[e, idx[e]] for e in range(E)])
                    for ii in range(inner_size):
                        if ii > 5:
                            break
                        sl = slice(ii * inner_batch, (ii + 1) * inner_batch)
                        bp, bs = points_sh[:, sl].contiguous(), speed_sh[:, sl].contiguous()
                        self.B = B[0, :]
                        loss_value, loss_n, _ = self.Loss(bp, bs, B, beta, gamma)
                        loss_value.backward()
                        self.optimizer.step()
                        self.optimizer.zero_grad()
                        total_train_loss += loss_value.detach()
                        total_diff += loss_n.detach()
                total_train_loss /= len(dataloader) * 5.0
                total_diff /= len(dataloader) * 5.0
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
        """Same checkpoint dict as the reference (:1143-1152)."""
        opt = getattr(self, "optimizer", None)
        torch.save({"epoch": epoch, "model_state_dict": self.network.state_dict(),
                    "optimizer_state_dict": opt.state_dict() if opt is not None else {},
                    "B_state_dict": getattr(self, "B", None),
                    "train_loss": self.total_train_loss, "val_loss": self.total_val_loss},
                   "{}/Model_Epoch_{}_ValLoss_{:.6e}.pt".format(
                       self.Params["ModelPath"], str(epoch).zfill(5), val_loss))

    def load(self, filepath):
        """Weights only, like the reference (:1154-1166; B is not restored, :1159)."""
        checkpoint = torch.load(filepath, map_location=torch.device(self.Params["Device"]),
                                weights_only=True)
        self.network = NN(self.Params["Device"], self.dim)
        self.network.load_state_dict(checkpoint["model_state_dict"], strict=True)
        self.network.to(torch.device(self.Params["Device"]))
        self.network.float()
        self.network.eval()

    def _dev(self):
        return torch.device(self.Params["Device"])

    # The epilogues run as fused kernels; when autograd records and the weights require grad
    # they are composed from the differentiable NN.out / out_grad / out_backgrad instead, so a
    # loss on them trains the weights as the reference's torch graphs do.
    def TravelTimes(self, Xp):
        """|x_g - x_s| / τ (:1173-1186), uses self.B."""
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            return compose_travel_time(self.network.out(Xp, self.B)[0], Xp, self.dim)
        return ops.travel_time(self.network.packed(), Xp, _as_table(self.B, Xp.device), None,
                               self.dim)

    def Tau(self, Xp):
        """τ (N,1) (:1188-1193), uses self.B."""
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            return self.network.out(Xp, self.B)[0]
        return ops.tau(self.network.packed(), Xp, _as_table(self.B, Xp.device), None,
                       self.dim).unsqueeze(1)

    def Speed(self, Xp):
        """Speed at the goal (:1195-1216), uses self.B."""
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            tau, dtau, _ = self.network.out_grad(Xp, self.B)
            return compose_speed(tau, dtau, Xp, self.dim)
        return ops.speed(self.network.packed(), Xp, _as_table(self.B, Xp.device), None,
                         self.dim)

    def Gradient(self, Xp, B, env=None):
        """Path velocity [v_s | v_g] (:1218-1248) from the out_backgrad sweep (quirk kept),
        per-row norms."""
        Xp = Xp.to(self._dev())
        if records_weights(self.network):
            tau, dtau, _ = self.network.out_backgrad(Xp, B, env)
            return compose_velocity(tau, dtau, Xp, self.dim)
        v, _ = ops.path_velocity(self.network.packed(), Xp, _as_table(B, Xp.device), env,
                                 self.dim, ops.GRAD_BACKGRAD_COMPAT)
        return v

    def Plan(self, XP, B, step=0.03, tol=0.06, max_iter=500, env=None,
             mode=ops.GRAD_BACKGRAD_COMPAT):
        """Batched test/gib_plan.py:74-86 loop on device: Q independent queries, each frozen
        once |x_g - x_s| <= tol.  Returns (path (Q, max_iter+2, 2dim), steps (Q,))."""
        XP = XP.to(self._dev())
        return ops.plan(self.network.packed(), XP, _as_table(B, XP.device), env, self.dim,
                        step, tol, max_iter, mode)

    def field_grid(self, limit=0.5):
        """The 80x80 evaluation grid of Model.plot (:1250-1275): start fixed at
        (-0.25, -0.25, 0, ...), goal swept over [-limit, limit)^2 in the first two axes;
        TravelTimes, Speed and Tau on the HIP kernels.  Returns numpy (X, Y, TT, V, TAU)."""
        spacing = limit / 40.0
        X, Y = np.meshgrid(np.arange(-limit, limit, spacing), np.arange(-limit, limit, spacing))
        XP = np.zeros((X.size, 2 * self.dim), np.float32)
        XP[:, 0] = -0.25
        XP[:, 1] = -0.25
        XP[:, self.dim + 0] = X.ravel()
        XP[:, self.dim + 1] = Y.ravel()
        XP = torch.from_numpy(XP).to(self._dev())
        with torch.no_grad():          # plotting values: nothing to differentiate
            tt = self.TravelTimes(XP)
            ss = self.Speed(XP)
            tau = self.Tau(XP)
            return (X, Y, tt.cpu().numpy().reshape(X.shape), ss.cpu().numpy().reshape(X.shape),
                    tau.cpu().numpy().reshape(X.shape))

    def plot(self, epoch, total_train_loss, alpha):
        """Model.plot (:1250-1293): speed and τ maps with travel-time contours, saved as
        <ModelPath>/plots<epoch>_<alpha>_<loss>_0.jpg and tauplots...; the field values come
        from field_grid (HIP)."""
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
