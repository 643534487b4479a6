"""CPU oracle for the P-NTFields τ/∇τ hot path — TEST INFRASTRUCTURE ONLY.

A from-scratch numpy restatement of the reference math (yhsong0804/P-NTFields,
`models/model_res_sigmoid_multi.py`, `models/model_res_sigmoid.py`, `test/gib_plan.py`,
`test/arm_plan.py`).  It is the *checker*: only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it.  The product path (`p-ntfields_amd/`) never
imports it and fails loudly without its HIP library.

Pinning: the restatement is checked against golden vectors produced by importing the
reference itself in the build container (`tests/golden/make_goldens.py` →
`tests/golden/*.npz`; `tests/test_oracle_golden.py`).

Every function computes in `dtype` (float64 by default, float32 for the CPU baseline
timing) on arrays shaped like the reference's:
    xp   (N, 2*dim)    [x_start | x_goal]
    B    (dim, 128) shared, or (n_env, dim, 128) with env (N,) int ids
    params: dict state-dict key -> array (reference key names)
"""
import numpy as np

SCALE = 10.0          # Softplus beta (model_res_sigmoid_multi.py:138-140)
THRESH = 20.0         # torch Softplus default threshold
H = 128

# ------------------------------------------------------------------ elementwise (A1)


def softplus10(y):
    """torch.nn.Softplus(beta=10) (model_res_sigmoid_multi.py:140): linear above beta*y>20."""
    by = SCALE * y
    with np.errstate(over="ignore"):
        soft = np.log1p(np.exp(np.minimum(by, THRESH))) / SCALE
    return np.where(by > THRESH, y, soft)


def sig10(y):
    """sigmoid(10 y) = softplus10' (`sigmoid`, model_res_sigmoid_multi.py:76-78)."""
    return 0.5 * (1.0 + np.tanh(0.5 * SCALE * y))


def sig_out(y):
    """sigmoid(0.1 y) head (`sigmoid_out`, model_res_sigmoid_multi.py:98-100)."""
    return 0.5 * (1.0 + np.tanh(0.05 * y))


def _lin(x, p, name):
    """Linear layer y = x W^T + b (torch.nn.Linear; weights stored (out, in))."""
    return x @ p[name + ".weight"].T + p[name + ".bias"]


def cast_params(params, dtype):
    return {k: np.asarray(v, dtype=dtype) for k, v in params.items()}


def _per_point_W(B, env, n, dtype):
    """W = 2*pi*B per point (input_mapping, model_res_sigmoid_multi.py:186-190)."""
    B = np.asarray(B, dtype=dtype)
    w = (2.0 * np.pi) * B
    if w.ndim == 2:
        return w, False
    assert env is not None, "per-env B table needs env ids"
    return w[np.asarray(env)], True


def _proj(x, w, per_point):
    return np.einsum("nd,ndf->nf", x, w) if per_point else x @ w


# ------------------------------------------------------------------ forward (A5)


def encoder_forward(p, phi):
    """Encoder on points (model_res_sigmoid_multi.py:227-234); returns z and saved pre-acts."""
    y0 = _lin(phi, p, "encoder.0")
    h = softplus10(y0)
    saved = {"e0": y0, "blk": []}
    for i in (1, 2):
        y1 = _lin(h, p, "encoder.%d" % i)
        a = softplus10(y1)
        y2 = _lin(a, p, "encoder1.%d" % i) + h
        h = softplus10(y2)
        saved["blk"].append((y1, y2))
    z = _lin(h, p, "encoder.3")
    return z, saved


def merge(zs, zg):
    """Smooth max/min over the two endpoints (model_res_sigmoid_multi.py:236-244)."""
    d = zs - zg
    c = np.log1p(np.exp(-SCALE * np.abs(d))) / SCALE
    mx = np.maximum(zs, zg) + c
    mn = np.minimum(zs, zg) - c
    return np.concatenate([mx, mn], axis=1), sig10(d)


def generator_forward(p, u):
    """Generator + head (model_res_sigmoid_multi.py:246-255)."""
    saved = {"blk": []}
    for i in (0, 1, 2):
        y1 = _lin(u, p, "generator.%d" % i)
        a = softplus10(y1)
        y2 = _lin(a, p, "generator1.%d" % i) + u
        u = softplus10(y2)
        saved["blk"].append((y1, y2))
    y3 = _lin(u, p, "generator.3")
    v = softplus10(y3)
    y4 = _lin(v, p, "generator.4")
    tau = sig_out(y4)
    saved["g3"] = y3
    return tau, saved


def forward(params, xp, B, env=None, dim=3, dtype=np.float64, keep=False):
    """NN.out (model_res_sigmoid_multi.py:215-259): tau (N,1)."""
    p = cast_params(params, dtype)
    xp = np.asarray(xp, dtype=dtype)
    n = xp.shape[0]
    w, per = _per_point_W(B, env, n, dtype)
    q_s = _proj(xp[:, :dim], w, per)
    q_g = _proj(xp[:, dim:], w, per)
    q = np.concatenate([q_s, q_g])
    phi = np.concatenate([np.sin(q), np.cos(q)], axis=1)
    z, enc = encoder_forward(p, phi)
    u, s0 = merge(z[:n], z[n:])
    tau, gen = generator_forward(p, u)
    if not keep:
        return tau
    return tau, dict(p=p, q=q, w=w, per=per, enc=enc, s0=s0, gen=gen, n=n, dim=dim)


def softplus_saturation(params, xp, B, dim=3):
    """Fraction of all softplus pre-activations (encoder, generator, generator[3]) that take
    torch Softplus's identity branch (10y > 20) — how much of that branch a fixture covers."""
    _, st = forward(params, xp, B, dim=dim, keep=True)
    ys = [st["enc"]["e0"], st["gen"]["g3"]]
    for blk in st["enc"]["blk"] + st["gen"]["blk"]:
        ys += list(blk)
    return sum(float((SCALE * y > THRESH).sum()) for y in ys) / sum(y.size for y in ys)


# ------------------------------------------------------------------ reverse mode (A6/A7)


def tau_grad(params, xp, B, env=None, dim=3, dtype=np.float64, compat=False):
    """tau and d tau / d xp.

    compat=False: exact reverse mode == Model.gradient(NN.out) (model_res_sigmoid_multi.py:890-896).
    compat=True : NN.out_backgrad (model_res_sigmoid_multi.py:402-647) including its encoder[0]
                  quirk, act' evaluated at the *activated* value (:435-438).
    """
    tau, st = forward(params, xp, B, env, dim, dtype, keep=True)
    p, n = st["p"], st["n"]
    # head + G3 (A9 of appendix A)
    d = 0.1 * tau * (1.0 - tau)                                   # dactout, :592-593
    dv = d * p["generator.4.weight"][0][None, :] * sig10(st["gen"]["g3"])
    du = dv @ p["generator.3.weight"]
    for i in (2, 1, 0):                                           # :615-618
        y1, y2 = st["gen"]["blk"][i]
        dr = du * sig10(y2)
        da = (dr @ p["generator1.%d.weight" % i]) * sig10(y1)
        du = da @ p["generator.%d.weight" % i] + dr
    s0 = st["s0"]
    s1 = 1.0 - s0
    dM, dm = du[:, :H], du[:, H:]
    dz = np.concatenate([s0 * dM + s1 * dm, s1 * dM + s0 * dm])   # :620-627
    dh = dz @ p["encoder.3.weight"]
    for i in (2, 1):                                              # :633-636
        y1, y2 = st["enc"]["blk"][i - 1]
        dr = dh * sig10(y2)
        da = (dr @ p["encoder1.%d.weight" % i]) * sig10(y1)
        dh = da @ p["encoder.%d.weight" % i] + dr
    y0 = st["enc"]["e0"]
    act0 = sig10(softplus10(y0)) if compat else sig10(y0)         # quirk :435-438
    dphi = (dh * act0) @ p["encoder.0.weight"]                    # :639
    q = st["q"]
    g = dphi[:, :H] * np.cos(q) - dphi[:, H:] * np.sin(q)         # :419, :640
    w = st["w"]
    if st["per"]:
        ww = np.concatenate([w, w])
        dp = np.einsum("nf,ndf->nd", g, ww)
    else:
        dp = g @ w.T                                              # :641
    dtau = np.concatenate([dp[:n], dp[n:]], axis=1)               # :643-645
    return tau, dtau


def tau_weight_grad(params, xp, B, wt, env=None, dim=3, dtype=np.float64):
    """Gradient of Σ_p wt_p·τ_p w.r.t. every trained parameter and the coordinates — what
    `(net.out(xp, B)[0][:, 0] * wt).sum().backward()` leaves in the reference's `.grad`
    (models/model_res_sigmoid_multi.py:215-259 is plain nn.Linear + autograd).  Returns
    (tau (n,), grads {key: array}, dcoords (n, 2dim)); encoder1.0 (never used, :160, :227)
    gets no entry."""
    tau, st = forward(params, xp, B, env, dim, dtype, keep=True)
    p, n = st["p"], st["n"]
    g = {}

    def acc(name, gy, x):                                          # y = x W^T + b
        g[name + ".weight"] = gy.T @ x
        g[name + ".bias"] = gy.sum(axis=0)
        return gy @ p[name + ".weight"]

    enc, gen = st["enc"], st["gen"]
    q = st["q"]
    phi = np.concatenate([np.sin(q), np.cos(q)], axis=1)
    h_in = [softplus10(enc["e0"]), softplus10(enc["blk"][0][1])]
    h2 = softplus10(enc["blk"][1][1])
    z = _lin(h2, p, "encoder.3")
    u_in = [merge(z[:n], z[n:])[0]] + [softplus10(gen["blk"][i][1]) for i in (0, 1)]
    u3 = softplus10(gen["blk"][2][1])
    v = softplus10(gen["g3"])
    t = tau[:, 0]
    gy4 = (np.asarray(wt, dtype) * 0.1 * t * (1.0 - t))[:, None]   # d sigmoid(0.1 y)/dy
    gv = acc("generator.4", gy4, v)
    gu = acc("generator.3", gv * sig10(gen["g3"]), u3)
    for i in (2, 1, 0):
        y1, y2 = gen["blk"][i]
        gy2 = gu * sig10(y2)
        ga = acc("generator1.%d" % i, gy2, softplus10(y1))
        gu = acc("generator.%d" % i, ga * sig10(y1), u_in[i]) + gy2
    s0 = st["s0"]
    s1 = 1.0 - s0
    gM, gm = gu[:, :H], gu[:, H:]
    gz = np.concatenate([s0 * gM + s1 * gm, s1 * gM + s0 * gm])
    gh = acc("encoder.3", gz, h2)
    for i in (2, 1):
        y1, y2 = enc["blk"][i - 1]
        gy2 = gh * sig10(y2)
        ga = acc("encoder1.%d" % i, gy2, softplus10(y1))
        gh = acc("encoder.%d" % i, ga * sig10(y1), h_in[i - 1]) + gy2
    dphi = acc("encoder.0", gh * sig10(enc["e0"]), phi)
    gq = dphi[:, :H] * np.cos(q) - dphi[:, H:] * np.sin(q)
    w = st["w"]
    dp = np.einsum("nf,ndf->nd", gq, np.concatenate([w, w])) if st["per"] else gq @ w.T
    return t, g, np.concatenate([dp[:n], dp[n:]], axis=1)


# ------------------------------------------------------------------ epilogues (A9/A10)


def path_velocity(xp, tau, dtau, dim=3, row_norm=True):
    """Model.Gradient formula (model_res_sigmoid_multi.py:1223-1248): [v_s | v_g].

    row_norm=False reproduces the arm model's whole-tensor torch.norm
    (models/model_res_sigmoid.py:1268,1278), identical for a batch of one."""
    xp = np.asarray(xp, dtype=dtau.dtype)
    D = xp[:, dim:] - xp[:, :dim]
    T0 = np.sqrt(np.sum(D * D, axis=1))
    t = tau[:, 0]
    T3 = t * t
    out = []
    for sign, dt in ((-1.0, dtau[:, :dim]), (1.0, dtau[:, dim:])):
        Y1 = (1.0 / (T0 * t))[:, None] * (sign * D)
        Y2 = (T0 / T3)[:, None] * dt
        Yp = -(Y1 - Y2)
        S = np.sqrt(np.sum(Yp * Yp, axis=1))[:, None] if row_norm else np.sqrt(np.sum(Yp * Yp))
        out.append(Yp / S ** 2)
    return np.concatenate(out, axis=1)


def speed(xp, tau, dtau, dim=3):
    """Model.Speed (model_res_sigmoid_multi.py:1195-1216), at the goal."""
    xp = np.asarray(xp, dtype=dtau.dtype)
    D = xp[:, dim:] - xp[:, :dim]
    T0 = np.sum(D * D, axis=1)
    DT1 = dtau[:, dim:]
    t = tau[:, 0]
    S = T0 * np.sum(DT1 * DT1, axis=1) - 2 * t * np.sum(DT1 * D, axis=1) + t * t
    return t * t / np.sqrt(S)


def travel_time(xp, tau, dim=3):
    """Model.TravelTimes (model_res_sigmoid_multi.py:1173-1186)."""
    xp = np.asarray(xp, dtype=tau.dtype)
    D = xp[:, dim:] - xp[:, :dim]
    return np.sqrt(np.sum(D * D, axis=1)) / tau[:, 0]


# ------------------------------------------------------------------ Taylor mode (A11)


def _taylor_act(y, J, L):
    """act_laplace (model_res_sigmoid_multi.py:675-691); J, L carry a direction axis 1."""
    s = sig10(y)
    ds = SCALE * s * (1.0 - s)
    return softplus10(y), J * s[:, None], J * J * ds[:, None] + L * s[:, None]


def _taylor_lin(x, J, L, p, name, res=None):
    """linear_laplace (:663-673), optional residual add (:744, :828)."""
    W, b = p[name + ".weight"], p[name + ".bias"]
    y, J2, L2 = x @ W.T + b, J @ W.T, L @ W.T
    if res is not None:
        y, J2, L2 = y + res[0], J2 + res[1], L2 + res[2]
    return y, J2, L2


def laplace(params, xp, B, env=None, dim=3, dtype=np.float64):
    """NN.out_laplace (model_res_sigmoid_multi.py:710-848) on flat pairs.

    Returns tau (N,1), dtau (N,2dim), ltau (N,2dim) (diagonal second derivatives)."""
    p = cast_params(params, dtype)
    xp = np.asarray(xp, dtype=dtype)
    n = xp.shape[0]
    w, per = _per_point_W(B, env, n, dtype)
    ww = np.concatenate([w, w]) if per else w
    x = np.concatenate([xp[:, :dim], xp[:, dim:]])
    q = _proj(x, ww, per)
    sq, cq = np.sin(q), np.cos(q)
    if per:
        wd = ww                                                  # (2n, dim, 128)
    else:
        wd = np.broadcast_to(w[None], (2 * n, dim, H))
    h = np.concatenate([sq, cq], axis=1)                          # input_mapping_laplace :199-213
    J = np.concatenate([wd * cq[:, None], -wd * sq[:, None]], axis=2)
    L = np.concatenate([-wd * wd * sq[:, None], -wd * wd * cq[:, None]], axis=2)
    y, J, L = _taylor_lin(h, J, L, p, "encoder.0")
    h, J, L = _taylor_act(y, J, L)
    for i in (1, 2):
        r = (h, J, L)
        y, J, L = _taylor_lin(h, J, L, p, "encoder.%d" % i)
        h, J, L = _taylor_act(y, J, L)
        y, J, L = _taylor_lin(h, J, L, p, "encoder1.%d" % i, res=r)
        h, J, L = _taylor_act(y, J, L)
    z, J, L = _taylor_lin(h, J, L, p, "encoder.3")
    zs, zg = z[:n], z[n:]
    Js, Jg, Ls, Lg = J[:n], J[n:], L[:n], L[n:]
    u, s0 = merge(zs, zg)                                         # :761-766
    s1 = 1.0 - s0
    c = SCALE * s0 * s1                                           # :790
    S0, S1, C = s0[:, None], s1[:, None], c[:, None]
    Jst = np.concatenate([Js * S0, Js * S1], axis=2)              # start directions :776-786
    Jgo = np.concatenate([Jg * S1, Jg * S0], axis=2)              # goal directions
    Lst = np.concatenate([Js * C * Js + Ls * S0, -Js * C * Js + Ls * S1], axis=2)   # :793-811
    Lgo = np.concatenate([Jg * C * Jg + Lg * S1, -Jg * C * Jg + Lg * S0], axis=2)
    J = np.concatenate([Jst, Jgo], axis=1)                        # (n, 2dim, 256)
    L = np.concatenate([Lst, Lgo], axis=1)
    for i in (0, 1, 2):
        r = (u, J, L)
        y, J, L = _taylor_lin(u, J, L, p, "generator.%d" % i)
        u, J, L = _taylor_act(y, J, L)
        y, J, L = _taylor_lin(u, J, L, p, "generator1.%d" % i, res=r)
        u, J, L = _taylor_act(y, J, L)
    y, J, L = _taylor_lin(u, J, L, p, "generator.3")
    u, J, L = _taylor_act(y, J, L)
    y, J, L = _taylor_lin(u, J, L, p, "generator.4")
    t = sig_out(y)                                                # actout_laplace :693-708
    dt = 0.1 * t * (1.0 - t)
    ddt = 0.1 * dt * (1.0 - 2.0 * t)
    Lo = J * J * ddt[:, None] + L * dt[:, None]
    Jo = J * dt[:, None]
    return t, Jo[:, :, 0], Lo[:, :, 0]


def eikonal_residual(params, xp, yobs, B, env=None, dim=3, gamma=1e-3, dtype=np.float64):
    """Model.Loss per-pair residual (model_res_sigmoid_multi.py:914-946).

    Returns tau, dtau, ltau, diff (N,).  The scalar loss_n adds the B regulariser on the
    caller side (:947)."""
    tau, dtau, ltau = laplace(params, xp, B, env, dim, dtype)
    xp = np.asarray(xp, dtype=dtype)
    yobs = np.asarray(yobs, dtype=dtype)
    D = xp[:, dim:] - xp[:, :dim]
    T0 = np.sum(D * D, axis=1)
    lap0 = ltau[:, :dim].sum(-1)
    lap1 = ltau[:, dim:].sum(-1)
    DT0, DT1 = dtau[:, :dim], dtau[:, dim:]
    t = tau[:, 0]
    T01 = T0 * np.sum(DT0 * DT0, axis=1)
    T02 = -2 * t * np.sum(DT0 * D, axis=1)
    T11 = T0 * np.sum(DT1 * DT1, axis=1)
    T12 = 2 * t * np.sum(DT1 * D, axis=1)
    T3 = t * t
    S0 = T01 - T02 + T3
    S1 = T11 - T12 + T3
    yp0 = 1.0 / (np.sqrt(S0) / T3 + gamma * lap0)
    yp1 = 1.0 / (np.sqrt(S1) / T3 + gamma * lap1)
    y0, y1 = yobs[:, 0], yobs[:, 1]
    diff = yp0 / y0 + y0 / yp0 + yp1 / y1 + y1 / yp1 - 4.0
    return tau, dtau, ltau, diff


def eikonal_residual_arm(params, xp, yobs, B, dim=6, gamma=1e-3, dtype=np.float64):
    """The arm model's residual (models/model_res_sigmoid.py:869-935): square-root speeds
    and viscosity applied to 1/Ypred; B is the (dim, 128) = B_state_dict.T table."""
    tau, dtau, ltau = laplace(params, xp, B, None, dim, dtype)
    xp = np.asarray(xp, dtype=dtype)
    yobs = np.asarray(yobs, dtype=dtype)
    D = xp[:, dim:] - xp[:, :dim]
    T0 = np.sum(D * D, axis=1)
    lap0, lap1 = ltau[:, :dim].sum(-1), ltau[:, dim:].sum(-1)
    DT0, DT1 = dtau[:, :dim], dtau[:, dim:]
    t = tau[:, 0]
    T3 = t * t
    S0 = T0 * np.sum(DT0 * DT0, 1) + 2 * t * np.sum(DT0 * D, 1) + T3
    S1 = T0 * np.sum(DT1 * DT1, 1) - 2 * t * np.sum(DT1 * D, 1) + T3
    yp0 = np.sqrt(1.0 / (1.0 / (T3 / np.sqrt(S0)) + gamma * lap0))
    yp1 = np.sqrt(1.0 / (1.0 / (T3 / np.sqrt(S1)) + gamma * lap1))
    y0, y1 = np.sqrt(yobs[:, 0]), np.sqrt(yobs[:, 1])
    diff = yp0 / y0 + y0 / yp0 + yp1 / y1 + y1 / yp1 - 4
    return tau, dtau, ltau, diff


# ------------------------------------------------------------------ training step (§8f rank 1)
# Reverse mode through the Taylor-mode graph: what `loss.backward()` computes for the weights
# in Model.train (model_res_sigmoid_multi.py:1040-1048; arm models/model_res_sigmoid.py:
# 1062-1071).  Hand-derived adjoints of act_laplace (:675-691), linear_laplace (:663-673),
# the merge (:761-811), actout_laplace (:693-708) and Model.Loss (:897-951).


_BLOCK_HEADS = ("encoder.1", "encoder.2", "generator.0", "generator.1", "generator.2")


def _tact_bwd(y, J, L, gh, gJ, gL):
    """Adjoint of act_laplace: h = sp(y), J' = σJ, L' = σ'J² + σL, σ = σ(10y)."""
    s = sig10(y)
    ds = SCALE * s * (1.0 - s)
    dds = SCALE * ds * (1.0 - 2.0 * s)
    S, DS, DDS = s[:, None], ds[:, None], dds[:, None]
    gy = gh * s + np.sum(gJ * J * DS + gL * (J * J * DDS + L * DS), axis=1)
    return gy, gJ * S + 2.0 * gL * J * DS, gL * S


def _tlin_bwd(x, J, L, W, gy, gJ, gL, grads, name):
    """Adjoint of linear_laplace: the bias enters the value row only."""
    grads[name + ".weight"] = grads.get(name + ".weight", 0) + (
        gy.T @ x + np.einsum("nko,nki->oi", gJ, J) + np.einsum("nko,nki->oi", gL, L))
    grads[name + ".bias"] = grads.get(name + ".bias", 0) + gy.sum(0)
    return gy @ W, gJ @ W, gL @ W


def _loss_bwd(xp, yobs, tau, dtau, ltau, dim, gamma, scale, arm):
    """diff per pair and d(scale·Σdiff)/d(τ, ∇τ, Δτ rows) (Model.Loss :914-946; arm :869-935)."""
    D = xp[:, dim:] - xp[:, :dim]
    T0 = np.sum(D * D, 1)
    t = tau[:, 0]
    gt = np.zeros_like(t)
    gd = np.zeros_like(dtau)
    gl = np.zeros_like(ltau)
    diff = -4.0
    for k, sgn in ((0, 1.0), (1, -1.0)):
        DT = dtau[:, k * dim:(k + 1) * dim]
        lap = ltau[:, k * dim:(k + 1) * dim].sum(1)
        dd = np.sum(DT * D, 1)
        S = T0 * np.sum(DT * DT, 1) + sgn * 2.0 * t * dd + t * t
        rS = np.sqrt(S)
        Q = rS / (t * t) + gamma * lap
        yp = 1.0 / Q
        y = yobs[:, k]
        if arm:
            a, b = np.sqrt(yp), np.sqrt(y)
            diff = diff + a / b + b / a
            dfy = (1.0 / b - b / (a * a)) / (2.0 * a)
        else:
            diff = diff + yp / y + y / yp
            dfy = 1.0 / y - y / (yp * yp)
        gQ = -scale * dfy * yp * yp
        gS = gQ / (2.0 * rS * t * t)
        gt += gQ * (-2.0 * rS / (t * t * t)) + gS * (sgn * 2.0 * dd + 2.0 * t)
        gd[:, k * dim:(k + 1) * dim] = gS[:, None] * (2.0 * T0[:, None] * DT + sgn * 2.0 * t[:, None] * D)
        gl[:, k * dim:(k + 1) * dim] = (gQ * gamma)[:, None]
    return diff, gt, gd, gl


def _tact_q(y, J, L):
    """encoder[0]'s act in NN.out_backgrad (model_res_sigmoid_multi.py:435-438): the
    derivative row is multiplied by σ(10·softplus(y)) instead of σ(10y); first order only."""
    h = softplus10(y)
    return h, J * sig10(h)[:, None], np.zeros_like(L)


def _tact_q_bwd(y, J, L, gh, gJ, gL):
    """Adjoint of _tact_q: d σ(10 sp(y)) / dy = 10 σq (1 - σq) σ(10y)."""
    s = sig10(y)
    sq = sig10(softplus10(y))
    dq = SCALE * sq * (1.0 - sq) * s
    gy = gh * s + np.sum(gJ * J * dq[:, None], axis=1)
    return gy, gJ * sq[:, None], np.zeros_like(gL)


def _taylor_tape(p, xp, B, env, dim, dtype, compat=False):
    """Taylor-mode forward of NN.out_laplace (model_res_sigmoid_multi.py:710-848; arm
    models/model_res_sigmoid.py:676-826) with every Linear input and pre-activation kept for
    the reverse sweep.  compat: encoder[0]'s J row uses the out_backgrad quirk (_tact_q)."""
    n = xp.shape[0]
    w, per = _per_point_W(B, env, n, dtype)
    ww = np.concatenate([w, w]) if per else w
    x = np.concatenate([xp[:, :dim], xp[:, dim:]])
    q = _proj(x, ww, per)
    sq, cq = np.sin(q), np.cos(q)
    wd = ww if per else np.broadcast_to(w[None], (2 * n, dim, H))
    phi = (np.concatenate([sq, cq], 1), np.concatenate([wd * cq[:, None], -wd * sq[:, None]], 2),
           np.concatenate([-wd * wd * sq[:, None], -wd * wd * cq[:, None]], 2))
    tape = []

    def lin(t3, name, res=None):
        out = _taylor_lin(*t3, p, name, res)
        tape.append(("lin", name, t3, res is not None))
        return out

    def act(y3, quirk=False):
        tape.append(("actq" if quirk else "act", y3))
        return _tact_q(*y3) if quirk else _taylor_act(*y3)

    h = act(lin(phi, "encoder.0"), quirk=compat)
    for i in (1, 2):
        a = act(lin(h, "encoder.%d" % i))
        h = act(lin(a, "encoder1.%d" % i, res=h))
    z, Jz, Lz = lin(h, "encoder.3")
    zs, zg, Js, Jg, Ls, Lg = z[:n], z[n:], Jz[:n], Jz[n:], Lz[:n], Lz[n:]
    u, s0 = merge(zs, zg)
    s1 = 1.0 - s0
    c = SCALE * s0 * s1
    S0, S1, C = s0[:, None], s1[:, None], c[:, None]
    J = np.concatenate([np.concatenate([Js * S0, Js * S1], 2),
                        np.concatenate([Jg * S1, Jg * S0], 2)], 1)
    L = np.concatenate([np.concatenate([Js * C * Js + Ls * S0, -Js * C * Js + Ls * S1], 2),
                        np.concatenate([Jg * C * Jg + Lg * S1, -Jg * C * Jg + Lg * S0], 2)], 1)
    u3 = (u, J, L)
    for i in (0, 1, 2):
        a = act(lin(u3, "generator.%d" % i))
        u3 = act(lin(a, "generator1.%d" % i, res=u3))
    v3 = act(lin(u3, "generator.3"))
    y, Jy, Ly = lin(v3, "generator.4")
    return dict(n=n, dim=dim, tape=tape, y=y[:, 0], Jy=Jy[:, :, 0], Ly=Ly[:, :, 0],
                merge=(Js, Jg, Ls, Lg, s0), q=q, wd=wd)


def _taylor_head(st):
    """actout_laplace (:693-708): τ (n,1), ∇τ (n,2dim), diagonal ∇²τ (n,2dim) and the
    derivatives of σ(0.1y) it needs for the adjoint."""
    y, Jy, Ly = st["y"], st["Jy"], st["Ly"]
    t = sig_out(y)
    dt = 0.1 * t * (1.0 - t)
    ddt = 0.1 * dt * (1.0 - 2.0 * t)
    dddt = 0.1 * (ddt * (1.0 - 2.0 * t) - 2.0 * dt * dt)
    return (t[:, None], Jy * dt[:, None], Jy * Jy * ddt[:, None] + Ly * dt[:, None],
            (t, dt, ddt, dddt))


def _taylor_adjoint(st, p, gt, gd, gl, want_x=False):
    """Reverse sweep of the Taylor tape from d/d(τ, ∇τ rows, ∇²τ rows): weight gradients of
    every Linear used and, with want_x, d/dxp through the Fourier features (:199-213)."""
    dim, n = st["dim"], st["n"]
    Jy, Ly = st["Jy"], st["Ly"]
    _, _, _, (t, dt, ddt, dddt) = _taylor_head(st)
    g = (gt * dt + np.sum(gd * Jy * ddt[:, None]
                          + gl * (Jy * Jy * dddt[:, None] + Ly * ddt[:, None]), 1),
         gd * dt[:, None] + 2.0 * gl * Jy * ddt[:, None], gl * dt[:, None])
    g = (g[0][:, None], g[1][:, :, None], g[2][:, :, None])
    Js, Jg, Ls, Lg, s0 = st["merge"]
    s1 = 1.0 - s0
    c = SCALE * s0 * s1
    S0, S1, C = s0[:, None], s1[:, None], c[:, None]
    grads = {}
    res_pending = []
    for op in reversed(st["tape"]):
        if op[0] == "act":
            g = _tact_bwd(*op[1], *g)
            continue
        if op[0] == "actq":
            g = _tact_q_bwd(*op[1], *g)
            continue
        _, name, x3, has_res = op
        gin = _tlin_bwd(*x3, p[name + ".weight"], *g, grads, name)
        if has_res:
            res_pending.append(g)
        if name in _BLOCK_HEADS:                   # the block input also feeds the residual
            gin = tuple(a + b for a, b in zip(gin, res_pending.pop()))
        g = gin
        if name == "generator.0":
            gu, gJ, gL = g
            gM, gm = gu[:, :H], gu[:, H:]
            gJsM, gJsm = gJ[:, :dim, :H], gJ[:, :dim, H:]
            gJgM, gJgm = gJ[:, dim:, :H], gJ[:, dim:, H:]
            gLsM, gLsm = gL[:, :dim, :H], gL[:, :dim, H:]
            gLgM, gLgm = gL[:, dim:, :H], gL[:, dim:, H:]
            g_s0 = np.sum((gJsM - gJsm) * Js - (gJgM - gJgm) * Jg
                          + (gLsM - gLsm) * Ls - (gLgM - gLgm) * Lg, 1)
            g_c = np.sum((gLsM - gLsm) * Js * Js + (gLgM - gLgm) * Jg * Jg, 1)
            k = (g_s0 + g_c * SCALE * (1.0 - 2.0 * s0)) * c
            gzs, gzg = gM * s0 + gm * s1 + k, gM * s1 + gm * s0 - k
            gJs = gJsM * S0 + gJsm * S1 + 2.0 * C * Js * (gLsM - gLsm)
            gJg = gJgM * S1 + gJgm * S0 + 2.0 * C * Jg * (gLgM - gLgm)
            gLs, gLg = gLsM * S0 + gLsm * S1, gLgM * S1 + gLgm * S0
            g = (np.concatenate([gzs, gzg]), np.concatenate([gJs, gJg]),
                 np.concatenate([gLs, gLg]))
    if not want_x:
        return grads, None
    # Fourier adjoint: Φ = [sin q | cos q], J_k = w_k [cos q | -sin q], L_k = -w_k² [sin q | cos q]
    gh, gJ, gL = g
    q, wd = st["q"], st["wd"]
    sq, cq = np.sin(q), np.cos(q)
    G = gh[:, :H] * cq - gh[:, H:] * sq
    G = G - np.sum(wd * (gJ[:, :, :H] * sq[:, None] + gJ[:, :, H:] * cq[:, None]), 1)
    G = G + np.sum(wd * wd * (-gL[:, :, :H] * cq[:, None] + gL[:, :, H:] * sq[:, None]), 1)
    gx = np.einsum("mj,mdj->md", G, wd)
    return grads, np.concatenate([gx[:n], gx[n:]], axis=1)


def taylor_vjp(params, xp, B, env=None, dim=3, g_tau=None, g_dtau=None, g_ltau=None,
               compat=False, want_x=True, dtype=np.float64):
    """Vector-Jacobian product of NN.out_laplace's outputs (models/model_res_sigmoid_multi.py:
    710-848; arm models/model_res_sigmoid.py:676-826), of NN.out_grad's (:303-400) and, with
    compat, of NN.out_backgrad's (:402-647, encoder[0] quirk :435-438; first order only):
    the gradients that `(Σ g_tau·τ + Σ g_dtau·∇τ + Σ g_ltau·∇²τ).backward()` leaves on every
    trained parameter and on the coordinates in the reference's autograd graph.
    g_tau (n,), g_dtau (n, 2dim), g_ltau (n, 2dim) or None (zero).  Returns
    ((τ (n,1), ∇τ (n,2dim), ∇²τ (n,2dim)), grads {key: array}, dcoords (n, 2dim) or None);
    encoder1.0 (never used, :160) gets no entry."""
    p = cast_params(params, dtype)
    xp = np.asarray(xp, dtype=dtype)
    n = xp.shape[0]
    if compat and g_ltau is not None:
        raise ValueError("out_backgrad has no second-derivative output")
    st = _taylor_tape(p, xp, B, env, dim, dtype, compat=compat)
    tau, dtau, ltau, _ = _taylor_head(st)
    z1 = np.zeros(n, dtype)
    z2 = np.zeros((n, 2 * dim), dtype)
    gt = z1 if g_tau is None else np.asarray(g_tau, dtype).reshape(n)
    gd = z2 if g_dtau is None else np.asarray(g_dtau, dtype).reshape(n, 2 * dim)
    gl = z2 if g_ltau is None else np.asarray(g_ltau, dtype).reshape(n, 2 * dim)
    grads, dx = _taylor_adjoint(st, p, gt, gd, gl, want_x)
    return (tau, dtau, ltau), grads, dx


def eikonal_loss_grad(params, xp, yobs, B, env=None, dim=3, gamma=1e-3, scale=1.0, arm=False,
                      dtype=np.float64):
    """Weight gradients of scale·Σ_pairs diff — loss.backward() of Model.Loss with
    scale = beta/(E·n) (multi, :947-948) or beta/N (arm).  The B regulariser of loss_n has no
    weight gradient.  Returns (diff (N,), grads {state-dict key: array}); encoder1.0 gets none
    (created :160 but never used)."""
    p = cast_params(params, dtype)
    xp = np.asarray(xp, dtype=dtype)
    yobs = np.asarray(yobs, dtype=dtype)
    st = _taylor_tape(p, xp, B, env, dim, dtype)
    tau, dtau, ltau, _ = _taylor_head(st)
    diff, gt, gd, gl = _loss_bwd(xp, yobs, tau, dtau, ltau, dim, gamma, scale, arm)
    grads, _ = _taylor_adjoint(st, p, gt, gd, gl)
    return diff, grads


def adamw_step(param, grad, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, wd=0.1):
    """torch.optim.AdamW single-tensor update (the reference's optimizer, :959-961); in place
    on float64 copies; `step` is the 1-based step count after this update."""
    param *= 1.0 - lr * wd
    m += (1.0 - betas[0]) * (grad - m)
    v *= betas[1]
    v += (1.0 - betas[1]) * grad * grad
    bc1 = 1.0 - betas[0] ** step
    bc2 = 1.0 - betas[1] ** step
    param -= (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + eps)
    return param


def loss_n(diff, B_table, n_env, n_per_env):
    """loss_n (model_res_sigmoid_multi.py:947): sum(diff)/E/n + 0.01 ||B||^2 /E/n."""
    B = np.asarray(B_table, dtype=np.float64)
    return float(np.sum(diff) / n_env / n_per_env + 0.01 * np.sum(B * B) / n_env / n_per_env)


# ------------------------------------------------------------------ planners (A12/A13)


def plan(params, xp0, B, env=None, dim=3, step=0.03, tol=0.06, max_iter=500,
         compat=True, row_norm=True, dtype=np.float64):
    """Batched bidirectional planner == Q independent copies of the batch-1 loop.

    Gibson (`test/gib_plan.py:74-86`): step 0.03, tol 0.06, cap 500, out_backgrad (compat).
    Arm   (`test/arm_plan.py:140-152`): step 0.015, tol 0.03, cap 300, autograd (exact).
    A query freezes once |xg - xs| <= tol; the loop body runs at most max_iter+1 times
    (`iter>max_iter` break after the increment).  Returns (path (Q, max_iter+2, 2dim) with
    frozen rows repeated, steps (Q,) int)."""
    xp = np.array(xp0, dtype=dtype)
    q = xp.shape[0]
    cap = max_iter + 1
    path = np.zeros((q, cap + 1, 2 * dim), dtype=dtype)
    path[:, 0] = xp
    steps = np.zeros(q, dtype=np.int32)
    active = np.linalg.norm(xp[:, dim:] - xp[:, :dim], axis=1) > tol
    for it in range(cap):
        if not active.any():
            path[:, it + 1:] = xp[:, None]
            break
        idx = np.nonzero(active)[0]
        e = None if env is None else np.asarray(env)[idx]
        tau, dtau = tau_grad(params, xp[idx], B, e, dim, dtype, compat=compat)
        g = path_velocity(xp[idx], tau, dtau, dim, row_norm=row_norm)
        xp[idx] = xp[idx] + step * g
        steps[idx] += 1
        path[:, it + 1] = xp
        dis = np.linalg.norm(xp[idx, dim:] - xp[idx, :dim], axis=1)
        active[idx[dis <= tol]] = False
    return path, steps
