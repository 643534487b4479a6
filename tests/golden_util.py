"""Shared helpers for the parity tests: golden fixtures, seeded weights, comparisons."""
import os

import numpy as np

from pntf import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def weights():
    return synth.make_weights(0)


def weight_checksum(w):
    return np.array([float(np.sum(np.abs(v.astype(np.float64)))) for v in w.values()])


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def max_rel(a, b, floor):
    """max |a-b| / max(|b|, floor) elementwise."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


# ---- compact digests of full weight gradients (tests/golden/make_out_grad_goldens.py
# --stage vjp): a 540 K-float gradient per case would be ~2 MB; instead the fixture holds the
# bias / head gradients whole and, per weight matrix, DIGEST_ROWS seeded rows plus a sketch of
# the whole matrix (DIGEST_SKETCH unit-norm Gaussian projections, |P·(g - g_ref)| <= ||g - g_ref||)
DIGEST_ROWS = 6
DIGEST_SKETCH = 16


def _digest_rng(key):
    import zlib
    return np.random.Generator(np.random.PCG64(zlib.crc32(key.encode())))


def digest_rows(key, shape):
    """The seeded row subset of a (out, in) weight gradient."""
    return np.sort(_digest_rng(key).choice(shape[0], size=min(DIGEST_ROWS, shape[0]),
                                           replace=False))


def digest_proj(key, size):
    rng = _digest_rng(key + "/sketch")
    P = rng.standard_normal((DIGEST_SKETCH, size))
    return P / np.linalg.norm(P, axis=1, keepdims=True)


def grad_digest(key, g):
    """{'rows', 'rowsel', 'sketch'} of a weight gradient, or {'full'} of a small tensor."""
    g = np.asarray(g, np.float64)
    if g.ndim < 2 or g.shape[0] == 1:
        return {"full": g.astype(np.float32)}
    idx = digest_rows(key, g.shape)
    return {"rowsel": idx.astype(np.int32), "rows": g[idx].astype(np.float32),
            "sketch": digest_proj(key, g.size) @ g.ravel(), "norm": np.linalg.norm(g)}


def digest_error(key, g, ref):
    """(elementwise max|Δ| / max|ref| over the stored rows or the full tensor, sketch
    max|Δ| / ||ref||_2 — an estimate of the relative L2 error of the whole matrix) of a
    gradient against its fixture digest `ref` (dict of arrays)."""
    g = np.asarray(g, np.float64)
    if "full" in ref:
        r = np.asarray(ref["full"], np.float64)
        return float(np.abs(g - r).max() / max(np.abs(r).max(), 1e-30)), 0.0
    rows = np.asarray(ref["rows"], np.float64)
    e_rows = float(np.abs(g[np.asarray(ref["rowsel"])] - rows).max() /
                   max(np.abs(rows).max(), 1e-30))
    sk = digest_proj(key, g.size) @ g.ravel()
    e_sk = float(np.abs(sk - np.asarray(ref["sketch"])).max() / max(float(ref["norm"]), 1e-30))
    return e_rows, e_sk


# ---- the north star per pair: every pair of every τ / ∇τ / Δτ golden
# comparison within 1e-4 relative of the reference's fp32 value, or — where that fp32 value
# is itself farther than 1e-4 from exact — within 1e-4 of the fp64 oracle on the same inputs.
NORTH_STAR = 1e-4
_F64 = {}


def golden_weights(name):
    """Weights a golden file was recorded at: the W2 checkpoints for *_w2_*, else the seeded
    init weights."""
    if "_w2_" not in name:
        return weights()
    import torch
    dim = 6 if name.endswith("d6.npz") else 3
    sd = torch.load(os.path.join(GOLDEN, "ckpt_w2_d%d.pt" % dim), map_location="cpu",
                    weights_only=True)["model_state_dict"]
    return {k: v.numpy().astype(np.float32) for k, v in sd.items()}


def fp64_of(name):
    """fp64 oracle outputs on a golden file's own inputs, under the golden's keys (cached)."""
    if name in _F64:
        return _F64[name]
    from oracle import pntf_oracle as O
    f = load(name)
    W = golden_weights(name)
    out = {}
    if name.startswith("fwd_grad"):
        dim = f["xp"].shape[1] // 2
        if "B_table" in f.files:
            B, env = f["B_table"], f["env"]
        else:
            B, env = (f["B"] if dim == 3 else f["B"].T), None
        t, d = O.tau_grad(W, f["xp"], B, env, dim=dim)
        out.update(tau=t, dtau=d, dtau_fwdmode=d, speed=O.speed(f["xp"], t, d, dim),
                   travel_time=O.travel_time(f["xp"], t, dim))
        if dim == 3:
            tc, dc = O.tau_grad(W, f["xp"], B, env, dim=dim, compat=True)
            out.update(tau_backgrad=tc, dtau_backgrad=dc,
                       gradient=O.path_velocity(f["xp"], tc, dc, dim))
        else:
            out["gradient16"] = O.path_velocity(f["xp"][:16], t[:16], d[:16], dim)
    elif name.startswith("loss"):
        if "B_table" in f.files:
            E, n, _ = f["pts"].shape
            xp = f["pts"].reshape(E * n, -1)
            env = np.repeat(np.arange(E), n).astype(np.int32)
            t, d, lt, df = O.eikonal_residual(W, xp, f["yobs"].reshape(E * n, 2), f["B_table"],
                                              env, dim=3, gamma=float(f["gamma"]))
        else:
            t, d, lt, df = O.eikonal_residual_arm(W, f["pts"], f["yobs"], f["B"].T, dim=6,
                                                  gamma=float(f["gamma"]))
        out.update(tau=t, dtau=d, ltau=lt, diff=df)
    else:
        raise KeyError(name)
    _F64[name] = out
    return out


def per_pair_rel(got, ref):
    """||got_p - ref_p|| / ||ref_p|| per pair (rows: the last axis is the pair's components
    unless the arrays are one value per pair)."""
    ref = np.asarray(ref, np.float64)
    got = np.asarray(got, np.float64).reshape(ref.shape)
    n = ref.shape[0] if ref.ndim < 3 else ref.shape[0] * ref.shape[1]
    a, b = got.reshape(n, -1), ref.reshape(n, -1)
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-30)


def north_star_pairs(what, got, ref, f64, tol=NORTH_STAR, diff=False):
    """Assert the north star per pair for `got` against the fp32 golden `ref`, adjudicating the
    pairs where ref itself is off by >= tol against the fp64 oracle `f64`.  diff=True: the
    Eikonal residual Σ_e(Ŝ/Y + Y/Ŝ) - 4 cancels, so its error is taken relative to |diff| + 4
    (the magnitude of its summands).  Returns (max error vs the golden, [(pair, e_golden,
    e_fp64, golden_vs_fp64)] of the adjudicated pairs)."""
    ref = np.asarray(ref, np.float64)
    got = np.asarray(got, np.float64).reshape(ref.shape)
    f64 = np.asarray(f64, np.float64).reshape(ref.shape)
    if diff:
        flat = lambda a: a.reshape(-1)  # noqa: E731
        e = np.abs(flat(got) - flat(ref)) / (np.abs(flat(ref)) + 4.0)
        e64 = np.abs(flat(got) - flat(f64)) / (np.abs(flat(f64)) + 4.0)
        r64 = np.abs(flat(ref) - flat(f64)) / (np.abs(flat(f64)) + 4.0)
    else:
        e, e64, r64 = per_pair_rel(got, ref), per_pair_rel(got, f64), per_pair_rel(ref, f64)
    adj = [(int(p), float(e[p]), float(e64[p]), float(r64[p])) for p in np.nonzero(e >= tol)[0]]
    bad = [a for a in adj if not a[2] < tol]
    print("north star %s: max per-pair rel vs golden %.2e (pair %d); %d pair(s) adjudicated "
          "against fp64%s" % (what, float(e.max()) if e.size else 0.0,
                              int(e.argmax()) if e.size else -1, len(adj),
                              "".join(" [pair %d: golden %.2e, fp64 %.2e, golden-vs-fp64 %.2e]"
                                      % a for a in adj[:8])))
    assert not bad, "%s: pairs off by >= %.0e from both the golden and fp64: %s" % (
        what, tol, bad[:8])
    return (float(e.max()) if e.size else 0.0), adj
