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
