"""CPU oracle for point -> triangle-mesh unsigned distance — TEST INFRASTRUCTURE ONLY.

Restates what `point_obstacle_distance` (dataprocessing/speed_sampling_gpu.py:325-336)
returns: sqrt of the minimum over triangles of the squared point-to-triangle distance, as
computed by the reference's CUDA dependency bvh_distance_queries (un-vendored submodule,
.gitmodules:1-3, github.com/YuliangXiu/bvh-distance-queries, no commit pinned; its BVH only
prunes triangles, the distance per (point, triangle) is the exact closest point of Ericson,
"Real-Time Collision Detection" §5.1.5).  Only `tests/` may import this module.

Pinning: the dependency is absent here and the reference's tests hold no vectors for it, so
the restatement is pinned by analytic known answers instead (distance to the surface of an
axis-aligned box mesh, inside and outside; tests/test_mesh.py) — "parity pinned by
geometry, not by reference outputs" (DESIGN.md).
"""
import numpy as np


def _seg_d2(p, a, e):
    q = p - a
    ee = np.einsum("...k,...k->...", e, e)
    t = np.where(ee > 0, np.einsum("...k,...k->...", q, e) / np.where(ee > 0, ee, 1.0), 0.0)
    t = np.clip(t, 0.0, 1.0)
    r = q - t[..., None] * e
    return np.einsum("...k,...k->...", r, r)


def tri_d2(p, tri):
    """Squared distance from points p (..., 3) to triangles tri (..., 3, 3), broadcasting;
    Ericson §5.1.5 region tests; in the interior region a (near-)zero-area triangle
    (sin^2 of the angle at a <= 1e-12, same test as the kernel) -> nearest edge."""
    p = np.asarray(p, np.float64)
    a, b, c = tri[..., 0, :], tri[..., 1, :], tri[..., 2, :]
    ab, ac = b - a, c - a
    dot = lambda x, y: np.einsum("...k,...k->...", x, y)
    ap, bp, cp = p - a, p - b, p - c
    d1, d2 = dot(ab, ap), dot(ac, ap)
    d3, d4 = dot(ab, bp), dot(ac, bp)
    d5, d6 = dot(ab, cp), dot(ac, cp)
    vc = d1 * d4 - d3 * d2
    vb = d5 * d2 - d1 * d6
    va = d3 * d6 - d5 * d4
    s = va + vb + vc
    safe = lambda x: np.where(x != 0, x, 1.0)
    inner = a + ab * (vb / safe(s))[..., None] + ac * (vc / safe(s))[..., None]
    q = inner
    # later regions first, so the earliest matching region (Ericson's order) wins
    r6 = (va <= 0) & ((d4 - d3) >= 0) & ((d5 - d6) >= 0)
    w6 = (d4 - d3) / safe((d4 - d3) + (d5 - d6))
    q = np.where(r6[..., None], b + w6[..., None] * (c - b), q)
    r5 = (vb <= 0) & (d2 >= 0) & (d6 <= 0)
    q = np.where(r5[..., None], a + (d2 / safe(d2 - d6))[..., None] * ac, q)
    r4 = (d6 >= 0) & (d5 <= d6)
    q = np.where(r4[..., None], c, q)
    r3 = (vc <= 0) & (d1 >= 0) & (d3 <= 0)
    q = np.where(r3[..., None], a + (d1 / safe(d1 - d3))[..., None] * ab, q)
    r2 = (d3 >= 0) & (d4 <= d3)
    q = np.where(r2[..., None], b, q)
    r1 = (d1 <= 0) & (d2 <= 0)
    q = np.where(r1[..., None], a, q)
    r = p - q
    d2q = dot(r, r)
    n = np.cross(ab, ac)
    flat = dot(n, n) <= 1e-12 * dot(ab, ab) * dot(ac, ac)
    degen = ~(r1 | r2 | r3 | r4 | r5 | r6) & (~(s > 0) | flat)
    if np.any(degen):
        de = np.minimum(np.minimum(_seg_d2(p, a, ab), _seg_d2(p, a, ac)), _seg_d2(p, b, c - b))
        d2q = np.where(degen, de, d2q)
    return d2q


def point_mesh_distance(pts, tris, chunk=256):
    """Unsigned distance (n,) from pts (n, 3) to the mesh tris (t, 3, 3), float64."""
    pts = np.asarray(pts, np.float64)
    tris = np.asarray(tris, np.float64)
    out = np.empty(len(pts))
    for s in range(0, len(pts), chunk):
        d2 = tri_d2(pts[s:s + chunk, None, :], tris[None, :, :, :])
        out[s:s + chunk] = np.sqrt(d2.min(axis=1))
    return out


def box_mesh(lo, hi):
    """12-triangle mesh of the axis-aligned box [lo, hi] (3,) -> (12, 3, 3)."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    v = np.array([[(hi if (i >> k) & 1 else lo)[k] for k in range(3)] for i in range(8)])
    quads = [(0, 2, 6, 4), (1, 5, 7, 3), (0, 4, 5, 1), (2, 3, 7, 6), (0, 1, 3, 2), (4, 6, 7, 5)]
    f = []
    for q0, q1, q2, q3 in quads:
        f += [(q0, q1, q2), (q0, q2, q3)]
    return v[np.array(f)]


def box_distance(pts, lo, hi):
    """Analytic unsigned distance from pts (n, 3) to the SURFACE of the box [lo, hi]."""
    pts = np.asarray(pts, np.float64)
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    out = np.maximum(np.maximum(lo - pts, pts - hi), 0.0)
    outside = np.linalg.norm(out, axis=1)
    inside = np.minimum(pts - lo, hi - pts).min(axis=1)
    is_in = np.all((pts >= lo) & (pts <= hi), axis=1)
    return np.where(is_in, inside, outside)


def speed_from_distance(y, offset, margin):
    """speed = clip(d, offset, margin) / margin (speed_sampling_gpu.py:414-419)."""
    return np.clip(y, offset, margin) / margin
