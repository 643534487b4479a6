"""Speed-sample generator: point -> triangle-mesh unsigned distance
(dataprocessing/speed_sampling_gpu.py:325-336, the reference's bvh_distance_queries call)
and the point sampler around it (:338-421).

Pinning: bvh_distance_queries is an un-vendored submodule (.gitmodules:1-3) and the
reference holds no vectors for it, so the oracle (oracle/mesh_oracle.py) is pinned by
analytic box distances (CPU tests below).  GPU tolerance: the kernel computes in fp32 on
coordinates in [-0.5, 0.5]; distances agree with the fp64 oracle to 2e-6 absolute.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import mesh_oracle as M
from pntf import _lib

TOL = 2e-6


def random_mesh(rng, t, scale=0.2):
    c = rng.uniform(-0.4, 0.4, (t, 1, 3))
    return c + rng.normal(0, scale, (t, 3, 3)) * rng.uniform(0.05, 1.0, (t, 1, 1))


# ------------------------------------------------------------------ CPU: oracle pinning


def test_oracle_matches_analytic_box_distance():
    rng = np.random.default_rng(0)
    lo, hi = np.array([-0.3, -0.2, -0.1]), np.array([0.25, 0.3, 0.2])
    pts = rng.uniform(-0.5, 0.5, (2000, 3))
    d = M.point_mesh_distance(pts, M.box_mesh(lo, hi))
    np.testing.assert_allclose(d, M.box_distance(pts, lo, hi), atol=1e-12)


def test_oracle_against_dense_triangle_sampling():
    """Closest point is never farther than any sampled point of the triangle, and a dense
    barycentric sampling gets within its resolution of it."""
    rng = np.random.default_rng(1)
    tri = random_mesh(rng, 1)[0]
    pts = rng.uniform(-0.5, 0.5, (200, 3))
    k = 200
    u, v = np.meshgrid(np.linspace(0, 1, k), np.linspace(0, 1, k))
    m = (u + v) <= 1
    s = tri[0] + u[m, None] * (tri[1] - tri[0]) + v[m, None] * (tri[2] - tri[0])
    dense = np.sqrt(((pts[:, None, :] - s[None]) ** 2).sum(-1)).min(1)
    d = M.point_mesh_distance(pts, tri[None])
    assert np.all(d <= dense + 1e-12)
    assert np.all(dense - d < 0.02)


def test_oracle_degenerate_triangle_is_segment_distance():
    tri = np.array([[[0.0, 0, 0], [0.2, 0, 0], [0.1, 0, 0]]])
    pts = np.array([[0.1, 0.3, 0.0], [-0.3, 0.0, 0.4], [0.5, 0.0, 0.0]])
    np.testing.assert_allclose(M.point_mesh_distance(pts, tri), [0.3, 0.5, 0.3], atol=1e-12)


def test_mesh_symbols_and_chunk_planner_without_gpu():
    L = _lib.load()
    assert L.pntf_mesh_chunks(0, 10) == 1
    assert L.pntf_mesh_chunks(1 << 20, 10) == 1          # one tile of triangles
    assert L.pntf_mesh_chunks(256, 100000) == 391         # all 391 tiles, fills the chip
    # argument validation before any device access
    assert L.pntf_point_mesh_distance(None, 5, None, 3, None, 0, None) == 1
    assert b"bad arguments" in L.pntf_mesh_last_error()
    assert L.pntf_point_mesh_distance(None, 0, None, 0, None, 0, None) == 0


def test_mesh_distance_has_no_cpu_path():
    from pntf import ops
    with pytest.raises(_lib.PntfError):
        ops.point_mesh_distance(torch.zeros(4, 3), torch.zeros(1, 3, 3))


# ------------------------------------------------------------------ GPU parity


@pytest.mark.gpu
@pytest.mark.parametrize("n,t", [(1, 1), (255, 7), (1000, 300), (4097, 1500), (300, 20000)])
def test_hip_distance_matches_oracle(n, t):
    from pntf import ops
    rng = np.random.default_rng(n * 31 + t)
    tris = random_mesh(rng, t).astype(np.float32)
    pts = rng.uniform(-0.5, 0.5, (n, 3)).astype(np.float32)
    d = ops.point_mesh_distance(torch.from_numpy(pts).cuda(),
                                torch.from_numpy(tris).cuda()[None]).detach().cpu().numpy()
    ref = M.point_mesh_distance(pts, tris)
    assert d.shape == (n,)
    assert np.abs(d - ref).max() < TOL


@pytest.mark.gpu
def test_hip_distance_culling_on_large_sorted_query():
    """Morton-ordered query with tile culling on a mesh of small clustered triangles:
    matches the oracle and the unordered query bit for bit."""
    from pntf import ops
    rng = np.random.default_rng(8)
    tris = random_mesh(rng, 4000, scale=0.01).astype(np.float32)
    pts = rng.uniform(-0.5, 0.5, (20000, 3)).astype(np.float32)
    P, T = torch.from_numpy(pts).cuda(), torch.from_numpy(tris).cuda()
    a = ops.point_mesh_distance(P, T, order=True)
    b = ops.point_mesh_distance(P, T, order=False)
    assert torch.equal(a, b)
    sub = rng.choice(20000, 1500, replace=False)
    assert np.abs(a.detach().cpu().numpy()[sub] - M.point_mesh_distance(pts[sub], tris)).max() < TOL


@pytest.mark.gpu
def test_hip_distance_bits_independent_of_triangle_split():
    from pntf import ops
    rng = np.random.default_rng(5)
    tris = torch.from_numpy(random_mesh(rng, 3000).astype(np.float32)).cuda()
    pts = torch.from_numpy(rng.uniform(-0.5, 0.5, (777, 3)).astype(np.float32)).cuda()
    outs = [ops.point_mesh_distance(pts, tris, chunks=c, order=o) for c in (1, 2, 5, 12, 0)
            for o in (False, True)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    # axis-aligned walls (Gibson-like rooms): many triangles whose true distance equals the
    # culling box gap to the last ulp; points on a lattice aligned with the walls
    walls = np.concatenate([M.box_mesh(np.array([-0.4, -0.3, -0.25]) + 0.1 * k,
                                       np.array([-0.2, 0.1, 0.05]) + 0.1 * k)
                            for k in range(6)]).astype(np.float32)
    g = np.linspace(-0.5, 0.5, 41, dtype=np.float32)
    lat = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    W, P = torch.from_numpy(walls).cuda(), torch.from_numpy(lat).cuda()
    ref = ops.point_mesh_distance(P, W, chunks=1, order=False)
    for c in (1, 3, 0):
        assert torch.equal(ops.point_mesh_distance(P, W, chunks=c, order=True), ref)
    sub = rng.choice(lat.shape[0], 1500, replace=False)
    assert np.abs(ref.detach().cpu().numpy()[sub] - M.point_mesh_distance(lat[sub], walls)).max() < TOL


@pytest.mark.gpu
def test_hip_box_analytic_and_degenerate():
    from pntf import ops
    rng = np.random.default_rng(6)
    lo, hi = np.array([-0.3, -0.2, -0.1]), np.array([0.25, 0.3, 0.2])
    tris = np.concatenate([M.box_mesh(lo, hi),
                           [[[0.0, 0, 0], [0.2, 0, 0], [0.1, 0, 0]]]]).astype(np.float32)
    pts = rng.uniform(-0.5, 0.5, (5000, 3)).astype(np.float32)
    d = ops.point_mesh_distance(torch.from_numpy(pts).cuda(),
                                torch.from_numpy(tris).cuda()).detach().cpu().numpy()
    assert np.all(np.isfinite(d))
    assert np.abs(d - M.point_mesh_distance(pts, tris)).max() < TOL
    assert ops.point_mesh_distance(torch.zeros(0, 3, device="cuda"),
                                   torch.from_numpy(tris).cuda()).shape == (0,)


@pytest.mark.gpu
def test_point_sampler_properties():
    """point_rand_sample_bound_points: shapes, box membership, offset < d(x0) < margin, and
    every returned distance recomputed by the oracle."""
    from dataprocessing import speed_sampling_gpu as S
    torch.manual_seed(0)
    lo, hi = np.array([-0.2, -0.2, -0.2]), np.array([0.2, 0.2, 0.2])
    tris = M.box_mesh(lo, hi)
    v = tris.reshape(-1, 3)
    f = np.arange(len(v)).reshape(-1, 3)
    offset, margin, n = 0.001, 0.05, 3000
    X, speed = S.point_rand_sample_bound_points(n, 3, v, f, offset, margin)
    assert X.shape == (n, 6) and X.dtype == np.float32 and speed.shape == (n, 2)
    assert np.all(np.abs(X) <= 0.5)
    d0 = M.point_mesh_distance(X[:, :3], tris)
    d1 = M.point_mesh_distance(X[:, 3:], tris)
    assert np.all((d0 > offset - TOL) & (d0 < margin + TOL))
    np.testing.assert_allclose(speed[:, 0], M.speed_from_distance(d0, offset, margin),
                               atol=TOL / margin)
    np.testing.assert_allclose(speed[:, 1], M.speed_from_distance(d1, offset, margin),
                               atol=TOL / margin)
    d = S.point_obstacle_distance(torch.from_numpy(X[:5, :3]).cuda(),
                                  torch.from_numpy(tris.astype(np.float32)).cuda()[None])
    np.testing.assert_allclose(d.detach().cpu().numpy(), d0[:5], atol=TOL)
