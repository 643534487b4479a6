"""CPU-only checks of the boundary: libpntf.so loads and exports exactly the C ABI of
include/pntf.h; host logic (state-dict layout, packing layout, argument validation, no
CPU fallback) behaves like the reference interface."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from pntf import _lib, ops, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pntf.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(pntf_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from pntf import build
        build.build()
    return ctypes.CDLL(_lib.LIB_PATH)


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ("pntf_pack_weights", "pntf_tau", "pntf_tau_grad", "pntf_path_velocity",
              "pntf_speed", "pntf_travel_time", "pntf_plan", "pntf_workspace_bytes"):
        assert s in syms


def test_library_exports_every_header_symbol(lib):
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert set(header_symbols()) == set(_lib.SIGNATURES)


def test_pure_queries_without_gpu(lib):
    lib.pntf_abi_version.restype = ctypes.c_int
    assert lib.pntf_abi_version() == 1
    lib.pntf_packed_floats.restype = ctypes.c_size_t
    # forward + transposed fragments of 13 matrices + biases/head (16x16 blob), then the same
    # matrices in wide fragment order + 19 bias-column fragments + 16 head fragments + head bias
    mats = 128 * 256 + 4 * 128 * 128 + 128 * 128 + 6 * 256 * 256 + 128 * 256
    plain = 128 + 4 * 128 + 128 + 6 * 256 + 128 + 128 + 4
    wide = 2 * mats + 19 * 256 + 16 * 256 + 4
    # then (64-float aligned) the quad streams: both directions once more, and per wave (8 per
    # quad workgroup) 14 bias / head fragments
    off_quad = (2 * mats + plain + wide + 63) // 64 * 64
    # then (64-float aligned) two split-bf16 copies of the wide matrices (3 bf16 terms per
    # weight; the second in block-major order for the encoder layers)
    off_x6 = (off_quad + 2 * mats + 8 * 14 * 256 + 63) // 64 * 64
    # then the forward matrices split for the residual kernel's 16x16x32 Taylor layers
    off_nx6 = (off_x6 + 2 * 3 * mats + 63) // 64 * 64
    assert lib.pntf_packed_floats() == off_nx6 + 3 * mats // 2
    lib.pntf_status_string.restype = ctypes.c_char_p
    assert lib.pntf_status_string(1) == b"invalid argument"


def test_argument_validation_without_gpu(lib):
    L = _lib.load()
    # dim must be 3 or 6; checked before any device access
    st = L.pntf_tau(None, 4, None, 10, None, None, 1, None, None)
    assert st == 1 and b"dim" in L.pntf_last_error()
    # empty batch is a no-op whatever the pointers are
    assert L.pntf_tau_grad(None, 3, None, 0, None, None, 1, 0, None, None, None, 0, None) == 0
    assert L.pntf_plan(None, 6, None, 0, None, None, 1, 0, 0.1, 0.1, 5, None, None, None, 0,
                       None) == 0
    assert L.pntf_plan(None, 6, None, 4, None, None, 1, 0, 0.1, 0.1, -1, None, None, None, 0,
                       None) == 1
    # unknown planner schedule, rejected before any device access
    fake = ctypes.c_void_p(64)
    assert L.pntf_plan_ex(fake, 6, fake, 4, fake, None, 1, 0, 0.1, 0.1, 5, fake, fake, fake,
                          1 << 20, 7, None) == 1
    assert b"schedule" in L.pntf_last_error()
    assert L.pntf_set_field_schedule(7) == 1
    assert L.pntf_set_field_schedule(0) == 0


def test_no_cpu_fallback():
    W = synth.make_weights(0)
    with pytest.raises(_lib.PntfError, match="HIP device"):
        ops.pack_weights([torch.from_numpy(v) for v in W.values()])
    with pytest.raises(_lib.PntfError, match="HIP device"):
        ops.tau(None, torch.zeros(4, 6), torch.zeros(3, 128))


def test_drop_in_state_dict_matches_reference_layout():
    from models import model_res_sigmoid as ma
    from models import model_res_sigmoid_multi as md
    net = md.NN("cpu", 3)
    assert list(net.state_dict().keys()) == synth.state_dict_keys()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    for name, fo, fi in synth.LAYER_SHAPES:
        assert shapes[name + ".weight"] == (fo, fi) and shapes[name + ".bias"] == (fo,)
    W = synth.make_weights(0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    arm = ma.NN("cpu", 6, torch.zeros(128, 6))
    assert list(arm.state_dict().keys()) == synth.state_dict_keys()
    assert tuple(arm.B.shape) == (6, 128)
    net.apply(net.init_weights)   # reference init U(±2/sqrt(fan_in))
    w = net.generator[0].weight.detach().numpy()
    assert np.abs(w).max() <= 2 / np.sqrt(256) + 1e-7


def test_models_raise_on_cpu_compute():
    from models import model_res_sigmoid_multi as md
    m = md.Model(".", ".", 3, 2, device="cpu")
    m.network = md.NN("cpu", 3)
    with pytest.raises(_lib.PntfError):
        m.network.out(torch.zeros(4, 6), torch.zeros(3, 128))
    with pytest.raises(_lib.PntfError):
        m.train()
    pts = torch.zeros(1, 4, 6, requires_grad=True)
    with pytest.raises(_lib.PntfError):      # the training loss has no CPU path either
        m.Loss(pts, torch.ones(1, 4, 2), torch.zeros(1, 3, 128), 1.0, 1e-3)


def _pack_index_numpy(W, trans):
    """numpy restatement of pack_kernel's index map (pntf_field.h)."""
    M = W.T if trans else W
    rows, cols = M.shape
    o = np.arange(rows * cols)
    s, lane, rest = o & 3, (o >> 2) & 63, o >> 8
    KT = cols // 16
    kt, ot = rest % KT, rest // KT
    n = 16 * ot + (lane & 15)
    k = 16 * kt + 4 * (lane >> 4) + s
    return M[n, k]


def test_pack_layout_is_a_permutation_and_feeds_mfma_fragments():
    rng = np.random.default_rng(0)
    W = rng.standard_normal((128, 256)).astype(np.float32)
    P = _pack_index_numpy(W, False)
    assert np.array_equal(np.sort(P), np.sort(W.ravel()))
    # fragment (ot, kt), lane (i, g), s  ==  W[16 ot + i][16 kt + 4 g + s]
    frag = P.reshape(8, 16, 64, 4)
    ot, kt, i, g = 3, 11, 5, 2
    np.testing.assert_array_equal(frag[ot, kt, g * 16 + i], W[16 * ot + i, 16 * kt + 4 * g:16 * kt + 4 * g + 4])
    PT = _pack_index_numpy(W, True)
    fragT = PT.reshape(16, 8, 64, 4)
    ot, kt = 13, 6
    np.testing.assert_array_equal(fragT[ot, kt, g * 16 + i],
                                  W.T[16 * ot + i, 16 * kt + 4 * g:16 * kt + 4 * g + 4])


def _pack_wide_numpy(W):
    """Restatement of pack_wide_kernel (pntf_wide.h): element o of the wide fragment stream."""
    rows, cols = W.shape
    o = np.arange(rows * cols)
    s, lane, u, rest = o & 3, (o >> 2) & 63, (o >> 8) & 3, o >> 10
    KT = cols // 32
    kt, ot = rest % KT, rest // KT
    return W[32 * ot + (lane & 31), 32 * kt + 8 * u + 4 * (lane >> 5) + s]


def test_wide_pack_layout_feeds_32x32x2_fragments():
    """Wide fragment (ot, kt, u), lane (i, h), element s holds W[32 ot + i][32 kt + 8u + 4h + s]:
    the A operand of the MFMA that takes register r = 4u + s of input tile kt as B, whose
    k rows are row(r, h) = (r & 3) + 8 (r >> 2) + 4 h (v_mfma_f32_32x32x2_f32 C/D layout)."""
    rng = np.random.default_rng(1)
    W = rng.standard_normal((256, 128)).astype(np.float32)
    P = _pack_wide_numpy(W)
    assert np.array_equal(np.sort(P), np.sort(W.ravel()))
    frag = P.reshape(8, 4, 4, 64, 4)          # (ot, kt, u, lane, s)
    row = lambda r, h: (r & 3) + 8 * (r >> 2) + 4 * h   # noqa: E731
    for ot, kt, r, i, h in [(0, 0, 0, 0, 0), (5, 3, 13, 17, 1), (7, 1, 6, 31, 0)]:
        u, s = r // 4, r % 4
        assert frag[ot, kt, u, 32 * h + i, s] == W[32 * ot + i, 32 * kt + row(r, h)]


def _pack_quad_numpy(W, dir_, waves=8):
    """Restatement of pack_quad_kernel (pntf_quad.h): the wave streams of one layer,
    shape (wave, groups, IN/16, 64 lanes, 4); block (og, kb) rows rotated by kb."""
    A = W.T if dir_ else W
    OUT, IN = A.shape
    w, g, q, lane, e = np.meshgrid(np.arange(waves), np.arange(OUT // (16 * waves)),
                                   np.arange(IN // 16), np.arange(64), np.arange(4),
                                   indexing="ij")
    kb = (lane >> 2) & 3
    row = w * (OUT // waves) + 16 * g + 4 * (lane >> 4) + ((lane + kb) & 3)
    k = 16 * q + 4 * e + kb
    return A[row, k]


def _ror16(x, n):
    """DPP row_ror:n: lane i of each 16-lane row reads lane (i - n) mod 16."""
    lane = np.arange(64)
    return x[(lane & ~15) | ((lane - n) & 15)]


def test_quad_pack_feeds_4x4x1_blocks():
    """Emulate one quad layer on the packed stream: v_mfma_f32_4x4x1_16b_f32 gives lane l
    D[i] += A(lane 4 (l >> 2) + i) * B(lane l) (block l >> 2, row i, column l & 3; layout
    measured by tests/diag/quad_probe.hip), B lane l = act[4 s + kb][pair l & 3]; the DPP tree
    of qring_sum leaves lane (og, kb, j) with the layer output at row
    w·OUT/8 + 16 g + 4 og + kb, pair j.  The SOLO layer (VALU, one pair; qring_sum_solo) reads
    the same partials from its lanes and sums them in the same association: bit-identical."""
    rng = np.random.default_rng(2)
    for (rows, cols, dir_) in [(128, 256, 0), (256, 128, 1), (256, 256, 0)]:
        W = rng.standard_normal((rows, cols)).astype(np.float32)
        P = _pack_quad_numpy(W, dir_)
        A = W.T if dir_ else W
        OUT, IN = A.shape
        act = rng.standard_normal((IN, 4)).astype(np.float32)
        ref = A.astype(np.float64) @ act.astype(np.float64)
        lane = np.arange(64)
        og, kb, j = lane >> 4, (lane >> 2) & 3, lane & 3
        for w in range(8):
            for g in range(OUT // 128):
                D = np.zeros((64, 4), np.float32)
                for q in range(IN // 16):
                    for e in range(4):
                        s = 4 * q + e
                        a = P[w, g, q, :, e]
                        b = act[4 * s + kb, j]
                        for i in range(4):
                            D[:, i] += a[4 * (lane >> 2) + i] * b
                b = D[:, 0] + _ror16(D[:, 1], 4)
                a = D[:, 2] + _ror16(D[:, 3], 4)
                p = b + _ror16(a, 8)
                rws = w * (OUT // 8) + 16 * g + 4 * og + kb
                np.testing.assert_allclose(p, ref[rws, j], rtol=1e-4, atol=1e-3)
                # the unrotated layout's butterflies (rounds 1-4) sum the same partials in the
                # same association: identical bits
                S = np.zeros((64, 4), np.float32)
                for i in range(4):
                    S[lane, (i + kb) & 3] = D[:, i]
                S = S + S[(lane & ~15) | ((lane - 4) & 15)]
                S = S + S[(lane & ~15) | ((lane - 8) & 15)]
                assert np.array_equal(p, S[lane, kb])
                # SOLO for pair 0: lane (og, kb, r) holds its own-row partial, = D[4 (l >> 2)
                # + 0][r] of the MFMA path (row (r + kb) & 3, pair 0)
                t = D[4 * (lane >> 2), lane & 3]
                bs = t + _ror16(t, 3)
                solo = (bs + _ror16(bs, 6))[lane & ~3]
                assert np.array_equal(solo, p[lane & ~3])


def test_synth_is_deterministic():
    np.testing.assert_array_equal(synth.make_pairs(100, 3, 2), synth.make_pairs(100, 3, 2))
    x = synth.make_pairs(5000, 3, 2)
    assert x.shape == (5000, 6) and np.all(np.abs(x) <= 0.5)
    e = synth.make_env_ids(1048576, 10)
    assert e.min() == 0 and e.max() == 9 and np.all(np.diff(e) >= 0)


def test_field_ex_validates_kind_and_schedule_without_gpu():
    L = _lib.load()
    fake = ctypes.c_void_p(16)
    assert L.pntf_field_ex(9, fake, 3, fake, 4, fake, None, 1, 0, fake, fake, fake, 1 << 30, 0,
                           None) == 1
    assert b"kind" in L.pntf_last_error()
    assert L.pntf_field_ex(1, fake, 3, fake, 4, fake, None, 1, 0, fake, fake, fake, 1 << 30, 5,
                           None) == 1
    assert b"schedule" in L.pntf_last_error()
    # empty batch: valid for every kind and schedule, nothing launched
    for kind in range(5):
        for sched in range(5):
            assert L.pntf_field_ex(kind, None, 3, None, 0, None, None, 1, 0, None, None, None, 0,
                                   sched, None) == 0


def test_build_info_names_every_kernel_unit():
    from pntf import build
    info = _lib.build_info()
    assert set(info) == {u[0] for u in build.UNITS}
    assert info == build.unit_ids()          # the loaded library is the current source


def _asm(unit):
    from pntf import build
    import glob
    files = glob.glob(os.path.join(build.BUILD, unit, "*amdgcn*gfx950*.s"))
    if not files:
        pytest.skip("device assembly of %s not kept (build dir absent)" % unit)
    return open(files[0]).read()


@pytest.mark.parametrize("unit", ["field_d3_k1", "field_d6_k1", "plan_d6", "fsplit_d3_k1",
                                  "residual_d3"])
def test_scratch_reloads_bypass_l1(unit):
    """Regression guard for DESIGN §7.3: a persistent wave rewrites its saved-σ slot for every
    tile and its stores do not refresh the CU's L1, so every load through the scratch buffer
    resource must carry the `nt` policy (a build without it returned stale σ tiles).  The same
    check runs inside pntf.build for every scratch-holding unit and fails the build."""
    from pntf import build
    descs, good, bad = build.scratch_policy_violations(_asm(unit))
    assert descs and good > 0 and bad == 0, (descs, good, bad)


def test_scratch_guard_catches_a_build_without_nt_loads(tmp_path):
    """A build variant whose scratch loads drop the nt bit (-DPNTF_SCRATCH_LOAD_AUX=0) must be
    rejected by the build guard: compile the split τ+∇τ kernel that way (device code only) and
    check that the guard counts its scratch loads as violations."""
    import subprocess
    from pntf import build
    out = str(tmp_path / "variant.s")
    cmd = ([build.hipcc()] + [f for f in build.CXXFLAGS if not f.startswith(("-save-temps",
                                                                            "-Rpass"))]
           + ["-DPNTF_DIM=3", "-DPNTF_KIND=1", "-DPNTF_SPLIT_FIELD",
              "-DPNTF_SCRATCH_LOAD_AUX=0", "--cuda-device-only", "-S",
              os.path.join(build.CSRC, "pntf_kernels.hip"), "-o", out])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "not found" in r.stderr:
        pytest.skip("hipcc unavailable")
    assert r.returncode == 0, r.stderr[-2000:]
    descs, good, bad = build.scratch_policy_violations(open(out).read())
    assert descs and bad > 0 and good == 0, (descs, good, bad)


def test_store_data_guard_on_snippets():
    """the build guard flags a VALU write of a 16-byte store's data VGPRs in the
    very next instruction (MUBUF: vdata first; global: vaddr, then vdata), and nothing once a
    wait state separates them or the writer is a load."""
    from pntf import build
    hz = build.store_data_hazards
    st = "\tbuffer_store_dwordx4 v[4:7], v9, s[0:3], s5 offen nt\n"
    assert len(hz(st + "\tv_add_f32_e32 v6, v1, v2\n")) == 1
    assert hz(st + "\ts_nop 0\n\tv_add_f32_e32 v6, v1, v2\n") == []
    assert hz(st + "\tv_add_f32_e32 v8, v1, v2\n") == []
    assert hz(st + "\tbuffer_load_dwordx4 v[4:7], v9, s[0:3], 0 offen\n") == []
    gst = "\tglobal_store_dwordx4 v[0:1], v[4:7], off\n"
    assert hz(gst + "\tv_mov_b32_e32 v0, 0\n") == []
    assert len(hz(gst + "\tv_accvgpr_read_b32 v5, a0\n")) == 1
    assert hz("\tbuffer_store_dwordx2 v[4:5], v9, s[0:3], 0 offen\n\tv_mov_b32 v4, 0\n") == []


@pytest.mark.parametrize("unit", ["wide_d3_k1", "wide_d6_k3", "fsplit_d3_k1", "gemm", "train"])
def test_store_data_guard_clean_on_built_units(unit):
    from pntf import build
    assert build.store_data_hazards(_asm(unit)) == []


def test_store_data_guard_catches_an_unguarded_build(tmp_path):
    """Without bstore's keep-alive s_nop (-DPNTF_BSTORE_UNGUARDED) the headline wide τ+∇τ
    kernel has the hazard that corrupted lanes 12-15: the guard must see it."""
    import subprocess
    from pntf import build
    out = str(tmp_path / "variant.s")
    cmd = ([build.hipcc()] + [f for f in build.CXXFLAGS if not f.startswith(("-save-temps",
                                                                            "-Rpass"))]
           + ["-DPNTF_DIM=3", "-DPNTF_KIND=1", "-DPNTF_WIDE_FIELD", "-DPNTF_PF_STEPS=2", "-DPNTF_BSTORE_UNGUARDED",
              "--cuda-device-only", "-S", os.path.join(build.CSRC, "pntf_kernels.hip"),
              "-o", out])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "not found" in r.stderr:
        pytest.skip("hipcc unavailable")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(build.store_data_hazards(open(out).read())) > 0


def test_field_schedule_resolution_and_wide_index_guard():
    """AUTO's kernel choice (include/pntf.h), and the guard of ADVICE r02: the wide kernel
    keeps 32-bit tile indices, so no batch above 2^31 - 32 pairs may reach it, whatever
    schedule is asked for (those run the int64-indexed wave-tile kernel).  Host-only: without
    a GPU the CU count is 256."""
    L = _lib.load()
    AUTO, WAVE, SPLIT, WIDE, QUAD = range(5)
    cus = 256
    assert L.pntf_field_schedule_for(1, AUTO) == QUAD
    assert L.pntf_field_schedule_for(4 * cus, AUTO) == QUAD
    assert L.pntf_field_schedule_for(4 * cus + 1, AUTO) == SPLIT
    assert L.pntf_field_schedule_for(32 * cus, AUTO) == SPLIT
    assert L.pntf_field_schedule_for(32 * cus + 1, AUTO) == WIDE
    assert L.pntf_field_schedule_for(1 << 20, AUTO) == WIDE
    lim = (1 << 31) - 32
    for sched in (AUTO, WIDE):
        assert L.pntf_field_schedule_for(lim, sched) == WIDE
        assert L.pntf_field_schedule_for(lim + 1, sched) == WAVE
        assert L.pntf_field_schedule_for(1 << 33, sched) == WAVE
    assert L.pntf_field_schedule_for(1 << 20, WAVE) == WAVE
    assert L.pntf_field_schedule_for(1 << 20, SPLIT) == SPLIT
    assert L.pntf_field_schedule_for(5, QUAD) == QUAD
    assert L.pntf_field_schedule_for(-1, AUTO) == -1 and L.pntf_field_schedule_for(4, 9) == -1


def test_gemm_rejects_rows_beyond_lds_tiled_grid_without_gpu():
    """the LDS-tiled GEMM puts row tiles on grid.y (limit 65535); an M past
    65535 * 128 rows on that path is rejected with a clear error before any launch."""
    L = _lib.load()
    fake = ctypes.c_void_p(256)
    M = 65535 * 128 + 1
    st = L.pntf_tt_gemm(1, 0, M, 128, 256, fake, M, fake, 128, fake, 128, 0.0, fake, 1 << 40,
                        None)
    assert st == 1 and b"grid" in L.pntf_tt_gemm_last_error()
