"""The split-bf16 copies of the wide weight fragments (pntf_wide.h pack_x6_kernel, DESIGN.md §3
"split-bf16 layers"), read back from the packed blob and checked against their definition:

  * every weight of the fp32 wide region (both directions, every matrix) appears once in each
    copy, at the fragment the wide kernel's step order reads it from: per 32 x 32 step (ot, kt)
    and k block b, element i of lane l holds M[32 ot + (l & 31)][32 kt + (i & 3) + 16 b +
    8 (i >> 2) + 4 (l >> 5)], i.e. element i & 3 of fp32 fragment 2b + (i >> 2);
  * step order of the first copy (OFF_X6): every layer's out tiles in one group, steps
    (kt, ot), fragments 3b + term, for the accumulate-in-bank engine (round 6; encoder[0]^T, the
    Fourier fold, in two passes (p, kt, ot_local) of its sin/cos tiles 2p, 2p + 1); round 5's
    groups of 4 / per tile with X6_ACC = False; the second copy (OFF_X6BM) block-major
    (g of 2 tiles, kt, b), fragments 3o + term, for the two-column layers;
  * the three terms are the round-to-nearest-even bf16 splits x0 = bf16(x), x1 = bf16(x - x0),
    x2 = bf16(x - x0 - x1), bit for bit, and x0 + x1 + x2 == x exactly.
"""
import numpy as np
import pytest
import torch

from golden_util import weights
from pntf import ops

pytestmark = pytest.mark.gpu

SZ_DIR = 128 * 256 + 4 * 128 * 128 + 128 * 128 + 6 * 256 * 256 + 128 * 256
SZ_BIAS = 128 + 4 * 128 + 128 + 6 * 256 + 128 + 128 + 4
# forward direction: (float offset, out, in, columns sharing the weights) in the OFF_* order
# the narrow (16x16x32) split copy of the forward direction (pntf_taylor.h pack_nx6_kernel)
NX6_SZ = 3 * SZ_DIR // 2
NX6_G = 16
NAMES = ["encoder.0", "encoder.1", "encoder1.1", "encoder.2", "encoder1.2", "encoder.3",
         "generator.0", "generator1.0", "generator.1", "generator1.1", "generator.2",
         "generator1.2", "generator.3"]
MATS = ([(0, 128, 256, 2)] + [(32768 + 16384 * i, 128, 128, 2) for i in range(5)] +
        [(114688 + 65536 * i, 256, 256, 1) for i in range(6)] + [(507904, 128, 256, 1)])


def bf16_rne(x):
    """float32 -> the float32 value of its round-to-nearest-even bf16 (finite inputs)."""
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return (r & 0xFFFFFFFF).astype(np.uint32).view(np.float32)


# The step order of the first copy follows the wide kernel's layer engine (pntf_wide.h):
# PNTF_X6_ACC = 1 (round 6, the accumulate-in-bank xlayer): every layer's out tiles in one group,
# steps (kt, ot); encoder[0]^T (the Fourier fold) in two passes of 4 out tiles.  Round 5's
# engine: groups of 4 (one-column) / per tile (two-column layers).
X6_ACC = True


def frag_index(gf, j, OT, KT, nc, b, bm, fold=False):
    ot, kt = divmod(j, KT)
    base = gf - j
    if nc == 2 and bm:
        return (base + ((ot // 2) * KT + kt) * 2 + b) * 6 + (ot % 2) * 3
    if X6_ACC and fold:
        p, ol = (ot % 4) // 2, ((ot % 4) % 2) * 2 + ot // 4
        return (base + (p * KT + kt) * 4 + ol) * 6 + 3 * b
    if X6_ACC:
        G = min(OT, 8) if nc == 1 else 4
    else:
        G = 1 if nc == 2 else 4
    return (base + (ot // G) * KT * G + kt * G + ot % G) * 6 + 3 * b


def test_x6_copies_match_their_definition():
    dev = torch.device("cuda:0")
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in weights().values()])
    P = packed.cpu().numpy()
    x6_sz = 3 * SZ_DIR
    off_bm = P.size - NX6_SZ - x6_sz      # the narrow split copy (round 6) comes last
    off_x6 = off_bm - x6_sz
    off_wide = 2 * SZ_DIR + SZ_BIAS
    wide = P[off_wide:off_wide + 2 * SZ_DIR].reshape(-1, 4, 64, 4)     # step, u, lane, s
    # fp32 values of (step, block, lane, i): element i & 3 of fragment 2b + (i >> 2)
    vals = wide.reshape(-1, 2, 2, 64, 4).transpose(0, 1, 3, 2, 4).reshape(-1, 2, 64, 8)
    x0 = bf16_rne(vals)
    x1 = bf16_rne(vals - x0)
    x2 = bf16_rne(vals - x0 - x1)
    assert np.array_equal(x0.astype(np.float64) + x1 + x2, vals.astype(np.float64))
    want = np.stack([x0, x1, x2], axis=2)                              # step, b, term, lane, i
    for off, bm in ((off_x6, False), (off_bm, True)):
        bits = P[off:off + x6_sz].view(np.uint16).reshape(-1, 64, 8).astype(np.uint32) << 16
        got = bits.view(np.float32)                                   # fragment, lane, i
        seen = np.zeros(got.shape[0], dtype=np.int32)
        for d in (0, 1):
            for m0, out, inn, nc in MATS:
                if d:
                    out, inn = inn, out
                OT, KT = out // 32, inn // 32
                for j in range(OT * KT):
                    gf = (d * SZ_DIR + m0) // 1024 + j
                    for b in range(2):
                        fr = frag_index(gf, j, OT, KT, nc, b, bm, fold=(d == 1 and m0 == 0))
                        for p in range(3):
                            assert np.array_equal(got[fr + p], want[gf, b, p]), (d, m0, j, b, p, bm)
                            seen[fr + p] += 1
        assert (seen == 1).all(), "every fragment written once"


def test_nx6_copy_matches_its_definition():
    """The residual kernel's split-bf16 Taylor layers (pntf_taylor.h taylor_layer_x6, round 6)
    read the forward matrices pre-split for v_mfma_f32_16x16x32_bf16: step st = (g·NB + b)·G + o
    (out tile ot = g·G + o of 16 rows, k block b of 32 features, G = min(OT, 8)) holds at lane
    l = (r, q) = (l & 15, l >> 4), element i, the three RNE bf16 terms of
    M[16 ot + r][16 (2b + (i >> 2)) + 4 q + (i & 3)], fragment 3 st + term; a matrix at forward
    offset o starts at 1.5 o."""
    dev = torch.device("cuda:0")
    W = weights()
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    P = packed.cpu().numpy()
    nx6 = P[P.size - NX6_SZ:]
    seen = 0
    for (m0, out, inn, _), name in zip(MATS, NAMES):
        M = np.asarray(W[name + ".weight"], np.float32)
        assert M.shape == (out, inn)
        OT, NB = out // 16, inn // 32
        G = min(OT, NX6_G)
        st = np.arange(OT * NB)
        o, b, ot = st % G, (st // G) % NB, (st // (G * NB)) * G + st % G
        lane, i = np.arange(64), np.arange(8)
        r, q = lane & 15, lane >> 4
        rows = 16 * ot[:, None, None] + r[None, :, None]
        cols = 16 * (2 * b[:, None, None] + (i[None, None, :] >> 2)) + 4 * q[None, :, None] + \
            (i[None, None, :] & 3)
        vals = M[rows, cols]                                              # step, lane, i
        x0 = bf16_rne(vals)
        x1 = bf16_rne(vals - x0)
        x2 = bf16_rne(vals - x0 - x1)
        assert np.array_equal(x0.astype(np.float64) + x1 + x2, vals.astype(np.float64))
        off = m0 * 3 // 2
        n = OT * NB * 3 * 256                          # floats of the copy (1 KiB fragments)
        bits = nx6[off:off + n].view(np.uint16).reshape(OT * NB, 3, 64, 8).astype(np.uint32)
        got = (bits << 16).view(np.float32)
        for p, want in enumerate((x0, x1, x2)):
            assert np.array_equal(got[:, p], want), (name, p)
        seen += n
    assert seen == NX6_SZ
