"""Seeded synthetic inputs for the τ/∇τ hot path.

No pretrained checkpoints or Gibson datasets exist offline, so every
parity case and every benchmark runs on inputs drawn here from numpy's PCG64 with fixed
seeds.  The generator is pure numpy: the GPU box regenerates the exact same arrays.

* weights  : state-dict order, W and b ~ U(-2/sqrt(fan_in), +2/sqrt(fan_in))
             (reference NN.init_weights, models/model_res_sigmoid_multi.py:177-183)
* B        : 0.5 * N(0, 1), shape (dim, 128) for the multi-env model
             (dataprocessing/speed_sampling_gpu.py:493) or (128, dim) for the arm model
             (models/model_res_sigmoid.py:942)
* pairs    : xs ~ U[-0.5,0.5]^dim, xg = xs + normalize(U[-0.5,0.5]^dim) * U[0, sqrt(dim)),
             kept only if xg is inside the box (dataprocessing/speed_sampling_gpu.py:346-356)
* speeds   : Yobs ~ U[0.1, 1]^2 (range of speed_sampling_gpu.py:418-419)
"""
import numpy as np

H = 128  # hidden width (models/model_res_sigmoid_multi.py:134)

# (state-dict key prefix, out_features, in_features) in reference state-dict order
# (NN.__init__, models/model_res_sigmoid_multi.py:155-175).
LAYER_SHAPES = (
    [("encoder.0", H, 2 * H)]
    + [("encoder.%d" % i, H, H) for i in (1, 2, 3)]
    + [("encoder1.0", H, 2 * H)]
    + [("encoder1.%d" % i, H, H) for i in (1, 2)]
    + [("generator.%d" % i, 2 * H, 2 * H) for i in (0, 1, 2)]
    + [("generator.3", H, 2 * H), ("generator.4", 1, H)]
    + [("generator1.%d" % i, 2 * H, 2 * H) for i in (0, 1, 2)]
)


def state_dict_keys():
    keys = []
    for name, _, _ in LAYER_SHAPES:
        keys += [name + ".weight", name + ".bias"]
    return keys


def make_weights(seed=0):
    """Seeded stand-in for NN.init_weights (model_res_sigmoid_multi.py:177-183).

    Returns an ordered dict key -> float32 array in the reference state-dict order."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, fo, fi in LAYER_SHAPES:
        stdv = 2.0 / np.sqrt(fi)
        out[name + ".weight"] = rng.uniform(-stdv, stdv, size=(fo, fi)).astype(np.float32)
        out[name + ".bias"] = rng.uniform(-stdv, stdv, size=(fo,)).astype(np.float32)
    return out


def make_B(dim=3, seed=1, arm=False):
    """B = 0.5*N(0,1); (dim,128) multi-env layout, (128,dim) arm layout."""
    rng = np.random.Generator(np.random.PCG64(seed))
    b = (0.5 * rng.standard_normal((dim, H))).astype(np.float32)
    return np.ascontiguousarray(b.T) if arm else b


def make_B_table(n_env=10, dim=3, first_seed=1):
    """Per-env B table (n_env, dim, 128), env e drawn with seed first_seed+e."""
    return np.stack([make_B(dim, first_seed + e) for e in range(n_env)])


def make_pairs(n, dim=3, seed=2):
    """(n, 2*dim) float32 [xs | xg] pairs, Gibson-style rejection sampling."""
    rng = np.random.Generator(np.random.PCG64(seed))
    chunks, have = [], 0
    while have < n:
        m = max(2 * (n - have), 1024)
        p = rng.uniform(-0.5, 0.5, size=(m, dim))
        dp = rng.uniform(-0.5, 0.5, size=(m, dim))
        rl = rng.uniform(0.0, 1.0, size=(m, 1)) * np.sqrt(dim)
        nrm = np.maximum(np.linalg.norm(dp, axis=1, keepdims=True), 1e-12)
        q = p + dp / nrm * rl
        ok = np.all((q <= 0.5) & (q >= -0.5), axis=1)
        c = np.concatenate([p[ok], q[ok]], axis=1)
        chunks.append(c)
        have += c.shape[0]
    return np.concatenate(chunks)[:n].astype(np.float32)


def make_box_pairs(n, dim=6, seed=3):
    """(n, 2*dim) float32 uniform [-0.5,0.5] start/goal queries (arm joint space)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(-0.5, 0.5, size=(n, 2 * dim)).astype(np.float32)


def make_env_ids(n, n_env, contiguous=True, seed=4):
    """Env id per pair: contiguous blocks of ~n/n_env or random."""
    if contiguous:
        return (np.arange(n, dtype=np.int64) * n_env // max(n, 1)).astype(np.int32)
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, n_env, size=n).astype(np.int32)


def make_speeds(n, seed=5, lo=0.1, hi=1.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(lo, hi, size=(n, 2)).astype(np.float32)
