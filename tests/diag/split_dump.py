"""Stage dumps (PNTF_DUMPX in pntf_split.h: the full activation bank after every LDS exchange,
block 0 / wave 0 / its first tile) of two split-width builds, compared stage by stage.
Diagnostics only: python tests/diag/split_dump.py s4d s8d"""
import ctypes, os, sys
import numpy as np
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "p-ntfields_amd"))
from pntf import ops, synth


def run(name, packed, xp, B, n):
    dev = xp.device
    lib = ctypes.CDLL(os.path.join(HERE, "libperf_%s.so" % name))
    V = lambda t: ctypes.c_void_p(t.data_ptr())
    split = lib.perf_split_width()
    grid = 1
    ws = torch.zeros(grid * split * 96 * 1024 * 4, dtype=torch.uint8, device=dev)
    dbg = torch.zeros(64 * 16 * 64 * 4, device=dev)
    assert lib.perf_set_dbg(V(dbg)) == 0
    t = torch.empty(n, device=dev)
    d = torch.empty(n, 6, device=dev)
    lib.perf_tau_grad.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
        [ctypes.c_void_p] * 5
    assert lib.perf_tau_grad(grid, V(packed), V(xp), n, V(B), V(t), V(d), V(ws),
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    return dbg.cpu().numpy().reshape(64, 16, 64, 4), d.cpu().numpy()


def main(a, b):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    n = 16
    xp = torch.from_numpy(synth.make_pairs(n, 3)).to(dev).contiguous()
    B = torch.from_numpy(synth.make_B(3)).to(dev).contiguous()
    da, oa = run(a, packed, xp, B, n)
    db, ob = run(b, packed, xp, B, n)
    for k in list(range(8)) + list(range(20, 29)) + [30]:
        x, y = da[k], db[k]
        sc = max(np.abs(x).max(), 1e-30)
        e = np.abs(x - y) / sc            # (tile, lane, r)
        bad_t = np.nonzero(e.max((1, 2)) > 1e-5)[0].tolist()
        bad_l = np.nonzero(e.max((0, 2)) > 1e-5)[0].tolist()
        print("stage %2d scale %.3g maxrel %.3g bad tiles %s bad lanes %s" % (
            k, sc, e.max(), bad_t, bad_l[:24]), flush=True)
    print("out dtau maxrel", float(np.abs(oa - ob).max() / np.abs(oa).max()))






def local(a, b):
    """Wave-local e3ᵀ tiles (stage 31: output L, 32: its σ tiles): build a = SPLIT 8 dumping
    wave 4 (global tiles 4, 12), build b = SPLIT 4 dumping wave 2 (global tiles 4, 5, 12, 13)."""
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(W[k]).to(dev) for k in synth.state_dict_keys()])
    n = 16
    xp = torch.from_numpy(synth.make_pairs(n, 3)).to(dev).contiguous()
    B = torch.from_numpy(synth.make_B(3)).to(dev).contiguous()
    da, _ = run(a, packed, xp, B, n)
    db, _ = run(b, packed, xp, B, n)
    # stage 40 + w: wave w's e3ᵀ output tiles (SPLIT 8: global c*8 + w; SPLIT 4: c*8 + 2w + t)
    for w in range(8):
        for c in range(2):
            x = da[40 + w, c]
            y = db[40 + w // 2, c * 2 + w % 2]
            e = np.abs(x - y) / max(np.abs(y).max(), 1e-30)
            print("wave %d col %d: maxrel %.3g bad lanes %s" % (
                w, c, e.max(), np.nonzero(e.max(1) > 1e-5)[0].tolist()[:8]), flush=True)
    x, y = da[24], db[24]
    e = np.abs(x - y) / max(np.abs(y).max(), 1e-30)
    print("stage 24 (exchanged) bad tiles", np.nonzero(e.max((1, 2)) > 1e-5)[0].tolist())


if __name__ == "__main__":
    if sys.argv[1] == "--local":
        local(*sys.argv[2:4])
    else:
        main(*sys.argv[1:3])
