"""C2 vs headline per-tile cost: the wide τ+∇τ kernel at 262 144 pairs
(8 wide tiles per wave) and 1 048 576 pairs (32 per wave), single B and the 10-env table,
launched back to back with HIP events per launch on the launch stream, plus a 262 144-pair run
after a warm 1M run (clock state).  Run under rocprofv3 --kernel-trace --stats to get the
per-launch kernel durations.

    python tools/c2_probe.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pntf import ops, synth  # noqa: E402


def events(fn, reps):
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) for a, b in evs])


def main(reps=20):
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    B = torch.from_numpy(synth.make_B(3, seed=1)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
    cases = {}
    for n in (262144, 1 << 20):
        xp = torch.from_numpy(synth.make_pairs(n, 3, seed=2)).to(dev)
        env = torch.from_numpy(synth.make_env_ids(n, 10)).to(dev)
        cases[n] = (xp, env)
    out = []
    for n in (262144, 1 << 20, 262144):
        xp, env = cases[n]
        for tag, fn in (("1env", lambda: ops.tau_grad(packed, xp, B, dim=3)),
                        ("10env", lambda: ops.tau_grad(packed, xp, Bt, env, dim=3))):
            fn()
            torch.cuda.synchronize()
            ms = events(fn, reps)
            tiles_per_wave = n / 32 / (torch.cuda.get_device_properties(0).multi_processor_count * 4)
            out.append("n=%7d %-5s  mean %.3f ms  min %.3f  max %.3f  per wave-tile %.4f ms  "
                       "pairs/s %.3e" % (n, tag, ms.mean(), ms.min(), ms.max(),
                                         ms.mean() / tiles_per_wave, n / ms.mean() * 1e3))
            print(out[-1], flush=True)
    return out


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
