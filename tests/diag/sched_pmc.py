"""Diagnostic: run the τ+∇τ entry point at 1M pairs under each schedule (6 launches each) so a
rocprofv3 --pmc pass can compare field_kernel (16-pair) and wide_field_kernel (32-pair).

    rocprofv3 --kernel-trace --pmc <counters> -- python tests/diag/sched_pmc.py
    python tests/diag/sched_pmc.py --parse <outdir>
"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-ntfields_amd")]


def run():
    import torch
    from pntf import ops, synth
    dev = torch.device("cuda:0")
    W = synth.make_weights(0)
    packed = ops.pack_weights([torch.from_numpy(v).to(dev) for v in W.values()])
    n = 1 << 20
    xp = torch.from_numpy(synth.make_pairs(n, 3, seed=1000)).to(dev)
    Bt = torch.from_numpy(synth.make_B_table(10, 3)).to(dev)
    env = torch.from_numpy(synth.make_env_ids(n, 10)).to(dev)
    for sched in ("wave_tile", "wide_tile"):
        for _ in range(6):
            ops.tau_grad(packed, xp, Bt, env, dim=3, schedule=sched)
        torch.cuda.synchronize()


def parse(out):
    rows = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(glob.glob(out + "/**/run_counter_collection.csv", recursive=True)[0])):
        if "field_kernel" in r["Kernel_Name"]:
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
            names[d] = "wide" if "wide" in r["Kernel_Name"] else "narrow"
    dur = {}
    for r in csv.DictReader(open(glob.glob(out + "/**/run_kernel_trace.csv", recursive=True)[0])):
        if "field_kernel" in r["Kernel_Name"]:
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for kind in ("narrow", "wide"):
        ids = sorted(d for d in rows if names[d] == kind)[1:]
        m = {k: sum(rows[d][k] for d in ids) / len(ids) for k in rows[ids[0]]}
        t = sum(dur[d] for d in ids) / len(ids)
        ghz = m.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9
        simd = 1024 * t * ghz * 1e9
        print("%-7s %8.3f ms %6.3f GHz  " % (kind, t * 1e3, ghz) + "  ".join(
            "%s=%.1f%%" % (k[3:], 100 * (v if k.startswith("SQ_VALU_MFMA") else 4 * v) / simd)
            for k, v in sorted(m.items()) if k != "GRBM_GUI_ACTIVE"))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run()
