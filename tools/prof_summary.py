"""Summarise rocprofv3 outputs (gpurun_out/) into committed profiles/ files.

    python tools/prof_summary.py --tag r02 --pairs 1048576 [--kernel wide_field_kernel<3, 1>]

Reads gpurun_out/prof_stats/run_kernel_stats.csv (kernel-trace --stats) and the separate
PMC passes gpurun_out/pmc_{fetch,write,mfma}/run_counter_collection.csv, applies the gfx950
corrections of MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of 16-B/lane streaming
reads: doubled; WRITE_SIZE exact for 16-B/lane stores; both in KiB), and writes
profiles/<tag>_kernel_stats.csv and profiles/<tag>_pmc_tau_grad.json; the latter is also
copied to profiles/pmc_tau_grad.json, which bench.py reads for roofline.traffic.
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
SRC = ""                 # gpurun_out prefix (--src)
PROF = os.path.join(ROOT, "profiles")


def counters(run, kernel):
    path = os.path.join(OUT, SRC + run, "run_counter_collection.csv")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--pairs", type=int, default=1 << 20)
    ap.add_argument("--kernel", default="wide_field_kernel<3, 1, true>")
    ap.add_argument("--unit", default="wide_d3_k1", help="build unit of --kernel")
    ap.add_argument("--src", default="", help="gpurun_out prefix of a tools/gpu_pass.sh pass "
                                              "(e.g. r05e: reads r05e_prof_stats, r05e_pmc_*)")
    a = ap.parse_args()
    global SRC
    SRC = a.src + "_" if a.src else ""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))
    from pntf import _lib
    unit_hash = _lib.build_info()[a.unit]      # the library these profiles were taken from
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, SRC + "prof_stats", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, "%s_kernel_stats.csv" % a.tag))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if a.kernel in r["Name"]:
            avg_ns = float(r["AverageNs"])
    fetch, nf = counters("pmc_fetch", a.kernel)
    write, nw = counters("pmc_write", a.kernel)
    mfma, nm = counters("pmc_mfma", a.kernel)
    fetch_b = fetch["FETCH_SIZE"] * 1024 * 2
    write_b = write["WRITE_SIZE"] * 1024
    flops = mfma["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512
    # the split-bf16 layers: six bf16 products per fp32 product
    flops_bf16 = mfma.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
    clock = mfma["GRBM_GUI_ACTIVE"] / 8 / (avg_ns * 1e-9) / 1e9
    simd_cycles = 1024 * avg_ns * 1e-9 * clock * 1e9
    j = {
        "kernel": a.kernel, "unit": a.unit, "unit_hash": unit_hash,
        "pairs_per_launch": a.pairs, "avg_duration_ns": avg_ns,
        "FETCH_SIZE_KiB": fetch["FETCH_SIZE"], "WRITE_SIZE_KiB": write["WRITE_SIZE"],
        "fetch_bytes_corrected_x2": fetch_b, "write_bytes": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "hbm_bytes_per_pair": (fetch_b + write_b) / a.pairs,
        "hbm_GBps": (fetch_b + write_b) / (avg_ns * 1e-9) / 1e9,
        "mfma_flops_per_launch": flops, "mfma_flops_per_pair": flops / a.pairs,  # fp32 MFMA
        "mfma_bf16_flops_per_launch": flops_bf16,
        "mfma_fp32_equivalent_flops_per_pair": (flops + flops_bf16 / 6) / a.pairs,
        "mfma_busy_cycles": mfma["SQ_VALU_MFMA_BUSY_CYCLES"],
        "mfma_busy_frac_of_simd_cycles": mfma["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
        "effective_clock_GHz": clock, "sq_waves": mfma.get("SQ_WAVES"),
        "dispatches_averaged": {"fetch": nf, "write": nw, "mfma": nm},
        "notes": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts half of 16-B/lane "
                 "streaming reads); Infinity-Cache hits are counted as fetches.",
    }
    p = os.path.join(PROF, "%s_pmc_tau_grad.json" % a.tag)
    with open(p, "w") as fh:
        json.dump(j, fh, indent=1)
    shutil.copy(p, os.path.join(PROF, "pmc_tau_grad.json"))
    print(json.dumps(j, indent=1))
    if os.path.exists(os.path.join(OUT, SRC + "pmc_stall", "run_counter_collection.csv")):
        st, ns = counters("pmc_stall", a.kernel)
        k = {"kernel": a.kernel, "unit": a.unit, "unit_hash": unit_hash,
             "dispatches": ns.get("SQ_WAIT_ANY"), **{c: st[c] for c in sorted(st)},
             "wait_any_frac_of_wave_cycles": st["SQ_WAIT_ANY"] / st["SQ_WAVE_CYCLES"],
             "wait_inst_any_frac_of_wave_cycles": st["SQ_WAIT_INST_ANY"] / st["SQ_WAVE_CYCLES"],
             "notes": "SQ_WAIT_ANY: wave parked on s_waitcnt (memory); SQ_WAIT_INST_ANY also "
                      "counts waits for the MFMA pipe, which an MFMA-bound kernel spends most "
                      "cycles in."}
        with open(os.path.join(PROF, "%s_pmc_stall_tau_grad.json" % a.tag), "w") as fh:
            json.dump(k, fh, indent=1)
        print("stall: SQ_WAIT_ANY %.4f of wave-cycles" % k["wait_any_frac_of_wave_cycles"])


if __name__ == "__main__":
    main()
