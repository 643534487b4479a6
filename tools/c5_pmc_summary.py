"""Summarise the C5 planner profiles of tools/gpu_pass.sh's c5 step (gpurun_out/<src>_c5_stats, <src>_c5_pmc_*)
into profiles/<tag>_c5_kernel_stats.csv and profiles/<tag>_pmc_c5_planner.json.

    python tools/c5_pmc_summary.py --tag r03 [--kernel "plan_quad_kernel<6, false>"]

Per launch (mean over the profiled dispatches).  Weight-stream bytes are derived from the
TCP->TCC read requests (128 B each on gfx950: 4.33 MB per tile-step x tile-steps checks it);
MFMA-executed FLOP from SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 (one v_mfma_f32_4x4x1_16b_f32 =
16 blocks x 4x4x1 x 2); the stall split from SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md PMC notes)."""
import argparse
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
WEIGHT_BYTES_PER_TILE_STEP = 2 * 540672 * 4      # both directions of the quad stream


def counters(tag, kernel, pre=""):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(OUT, pre + "c5_pmc_%s" % tag, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r03")
    ap.add_argument("--kernel", default="plan_quad_kernel<6, false>")
    ap.add_argument("--unit", default="plan_quad_d6")
    ap.add_argument("--src", default="", help="gpurun_out prefix of a tools/gpu_pass.sh pass "
                                              "(e.g. r05e: reads r05e_c5_stats, r05e_c5_pmc_*)")
    a = ap.parse_args()
    a.src = a.src + "_" if a.src else ""
    sys.path.insert(0, os.path.join(ROOT, "p-ntfields_amd"))
    from pntf import _lib
    stats = glob.glob(os.path.join(OUT, a.src + "c5_stats", "*kernel_stats.csv"))[0]
    shutil.copy(stats, os.path.join(PROF, "%s_c5_kernel_stats.csv" % a.tag))
    avg_ns = [float(r["AverageNs"]) for r in csv.DictReader(open(stats))
              if a.kernel in r["Name"]][0]
    probe = json.loads([ln for ln in open(os.path.join(OUT, a.src + "c5_stats.log"))
                        if ln.startswith("{")][-1])
    sq, tcc, lds, fetch = (counters(t, a.kernel, a.src) for t in ("sq", "tcc", "lds", "fetch"))
    clock = tcc["GRBM_GUI_ACTIVE"] / 8 / (avg_ns * 1e-9)
    simd_cycles = 1024 * avg_ns * 1e-9 * clock
    mfma = sq["SQ_INSTS_VALU_MFMA_MOPS_F32"]
    waves = lds["SQ_WAVES"]
    # 20 480 v_mfma_f32_4x4x1_16b_f32 per tile-step (both sweeps), whatever the wave count
    tile_steps = mfma / 20480.0
    req_bytes = tcc["TCP_TCC_READ_REQ_sum"] * 128
    wc = sq["SQ_WAVE_CYCLES"]
    j = {
        "kernel": a.kernel, "unit": a.unit, "unit_hash": _lib.build_info()[a.unit],
        "workload": "C5: 1024 arm queries (dim 6), <= 199 steps, per-query freeze; "
                    "tools/c5_probe.py",
        "avg_duration_ns": avg_ns, "probe": probe,
        "effective_clock_GHz": clock / 1e9,
        "tile_steps_per_launch": tile_steps,
        "tile_steps_check": "MFMA count / 20480 per tile-step (%d waves per tile)" % round(waves / 256),
        "weight_stream_bytes_per_launch_from_TCP_TCC_READ_REQ_x128": req_bytes,
        "weight_stream_bytes_expected": tile_steps * WEIGHT_BYTES_PER_TILE_STEP,
        "l2_hit_rate": tcc["TCC_HIT_sum"] / (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]),
        "fabric_fetch_bytes_x2": fetch["FETCH_SIZE"] * 1024 * 2,
        "per_CU_stream_GBps_avg_over_launch": req_bytes / (avg_ns * 1e-9) / 256 / 1e9,
        "mfma_instructions": mfma, "mfma_flops_executed": mfma * 512,
        "mfma_busy_frac_of_simd_cycles": sq["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
        "mfma_busy_cycles_per_instruction": sq["SQ_VALU_MFMA_BUSY_CYCLES"] / mfma,
        "wave_cycles_split": {"wait_any": sq["SQ_WAIT_ANY"] / wc,
                              "wait_inst_any": sq["SQ_WAIT_INST_ANY"] / wc,
                              "active_inst_any": sq["SQ_ACTIVE_INST_ANY"] / wc,
                              "wait_inst_lds": sq["SQ_WAIT_INST_LDS"] / wc},
        "instructions_per_wave_per_tile_step": {
            k: lds[k] / waves / (tile_steps / 256)
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS")},
        "lds_bank_conflict_frac": lds["SQ_LDS_BANK_CONFLICT"] / lds["SQ_LDS_IDX_ACTIVE"],
        "raw": {"sq": sq, "tcc": tcc, "lds": lds, "fetch": fetch},
    }
    p = os.path.join(PROF, "%s_pmc_c5_planner.json" % a.tag)
    with open(p, "w") as fh:
        json.dump(j, fh, indent=1)
    print(json.dumps({k: v for k, v in j.items() if k != "raw"}, indent=1))


if __name__ == "__main__":
    main()
