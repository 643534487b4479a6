"""Summarise pmc_variants.sh output per variant (mean over each variant's 5 timed launches)."""
import collections
import csv
import glob
import sys

out, names = sys.argv[1], sys.argv[2:]
rows = collections.defaultdict(dict)
for r in csv.DictReader(open(glob.glob(out + "/**/run_counter_collection.csv", recursive=True)[0])):
    if "field_kernel" in r["Kernel_Name"]:
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
dur = {}
kt = glob.glob(out + "/**/run_kernel_trace.csv", recursive=True)
if kt:
    for r in csv.DictReader(open(kt[0])):
        if "field_kernel" in r["Kernel_Name"]:
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
ids = sorted(rows)[1:]            # drop the shipped-kernel reference launch
keys = sorted(rows[ids[0]])
print("%-10s %8s %7s " % ("variant", "ms", "GHz") + " ".join("%14s" % k[3:17] for k in keys))
for i, nm in enumerate(names):
    sel = ids[6 * i + 1: 6 * i + 6]
    m = {k: sum(rows[d][k] for d in sel) / len(sel) for k in rows[sel[0]]}
    t = sum(dur.get(d, 0) for d in sel) / len(sel)
    ghz = m["GRBM_GUI_ACTIVE"] / 8 / t / 1e9 if t and "GRBM_GUI_ACTIVE" in m else 0
    # per-SIMD-cycle fractions: SQ_* wave/inst counters count quad-cycles per wave (x4),
    # SQ_VALU_MFMA_* count cycles; 1024 waves = one per SIMD
    simd = 1024 * t * ghz * 1e9
    vals = []
    for k in keys:
        v = m[k]
        if k == "GRBM_GUI_ACTIVE":
            vals.append("%14.4g" % v)
        elif k.startswith("SQ_VALU_MFMA") and simd:
            vals.append("%13.1f%%" % (100 * v / simd))
        elif simd:
            vals.append("%13.1f%%" % (100 * 4 * v / simd))
        else:
            vals.append("%14.4g" % v)
    print("%-10s %8.3f %7.3f " % (nm, t * 1e3, ghz) + " ".join(vals))
