"""Busy time vs idle gaps of a rocprofv3 --kernel-trace run (kernel_trace.csv):

    python tools/trace_gaps.py <kernel_trace.csv> [first_kernel_regex]

Prints the span from the first to the last kernel, the time some kernel was running (the
union of [start, end) intervals), the idle gaps between kernels, and the top kernels by time.
With a regex, the span starts at the first kernel whose name matches (skip set-up)."""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if len(sys.argv) > 2:
        pat = re.compile(sys.argv[2])
        i = next(i for i, k in enumerate(ks) if pat.search(k[2]))
        ks = ks[i:]
    busy, cur_s, cur_e, gaps = 0, ks[0][0], ks[0][1], []
    for s, e, _ in ks[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = ks[-1][1] - ks[0][0]
    gaps.sort()
    print("kernels %d  span %.3f ms  busy %.3f ms  idle %.3f ms (%.1f %%)  gaps: n %d, median "
          "%.1f us, p90 %.1f us, max %.1f us" % (
              len(ks), span / 1e6, busy / 1e6, (span - busy) / 1e6, 100.0 * (span - busy) / span,
              len(gaps), gaps[len(gaps) // 2] / 1e3 if gaps else 0,
              gaps[int(len(gaps) * 0.9)] / 1e3 if gaps else 0, gaps[-1] / 1e3 if gaps else 0))


if __name__ == "__main__":
    main()
