#!/usr/bin/env python3
"""GPU idle gaps from a rocprofv3 kernel trace (run_kernel_trace.csv): host stalls show up as gaps
between consecutive kernels.  Usage: trace_gaps.py <kernel_trace.csv> [min_gap_ms]"""
import csv
import sys


def main(path, min_ms=0.5):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70])
                for r in csv.DictReader(open(path)))
    t0, end = ev[0][0], ev[0][1]
    busy = ev[0][1] - ev[0][0]
    gaps = []
    for s, e, n in ev[1:]:
        if s - end > min_ms * 1e6:
            gaps.append(((end - t0) / 1e6, (s - end) / 1e6, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = (end - t0) / 1e6
    print(f"span {span:.1f} ms, busy {busy / 1e6:.1f} ms ({100 * busy / 1e6 / span:.1f}%), "
          f"{len(gaps)} gaps > {min_ms} ms totalling {sum(g[1] for g in gaps):.1f} ms")
    # every inter-kernel gap (host stalls between graph replays show up as many short gaps), by size
    allg = []
    end = ev[0][1]
    for s, e, n in ev[1:]:
        if s > end:
            allg.append((s - end) / 1e6)
        end = max(end, e)
    for lo, hi in ((0, 0.005), (0.005, 0.02), (0.02, 0.1), (0.1, 0.5), (0.5, 5), (5, 1e9)):
        sel = [g for g in allg if lo <= g < hi]
        print(f"  gaps in [{lo}, {hi}) ms: {len(sel)} totalling {sum(sel):.1f} ms")
    for at, g, n in gaps:
        print(f"  at {at:9.1f} ms  gap {g:8.2f} ms  before {n}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5)
