#!/usr/bin/env python3
"""Per-call-site kernel times from a rocprofv3 kernel trace (run_kernel_trace.csv).

One kernel name covers several call sites (hipBLASLt's ``Cijk_*`` runs o, down and lm_head; gemm4w's
instances run several shapes), so a dispatch is keyed by (kernel, the kernel before it on the same queue):
in the decode step o follows the attention kernel, down follows gate|up, lm_head follows the last down.
Prints calls, median, mean, p10 and p90 per key, sorted by total time.

Usage: trace_shapes.py <kernel_trace.csv> [top]"""
import csv
import statistics
import sys


def short(name: str) -> str:
    name = name.split("(")[0]
    if name.startswith("void "):
        name = name[5:]
    if "Cijk_" in name:
        return "Cijk_" + ("SK" if "_SK" in name else "") + name.split("_MT")[1][:12] if "_MT" in name else "Cijk"
    return name[:60]


def main(path: str, top: int = 30) -> None:
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(path)))
    by = {}
    prev = ""
    for s, e, n in ev:
        k = (short(n), prev)
        by.setdefault(k, []).append((e - s) / 1e3)
        prev = short(n)
    tot = sum(sum(v) for v in by.values())
    rows = sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]
    print(f"total {tot / 1e3:.1f} ms over {len(ev)} dispatches")
    print("| kernel | after | calls | median us | mean us | p10 | p90 | total ms | % |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|")
    for (k, p), v in rows:
        v = sorted(v)
        print(f"| `{k}` | `{p}` | {len(v)} | {statistics.median(v):.1f} | {statistics.fmean(v):.1f} | "
              f"{v[len(v) // 10]:.1f} | {v[(9 * len(v)) // 10]:.1f} | {sum(v) / 1e3:.1f} | {100 * sum(v) / tot:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
