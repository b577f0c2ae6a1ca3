#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV (kernel_stats.csv) into a markdown table."""
import csv
import sys


def main(path, title, out):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {title}", "", f"Total GPU kernel time: {tot / 1e6:.1f} ms", "",
             "| kernel | calls | avg us | total ms | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:40]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:20]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
