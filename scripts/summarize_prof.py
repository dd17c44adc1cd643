"""Compact per-kernel summary of a rocprofv3 --stats kernel_stats.csv."""
import csv
import re
import sys


def short(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        return f"hipblaslt_{m.group(1) if m else '?'}"
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def main(path, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.1f} ms")
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['Percentage']):6.2f}% {int(r['Calls']):7d} calls "
              f"{float(r['AverageNs']) / 1e3:9.1f} us  {short(r['Name'])}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
