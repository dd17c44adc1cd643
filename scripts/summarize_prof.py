"""Summarize a rocprofv3 --kernel-trace --stats CSV (run_kernel_stats.csv) by kernel family.

usage: python scripts/summarize_prof.py <kernel_stats.csv> [title]
"""
import csv
import sys

FAMILIES = [
    ("hipblaslt (library GEMM)", lambda n: "Cijk" in n),
    ("gemm_tile (owned 256x256 MFMA GEMM)", lambda n: "gemm_tile" in n),
    ("gemm_decode / gemm_w4 (owned decode GEMMs)", lambda n: "gemm_dec" in n or "gemm_w4" in n),
    ("splitk_reduce", lambda n: "splitk_reduce" in n),
    ("other owned gemm (skinny/stream)", lambda n: "gemm_skinny" in n or "gemm_stream" in n),
    ("attention (prefill+decode+combine)", lambda n: "attn" in n or "paged_decode" in n),
    ("ivf/topk", lambda n: "topk" in n.lower() or "ivf" in n),
    ("norms", lambda n: "norm" in n),
    ("rope/kv", lambda n: "rope" in n),
    ("sampling", lambda n: "samp" in n),
]


def main(path, title=""):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    if title:
        print(title)
    print(f"total kernel time {tot / 1e6:.1f} ms")
    for name, f in FAMILIES:
        s = sum(float(r["TotalDurationNs"]) for r in rows if f(r["Name"]))
        print(f"{name:44s} {s / 1e6:9.1f} ms {100 * s / tot:6.2f} %")
    print()
    for r in rows[:25]:
        print(f"{float(r['Percentage']):6.2f}% {float(r['TotalDurationNs']) / 1e6:9.2f}ms n={r['Calls']:>6} "
              f"avg={float(r['AverageNs']) / 1e3:8.1f}us {r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], " ".join(sys.argv[2:]))
