"""Per-kernel table from rocprofv3 --pmc passes (scripts/pmc_kernels.sh).

Every pass runs the same workload, so counters are summed per kernel name
within a pass and joined across passes by name; durations come from the
kernel trace of the pass that collected the counter (PMC serialises
dispatches, so the times are per-kernel isolated times).

Derived columns:
  rd/wr GB/s   FETCH_SIZE / WRITE_SIZE (KiB) over the kernel time (HBM + MALL traffic seen by L2)
  bf16 TF/s    SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP over the kernel time
  %peak        bf16 TF/s over the 2.5 PFLOP/s dense bf16 MFMA peak of MI355X
  lds cf/inst  SQ_LDS_BANK_CONFLICT cycles per LDS instruction
"""
import csv
import glob
import os
import sys
from collections import defaultdict



def short(name: str, n: int = 90) -> str:
    """Kernel name without the argument list, cut to n characters."""
    return name.split("(")[0][:n]


def load(out):
    counters = defaultdict(float)  # (kernel, counter) -> sum
    dur_ns = defaultdict(float)  # kernel -> ns (max over passes)
    calls = defaultdict(int)
    for d in sorted(glob.glob(os.path.join(out, "p*"))):
        if not os.path.isdir(d):
            continue
        pdur = defaultdict(float)
        pcalls = defaultdict(set)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                counters[(k, r["Counter_Name"])] += float(r["Counter_Value"])
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                if did not in pcalls[k]:
                    pcalls[k].add(did)
                    if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                        pdur[k] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        if not any(pdur.values()):
            for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    pdur[short(r["Kernel_Name"])] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for k, v in pdur.items():
            dur_ns[k] = max(dur_ns[k], v)
        for k, s in pcalls.items():
            calls[k] = max(calls[k], len(s))
    return counters, dur_ns, calls


def main(out, top=30):
    c, dur, calls = load(out)
    names = sorted(dur, key=lambda k: -dur[k])[:top]
    hdr = f"{'kernel':60s} {'calls':>6s} {'ms':>8s} {'rd GB/s':>8s} {'wr GB/s':>8s} {'bf16 TF/s':>9s} " \
          f"{'%peak':>9s} {'lds cf/inst':>11s} {'waves':>9s}"
    print(hdr)
    for k in names:
        t = dur[k] * 1e-9
        g = lambda n: c.get((k, n), 0.0)  # noqa: E731
        rd = g("FETCH_SIZE") * 1024 / t / 1e9 if t else 0
        wr = g("WRITE_SIZE") * 1024 / t / 1e9 if t else 0
        tf = g("SQ_INSTS_VALU_MFMA_MOPS_BF16") * 512 / t / 1e12 if t else 0
        mf = 100.0 * tf / 2500.0
        lds = g("SQ_INSTS_LDS")
        cf = g("SQ_LDS_BANK_CONFLICT") / lds if lds else 0
        print(f"{k[:60]:60s} {calls[k]:6d} {dur[k] / 1e6:8.2f} {rd:8.0f} {wr:8.0f} {tf:9.1f} {mf:9.1f} {cf:11.3f} "
              f"{g('SQ_WAVES'):9.0f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
