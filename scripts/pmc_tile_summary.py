"""Derived tile-GEMM counter figures from scripts/pmc_tile.sh output directories.

python scripts/pmc_tile_summary.py gpurun_out/pmc_TAG [...]

Counters are taken per dispatch, per pass (a counter repeated in two passes, e.g. GRBM_GUI_ACTIVE, is read from
each pass on its own, never summed across them) and the per-dispatch median is reported.  Clock = GRBM_GUI_ACTIVE /
8 XCDs / dispatch time; MFMA busy is SQ_VALU_MFMA_BUSY_CYCLES over (clock cycles x 256 CUs), i.e. percent of
CU-cycles (400 % = all four SIMDs busy), also shown per SIMD.
"""
import collections
import csv
import glob
import statistics
import sys

KERNEL = "gemm_tile_kernel"


def passes(out):
    per = []
    for d in sorted(glob.glob(out + "/p[0-9]*")):
        vals = collections.defaultdict(lambda: collections.defaultdict(float))
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if KERNEL not in r["Kernel_Name"]:
                    continue
                vals[r["Counter_Name"]][r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
        dur = []
        for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if KERNEL in r["Kernel_Name"]:
                    dur.append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
        per.append((vals, dur))
    return per


def main():
    for out in sys.argv[1:]:
        wall = open(out + "/wall.log").read().strip().splitlines()
        print("==", out + ":", wall[-1] if wall else "")
        med = {}
        gui_t = []
        for vals, dur in passes(out):
            t = statistics.median(dur) if dur else float("nan")
            for c, by in vals.items():
                med.setdefault(c, statistics.median(by.values()))
            if "GRBM_GUI_ACTIVE" in vals:
                gui_t.append((statistics.median(vals["GRBM_GUI_ACTIVE"].values()), t))
        gui, t = gui_t[0]
        cyc = gui / 8
        print("   median profiled dispatch %.1f us" % t)
        print("   clock %.2f GHz (GRBM_GUI_ACTIVE / 8 / time)" % (cyc / t / 1e3))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
            g2, _ = gui_t[-1]
            busy = med["SQ_VALU_MFMA_BUSY_CYCLES"] / (g2 / 8 * 256) * 100
            print("   MFMA busy %.1f %% of CU-cycles (256 CUs) = %.1f %% per SIMD" % (busy, busy / 4))
        wc = med.get("SQ_WAVE_CYCLES")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if wc and c in med:
                print("   %-22s %5.1f %% of wave-cycles" % (c, med[c] / wc * 100))
        for c in ("SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT",
                  "FETCH_SIZE", "TCC_HIT_sum", "SQ_WAVES", "SQ_BUSY_CYCLES"):
            if c in med:
                print("   %-22s %.4g" % (c, med[c]))


if __name__ == "__main__":
    main()
