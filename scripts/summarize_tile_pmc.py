"""Per-dispatch averages of the tile-GEMM counter passes (scripts/pmc_tile.sh) and derived ratios.

python scripts/summarize_tile_pmc.py gpurun_out/pmc_tile_gu [...]
Derived: clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (CUs x
GRBM_GUI_ACTIVE / 8); wait shares of SQ_WAVE_CYCLES (quad-cycle units, all three counted alike).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(list)
    durs = []
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        if not os.path.isdir(p):
            continue
        per = defaultdict(float)
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "gemm_tile" not in r["Kernel_Name"]:
                    continue
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (did, c), v in per.items():
            vals[c].append(v)
        for f in glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "gemm_tile" in r["Kernel_Name"]:
                    durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    avg = {c: sum(v) / len(v) for c, v in vals.items()}
    return avg, sorted(durs)[len(durs) // 2] if durs else 0


def main():
    for d in sys.argv[1:]:
        avg, dur_ns = load(d)
        wall = open(os.path.join(d, "wall.log")).read().strip().splitlines()[-1]
        print(f"== {d}: {wall}")
        print(f"   median profiled dispatch {dur_ns / 1e3:.1f} us")
        g = avg.get("GRBM_GUI_ACTIVE", 0)
        if g and dur_ns:
            print(f"   clock {g / 8 / dur_ns:.2f} GHz (GRBM_GUI_ACTIVE / 8 / time)")
        mf = avg.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if mf and g:
            print(f"   MFMA busy {mf / (256 * g / 8) * 100:.1f} % of CU-cycles (256 CUs)")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in avg:
                    print(f"   {k:22s} {avg[k] / wc * 100:5.1f} % of wave-cycles")
        for k in ("SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT",
                  "SQ_ACTIVE_INST_VALU", "FETCH_SIZE", "TCC_HIT_sum", "SQ_WAVES", "SQ_BUSY_CYCLES"):
            if k in avg:
                print(f"   {k:22s} {avg[k]:.4g}")


if __name__ == "__main__":
    main()
