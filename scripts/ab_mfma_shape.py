"""Same-process interleaved A/B of the tile GEMM's two MFMA shapes (csrc/kernels/gemm_tile.hip ``Shape``:
v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 at the same 64x32 quadrant per wave) on the bench's
prefill shapes with random operands (cdna guide §5.4 rule 28 / MI355X_MICROARCH 'DVFS give-back' item 7:
rank by wall on random data).  Each arm is run back to back for >= 0.5 s per round so the clock settles.

python scripts/ab_mfma_shape.py --M 7104 --rounds 5 --out gpurun_out/ab_mfma.json
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv": (4608, 3584), "o": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[7104])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    for M in a.M:
        for name, (N, K) in SHAPES.items():
            silu = name == "gate_up"
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
            ks, sk = G.schedule(M, N, K, silu)
            G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
            fn = (lambda: G.gemm_silu(x, w, ksplit=ks, sk=sk)) if silu else (lambda: G.gemm(x, w, ksplit=ks, sk=sk))
            outs, times = {}, {16: [], 32: []}
            for mf in (16, 32):
                G.set_mfma(mf)
                outs[mf] = fn().float()
            for _ in range(a.rounds):
                for mf in (16, 32):
                    G.set_mfma(mf)
                    for _ in range(5):
                        fn()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.reps):
                        fn()
                    e.record()
                    e.synchronize()
                    times[mf].append(s.elapsed_time(e) * 1e3 / a.reps)
            G.set_mfma(16)
            fl = 2 * M * N * K
            r = {f"mf{mf}": {"median_us": round(statistics.median(t), 1), "min_us": round(min(t), 1),
                             "TF_s_median": round(fl / statistics.median(t) / 1e6, 1)} for mf, t in times.items()}
            r["sched"] = [ks, sk]
            r["max_abs_diff_32_vs_16"] = round((outs[32] - outs[16]).abs().max().item(), 5)
            r["speedup_32_over_16"] = round(statistics.median(times[16]) / statistics.median(times[32]), 4)
            res[f"{name}_M{M}"] = r
            print(name, M, json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
