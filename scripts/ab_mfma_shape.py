"""Same-process interleaved A/B of tile GEMM arms (csrc/kernels/gemm_tile.hip): ``mf16`` (v_mfma_f32_16x16x32_bf16,
the 12/4/8/0-read phase schedule), ``mf32`` (v_mfma_f32_32x32x16_bf16 at the same 64x32 quadrant per wave) and
``s1`` (16x16x32 with the balanced 8/4/8/4-read schedule, ``SCHED`` 1) on the bench's
prefill shapes with random operands (cdna guide §5.4 rule 28 / MI355X_MICROARCH 'DVFS give-back' item 7:
rank by wall on random data).  Each arm is run back to back for >= 0.5 s per round so the clock settles.

python scripts/ab_mfma_shape.py --M 7104 --rounds 5 --arms mf16,s1 --out gpurun_out/ab_mfma.json
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
    ap.add_argument("--arms", default="mf16,mf32")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    arms = a.arms.replace(":", ",").split(",")  # ':' too (scripts/gpu_run.sh turns ',' into spaces)

    def use(arm):
        G.set_mfma(32 if arm == "mf32" else 16)
        G.set_sched(2 if arm == "s2" else 1 if arm == "s1" else 0)
    dev = torch.device("cuda")
    res = {}
    for M in a.M:
        for name in a.shapes.replace(":", ",").split(","):
            N, K = SHAPES[name]
            silu = name == "gate_up"
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
            ks, sk = G.schedule(M, N, K, silu)
            G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
            fn = (lambda: G.gemm_silu(x, w, ksplit=ks, sk=sk)) if silu else (lambda: G.gemm(x, w, ksplit=ks, sk=sk))
            outs, times = {}, {arm: [] for arm in arms}
            for arm in arms:
                use(arm)
                outs[arm] = fn().float()
            for _ in range(a.rounds):
                for arm in arms:
                    use(arm)
                    for _ in range(5):
                        fn()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.reps):
                        fn()
                    e.record()
                    e.synchronize()
                    times[arm].append(s.elapsed_time(e) * 1e3 / a.reps)
            use("mf16")
            fl = 2 * M * N * K
            r = {arm: {"median_us": round(statistics.median(t), 1), "min_us": round(min(t), 1),
                       "TF_s_median": round(fl / statistics.median(t) / 1e6, 1)} for arm, t in times.items()}
            r["sched"] = [ks, sk]
            b0 = arms[0]
            for arm in arms[1:]:
                r[f"max_abs_diff_{arm}_vs_{b0}"] = round((outs[arm] - outs[b0]).abs().max().item(), 5)
                r[f"bitwise_equal_{arm}_vs_{b0}"] = bool(torch.equal(outs[arm], outs[b0]))
                r[f"speedup_{arm}_over_{b0}"] = round(statistics.median(times[b0]) / statistics.median(times[arm]), 4)
            res[f"{name}_M{M}"] = r
            print(name, M, json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
