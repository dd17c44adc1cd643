"""qkv / o projections of Qwen2-7B at 129-224 decode rows as deferred split-K planes (what the decoder runs):
the decode kernel's current plan (ops/gemm.py dec_plan) against K-split / wave-count variants, hipGraph-timed
over weight copies that exceed the Infinity Cache (cold, as in serving).

usage: python scripts/sweep_dec_mid.py [--ms 144,176,192,224] [--out f.json]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv": (4608, 3584), "o": (3584, 3584)}


def graph_us(fn, copies, reps=3):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for w in copies[:2]:
            fn(w)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for w in copies:
            fn(w)
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / len(copies))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="144,176,192,224")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = {}
    for name, (N, K) in SHAPES.items():
        copies = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(12)]
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            base = G.dec_plan(M, N, K)
            arms = {"current": base}
            if base is not None:
                mt = base[0]
                for nwv in (4, 5, 8):
                    for ks in (7, 14, 28):
                        if N % (16 * nwv * 2) == 0 and (mt, nwv, 2) in G.DEC_VARIANTS:
                            arms[f"mt{mt}_w{nwv}_ks{ks}"] = (mt, nwv, 2, ks)
            row = {}
            for arm, plan in arms.items():
                if plan is None:
                    continue
                how = ("decode", G.dec_ksplit(K, plan[3]), plan)
                try:
                    row[arm] = round(graph_us(lambda w, how=how: G.gemm_deferred(x, w, how), copies), 2)
                except Exception as e:  # a plan the launcher refuses
                    row[arm] = str(e)[:80]
            row["plan"] = list(base) if base else None
            res[f"{name}_M{M}"] = row
            print(name, M, row, flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
