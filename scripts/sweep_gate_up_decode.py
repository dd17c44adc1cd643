"""Fused gate/up SwiGLU GEMM at 257-512-row decode batches: owned tile kernel schedules.

At M = 257..512 the interleaved gate/up weight (Qwen2-7B: N = 37888, K = 3584) is 2 x 148 = 296
256x256 tiles: one full round on 256 CUs plus a 40-tile tail, so whole-tile scheduling runs ~2 rounds.
Times (CUDA events, median) the whole-tile schedule against K-splits (fp32 planes + the SwiGLU
reduce) and the tail-only stream-K round (sk < 0), checks each against the whole-tile output, and
prints one JSON line per (M, arm).

usage: python scripts/sweep_gate_up_decode.py [--n 37888 --k 3584]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.ops import gemm as G  # noqa: E402


def med_us(fn, reps=15):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=37888)
    ap.add_argument("--k", type=int, default=3584)
    ap.add_argument("--ms", default="288,320,384,448,512")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    N, K = a.n, a.k
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    big = torch.empty(256 << 20, dtype=torch.uint8, device=dev)  # flushes L2/MALL between reps
    for M in [int(m) for m in a.ms.split(",")]:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        arms = [(1, 0), (2, 0), (3, 0), (4, 0)]
        arms += [(1, -s) for s in (64, 96, 128, 160, 192, 256) if G.sk_ok(M, N, K, 1, -s)]
        arms = [ar for ar in arms if G.sk_ok(M, N, K, *ar)]
        ref = G.gemm_silu(x, w, ksplit=1, sk=0)
        for ks, sk in arms:
            G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
            if sk:
                G.WS.counters(dev)
            y = G.gemm_silu(x, w, ksplit=ks, sk=sk)
            err = (y.float() - ref.float()).abs().max().item()

            def run():
                big.zero_()
                G.gemm_silu(x, w, ksplit=ks, sk=sk, out=y)

            t = med_us(run)
            tz = med_us(lambda: big.zero_())
            print(json.dumps({"M": M, "N": N, "K": K, "ksplit": ks, "sk": sk, "us": round(t - tz, 1),
                              "maxdiff_vs_whole_tile": err}), flush=True)


if __name__ == "__main__":
    main()
