"""W4A16 decode GEMM (csrc/kernels/gemm_w4.hip) against the bf16 path linear() / mlp_gate_up() would take,
per batch size and Qwen2-7B projection, interleaved in one process on cold weights (copies rotate past the
Infinity Cache).  One JSON line per (shape, arm): median us.

usage: python scripts/w4_probe.py [--ms 1,8,16,32,64,96,128,192,256] [--reps 15] [--graph] [--out f.jsonl]

--graph: each arm is captured in a hipGraph of ``--calls`` back-to-back launches (as the decode step is
served) and timed per launch over replays; without it every launch is timed alone between events, which
adds the host launch gap to every arm.
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
from githubrepostorag_amd.ops import w4 as W  # noqa: E402
from githubrepostorag_amd.ops.linear import enable_tuned_gemms, linear  # noqa: E402

Q7 = {"qkv": (4608, 3584, False), "o": (3584, 3584, False), "gate_up": (37888, 3584, True),
      "down": (3584, 18944, False)}


def timeit(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,8,16,32,64,96,128,192,256")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--out", default=None)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--calls", type=int, default=12)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    enable_tuned_gemms()
    fh = open(args.out, "a") if args.out else None
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, (N, K, silu) in Q7.items():
        ncopy = max(1, min(6, (600 << 20) // (N * K * 2) + 1))
        ws = [((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16).to(dev) for _ in range(ncopy)]
        qs = [W.W4Linear.quantize(w, silu=silu) for w in ws]
        for q in qs:
            q.release_codes()
        for M in map(int, args.ms.split(",")):
            x = ((torch.rand(M, K, generator=g) * 2 - 1)).to(torch.bfloat16).to(dev)
            it = {"i": 0}
            arms = {}

            def bf16():
                w = ws[it["i"] % ncopy]
                it["i"] += 1
                return G.mlp_gate_up(x, w) if silu else linear(x, w)
            arms["bf16_dispatch"] = bf16
            need = -(-M // 16)
            for mt in (4, 8, 12, 16):
                if mt < need:
                    continue
                tiles = N // 128
                for ks in ([1] if silu else sorted({1, W.w4_ksplit(K, max(1, 256 // tiles)), W.w4_ksplit(K, 4)})):
                    G.WS.reserve(dev, ks * M * N)

                    def f(mt=mt, ks=ks):
                        q = qs[it["i"] % ncopy]
                        it["i"] += 1
                        return W.gemm_w4(x, q, plan_=(mt, 4, ks))
                    arms[f"w4_mt{mt}_ks{ks}"] = f
                break  # the smallest tiling that covers M (larger ones only pad rows)
            for f in arms.values():
                f(); f()
            torch.cuda.synchronize()
            times = {k: [] for k in arms}
            if args.graph:
                graphs = {}
                side = torch.cuda.Stream(dev)
                for k, f in arms.items():
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.stream(side):
                        with torch.cuda.graph(gr, stream=side):
                            for _ in range(args.calls):
                                f()
                    graphs[k] = gr
                torch.cuda.synchronize()
                for _ in range(args.reps):
                    for k, gr in graphs.items():
                        times[k] += [t / args.calls for t in timeit(gr.replay, 1)]
                del graphs
            else:
                for _ in range(args.reps):
                    for k, f in arms.items():
                        times[k] += timeit(f, 1)
            best = min(times, key=lambda k: statistics.median(times[k]))
            for k, ts in times.items():
                row = {"proj": name, "M": M, "N": N, "K": K, "arm": k, "graph": args.graph, "med_us": round(statistics.median(ts), 1),
                       "best": k == best}
                line = json.dumps(row)
                print(line, flush=True)
                if fh:
                    fh.write(line + "\n")
    if fh:
        fh.close()


if __name__ == "__main__":
    main()
