"""Time one GEMM shape under every owned schedule the launcher accepts (K-splits,
stream-K grids) against the library, interleaved in one process on the same
random operands (cdna guide §5.4 rules 24/25); weights rotate over copies that
exceed the Infinity Cache so decode-sized GEMMs are timed cold, as served.

usage: python scripts/gemm_probe.py --shapes 512:4608:3584,512:37888:3584:silu [--reps 15] [--out f.jsonl]
One JSON line per (shape, schedule): median / min us and TF/s.
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
from githubrepostorag_amd.ops.linear import enable_tuned_gemms  # noqa: E402


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


def schedules(M, N, K, silu):
    ncu = G._num_cus()
    kt = K // 64
    out = [(1, 0)]
    for ks in (2, 3, 4, 5, 6, 7, 8, 9, 12, 16):
        if G.sk_ok(M, N, K, ks, 0) and ks <= kt // 2:
            out.append((ks, 0))
    tiles = -(-M // 256) * -(-N // 256)
    tail = tiles % ncu
    for sk in (ncu, -ncu, ncu // 2, -ncu // 2, 192, -192, -tail, -2 * tail, -4 * tail):
        if sk and abs(sk) <= ncu and G.sk_ok(M, N, K, 1, sk):
            out.append((1, sk))
    for s_ in (2, 3, 4):  # K-aligned tail splits, more stream-K workgroups than CUs allowed
        if tail and G.sk_ok(M, N, K, 1, -s_ * tail):
            out.append((1, -s_ * tail))
    return list(dict.fromkeys(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", required=True)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-lib", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    enable_tuned_gemms()
    torch.manual_seed(0)
    fh = open(args.out, "a") if args.out else None
    for spec in args.shapes.split(","):
        parts = spec.split(":")
        M, N, K = int(parts[0]), int(parts[1]), int(parts[2])
        silu = len(parts) > 3 and parts[3] == "silu"
        wbytes = N * K * 2
        ncopy = max(1, min(32, (600 << 20) // wbytes + 1))  # > the 256 MB MALL: cold weights, as in decode
        ws = [(torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) * 0.05 for _ in range(ncopy)]
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        it = {"i": 0}
        scheds = schedules(M, N, K, silu)
        for ks, sk in scheds:
            G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
        G.WS.counters(dev)
        ref = torch.nn.functional.linear(x[:64].float(), ws[0].float())

        def mk(ks, sk):
            def f():
                w = ws[it["i"] % ncopy]
                it["i"] += 1
                return G.gemm_silu(x, w, ksplit=ks, sk=sk) if silu else G.gemm(x, w, ksplit=ks, sk=sk)
            return f

        def lib():
            w = ws[it["i"] % ncopy]
            it["i"] += 1
            y = torch.nn.functional.linear(x, w)
            if silu:
                y = y.view(M, -1, 2, 32)
                y = torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]
            return y

        arms = {f"own_ks{ks}_sk{sk}": mk(ks, sk) for ks, sk in scheds}
        if not args.no_lib:
            arms["library"] = lib
        errs = {}
        if not silu:
            for name, f in arms.items():
                if name == "library":
                    continue
                it["i"] = 0
                y = f()[:64].float()
                errs[name] = round(((y - ref).abs().max() / (ref.abs().max() + 1e-6)).item(), 5)
        for f in arms.values():
            f(); f()
        torch.cuda.synchronize()
        times = {k: [] for k in arms}
        for _ in range(args.reps):
            for k, f in arms.items():
                times[k] += timeit(f, 1)
        flop = 2.0 * M * N * K
        best = min(times, key=lambda k: statistics.median(times[k]))
        for k, ts in times.items():
            med = statistics.median(ts)
            row = {"M": M, "N": N, "K": K, "silu": silu, "arm": k, "med_us": round(med, 1),
                   "min_us": round(min(ts), 1), "tflops": round(flop / med / 1e6, 1), "err": errs.get(k),
                   "best": k == best}
            line = json.dumps(row)
            print(line, flush=True)
            if fh:
                fh.write(line + "\n")
    if fh:
        fh.close()


if __name__ == "__main__":
    main()
