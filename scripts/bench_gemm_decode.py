"""A/B of the decode-regime GEMM (csrc/kernels/gemm_decode.hip) against the
256x256 tile kernel and the library GEMM on the Qwen2-7B projections at decode
batches (M = 64..256).  Every variant (mt, waves, K-splits) is timed, so the
output doubles as the dispatch sweep for ops/gemm.py dec_plan.

Weights rotate over enough copies to exceed the 256 MB Infinity Cache (timed
cold, as in serving); all arms interleave in one process on the same operands.
Prints one JSON line per (shape, arm).

usage: python scripts/bench_gemm_decode.py [--ms 64,128,192,256] [--reps 30] [--out f.jsonl]
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

Q7 = {"qkv": (4608, 3584), "o": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944)}


def timeit(fn, reps):
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
    ap.add_argument("--ms", default="64,128,192,256")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--splits", default="1,2,3,4,5,7,9,14,18,28")
    ap.add_argument("--w4", action="store_true", help="add W4A16 (ops/w4.py) arms; their error is vs the 4-bit weight")
    ap.add_argument("--packed", action="store_true", help="add unit-packed weight arms (pk_*)")
    ap.add_argument("--dispatch", action="store_true", help="arms: library, tile kernel, dec_plan's choice")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    enable_tuned_gemms()
    torch.manual_seed(0)
    rows = []
    for sname in args.shapes.split(","):
        N, K = Q7[sname]
        silu = sname == "gate_up"
        wbytes = N * K * 2
        ncopy = max(2, min(10, (700 << 20) // wbytes + 1))
        ws = [(torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) * 0.05 for _ in range(ncopy)]
        for M in map(int, args.ms.split(",")):
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            ref = torch.nn.functional.linear(x.float(), ws[0].float())
            if silu:
                g, u = G.deinterleave_gate_up(ws[0].float())
                ref = torch.nn.functional.silu(x.float() @ g.T) * (x.float() @ u.T)
            it = {"i": 0}

            def nxt():
                it["i"] += 1
                return ws[it["i"] % ncopy]

            arms = {"lib": lambda w=None: torch.nn.functional.linear(x, w if w is not None else nxt())}
            pks = [G.DecPacked(w_, silu) for w_ in ws] if args.packed else []
            S, SK = G.plan(M, N, K)
            G.WS.reserve(dev, G._ws_floats(M, N, S, SK))
            arms["tile"] = (lambda w=None: G.gemm_silu(x, w if w is not None else nxt(), ksplit=S, sk=SK)) if silu \
                else (lambda w=None: G.gemm(x, w if w is not None else nxt(), ksplit=S, sk=SK))
            if args.dispatch:  # only the plan ops/gemm.py dec_plan picks
                pl = G.dec_plan(M, N, K, silu)
                if pl is not None:
                    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, pl[3])))
                    arms["plan_" + "_".join(map(str, pl))] = (
                        lambda w=None, plan=pl: G.gemm_decode(x, w if w is not None else nxt(),
                                                              epi=G.EPI_SILU if silu else G.EPI_STORE, plan=plan))
            for mt, nwv, ntw in [] if args.dispatch else G.dec_variants(M) + [
                    v for v in G.DEC_VARIANTS if v[1] == 5 and 16 * v[0] < M and -(-M // (16 * v[0])) <= 4]:
                seen = set()
                for req in map(int, args.splits.split(",")):
                    ks = G.dec_ksplit(K, req)
                    if ks in seen or (silu and ks > 1):
                        continue
                    seen.add(ks)
                    # plain tiling (nwv units per workgroup) and the balanced grid (about one workgroup per CU)
                    gss = {0: N // (16 * nwv * ntw)} if N % (16 * nwv * ntw) == 0 else {}
                    gb = G.dec_balanced_gs(N, ntw, nwv, ks)
                    if gb is not None and gb not in gss.values():
                        gss[gb] = gb
                    for gs, ngroups in gss.items():
                        if ngroups * ks * -(-M // (16 * mt)) > 1200:
                            continue
                        G.WS.reserve(dev, G.dec_ws_floats(M, N, ks))
                        plan = (mt, nwv, ntw, ks, gs)
                        epi = G.EPI_SILU if silu else G.EPI_STORE
                        arms[f"dec_mt{mt}_w{nwv}_n{ntw}_s{ks}" + (f"_g{gs}" if gs else "")] = (
                            lambda w=None, plan=plan, epi=epi: G.gemm_decode(x, w if w is not None else nxt(),
                                                                             epi=epi, plan=plan))
                        if args.packed:
                            arms[f"pk_mt{mt}_w{nwv}_n{ntw}_s{ks}" + (f"_g{gs}" if gs else "")] = (
                                lambda w=None, plan=plan, epi=epi: G.gemm_decode(
                                    x, ws[0], epi=epi, plan=plan,
                                    packed=pks[0] if w is not None else pks[it.__setitem__("i", it["i"] + 1)
                                                                            or it["i"] % len(pks)]))
            if args.w4:
                from githubrepostorag_amd.ops import w4 as W4

                w4s = [W4.W4Linear.quantize(w, silu=silu) for w in ws[:2]]
                for w4 in w4s:
                    w4.release_codes()
                w4ref = W4.W4Linear.quantize(ws[0], silu=silu)
                need = -(-M // 16)
                for mt, nwv in [v for v in W4.W4_VARIANTS if v[0] >= need and N % (32 * v[1]) == 0][:2]:
                    tiles = N // (32 * nwv)
                    for req in ((1,) if silu else map(int, args.splits.split(","))):
                        ks = 1 if silu else G.dec_ksplit(K, req)
                        name = f"w4_mt{mt}_w{nwv}_s{ks}"
                        if name in arms or tiles * ks > 1200:
                            continue
                        G.WS.reserve(dev, ks * M * N)
                        arms[name] = (lambda w=None, p_=(mt, nwv, ks): W4.gemm_w4(
                            x, w4ref if w is not None else w4s[it.__setitem__("i", it["i"] + 1) or it["i"] % 2],
                            plan_=p_))
            errs = {}
            for name, fn in arms.items():
                if name == "lib":
                    continue
                y = fn(ws[0]).float()
                r = ref
                if name.startswith("w4"):
                    d = w4ref.dequant(torch.float32)
                    if silu:
                        g_, u_ = G.deinterleave_gate_up(d)
                        r = torch.nn.functional.silu(x.float() @ g_.T) * (x.float() @ u_.T)
                    else:
                        r = x.float() @ d.T
                errs[name] = ((y - r).abs().max() / (r.abs().max() + 1e-9)).item()
            for _ in range(3):
                for fn in arms.values():
                    fn()
            torch.cuda.synchronize()
            times = {n: [] for n in arms}
            for _ in range(3):
                for n, fn in arms.items():
                    times[n].append(timeit(fn, max(1, args.reps // 3)))
            lib_us = statistics.median(times["lib"])
            for n in arms:
                us = statistics.median(times[n])
                wb = wbytes // 4 + N * (K // 128) * 8 if n.startswith("w4") else wbytes
                row = {"shape": sname, "M": M, "N": N, "K": K, "arm": n, "us": round(us, 2),
                       "TBps": round((wb + M * K * 2) / us / 1e6, 2), "vs_lib": round(lib_us / us, 3),
                       "relerr": None if n == "lib" else round(errs[n], 5)}
                print(json.dumps(row), flush=True)
                rows.append(row)
        del ws
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
