"""Measured prefill-GEMM dispatch: owned 256x256 tile kernel vs the library.

For every prefill/encoder weight shape and a dense sweep of row counts M
(the engine's prefill steps carry arbitrary token counts, and the library's
heuristic choice swings with M: Qwen2-7B down_proj runs at 1504 TF/s at
M = 4096 and 863 TF/s at M = 7104, profiles/gemm_tile_prefill_7k.jsonl),
time hipBLASLt (TunableOp results loaded, as in serving) and the owned kernel
under each tail schedule it has (whole tiles; stream-K round; tail-only
stream-K), check each owned arm against the library output, and record the
fastest arm per M.  Writes githubrepostorag_amd/tuning/gemm_prefill_gfx950.json,
which ops/linear.py (plain projections) and ops/gemm.py (fused SwiGLU) read.

Both arms run interleaved in one process on the same random operands
(cdna guide §5.4 rules 24/25); medians of CUDA-event timings.

usage: python scripts/sweep_prefill_gemm.py [--models qwen2-7b,bge-large] [--mmin 384 --mmax 16384 --mstep 256]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.ops import gemm as G  # noqa: E402
from githubrepostorag_amd.ops.linear import enable_tuned_gemms  # noqa: E402

SHAPES = {
    # name: [(label, N, K, silu)]  (N, K) of the [N, K] weight; silu: interleaved gate/up + SwiGLU epilogue
    "qwen2-7b": [("qkv", 4608, 3584, False), ("o", 3584, 3584, False), ("gate_up", 37888, 3584, True),
                 ("down", 3584, 18944, False)],
    "qwen2-1.5b": [("qkv", 2048, 1536, False), ("o", 1536, 1536, False), ("gate_up", 17920, 1536, True),
                   ("down", 1536, 8960, False)],
    "bge-large": [("qkv", 3072, 1024, False), ("o", 1024, 1024, False), ("ffn1", 4096, 1024, False),
                  ("ffn2", 1024, 4096, False)],
    "bge-base": [("qkv", 2304, 768, False), ("o", 768, 768, False), ("ffn1", 3072, 768, False),
                 ("ffn2", 768, 3072, False)],
}


def _tp_shapes(model: str, tp: int):
    """Per-rank projection shapes of a TP-sharded Qwen2 (models/qwen2.py: q heads / TP, kv heads / TP or
    one replicated, FFN zero-padded to a multiple of 64)."""
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import FFN_PAD

    c = decoder_config(model)
    hq, hkv, D, H = c.num_heads // tp, max(1, c.num_kv_heads // tp), c.head_dim, c.hidden_size
    inter = -(-(c.intermediate_size // tp) // FFN_PAD) * FFN_PAD
    return [("qkv", (hq + 2 * hkv) * D, H, False), ("o", H, hq * D, False), ("gate_up", 2 * inter, H, True),
            ("down", H, inter, False)]


# BASELINE config 4 (Qwen2-72B TP=8) and Qwen2-7B at TP 2 / 4 (28 heads: TP 8 does not divide them)
for _m, _tp in (("qwen2-72b", 8), ("qwen2-7b", 2), ("qwen2-7b", 4)):
    SHAPES[f"{_m}-tp{_tp}"] = _tp_shapes(_m, _tp)


def med_us(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def own_arms(M, N, K):
    """(ksplit, sk) schedules the owned kernel can run this shape with."""
    ncu = G._num_cus()
    arms = {(1, 0)}
    arms.add(G.plan(M, N, K))
    tiles = -(-M // 256) * -(-N // 256)
    if tiles > 2 * ncu and tiles % ncu:
        arms.add((1, ncu))
    kt = K // 64
    if tiles > ncu and tiles % ncu and (tiles % ncu) * kt >= ncu * ((kt + 3) // 4):
        arms.add((1, -ncu))
    # tail-only stream-K over a smaller grid: the last partial round's tiles shared by g workgroups
    # (g = 1x / 2x / 4x the leftover tiles, capped by the launcher's quarter-tile rule), so a thin
    # last round (e.g. 10 tiles after two full rounds) costs a fraction of a round instead of a round
    tail = tiles % ncu
    if tiles > ncu and tail:
        for f in (1, 2, 4):
            g = min(ncu, tail * f, (tail * kt) // ((kt + 3) // 4))
            if g >= 2 and G.sk_ok(M, N, K, 1, -g):
                arms.add((1, -g))
        # K-aligned tail splits: every leftover tile cut into s equal K parts (s x tail workgroups, more than
        # one per CU allowed): the parts of a round start at the same K offsets (L2 reuse, unlike a grid
        # that straddles tiles) and the tail costs ceil(s tail / CUs) / s of a round
        for s_ in (2, 3, 4):
            g = tail * s_
            if g > ncu // 2 and G.sk_ok(M, N, K, 1, -g):
                arms.add((1, -g))
    return sorted(arms)


def table_row(M, med):
    """[M, lib_us, best owned us, its ksplit, its sk] (owned fields null when no arm passed numerics)."""
    own = {a: t for a, t in med.items() if a != "lib"}
    if not own:
        return [M, round(med["lib"], 1), None, 1, 0]
    a = min(own, key=own.get)
    return [M, round(med["lib"], 1), round(own[a], 1), a[0], a[1]]


def table_from_log(path):
    """Rebuild the dispatch table from a --log file of an earlier sweep."""
    table = {}
    for line in open(path):
        r = json.loads(line)
        model, label = r["shape"].split("/")
        N, K, silu = next((n, k, s) for lb, n, k, s in SHAPES[model] if lb == label)
        med = {"lib": r["lib_us"]}
        for k, v in r.items():
            if k.startswith("own_") and k.endswith("_us"):
                ks, sk = k[4:-3].split("_")
                med[(int(ks), int(sk))] = v
        table.setdefault(f"{N},{K},{int(silu)}", []).append(table_row(r["M"], med))
    return table


def write_table(path, table, mstep, extra=None):
    out = {"arch": "gfx950", "note": "scripts/sweep_prefill_gemm.py: per (N, K, silu) and M bucket "
           "[M, library us, best owned us, its ksplit, its sk]; ops/linear.py prefill_plan() takes the library "
           "only where it won at both buckets around M", "mstep": mstep, "table": table, **(extra or {})}
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f)
    print(f"wrote {path} ({sum(len(v) for v in table.values())} buckets)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="qwen2-7b,bge-large")
    ap.add_argument("--mmin", type=int, default=384)
    ap.add_argument("--mmax", type=int, default=16384)
    ap.add_argument("--mstep", type=int, default=256)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="githubrepostorag_amd/tuning/gemm_prefill_gfx950.json")
    ap.add_argument("--log", default=None)
    ap.add_argument("--from-log", default=None, help="rebuild --out from an earlier sweep's --log, no GPU")
    ap.add_argument("--labels", default=None, help="only these shape labels (e.g. qkv,o)")
    ap.add_argument("--merge", action="store_true",
                    help="update only the swept (N, K, silu) keys of the existing --out table, keep the rest")
    args = ap.parse_args()
    if args.from_log:
        write_table(args.out, table_from_log(args.from_log), args.mstep)
        return
    dev = torch.device("cuda", 0)
    enable_tuned_gemms()
    torch.manual_seed(0)
    table, times = {}, {}
    logf = open(args.log, "w") if args.log else None
    t_start = time.time()
    for model in args.models.split(","):
        for label, N, K, silu in SHAPES[model]:
            if args.labels and label not in args.labels.split(","):
                continue
            key = f"{N},{K},{int(silu)}"
            ws = [((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(2)]
            xfull = (torch.rand(args.mmax, K, device=dev) * 2 - 1).to(torch.bfloat16)
            rows, trow = [], []
            for M in range(args.mmin, args.mmax + 1, args.mstep):
                x = xfull[:M]
                arms = own_arms(M, N, K)
                for ks, sk in arms:
                    G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
                    if sk:
                        G.WS.counters(dev)
                it = {"i": 0}

                def lib():
                    w = ws[it["i"] & 1]
                    it["i"] += 1
                    y = torch.nn.functional.linear(x, w)
                    if silu:
                        y = y.view(M, -1, 2, 32)
                        y = (torch.nn.functional.silu(y[:, :, 0].float()) * y[:, :, 1].float()).to(x.dtype).reshape(M, -1)
                    return y

                def own(ks, sk):
                    def f():
                        w = ws[it["i"] & 1]
                        it["i"] += 1
                        return G.gemm_silu(x, w, ksplit=ks, sk=sk) if silu else G.gemm(x, w, ksplit=ks, sk=sk)
                    return f

                # numerics: each owned arm against the library on the same weight
                it["i"] = 0
                ref = lib().float()
                scale = ref.abs().max().item() + 1e-6
                ok = {}
                for a in arms:
                    it["i"] = 0
                    y = own(*a)().float()
                    ok[a] = ((y - ref).abs().max().item() / scale) < 2e-2
                fns = {"lib": lib, **{a: own(*a) for a in arms if ok[a]}}
                for f in fns.values():  # warm
                    f()
                torch.cuda.synchronize()
                t = {k: [] for k in fns}
                for _ in range(args.reps):  # interleaved rounds
                    for k, f in fns.items():
                        t[k].append(med_us(f, 1))
                med = {k: statistics.median(v) for k, v in t.items()}
                best = min(med, key=med.get)
                choice = ["lib", 1, 0] if best == "lib" else ["own", best[0], best[1]]
                rows.append(table_row(M, med))
                trow.append({"M": M, "lib_us": round(med["lib"], 1),
                             **{f"own_{a[0]}_{a[1]}_us": round(med[a], 1) for a in arms if a in med},
                             "bad_arms": [list(a) for a in arms if not ok[a]], "best": choice})
                line = json.dumps({"shape": f"{model}/{label}", **trow[-1]})
                print(line, flush=True)
                if logf:
                    logf.write(line + "\n")
                    logf.flush()
            table[key] = rows
            times[f"{model}/{label}"] = trow
            del ws, xfull
            torch.cuda.empty_cache()
    extra = {"sweep_s": round(time.time() - t_start, 1)}
    if args.merge and os.path.exists(args.out):
        old = json.load(open(args.out))
        merged = dict(old["table"])
        for key, rows in table.items():  # rows below the sweep's range (decode-batch rows) are kept
            lo = min(r[0] for r in rows)
            merged[key] = sorted([r for r in merged.get(key, []) if r[0] < lo] + rows)
        extra = {k: v for k, v in old.items() if k not in ("arch", "note", "mstep", "table")}
        extra["resweep"] = f"{sorted(table)} re-swept ({round(time.time() - t_start, 1)} s)"
        table = merged
    write_table(args.out, table, args.mstep, extra)

if __name__ == "__main__":
    main()
