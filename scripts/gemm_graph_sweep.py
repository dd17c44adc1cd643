"""Graph-timed, cold-weight sweep of the Qwen2-7B decode projections at 1-256 rows.

Every arm is captured into one hipGraph of R launches that rotate over >= 1 GiB of weight copies (a decode
step streams 15 GB of weights, so each matrix arrives cold from HBM), replayed back to back; the time per
launch excludes Python / ctypes dispatch, unlike scripts/microbench.py's eager loop.  Arms per shape:
  linear      ops/linear.linear (or mlp_gate_up): the dispatched kernel plus its split-K reduce
  deferred    ops/linear.linear_deferred: the planes left for the consumer (RoPE / RMSNorm) to reduce,
              the form the decoder runs for qkv / o / down (decode batches)
Output: one JSON object {shape_M: {arm: {us, TB_s}}} (weights' bytes / time).

python scripts/gemm_graph_sweep.py --Ms 64,128,176,256 --out gpurun_out/gemm_sweep.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import gemm as G  # noqa: E402
from githubrepostorag_amd.ops._lib import lib  # noqa: E402
from githubrepostorag_amd.ops.linear import enable_tuned_gemms, kernel_for, linear, linear_deferred  # noqa: E402

SHAPES = {"qkv": (4608, 3584, False), "o": (3584, 3584, False), "gate_up": (37888, 3584, True),
          "down": (3584, 18944, False)}


def graph_time(fn, ws, reps: int) -> float:
    """us per launch of fn(w) over the rotating copies, captured as one graph of `reps` launches."""
    for w in ws[:2]:
        fn(w)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(ws[0])
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(ws[i % len(ws)])
    g.replay()
    torch.cuda.synchronize()
    best = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best.append(e0.elapsed_time(e1) * 1000.0 / reps)
    best.sort()
    return best[len(best) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Ms", default="64,128,176,256")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--packed", type=int, default=0,
                    help="1: also the decode kernel on the unit-packed weight layout (ops/gemm.py DecPacked) vs the "
                         "natural [N, K] layout, same plan (dec_plan, or --plan)")
    ap.add_argument("--tail", type=int, default=0, help="1: also the 8-wave tail-split decode schedules")
    ap.add_argument("--depths", default="", help="ring depths to A/B on the dispatched decode plan (e.g. 6,8)")
    ap.add_argument("--plan", default="", help="mt,nwv,ntw,ksplit[,gs] for the packed A/B (default dec_plan)")
    ap.add_argument("--hot", type=int, default=0, help="1: also every arm on one weight copy (cache-hot)")
    ap.add_argument("--tile", default="", help="stream-K grids of the 256x256 tile kernel to A/B (e.g. 256:192; "
                                               "k2 = 2-way split-K with the reduce)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    enable_tuned_gemms()
    dev = torch.device("cuda")
    out = {}
    with torch.inference_mode():
        for name in a.shapes.replace(":", ",").split(","):
            N, K, silu = SHAPES[name]
            ncopy = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
            ws = [((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
            for M in [int(m) for m in a.Ms.replace(":", ",").split(",")]:
                x = ((torch.rand(M, K, device=dev) * 2 - 1)).to(torch.bfloat16)
                arms = {}
                if silu:
                    arms["linear"] = lambda w: G.mlp_gate_up(x, w)
                else:
                    arms["linear"] = lambda w: linear(x, w)
                    arms["deferred"] = lambda w: linear_deferred(x, w)
                plan = tuple(int(v) for v in a.plan.replace(":", ",").split(",")) if a.plan else G.dec_plan(M, N, K, silu)
                if a.packed and plan is not None:
                    pks = [G.DecPacked(w, silu) for w in ws]
                    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
                    epi = G.EPI_SILU if silu else G.EPI_STORE
                    arms["dec_natural"] = lambda w, plan=plan, epi=epi: G.gemm_decode(x, w, epi=epi, plan=plan)
                    pk_of = {id(w): p for w, p in zip(ws, pks)}
                    arms["dec_packed"] = lambda w, plan=plan, epi=epi: G.gemm_decode(x, w, epi=epi, plan=plan,
                                                                                     packed=pk_of[id(w)])
                if a.tail:  # the 8-wave tail-split schedule at the K-splits that give 4-5 units per workgroup
                    epi = G.EPI_SILU if silu else G.EPI_STORE
                    for ks in ([1] if silu else [k for k in (4, 7, 8, 10, 14) if G.dec_ksplit(K, k) == k]):
                        tp = G.dec_tail_plan(M, N, ksplit=ks)
                        if tp is None:
                            continue
                        G.WS.reserve(dev, G.dec_ws_floats(M, N, ks))
                        arms[f"tail_ks{ks}"] = lambda w, tp=tp, epi=epi: G.gemm_decode(x, w, epi=epi, plan=tp)
                if plan is not None and M < 33:  # 1-32 rows: the 1- / 2-row-tile decode variants vs the dispatch
                    epi = G.EPI_SILU if silu else G.EPI_STORE
                    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
                    arms["decode"] = lambda w, plan=plan, epi=epi: G.gemm_decode(x, w, epi=epi, plan=plan)
                    ks = G.dec_ksplit(K, plan[3])
                    if not silu and ks > 1:  # the planes left for RoPE / RMSNorm (no reduce launch)
                        for kk in sorted({ks, G.dec_ksplit(K, 2 * plan[3])}):
                            pl = (plan[0], plan[1], plan[2], kk)
                            G.WS.reserve(dev, G.dec_ws_floats(M, N, kk))
                            arms[f"dec_deferred_ks{kk}"] = lambda w, pl=pl, kk=kk: G.gemm_deferred(
                                x, w, ("decode", kk, pl))
                for d in [int(v) for v in a.depths.replace(":", ",").split(",") if v.strip()]:
                    if plan is None or plan[1] not in (4, 5) or plan[0] > (2 if d == 12 else 4 if d == 8 else 8) \
                            or (plan[0] <= 2 and d == 6):
                        continue
                    epi = G.EPI_SILU if silu else G.EPI_STORE
                    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))

                    def deep(w, d=d, plan=plan, epi=epi):
                        prev = lib().grag_gemm_decode_depth(d)
                        try:
                            return G.gemm_decode(x, w, epi=epi, plan=plan)
                        finally:
                            lib().grag_gemm_decode_depth(prev)
                    arms[f"depth{d}"] = deep
                    if a.packed:
                        def deep_pk(w, d=d, plan=plan, epi=epi):
                            prev = lib().grag_gemm_decode_depth(d)
                            try:
                                return G.gemm_decode(x, w, epi=epi, plan=plan, packed=pk_of[id(w)])
                            finally:
                                lib().grag_gemm_decode_depth(prev)
                        arms[f"depth{d}_packed"] = deep_pk
                for t in [v for v in a.tile.replace(":", ",").split(",") if v.strip()]:
                    ks_t, sk_t = (int(t[1:]), 0) if t.startswith("k") else (1, int(t))
                    G.WS.reserve(dev, G._ws_floats(M, N, ks_t, sk_t))
                    if silu:
                        arms[f"tile_{t}"] = lambda w, ks_t=ks_t, sk_t=sk_t: G.gemm_silu(x, w, ksplit=ks_t, sk=sk_t)
                    else:
                        arms[f"tile_{t}"] = lambda w, ks_t=ks_t, sk_t=sk_t: G.gemm(x, w, ksplit=ks_t, sk=sk_t)
                if a.hot:  # the same weight every launch: served from the 256 MB MALL / L2 when it fits
                    for k in list(arms):
                        arms[k + "_hot"] = (lambda f: (lambda w, f=f: f(ws[0])))(arms[k])
                r = {"kernel": "mlp_gate_up" if silu else kernel_for(M, N, K), "plan": plan}
                gb = N * K * 2 / 1e9
                for k, fn in arms.items():
                    try:
                        us = graph_time(fn, ws, a.reps)
                    except RuntimeError as e:  # a schedule the launcher refuses for this shape
                        r[k] = {"error": str(e)[:120]}
                        continue
                    r[k] = {"us": round(us, 2), "TB_s": round(gb / (us * 1e-6) / 1e3, 3)}
                out[f"{name}_M{M}"] = r
                print(name, M, json.dumps(r), flush=True)
                if a.packed and plan is not None:
                    del pks, pk_of
            del ws
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
