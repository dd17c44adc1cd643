"""Graph-timed split-KV plan sweep of the paged decode attention (csrc/kernels/attention.hip
paged_decode_kernel + attn_combine_kernel) over batch x context: one hipGraph of R launches per arm (the
decode step replays attention from a graph too), K/V in random blocks, us per call incl. the combine.

python scripts/attn_sweep.py --grid 1:1024/1:4096/1:11600/4:4096/16:4096/176:1500 --splits 64:128:256:512
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.engine.llm_engine import _pow2_at_least, _split_len_for  # noqa: E402
from githubrepostorag_amd.ops import attention as A  # noqa: E402

VARIANTS = {"ns2": 3, "ns3": 8, "ns4": 7, "ns2_nt": 11, "ns3_nt": 12, "mw2": 22, "mw4": 24}


def graph_us(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / reps)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="1:1024,1:4096,1:11600,4:4096,4:11600,16:4096,16:11600,176:1500")
    ap.add_argument("--splits", default="64:128:256:512:1024")
    ap.add_argument("--variants", default="ns2:ns3:mw2:mw4")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    A.decode_counters(dev)
    Hq, Hkv, D, BS = 28, 4, 128, 16
    out = {}
    with torch.inference_mode():
        for cell in a.grid.replace("/", ",").split(","):  # ',' or '/' between cells (gpu_run.sh eats commas)
            B, ctx = (int(v) for v in cell.split(":"))
            nb = B * (-(-ctx // BS)) + 1
            kc = torch.randn(nb, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
            vc = torch.randn_like(kc)
            q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
            bt = (1 + torch.randperm(nb - 1, device=dev)[: B * (-(-ctx // BS))]).view(B, -1).to(torch.int32)
            gb = B * ctx * Hkv * D * 2 * 2 / 1e9
            res = {"bytes_gb": round(gb, 4), "engine_split_len": _split_len_for(B)}
            for sl in [int(v) for v in a.splits.replace(":", ",").split(",")]:
                if sl % 32:
                    continue
                ns = -(-ctx // sl)
                for vname in a.variants.replace(":", ",").split(","):
                    if VARIANTS[vname] not in A.DECODE_MW and sl % A.KV_TILE:
                        continue  # the single-wave kernel takes parts of whole 64-key tiles
                    meta = A.AttnMetadata(
                        q_start=torch.arange(B + 1, device=dev, dtype=torch.int32),
                        ctx_len=torch.full((B,), ctx, device=dev, dtype=torch.int32), block_tables=bt,
                        slot_mapping=torch.zeros(B, dtype=torch.int32, device=dev), max_q_len=1, num_seqs=B,
                        num_tokens=B, is_decode=True, num_splits=ns, split_len=sl,
                        part_o=torch.empty(ns * B * Hq * D, device=dev), part_ml=torch.empty(ns * B * Hq * 2, device=dev))
                    meta.extra = {"decode_nw": VARIANTS[vname]}
                    o = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=dev)
                    us = graph_us(lambda: A.paged_attention(q, kc, vc, meta, 0.088, out=o))
                    res[f"split{sl}_{vname}"] = {"us": round(us, 2), "TB_s": round(gb / (us * 1e-6) / 1e3, 3),
                                                 "waves": B * Hkv * ns}
            # the small-batch kernel at its own plan (ops/attention.decode_mw_plan)
            mns, msl = A.decode_mw_plan(B, Hkv, ctx, 11712, force=True)
            for vname in ("mw2", "mw4"):
                meta = A.AttnMetadata(
                    q_start=torch.arange(B + 1, device=dev, dtype=torch.int32),
                    ctx_len=torch.full((B,), ctx, device=dev, dtype=torch.int32), block_tables=bt,
                    slot_mapping=torch.zeros(B, dtype=torch.int32, device=dev), max_q_len=1, num_seqs=B,
                    num_tokens=B, is_decode=True, num_splits=mns, split_len=msl,
                    part_o=torch.empty(mns * B * Hq * D, device=dev), part_ml=torch.empty(mns * B * Hq * 2, device=dev))
                meta.extra = {"decode_nw": VARIANTS[vname]}
                o = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=dev)
                us = graph_us(lambda: A.paged_attention(q, kc, vc, meta, 0.088, out=o))
                res[f"mwplan_{vname}"] = {"us": round(us, 2), "TB_s": round(gb / (us * 1e-6) / 1e3, 3),
                                          "nsplit": mns, "split_len": msl}
            # the engine's own plan (llm_engine._run_decode: split_len by batch, nsplit a power of two)
            sl = _split_len_for(B)
            ns = _pow2_at_least(-(-ctx // sl))
            res["engine_plan"] = {"split_len": sl, "nsplit": ns, "variant": A.decode_variant(ns, sl, B * Hkv * ns)}
            best = min((v["us"], k) for k, v in res.items() if isinstance(v, dict) and "us" in v)
            res["best"] = best[1]
            out[f"B{B}_ctx{ctx}"] = res
            print(cell, json.dumps({k: (v["us"] if isinstance(v, dict) and "us" in v else v) for k, v in res.items()}),
                  flush=True)
            del kc, vc
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
