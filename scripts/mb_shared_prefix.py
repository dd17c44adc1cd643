"""Decode attention over prefix-sharing rows (ingest's regime: each chunk's summary / title / keyword
calls share the chunk's KV blocks): kernel time of one decode attention launch with the rows of a group
ADJACENT in the batch and the XCD placement on (csrc/kernels/attention.hip g_decode_xcd), adjacent with it
off, SHUFFLED, a batch with no sharing at all (every row its own blocks: the HBM-traffic upper bound), and the
shared-prefix decode (paged_decode_prefix_kernel + the per-row kernel over the suffix; --cascade-parts: its
prefix parts per group), checked against the plain kernel's output.

python scripts/mb_shared_prefix.py --B 192 --group 3 --prefix 1536 --suffix 256 --out gpurun_out/mb_shared.json
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.engine.llm_engine import _decode_plan  # noqa: E402
from githubrepostorag_amd.ops import attention as A  # noqa: E402
from githubrepostorag_amd.ops._lib import lib  # noqa: E402


class _M:  # the model attributes _decode_plan reads
    hkv = 4
    device = torch.device("cuda")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=192)
    ap.add_argument("--group", type=int, default=3)
    ap.add_argument("--prefix", type=int, default=1536)
    ap.add_argument("--suffix", type=int, default=256)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cascade-min-part", default="256", help="shortest prefix part (keys), one arm per value")
    ap.add_argument("--arms", default="adjacent_rr,no_sharing,cascade")
    ap.add_argument("--share-every", type=int, default=1,
                    help="only every Nth group shares its prefix (the rest: own blocks), a partly shared batch")
    a = ap.parse_args()
    dev = torch.device("cuda")
    Hq, Hkv, D, BS = 28, 4, 128, 16
    B, g = a.B, a.group
    npfx, nsfx = a.prefix // BS, -(-a.suffix // BS)
    ngroups = -(-B // g)
    nb_shared = ngroups * npfx + B * nsfx
    nb_flat = B * (npfx + nsfx)
    NB = max(nb_shared, nb_flat) + 8
    gen = torch.Generator(device="cpu").manual_seed(0)
    kc = (torch.randn(NB, Hkv, BS, D, generator=gen) * 0.5).to(torch.bfloat16).to(dev)
    vc = torch.randn(NB, Hkv, BS, D, generator=gen).to(torch.bfloat16).to(dev)
    q = torch.randn(B, Hq, D, generator=gen).to(torch.bfloat16).to(dev)
    ctx = npfx * BS + a.suffix
    width = npfx + nsfx
    perm = torch.randperm(NB - 8, generator=gen)

    def table(shared: bool, order):
        bt = torch.zeros(B, width, dtype=torch.int32)
        o = 0
        for gi in range(ngroups):
            sh = shared and gi % a.share_every == 0
            pf = perm[o:o + npfx] if sh else None
            if sh:
                o += npfx
            for j in range(g):
                r = gi * g + j
                if r >= B:
                    break
                if sh:
                    bt[r, :npfx] = pf
                else:
                    bt[r, :npfx] = perm[o:o + npfx]
                    o += npfx
                bt[r, npfx:] = perm[o:o + nsfx]
                o += nsfx
        return bt[order]

    nsplit, split_len = _decode_plan(_M(), B, ctx, 8192)
    res = {"B": B, "group": g, "ctx": ctx, "nsplit": nsplit, "split_len": split_len}
    scale = 1 / math.sqrt(D)
    shuffled = torch.randperm(B, generator=gen)
    ident = torch.arange(B)
    ref_out = None
    import numpy as np

    arms = [("adjacent_xcd", True, ident, 1, 0), ("adjacent_rr", True, ident, 0, 0),
            ("shuffled_xcd", True, shuffled, 1, 0), ("shuffled_rr", True, shuffled, 0, 0),
            ("no_sharing", False, ident, 0, 0)]
    arms += [(f"cascade_m{mp}", True, ident, 0, int(mp)) for mp in a.cascade_min_part.split(",") if mp]
    want = a.arms.split(",")
    arms = [x for x in arms if x[0] in want or ("cascade" in want and x[4])]
    for name, shared, order, xcd, csl in arms:
        bt_h = table(shared, order)
        bt = bt_h.to(dev)
        m = A.AttnMetadata(q_start=torch.arange(B + 1, dtype=torch.int32, device=dev),
                           ctx_len=torch.full((B,), ctx, dtype=torch.int32, device=dev), block_tables=bt,
                           slot_mapping=torch.zeros(B, dtype=torch.int32, device=dev), max_q_len=1, num_seqs=B,
                           num_tokens=B, is_decode=True, num_splits=nsplit, split_len=split_len,
                           part_o=torch.empty(nsplit * B * Hq * D, dtype=torch.float32, device=dev),
                           part_ml=torch.empty(nsplit * B * Hq * 2, dtype=torch.float32, device=dev))
        if csl:
            pre, spans, saved = A.prefix_groups(bt_h.numpy(), np.full(B, ctx), BS, Hq // Hkv)
            res.setdefault("saved_key_share", round(saved / (B * ctx), 3))
            nsp = A.CASCADE_MAX_PLANES
            part, items, used = A.cascade_layout(pre, spans, A.cascade_items(B), min_part=csl)
            m.cascade = A.Cascade(pre_len=torch.from_numpy(pre).to(dev), pre_part=torch.from_numpy(part).to(dev),
                                  items=torch.from_numpy(items.reshape(-1)).to(dev), planes=nsp,
                                  pre_o=torch.empty(nsp * B * Hq * D, device=dev),
                                  pre_ml=torch.empty(nsp * B * Hq * 2, device=dev))
        prev = lib().grag_attn_decode_xcd(xcd)
        try:
            out = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=dev)
            A.paged_attention(q, kc, vc, m, scale, out=out)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for _ in range(a.reps):
                    A.paged_attention(q, kc, vc, m, scale, out=out)
            gr.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gr.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000 / a.reps)
        finally:
            lib().grag_attn_decode_xcd(prev)
        if ref_out is None and shared:
            ref_out = out.float().cpu()
        elif shared and not csl:
            assert torch.equal(out.float().cpu(), ref_out), "placement changed the result"
        elif csl:
            err = (out.float().cpu() - ref_out).abs().max().item()
            assert err < 2e-2, f"shared-prefix decode differs from the plain kernel: {err}"
        us = sorted(ts)[len(ts) // 2]
        kv_bytes = B * ctx * Hkv * D * 2 * 2
        res[name] = {"us": round(us, 2), "TB_s_if_every_row_read": round(kv_bytes / us / 1e6, 2)}
        if csl:
            n_sh = len(range(0, ngroups, a.share_every))
            uniq = (n_sh * npfx * BS + (B - n_sh * g) * npfx * BS + B * (ctx - npfx * BS)) * Hkv * D * 2 * 2
            res[name].update(items=used, part_keys=int(part.max()), TB_s_unique_kv=round(uniq / us / 1e6, 2))
        print(name, res[name], flush=True)
    if "shuffled_xcd" in res and "adjacent_xcd" in res:
        res["speedup_adjacent_xcd_vs_shuffled"] = round(res["shuffled_xcd"]["us"] / res["adjacent_xcd"]["us"], 3)
        res["speedup_adjacent_xcd_vs_rr"] = round(res["adjacent_rr"]["us"] / res["adjacent_xcd"]["us"], 3)
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
