"""Interleaved A/B micro-benchmarks of hot ops on the real model shapes
(one process, several rounds, median/min per variant — cdna guide §5.4 rule 24)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import attention as A
from githubrepostorag_amd.ops import sampling as S
from githubrepostorag_amd.ops.linear import gemm_skinny


def timeit(fn, iters=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def rounds(variants, n=5, iters=50):
    res = {k: [] for k in variants}
    for _ in range(n):
        for k, fn in variants.items():
            res[k].append(timeit(fn, iters))
    return {k: {"median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2)} for k, v in res.items()}


def gemm_bench(M):
    out = {}
    dev = torch.device("cuda")
    for name, N, K in [("qkv", 4608, 3584), ("o_proj", 3584, 3584), ("gate_up", 37888, 3584), ("down", 3584, 18944),
                       ("lm_head", 152064, 3584)]:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        # rotate through >= 1 GiB of weight copies: in a real decode step the
        # other ~15 GB of weights evict each matrix from the 256 MB MALL
        ncopy = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        it = {"i": 0}

        def nxt():
            it["i"] = (it["i"] + 1) % ncopy
            return ws[it["i"]]

        r = rounds({"hipblaslt": lambda: torch.nn.functional.linear(x, nxt()),
                    "grag_skinny": lambda: gemm_skinny(x, nxt())})
        del ws
        gb = N * K * 2 / 1e9
        for k in r:
            r[k]["TB_s"] = round(gb / (r[k]["min_us"] * 1e-6) / 1e3, 2)
        out[f"{name}_M{M}"] = r
    return out


def midm_bench(Ms=(128, 176, 192, 224, 256)):
    """Qwen2-7B projections at 129-256 rows (ingest / agent decode batches): the dispatched kernel
    (ops/linear.kernel_for, ops/gemm.mlp_gate_up) vs tile-kernel schedules (whole tiles, split-K,
    stream-K rounds), on >= 1 GiB of rotating weight copies (cold weights, as in a decode step)."""
    from githubrepostorag_amd.ops import gemm as G
    from githubrepostorag_amd.ops.linear import kernel_for, linear

    dev = torch.device("cuda")
    out = {}
    for name, N, K, silu in [("qkv", 4608, 3584, False), ("o", 3584, 3584, False),
                             ("gate_up", 37888, 3584, True), ("down", 3584, 18944, False)]:
        ncopy = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
        ws = [((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
        it = {"i": 0}

        def nxt():
            it["i"] = (it["i"] + 1) % ncopy
            return ws[it["i"]]

        for M in Ms:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            arms = {"dispatched": (lambda: G.mlp_gate_up(x, nxt())) if silu else (lambda: linear(x, nxt()))}
            tiles = -(-M // 256) * -(-N // 256)
            scheds = [(1, 0), (1, 256), (1, -256), (2, 0), (3, 0), (4, 0)]
            for ks, sk in scheds:
                if not G.sk_ok(M, N, K, ks, sk) or (ks > 1 and tiles * ks > 4 * 256):
                    continue
                G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
                if sk:
                    G.WS.counters(dev)
                arms[f"tile_{ks}_{sk}"] = ((lambda ks=ks, sk=sk: G.gemm_silu(x, nxt(), ksplit=ks, sk=sk)) if silu
                                          else (lambda ks=ks, sk=sk: G.gemm(x, nxt(), ksplit=ks, sk=sk)))
            r = rounds(arms, n=5, iters=30)
            r["dispatched_kind"] = "mlp_gate_up" if silu else kernel_for(M, N, K)
            gb = N * K * 2 / 1e9
            for k, v in r.items():
                if isinstance(v, dict):
                    v["TB_s"] = round(gb / (v["min_us"] * 1e-6) / 1e3, 2)
            out[f"{name}_M{M}"] = r
            print(name, M, json.dumps(r), flush=True)
        del ws
        torch.cuda.empty_cache()
    return out


def attn_decode_bench(B, ctx, split_len):
    dev = torch.device("cuda")
    Hq, Hkv, D, BS = 28, 4, 128, 16
    nb = B * ((ctx + BS - 1) // BS) + 1
    kc = torch.randn(nb, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    bt = torch.randperm(nb - 1, device=dev)[: B * ((ctx + BS - 1) // BS)].view(B, -1).to(torch.int32) + 1
    ns = (ctx + split_len - 1) // split_len
    meta = A.AttnMetadata(q_start=torch.arange(B + 1, device=dev, dtype=torch.int32),
                          ctx_len=torch.full((B,), ctx, device=dev, dtype=torch.int32), block_tables=bt,
                          slot_mapping=torch.zeros(B, dtype=torch.int32, device=dev), max_q_len=1, num_seqs=B,
                          num_tokens=B, is_decode=True, num_splits=ns, split_len=split_len,
                          part_o=torch.empty(ns * B * Hq * D, device=dev), part_ml=torch.empty(ns * B * Hq * 2, device=dev))
    import copy

    arms = {}
    arms_codes = (("tk64", 1), ("tk32", 3), ("tk32_ns3", 8), ("tk32_ns4", 7))
    if os.environ.get("MB_DECODE_ARMS") == "nt":  # default vs non-temporal K/V loads
        arms_codes = (("tk32", 3), ("tk32_nt", 11), ("tk32_ns3", 8), ("tk32_ns3_nt", 12))
    for name, code in arms_codes:
        mm = copy.copy(meta)
        mm.extra = {"decode_nw": code}
        arms[f"paged_decode_{name}_split{split_len}"] = (lambda mm=mm: A.paged_attention(q, kc, vc, mm, 0.088))
    r = rounds(arms)
    gb = B * ctx * Hkv * D * 2 * 2 / 1e9
    for k in r:
        r[k]["TB_s"] = round(gb / (r[k]["min_us"] * 1e-6) / 1e3, 2)
    return r


def attn_prefill_bench(nseq, L):
    dev = torch.device("cuda")
    Hq, Hkv, D, BS = 28, 4, 128, 16
    nbs = (L + BS - 1) // BS
    kc = torch.randn(nseq * nbs + 1, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(nseq * L, Hq, D, device=dev, dtype=torch.bfloat16)
    bt = (torch.arange(nseq * nbs, device=dev, dtype=torch.int32) + 1).view(nseq, nbs)
    meta = A.AttnMetadata(q_start=torch.arange(0, nseq * L + 1, L, device=dev, dtype=torch.int32),
                          ctx_len=torch.full((nseq,), L, device=dev, dtype=torch.int32), block_tables=bt,
                          slot_mapping=torch.zeros(nseq * L, dtype=torch.int32, device=dev), max_q_len=L,
                          num_seqs=nseq, num_tokens=nseq * L)
    def run(code):
        meta.extra = {"prefill_nw": code}
        return A.paged_attention(q, kc, vc, meta, 0.088)

    r = rounds({"prefill_4wave": lambda: run(4), "prefill_8wave_dma": lambda: run(5),
                "prefill_8wave_dma_3stage": lambda: run(6)}, n=3, iters=10)
    ref = run(5).float()
    err = (run(6).float() - ref).abs().max().item()
    r["prefill_8wave_dma_3stage"]["max_abs_diff_vs_2stage"] = round(err, 5)
    fl = nseq * Hq * L * L / 2 * D * 4 / 1e12
    for k in r:
        r[k]["TFLOPs"] = round(fl / (r[k]["min_us"] * 1e-6), 1)
    return r


def elementwise_bench():
    """Prefill-size elementwise kernels: GB/s of silu_mul and fused add+RMSNorm."""
    from githubrepostorag_amd.ops import elementwise as E
    from githubrepostorag_amd.ops.norm import rmsnorm

    dev = torch.device("cuda")
    T, I, H = 14336, 18944, 3584
    gu = torch.randn(T, 2 * I, device=dev, dtype=torch.bfloat16)
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    res = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16)
    r = rounds({"silu_mul": lambda: E.silu_mul(gu), "add_rmsnorm": lambda: rmsnorm(x, w, 1e-6, residual=res)},
               n=3, iters=10)
    nbytes = {"silu_mul": T * I * 2 * 3, "add_rmsnorm": T * H * 2 * 4}
    for k in r:
        r[k]["GB_s"] = round(nbytes[k] / (r[k]["min_us"] * 1e-6) / 1e9, 1)
    return r


def sampler_bench(B):
    dev = torch.device("cuda")
    V = 152064
    st = S.SamplerState(B, V, dev)
    for i in range(B):
        st.reset_slot(i, 0.4, 0.8, 0, 1.2, list(range(0, 2000, 7)))
    logits = torch.randn(B, V, device=dev, dtype=torch.bfloat16) * 3
    slots = torch.arange(B, device=dev, dtype=torch.int32)
    out = torch.empty(B, dtype=torch.int32, device=dev)
    S.sample(logits, st, slots, out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        S.sample(logits, st, slots, out=out)
    return rounds({"sampler_top_p": lambda: S.sample(logits, st, slots), "sampler_top_p_graph": g.replay})


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all")
    ap.add_argument("--out", default=None, help="also write the JSON here")
    args = ap.parse_args()
    res = {}
    if args.what in ("all", "gemm"):
        for M in (1, 8, 64):
            res.update(gemm_bench(M))
    if args.what == "decode_splits":  # split-KV plan at the bench's 512-row step: fewer splits, no combine
        for sl in (256, 512, 1024, 2048):
            res[f"decode_B512_ctx1100_split{sl}"] = attn_decode_bench(512, 1100, sl)
        for sl in (256, 2048):
            res[f"decode_B256_ctx1100_split{sl}"] = attn_decode_bench(256, 1100, sl)
            res[f"decode_B128_ctx2048_split{sl}"] = attn_decode_bench(128, 2048, sl)
    if args.what == "decode_ring":  # LDS ring depth of the 32-key decode kernel at the bench's / ingest's shapes
        for B, ctx, sl in ((512, 1100, 2048), (1024, 1100, 2048), (256, 1100, 1024), (64, 1152, 256),
                           (176, 3000, 1024), (16, 6000, 256), (1, 4096, 64)):
            res[f"decode_B{B}_ctx{ctx}_split{sl}"] = attn_decode_bench(B, ctx, sl)
    if args.what == "decode_nt_splits":  # non-temporal K/V loads x split-KV part length at the serving batches
        os.environ["MB_DECODE_ARMS"] = "nt"
        for B, ctx, sl in ((512, 1100, 2048), (512, 1100, 1024), (512, 1100, 512), (1024, 1100, 2048),
                           (1024, 1100, 1024), (256, 1100, 1024), (256, 1100, 512)):
            res[f"decode_B{B}_ctx{ctx}_split{sl}"] = attn_decode_bench(B, ctx, sl)
    if args.what in ("all", "attn", "decode"):
        res["decode_B512_ctx1100_split256"] = attn_decode_bench(512, 1100, 256)  # the bench's decode step
    if args.what in ("all", "attn"):
        for sl in (256, 512):
            res[f"decode_B64_ctx1152_split{sl}"] = attn_decode_bench(64, 1152, sl)
        res["decode_B1_ctx4096_split64"] = attn_decode_bench(1, 4096, 64)
        res["prefill_16x1024"] = attn_prefill_bench(16, 1024)
    if args.what == "prefill":
        res["prefill_16x1024"] = attn_prefill_bench(16, 1024)
        res["prefill_4x4096"] = attn_prefill_bench(4, 4096)
        res["prefill_2x11712"] = attn_prefill_bench(2, 11712)  # the reference's --max-model-len
    if args.what == "midm":  # 129-256-row projections: dispatched kernel vs tile schedules
        res.update(midm_bench())
    if args.what in ("all", "elementwise"):
        res["elementwise_T14336"] = elementwise_bench()
    if args.what in ("all", "sampler"):
        res["sampler_B64"] = sampler_bench(64)
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
