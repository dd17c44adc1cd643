"""Measured decode-GEMM dispatch table: for every decode weight shape and
every graph batch bucket M, time the library GEMM (hipBLASLt/rocBLAS with the
tuned solutions loaded), grag_gemm_skinny and grag_gemm_stream on cold
rotating weights (CUDA events, interleaved rounds) and record the fastest.
Writes githubrepostorag_amd/tuning/gemm_dispatch_gfx950.json, which
ops/linear.py consults at run time."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.models.configs import decoder_config  # noqa: E402
from githubrepostorag_amd.ops import linear as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--models", default="qwen2-7b,qwen2-1.5b")
ap.add_argument("--out", default="githubrepostorag_amd/tuning/gemm_dispatch_gfx950.json")
ap.add_argument("--M", default="1,2,4,8,16,24,32,48,64,96,128")
ap.add_argument("--merge", action="store_true", help="update the measured (N, K) rows of --out, keep the rest")
a = ap.parse_args()
L.enable_tuned_gemms()
dev = torch.device("cuda")
table = {}
report = {}


def time_fn(fn, reps=20, rounds=5):
    """GPU time per call inside a captured hipGraph (how the decode step runs
    them): no host launch overhead in the number."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps * 1000)
    del g
    return statistics.median(out)


shapes = set()
for spec in a.models.split(","):  # "model" or "model:tp" (per-rank shapes of a TP-sharded Qwen2)
    name, _, tp = spec.partition(":")
    tp = int(tp or 1)
    c = decoder_config(name)
    H, D = c.hidden_size, c.head_dim
    hq, hkv = c.num_heads // tp, max(1, c.num_kv_heads // tp)
    from githubrepostorag_amd.models.qwen2 import FFN_PAD  # noqa: E402

    I = -(-(c.intermediate_size // tp) // FFN_PAD) * FFN_PAD if tp > 1 else c.intermediate_size
    vocab = -(-c.vocab_size // tp)
    shapes |= {((hq + 2 * hkv) * D, H), (H, hq * D), (H, I), (-(-vocab // 8) * 8 if tp > 1 else vocab, H)}
    if tp == 1:
        shapes.add((2 * I, H))  # gate/up at TP>1 runs the fused SwiGLU kernels (ops/gemm.py mlp_gate_up)
for N, K in sorted(shapes):
    ncopy = max(2, min(12, (1 << 30) // (N * K * 2) + 1))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
    it = {"i": 0}

    def nxt():
        it["i"] = (it["i"] + 1) % ncopy
        return ws[it["i"]]

    rows = []
    for M in map(int, a.M.split(",")):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        cand = {"library": lambda: torch.nn.functional.linear(x, nxt())}
        if K % 64 == 0 and M <= 64:
            cand["skinny"] = lambda: L.gemm_skinny(x, nxt())
        if K % 16 == 0 and N % 4 == 0 and M <= 128:
            cand["stream"] = lambda: L.gemm_stream(x, nxt())
        t = {k: time_fn(f) for k, f in cand.items()}
        t2 = {k: time_fn(f) for k, f in cand.items()}  # second interleaved round
        t = {k: min(t[k], t2[k]) for k in t}
        best = min(t, key=t.get)
        rows.append([M, best])
        report[f"{N}x{K}_M{M}"] = {k: round(v, 2) for k, v in t.items()}
        print(f"N={N:6d} K={K:6d} M={M:4d} " + "  ".join(f"{k} {v:8.1f}" for k, v in t.items()) + f"  -> {best}",
              flush=True)
    table[f"{N},{K}"] = rows
    del ws
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
if a.merge and os.path.exists(a.out):
    old = json.load(open(a.out))
    table = {**old.get("table", {}), **table}
    report = {**old.get("times_us", {}), **report}
with open(a.out, "w") as f:
    json.dump({"arch": "gfx950", "note": "fastest decode GEMM per (N,K) and batch bucket M; see scripts/"
               "gemm_dispatch_table.py", "table": table, "times_us": report}, f, indent=1)
print("wrote", a.out)
