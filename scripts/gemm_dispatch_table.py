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
for name in a.models.split(","):
    c = decoder_config(name)
    H, I, D = c.hidden_size, c.intermediate_size, c.head_dim
    shapes |= {((c.num_heads + 2 * c.num_kv_heads) * D, H), (H, c.num_heads * D), (2 * I, H), (H, I),
               (c.vocab_size, H)}
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
with open(a.out, "w") as f:
    json.dump({"arch": "gfx950", "note": "fastest decode GEMM per (N,K) and batch bucket M; see scripts/"
               "gemm_dispatch_table.py", "table": table, "times_us": report}, f, indent=1)
print("wrote", a.out)
