"""Decode-GEMM microbench: plain hipBLASLt ``F.linear`` vs split-K over the
library (strided-batched GEMM of K/S slices with fp32 output + reduce) for the
Qwen2-7B projections at continuous-batching decode sizes (M = 64..256).

Weights rotate over enough copies to defeat the 256 MB MALL (cold weights, as
in a real decode step) and every variant is timed inside a hipGraph so launch
overhead does not count.  Output: one JSON line per (shape, M, variant).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

SHAPES = [(3584, 18944, "down"), (3584, 3584, "o"), (4608, 3584, "qkv"), (37888, 3584, "gate_up")]
MS = [64, 96, 128, 160, 192, 224, 256]


def splitk(x, w, S):
    M, K = x.shape
    N = w.shape[0]
    xs = x.view(M, S, K // S).transpose(0, 1)  # [S, M, K/S]
    ws = w.view(N, S, K // S).transpose(0, 1).transpose(1, 2)  # [S, K/S, N]
    return torch.bmm(xs, ws, out_dtype=torch.float32).sum(0).to(x.dtype)


def timed(fn, ws, x, reps=8):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for w in ws:
            fn(x, w)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            for w in ws:
                fn(x, w)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * reps * len(ws))


def main():
    from githubrepostorag_amd.ops.linear import enable_tuned_gemms, linear

    if "--untuned" not in sys.argv:
        print("# tuned library GEMMs:", enable_tuned_gemms(), file=sys.stderr)
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    for N, K, name in SHAPES:
        copies = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in MS:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = F.linear(x.float(), ws[0].float())
            row = {"shape": name, "N": N, "K": K, "M": M,
                   "library_us": round(timed(lambda a, b: F.linear(a, b), ws, x), 1),
                   "dispatch_us": round(timed(lambda a, b: linear(a, b), ws, x), 1)}
            for S in (2, 4, 8, 16):
                if K % (S * 64):
                    continue
                y = splitk(x, ws[0], S)
                err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                row[f"splitk{S}_us"] = round(timed(lambda a, b, S=S: splitk(a, b, S), ws, x), 1)
                row[f"splitk{S}_relerr"] = float(f"{err:.2e}")
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
