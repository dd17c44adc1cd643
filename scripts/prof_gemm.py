"""Run a few decode-GEMM variants back to back (for rocprofv3 --pmc passes):
python scripts/prof_gemm.py --shape down --M 64 --reps 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops.linear import gemm_skinny, gemm_stream  # noqa: E402
from scripts.bench_gemm import SHAPES  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="down")
ap.add_argument("--M", type=int, default=64)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--variants", default="hipblaslt,stream,skinny")
a = ap.parse_args()
N, K = SHAPES[a.shape]
dev = torch.device("cuda")
x = torch.randn(a.M, K, device=dev, dtype=torch.bfloat16)
ncopy = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
fns = {"hipblaslt": lambda w: torch.nn.functional.linear(x, w), "stream": lambda w: gemm_stream(x, w),
       "skinny": lambda w: gemm_skinny(x, w)}
for v in a.variants.split(","):
    for i in range(a.reps):
        fns[v](ws[i % ncopy])
    torch.cuda.synchronize()
print("done")
