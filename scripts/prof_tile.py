"""Run the owned tile GEMM (csrc/kernels/gemm_tile.hip) on one prefill shape back to back on random
operands (for rocprofv3 --pmc passes, scripts/pmc_tile.sh) and print its wall-clock TF/s.

python scripts/prof_tile.py --shape gate_up --M 7104 --reps 40
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import gemm as G  # noqa: E402

Q7 = {"qkv": (4608, 3584), "o": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944)}
ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="gate_up")
ap.add_argument("--M", type=int, default=7104)
ap.add_argument("--reps", type=int, default=40)
ap.add_argument("--sched", default="", help="ksplit,sk (default: the dispatch table's)")
a = ap.parse_args()
N, K = Q7[a.shape]
silu = a.shape == "gate_up"
dev = torch.device("cuda")
x = (torch.rand(a.M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
ks, sk = map(int, a.sched.split(",")) if a.sched else G.schedule(a.M, N, K, silu)
G.WS.reserve(dev, G._ws_floats(a.M, N, ks, sk))
fn = (lambda: G.gemm_silu(x, w, ksplit=ks, sk=sk)) if silu else (lambda: G.gemm(x, w, ksplit=ks, sk=sk))
for _ in range(5):
    fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.reps):
    fn()
e.record()
e.synchronize()
us = s.elapsed_time(e) * 1e3 / a.reps
print(f"{a.shape} M={a.M} sched=({ks},{sk}) {us:.1f} us {2 * a.M * N * K / us / 1e6:.1f} TF/s")
