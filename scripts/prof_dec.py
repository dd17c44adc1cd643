"""Run one decode-GEMM plan (csrc/kernels/gemm_decode.hip) back to back on cold, rotating weights, for
rocprofv3 --pmc passes (scripts/pmc_dec.sh):
python scripts/prof_dec.py --shape gate_up --M 192 --plan 12,5,2,1,256 --reps 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import gemm as G  # noqa: E402

Q7 = {"qkv": (4608, 3584), "o": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944)}
ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="gate_up")
ap.add_argument("--M", type=int, default=192)
ap.add_argument("--plan", default="12,5,2,1,256", help="mt,nwv,ntw,ksplit[,gs] or 'tile'")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
N, K = Q7[a.shape]
silu = a.shape == "gate_up"
dev = torch.device("cuda")
x = torch.randn(a.M, K, device=dev, dtype=torch.bfloat16)
ncopy = max(2, min(10, (700 << 20) // (N * K * 2) + 1))
ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
if a.plan == "tile":
    S, SK = G.plan(a.M, N, K)
    G.WS.reserve(dev, G._ws_floats(a.M, N, S, SK))
    fn = (lambda w: G.gemm_silu(x, w, ksplit=S, sk=SK)) if silu else (lambda w: G.gemm(x, w, ksplit=S, sk=SK))
else:
    plan = G.dec_plan(a.M, N, K, silu) if a.plan == "auto" else tuple(int(v) for v in a.plan.split(","))
    print("plan", plan)
    G.WS.reserve(dev, G.dec_ws_floats(a.M, N, G.dec_ksplit(K, plan[3])))
    fn = lambda w: G.gemm_decode(x, w, epi=G.EPI_SILU if silu else G.EPI_STORE, plan=plan)  # noqa: E731
for i in range(a.reps):
    fn(ws[i % ncopy])
torch.cuda.synchronize()
print("done")
