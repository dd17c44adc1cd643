"""Time the fused qkv bias + RoPE + paged K/V store pass (csrc/kernels/elementwise.hip qkv_rope_kernel) on the
Qwen2-7B shapes at a few token counts, bf16 input (prefill) and deferred split-K planes (decode batches);
CUDA-event wall time per call over back-to-back launches.

python scripts/prof_rope.py --T 1:176:2048:8192
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import elementwise as E  # noqa: E402
from githubrepostorag_amd.ops.linear import linear_deferred  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--T", default="1:176:2048:8192")
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda")
Hq, Hkv, D, BS, K = 28, 4, 128, 16, 3584
N = (Hq + 2 * Hkv) * D
cs = E.rope_cos_sin(16384, D, 1e6, dev)
bias = torch.randn(N, device=dev, dtype=torch.bfloat16)
for T in [int(t) for t in a.T.replace(",", ":").split(":")]:
    NB = T // BS + 2
    kc = torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    pos = torch.arange(T, dtype=torch.int32, device=dev)
    slots = torch.arange(T, dtype=torch.int32, device=dev)
    qkv = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    arms = {"bf16": qkv}
    if T <= 512:
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        arms["planes"] = linear_deferred(x, w)
    for name, inp in arms.items():
        for _ in range(3):
            E.qkv_rope_kvstore(inp, bias, pos, cs, slots, kc, vc, Hq, Hkv, D)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            E.qkv_rope_kvstore(inp, bias, pos, cs, slots, kc, vc, Hq, Hkv, D)
        e.record()
        e.synchronize()
        print(f"qkv_rope T={T} {name}: {s.elapsed_time(e) * 1e3 / a.reps:.1f} us", flush=True)
