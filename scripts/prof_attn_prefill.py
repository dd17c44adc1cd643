"""Run the paged prefill attention (csrc/kernels/attention.hip attn_prefill_kernel, the engine's 8-wave
LDS-DMA arm) back to back on random operands at one (sequences x length) shape, for rocprofv3 --pmc passes
(scripts/pmc_py.sh), and print its wall-clock TF/s (causal FLOPs: 4 * L^2 / 2 * D per query head).

python scripts/prof_attn_prefill.py --nseq 2 --L 11712 --reps 20 [--nw 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import attention as A  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nseq", type=int, default=2)
ap.add_argument("--L", type=int, default=11712)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--nw", type=int, default=5, help="prefill arm code (ops/attention.py): 5 = 8-wave LDS-DMA ring")
a = ap.parse_args()
dev = torch.device("cuda")
Hq, Hkv, D, BS = 28, 4, 128, 16
nbs = (a.L + BS - 1) // BS
kc = torch.randn(a.nseq * nbs + 1, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
vc = torch.randn_like(kc)
q = torch.randn(a.nseq * a.L, Hq, D, device=dev, dtype=torch.bfloat16)
bt = (torch.arange(a.nseq * nbs, device=dev, dtype=torch.int32) + 1).view(a.nseq, nbs)
meta = A.AttnMetadata(q_start=torch.arange(0, a.nseq * a.L + 1, a.L, device=dev, dtype=torch.int32),
                      ctx_len=torch.full((a.nseq,), a.L, device=dev, dtype=torch.int32), block_tables=bt,
                      slot_mapping=torch.zeros(a.nseq * a.L, dtype=torch.int32, device=dev), max_q_len=a.L,
                      num_seqs=a.nseq, num_tokens=a.nseq * a.L)
meta.extra = {"prefill_nw": a.nw}
for _ in range(3):
    A.paged_attention(q, kc, vc, meta, 0.088)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.reps):
    A.paged_attention(q, kc, vc, meta, 0.088)
e.record()
e.synchronize()
us = s.elapsed_time(e) * 1e3 / a.reps
fl = a.nseq * Hq * a.L * a.L / 2 * D * 4
print(f"attn prefill nseq={a.nseq} L={a.L} nw={a.nw}: {us:.1f} us {fl / us / 1e6:.1f} TF/s")
