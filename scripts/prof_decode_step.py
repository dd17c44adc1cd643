"""One Qwen2-7B decode step at the bench's operating point (B live sequences, ~ctx cached tokens each,
random weights and KV), captured in a hipGraph and replayed back to back: wall time per step, and under
``rocprofv3 --kernel-trace --stats`` the per-kernel split of a decode step.

python scripts/prof_decode_step.py --B 512 --ctx 1100 --reps 30
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.models.configs import decoder_config  # noqa: E402
from githubrepostorag_amd.models.qwen2 import Qwen2Model  # noqa: E402
from githubrepostorag_amd.ops.attention import AttnMetadata  # noqa: E402
from githubrepostorag_amd.ops.linear import linear  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--ctx", type=int, default=1100)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--split-len", type=int, default=0, help="keys per split-KV part (0: the engine's plan, llm_engine._split_len_for)")
ap.add_argument("--model", default="qwen2-7b")
a = ap.parse_args()

dev = torch.device("cuda", 0)
cfg = decoder_config(a.model)
model = Qwen2Model(cfg, device=dev, seed=0)
B, ctx, BS = a.B, a.ctx, 16
nb = -(-(ctx + 1) // BS)
kv = model.allocate_kv_cache(B * nb + 1, BS)
for kc, vc in kv:  # random cached keys / values (zeros would collapse the softmax work)
    kc.normal_(0, 1)
    vc.normal_(0, 1)
i32 = dict(dtype=torch.int32, device=dev)
bt = (1 + torch.arange(B * nb, **i32)).view(B, nb)
pos = torch.full((B,), ctx, **i32)
slot = bt[:, ctx // BS] * BS + ctx % BS
from githubrepostorag_amd.engine.llm_engine import _pow2_at_least, _split_len_for  # noqa: E402

split_len = a.split_len or _split_len_for(B)
nsplit = -(-(ctx + 1) // split_len) if a.split_len else _pow2_at_least(-(-(ctx + 1) // split_len))
print(f"split-KV plan: {nsplit} parts of {split_len} keys")
hq, d = model.hq, model.head_dim
meta = AttnMetadata(q_start=torch.arange(B + 1, **i32), ctx_len=torch.full((B,), ctx + 1, **i32), block_tables=bt,
                    slot_mapping=slot, max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True, num_splits=nsplit,
                    split_len=split_len, part_o=torch.empty(nsplit * B * hq * d, dtype=torch.float32, device=dev),
                    part_ml=torch.empty(nsplit * B * hq * 2, dtype=torch.float32, device=dev))
ids = torch.randint(0, cfg.vocab_size, (B,), **i32)


def step():
    h = model.forward(ids, pos, meta, kv)
    return linear(h, model.lm_head)


with torch.inference_mode():
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    import time as _t
    host = []
    for _ in range(10):  # host cost of one replay call (hipGraphLaunch), GPU idle before it
        torch.cuda.synchronize()
        h0 = _t.perf_counter()
        g.replay()
        host.append((_t.perf_counter() - h0) * 1e3)
    torch.cuda.synchronize()
    print(f"graph replay host call: median {sorted(host)[len(host) // 2]:.3f} ms (min {min(host):.3f})")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    e1.synchronize()
print(f"decode step B={B} ctx={ctx}: {e0.elapsed_time(e1) / a.reps:.3f} ms per step (hipGraph, incl. LM head)")
