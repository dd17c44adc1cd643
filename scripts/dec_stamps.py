"""Where a decode-GEMM launch spends its time, per workgroup (csrc/kernels/gemm_decode.hip stamps): every
workgroup records s_memrealtime (100 MHz, one clock for the whole chip) at its start and at the end of its
main loop, plus its XCC.  Cold weights (rotating copies), eager launches with a sync between them.

python scripts/dec_stamps.py --shape o --M 176 [--plan auto|mt:nwv:ntw:ks[:gs]] [--packed 1]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops import gemm as G  # noqa: E402
from githubrepostorag_amd.ops._lib import lib  # noqa: E402

Q7 = {"qkv": (4608, 3584), "o": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944)}
ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="o")
ap.add_argument("--M", type=int, default=176)
ap.add_argument("--plan", default="auto")
ap.add_argument("--packed", type=int, default=0)
ap.add_argument("--reps", type=int, default=6)
a = ap.parse_args()
N, K = Q7[a.shape]
silu = a.shape == "gate_up"
dev = torch.device("cuda")
x = torch.randn(a.M, K, device=dev, dtype=torch.bfloat16)
ncopy = max(2, min(8, (700 << 20) // (N * K * 2) + 1))
ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
plan = G.dec_plan(a.M, N, K, silu) if a.plan == "auto" else tuple(int(v) for v in a.plan.split(":"))
pk = [G.DecPacked(w, silu) for w in ws] if a.packed else [None] * ncopy
G.WS.reserve(dev, G.dec_ws_floats(a.M, N, G.dec_ksplit(K, plan[3])))
epi = G.EPI_SILU if silu else G.EPI_STORE
buf = torch.zeros(4 * 4096, dtype=torch.int64, device=dev)
print(f"{a.shape} M={a.M} plan={plan} packed={a.packed}")
for i in range(a.reps + 1):
    buf.zero_()
    torch.cuda.synchronize()
    lib().grag_gemm_decode_stamps(buf.data_ptr() if i else None)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    G.gemm_decode(x, ws[i % ncopy], epi=epi, plan=plan, packed=pk[i % ncopy])
    e1.record()
    torch.cuda.synchronize()
    lib().grag_gemm_decode_stamps(None)
    if not i:
        continue
    st = buf.view(-1, 4).cpu()
    st = st[st[:, 0] > 0]
    t0 = int(st[:, 0].min())
    start = ((st[:, 0] - t0) * 10 / 1000.0).tolist()  # us
    end = ((st[:, 1] - t0) * 10 / 1000.0).tolist()
    life = [e - s for s, e in zip(start, end)]
    q = lambda v, f: sorted(v)[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
    print(f"rep {i}: event {e0.elapsed_time(e1) * 1000:.1f} us, WGs {len(st)}, span {max(end):.1f} us | start p50 "
          f"{q(start, .5):.1f} p90 {q(start, .9):.1f} max {max(start):.1f} | main-loop end p10 {q(end, .1):.1f} p50 "
          f"{q(end, .5):.1f} p90 {q(end, .9):.1f} | life p50 {statistics.median(life):.1f} max {max(life):.1f}")
    if i == a.reps:
        by = {}
        for row, s_, e_ in zip(st.tolist(), start, end):
            by.setdefault(row[2] & 15, []).append((s_, e_))
        for xcc in sorted(by):
            v = by[xcc]
            print(f"   xcc {xcc}: {len(v)} WGs, start max {max(s for s, _ in v):.1f}, end p50 "
                  f"{statistics.median(e for _, e in v):.1f} max {max(e for _, e in v):.1f}")
