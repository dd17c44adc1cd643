"""Minimal repro: sampler inside a captured hipGraph."""
import faulthandler
import sys

faulthandler.enable()
import torch  # noqa: E402

sys.path.insert(0, ".")
from githubrepostorag_amd.ops import sampling as S  # noqa: E402

dev = torch.device("cuda")
B, V = 8, 152064
st = S.SamplerState(B, V, dev)
for i in range(B):
    st.reset_slot(i, 0.4, 0.8, 0, 1.2, [1, 2, 3])
logits = torch.randn(B, V, device=dev, dtype=torch.bfloat16)
slots = torch.arange(B, device=dev, dtype=torch.int32)
out = torch.empty(B, dtype=torch.int32, device=dev)
S.sample(logits, st, slots, out=out)
torch.cuda.synchronize()
print("eager ok", out.tolist(), flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    S.sample(logits, st, slots, out=out)
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", out.tolist(), flush=True)
