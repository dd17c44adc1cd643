"""(Probe behind the variant restriction in csrc/kernels/gemm_w4.hip; exercises the (16, 4) tiling.)

Dense A x one-hot W probe of gemm_w4 (W[n, k] = 1 at k = kn): y[m, n] = A[m, kn] (debug aid)."""
import torch
from githubrepostorag_amd.ops import w4 as W

dev = torch.device("cuda", 0)
torch.manual_seed(0)
for plan, M, N, K, stride, off in [((16, 4, 1), 192, 256, 3584, 1, 0), ((16, 4, 1), 192, 256, 3584, 13, 5),
                                   ((16, 4, 1), 224, 128, 3584, 1, 0), ((16, 4, 1), 224, 128, 3584, 27, 3)]:
    kn = torch.arange(N, device=dev) * stride + off
    w = torch.zeros(N, K, device=dev)
    w[torch.arange(N, device=dev), kn] = 1.0
    L = W.W4Linear.quantize(w)
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    y = W.gemm_w4(x, L, plan_=plan).float()
    ref = x.float()[:, kn]
    bad = (y - ref).abs() > 1e-2
    print(plan, stride, off, "bad rows", bad.any(1).nonzero().flatten().tolist()[:20], "bad n", bad.any(0).nonzero().flatten().tolist()[:20], flush=True)
    # dense both
    w2 = (torch.rand(N, K, device=dev) * 2 - 1) * 0.5
    L2 = W.W4Linear.quantize(w2)
    y2 = W.gemm_w4(x, L2, plan_=plan).float()
    r2 = x.float() @ L2.dequant(torch.float32).T
    e = (y2 - r2).abs()
    print("   dense rel", round((e.max() / r2.abs().max()).item(), 5), "worst rows", e.amax(1).topk(4).indices.tolist(), "worst n", e.amax(0).topk(4).indices.tolist())
