"""Data-parallel sharded index: each rank keeps a shard of the vectors in its
own HBM (288 GB per MI355X: a 10M x 1024 bf16 shard is 20.5 GB) and searches
it locally with the fused kernels.  Every rank brings its own query batch, so
one search is three steps over xGMI:
  C4  all-gather the query embeddings ([W, nq, d] bf16: every shard scores
      every rank's queries),
      local fused score + top-k of all W*nq queries against this shard,
  C3  all-to-all of the per-shard lists (slice j = the lists for rank j's
      queries: W*nq*k (score, id) pairs in, the same out, never the whole
      W x W*nq x k gather), then a local merge to the global top-k.
Query batches of different sizes are padded to the largest.  Global ids are
interleaved: global = local * world + rank, so shards never collide and no id
exchange is needed at insert time.
"""
from __future__ import annotations

import torch

from ..ops.topk import score_topk
from ..parallel.comm import Group
from ..utils.gpu_guard import guarded
from .ivf import IVFIndex


class ShardedIndex:
    def __init__(self, dim: int, group: Group | None = None, device="cuda", kind: str = "ivf", nlist: int = 1024,
                 nprobe: int = 16):
        self.group = group or Group([0])
        self.dim = dim
        self.device = torch.device(device)
        self.kind = kind
        self.nprobe = nprobe
        self.ivf = IVFIndex(dim, nlist, device) if kind == "ivf" else None
        self.flat = torch.zeros(0, dim, dtype=torch.bfloat16, device=self.device)

    def global_ids(self, local: torch.Tensor) -> torch.Tensor:
        return torch.where(local >= 0, local * self.group.size + self.group.rank, local)

    @torch.inference_mode()
    def build(self, X: torch.Tensor, train_sample: int = 131072, iters: int = 8, seed: int = 0) -> None:
        if self.kind == "ivf":
            m = min(train_sample, X.shape[0])
            g = torch.Generator(device="cpu")
            g.manual_seed(seed + self.group.rank)
            idx = torch.randperm(X.shape[0], generator=g)[:m].to(X.device)
            self.ivf.train(X[idx], iters=iters, seed=seed, group=self.group)
            self.ivf.add(X)
        else:
            self.flat = X.to(self.device, torch.bfloat16).contiguous()

    @property
    def local_size(self) -> int:
        return self.ivf.ntotal if self.kind == "ivf" else int(self.flat.shape[0])

    def _local(self, Q: torch.Tensor, k: int):
        if self.kind == "ivf":
            s, i = self.ivf.search(Q, k, self.nprobe)
        else:
            s, i = score_topk(self.flat, Q.to(self.device, torch.bfloat16), k)
        return s.float(), self.global_ids(i)

    @guarded
    @torch.inference_mode()
    def search(self, Q: torch.Tensor, k: int):
        """This rank's queries Q [nq, d] -> global top-k (scores fp32, ids int64)."""
        g = self.group
        Q = Q.to(self.device, torch.bfloat16)
        if g.trivial:
            return self._local(Q, k)
        nq = Q.shape[0]
        sizes = g.all_gather(torch.tensor([nq], dtype=torch.int64, device=self.device)).view(-1)
        qmax = int(sizes.max())
        Qp = torch.zeros(qmax, Q.shape[1], dtype=Q.dtype, device=self.device)
        Qp[:nq] = Q
        Qall = g.all_gather(Qp).view(g.size * qmax, -1)  # C4
        s, i = self._local(Qall, k)
        kk = s.shape[1]
        packed = torch.empty(g.size * qmax, kk, 2, dtype=torch.int64, device=self.device)
        packed[..., 0] = i
        packed[..., 1] = s.view(torch.int32).to(torch.int64)
        recv = g.all_to_all(packed.view(g.size, qmax, kk, 2))  # C3: [shard, my query, k, 2]
        ids = recv[..., 0].permute(1, 0, 2).reshape(qmax, -1)[:nq]
        sc = recv[..., 1].to(torch.int32).view(torch.float32).permute(1, 0, 2).reshape(qmax, -1)[:nq]
        sc = torch.where(ids >= 0, sc, torch.full_like(sc, float("-inf")))
        top, sel = sc.topk(min(k, sc.shape[1]), dim=1)
        return top, ids.gather(1, sel)
