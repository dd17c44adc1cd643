"""IVF (inverted-file) cosine index for large static shards.

* training: spherical k-means on a sample; the assignment step is the fused
  score+top-k kernel with k=1 over the centroids (MFMA GEMM + argmax), the
  update is an index_add of member vectors followed by re-normalisation;
  empty lists are re-seeded from random points.  Across DP shards the
  centroid sums/counts are all-reduced (collective C6) so every shard trains
  the same quantiser.
* storage: vectors re-ordered list-contiguous in HBM ([N, d] bf16 +
  list offsets + original ids), so a probe is one contiguous range scan.
* search: coarse top-nprobe over the centroids, then the (query, list) probe
  pairs are grouped per list into work items of up to 16 queries and scanned
  by ``grag_score_topk_work`` in ONE launch; per-query candidates are merged
  with a device-side gather + topk.  Work-item construction is all on
  device (sort + segment ranks), no host loop.
"""
from __future__ import annotations

import torch

from ..ops.topk import num_waves, score_topk, score_topk_work


def _normalize(x: torch.Tensor) -> torch.Tensor:
    xf = x.float()
    return (xf / xf.norm(dim=-1, keepdim=True).clamp_min(1e-12)).to(x.dtype)


class IVFIndex:
    def __init__(self, dim: int, nlist: int, device="cuda", dtype=torch.bfloat16):
        self.dim = dim
        self.nlist = nlist
        self.device = torch.device(device)
        self.dtype = dtype
        self.centroids: torch.Tensor | None = None
        self.vectors = torch.zeros(0, dim, dtype=dtype, device=self.device)
        self.ids = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.offsets = torch.zeros(nlist + 1, dtype=torch.int64, device=self.device)
        self._offsets_host: list[int] = [0] * (nlist + 1)

    # ------------------------------------------------------------------ train
    def assign(self, X: torch.Tensor, chunk: int = 1 << 18) -> torch.Tensor:
        out = []
        for s in range(0, X.shape[0], chunk):
            _, ids = score_topk(self.centroids, X[s:s + chunk], 1)
            out.append(ids[:, 0])
        return torch.cat(out) if out else torch.zeros(0, dtype=torch.long, device=self.device)

    @torch.inference_mode()
    def train(self, sample: torch.Tensor, iters: int = 10, seed: int = 0, group=None) -> None:
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        X = _normalize(sample.to(self.device, self.dtype))
        m = X.shape[0]
        assert m >= self.nlist, "need at least nlist training points"
        init = torch.randperm(m, generator=g)[: self.nlist].to(self.device)
        C = X[init].clone()
        if group is not None and not group.trivial:
            group.broadcast(C)
        self.centroids = C
        for _ in range(iters):
            a = self.assign(X)
            sums = torch.zeros(self.nlist, self.dim, dtype=torch.float32, device=self.device)
            sums.index_add_(0, a, X.float())
            cnt = torch.bincount(a, minlength=self.nlist).float()
            if group is not None and not group.trivial:
                group.all_reduce(sums)
                group.all_reduce(cnt)
            empty = cnt == 0
            if bool(empty.any()):
                re = torch.randint(0, m, (int(empty.sum()),), generator=g).to(self.device)
                sums[empty] = X[re].float()
            self.centroids = _normalize(sums).to(self.dtype)

    # ------------------------------------------------------------------ add
    @torch.inference_mode()
    def add(self, X: torch.Tensor, ids: torch.Tensor | None = None) -> None:
        """(Re)build list storage with X [N, d] (bf16, normalised)."""
        X = X.to(self.device, self.dtype)
        if ids is None:
            ids = torch.arange(self.ids.numel(), self.ids.numel() + X.shape[0], device=self.device)
        a = self.assign(X)
        if self.vectors.shape[0]:
            a = torch.cat([self.assign(self.vectors), a])
            X = torch.cat([self.vectors, X])
            ids = torch.cat([self.ids, ids.to(self.device)])
        order = torch.argsort(a, stable=True)
        self.vectors = X[order].contiguous()
        self.ids = ids.to(self.device)[order].contiguous()
        cnt = torch.bincount(a, minlength=self.nlist)
        self.offsets = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        self.offsets[1:] = torch.cumsum(cnt, 0)
        self._offsets_host = self.offsets.cpu().tolist()

    @property
    def ntotal(self) -> int:
        return int(self.vectors.shape[0])

    # ------------------------------------------------------------------ search
    @torch.inference_mode()
    def search(self, Q: torch.Tensor, k: int, nprobe: int = 16):
        Q = _normalize(Q.to(self.device, self.dtype))
        nq = Q.shape[0]
        nprobe = min(nprobe, self.nlist)
        _, lists = score_topk(self.centroids, Q, nprobe)  # [nq, nprobe]
        if not Q.is_cuda:
            return self._search_ref(Q, lists, k)
        pair_q = torch.arange(nq, device=self.device).repeat_interleave(nprobe)
        pair_l = lists.reshape(-1).clamp_min(0)
        order = torch.argsort(pair_l, stable=True)
        sl, sq = pair_l[order], pair_q[order]
        P = sl.numel()
        # rank of each pair inside its list's group
        first = torch.ones(P, dtype=torch.bool, device=self.device)
        first[1:] = sl[1:] != sl[:-1]
        grp_start = torch.cummax(torch.where(first, torch.arange(P, device=self.device),
                                             torch.zeros(P, dtype=torch.long, device=self.device)), 0).values
        rank = torch.arange(P, device=self.device) - grp_start
        tile = rank // 16
        # one work item per (list, tile)
        new_item = first | (rank % 16 == 0)
        item = torch.cumsum(new_item.long(), 0) - 1
        W = int(item[-1]) + 1
        work_q = torch.full((W, 16), -1, dtype=torch.int32, device=self.device)
        work_q[item, rank % 16] = sq.to(torch.int32)
        work_l = torch.zeros(W, dtype=torch.long, device=self.device)
        work_l[item] = sl
        work_rows = torch.stack([self.offsets[work_l], self.offsets[work_l + 1]], 1).contiguous()
        del tile
        s, i = score_topk_work(self.vectors, Q, k, work_rows, work_q, 1, row_ids=self.ids)
        nw = num_waves()
        flat_s = s.reshape(W * 16, nw * k)
        flat_i = i.reshape(W * 16, nw * k)
        # candidates per query: its nprobe (item, slot) rows
        pos = item * 16 + rank % 16  # per sorted pair
        cand_idx = torch.empty(P, dtype=torch.long, device=self.device)
        cand_idx[order] = pos
        cand_idx = cand_idx.view(nq, nprobe)
        cs = flat_s[cand_idx].reshape(nq, -1)
        ci = flat_i[cand_idx].reshape(nq, -1)
        kk = min(k, cs.shape[1])
        bs, sel = cs.topk(kk, dim=1)
        return bs, ci.gather(1, sel)

    def _search_ref(self, Q, lists, k):
        nq = Q.shape[0]
        out_s = torch.full((nq, k), float("-inf"))
        out_i = torch.full((nq, k), -1, dtype=torch.long)
        off = self._offsets_host
        for qi in range(nq):
            rows = torch.cat([torch.arange(off[l], off[l + 1]) for l in lists[qi].tolist() if l >= 0])
            if rows.numel() == 0:
                continue
            sc = self.vectors[rows].float() @ Q[qi].float()
            kk = min(k, sc.numel())
            v, j = sc.topk(kk)
            out_s[qi, :kk] = v
            out_i[qi, :kk] = self.ids[rows[j]]
        return out_s, out_i
