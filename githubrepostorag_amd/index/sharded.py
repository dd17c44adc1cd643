"""Data-parallel sharded index over the product vector table: each rank keeps
a shard of the rows in its own HBM (288 GB per MI355X: a 10M x 1024 bf16
shard is 20.5 GB) as an ``index/store.py`` VectorTable (flat or IVF, with the
metadata columns, live bitmap and filters of the service store), and searches
it locally with the fused kernels.  Every rank brings its own query batch, so
one search is three steps over xGMI:
  C4  all-gather the query embeddings ([W, nq, d] bf16: every shard scores
      every rank's queries),
      local fused score + filter + top-k of all W*nq queries against this shard,
  C3  all-to-all of the per-shard lists (slice j = the lists for rank j's
      queries: W*nq*k (score, id) pairs in, the same out, never the whole
      W x W*nq x k gather), then a local merge to the global top-k.
Query batches of different sizes are padded to the largest.  Global ids are
interleaved: global = local * world + rank, so shards never collide and no id
exchange is needed at insert time.  The IVF quantiser is trained jointly:
the k-means sums/counts are all-reduced every iteration (C6), so every shard
probes the same lists.
"""
from __future__ import annotations

import torch

from ..ops.topk import merge_fits, merge_partials
from ..parallel.comm import Group
from ..utils.gpu_guard import guarded
from .store import VectorTable


class ShardView:
    """Virtual rows of one shard: local row j = global corpus row j * world + rank."""

    def __init__(self, corpus, rank: int, world: int):
        self.corpus, self.rank, self.world = corpus, rank, world

    def _g(self, j: int) -> int:
        return j * self.world + self.rank

    def row_id(self, j: int) -> str:
        return self.corpus.row_id(self._g(j))

    def text(self, j: int) -> str:
        return self.corpus.text(self._g(j))

    def meta(self, j: int) -> dict:
        return self.corpus.meta(self._g(j))

    def index_of(self, row_id: str):
        i = self.corpus.index_of(row_id)
        return None if i is None or i % self.world != self.rank else i // self.world

    def spec(self) -> dict:
        return {"kind": "shard", "corpus": self.corpus.spec(), "rank": self.rank, "world": self.world}

    def register(self, table) -> None:
        self.corpus.register(table)

    def columns(self, device) -> dict:
        n_local = self.n
        idx = torch.arange(n_local, device=device, dtype=torch.int64) * self.world + self.rank
        return {k: v[idx] for k, v in self.corpus.columns(device).items()}


class ShardedIndex:
    def __init__(self, dim: int, group: Group | None = None, device="cuda", kind: str = "ivf", nlist: int = 1024,
                 nprobe: int = 16):
        self.group = group or Group([0])
        self.dim = dim
        self.device = torch.device(device)
        self.kind = kind
        self.nprobe = nprobe
        self.table = VectorTable("shard", dim, self.device, index_kind=kind, nlist=nlist, nprobe=nprobe,
                                 compact_min=1 << 62)

    def global_ids(self, local: torch.Tensor) -> torch.Tensor:
        return torch.where(local >= 0, local * self.group.size + self.group.rank, local)

    def _finish(self, train_sample: int, iters: int, seed: int) -> None:
        if self.kind == "ivf":
            self.table.compact(train_iters=iters, sample=train_sample, seed=seed,
                               group=None if self.group.trivial else self.group)

    @torch.inference_mode()
    def build(self, X: torch.Tensor, train_sample: int = 131072, iters: int = 8, seed: int = 0) -> None:
        """Shard of anonymous vectors (local row j = global j * world + rank)."""
        from ..utils.synthetic import SyntheticCorpus

        view = ShardView(SyntheticCorpus(X.shape[0] * self.group.size, seed=seed), self.group.rank, self.group.size)
        self.table.add_virtual(view, X.to(self.device, torch.bfloat16), columns={})
        self._finish(train_sample, iters, seed)

    @torch.inference_mode()
    def build_corpus(self, corpus, X_local: torch.Tensor, train_sample: int = 131072, iters: int = 8,
                     seed: int = 0) -> None:
        """This rank's shard of a virtual corpus (rows i = rank (mod world)), with its
        metadata columns, so filtered searches run inside the scan."""
        view = ShardView(corpus, self.group.rank, self.group.size)
        view.n = X_local.shape[0]
        self.table.add_virtual(view, X_local)
        self._finish(train_sample, iters, seed)

    def recall(self, Q: torch.Tensor, k: int, flt: dict | None = None, nprobes=(None,)) -> dict:
        """recall@k of the IVF search against the exact scan over every shard, for each nprobe in
        ``nprobes`` (None: the index's own), with the wall time of each search (collective: every rank calls
        it with its own queries)."""
        import time

        def timed(fn):
            if Q.is_cuda:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            if Q.is_cuda:
                torch.cuda.synchronize()
            return out, time.perf_counter() - t0

        (_, truth), t_exact = timed(lambda: self.search(Q, k, flt, exact=True))
        truth = truth.cpu().tolist()
        out = {"queries": Q.shape[0], "k": k, "exact_scan_ms": round(t_exact * 1000, 2), "by_nprobe": []}
        keep = self.table.nprobe
        try:
            for npb in nprobes:
                self.table.nprobe = int(npb or keep)
                self.search(Q, k, flt)  # warm the plan for this nprobe
                (_, got), t = timed(lambda: self.search(Q, k, flt))
                got = got.cpu().tolist()
                hit = sum(len({x for x in a if x >= 0} & {x for x in b if x >= 0}) for a, b in zip(got, truth))
                tot = sum(len([x for x in b if x >= 0]) for b in truth)
                out["by_nprobe"].append({"nprobe": self.table.nprobe, "recall_at_k": round(hit / max(1, tot), 4),
                                         "search_ms": round(t * 1000, 2)})
        finally:
            self.table.nprobe = keep
        return out

    @property
    def local_size(self) -> int:
        return self.table.count()

    def _local(self, Q: torch.Tensor, k: int, flt: dict | None = None, exact: bool = False):
        """This shard's top-k for every query, with the whole filter applied the way
        ``VectorTable.search`` applies it: up to four predicates fused in the scan,
        further ones ANDed into the row bitmap, and host-side checks (unindexed
        fields; the exact test behind a multi-value field's bloom bit) on an
        over-fetched candidate list, so no filter is dropped."""
        from .store import OP_EQ, _and_bitmap

        t = self.table
        nq = Q.shape[0]
        empty = (torch.full((nq, k), float("-inf"), device=Q.device),
                 torch.full((nq, k), -1, dtype=torch.long, device=Q.device))
        with t.lock:
            pc = t.predicates(flt)
            if pc is None or t.n == 0:
                return empty
            preds, checks = pc
            bitmap = t.live
            if len(preds) > 4:
                m = torch.ones(t.n, dtype=torch.bool, device=self.device)
                for p in preds[4:]:
                    c = p.column[: t.n]
                    m &= (c == p.value) if p.op == OP_EQ else ((c & p.value) != 0)
                bitmap = _and_bitmap(t.live, m)
                preds = preds[:4]
            kk = max(k, min(32, k + 8)) if checks else k
            if exact and t.n:  # every live row of the shard (IVF: the same fused scan over all slots)
                from ..ops.topk import score_topk

                s, i = score_topk(t.vectors[: t.n], Q.to(self.device, t.dtype), kk, preds=preds, bitmap=bitmap,
                                  row_ids=t.slot_row if t.ivf else None)
            else:
                s, i = t._scan(Q.to(self.device, t.dtype), kk, preds, bitmap, None)
            t._track_read()
        if checks:  # exact host checks on the over-fetched rows, then back to [nq, k]
            sl, il = s.float().cpu().tolist(), i.cpu().tolist()
            out_s = torch.full((nq, k), float("-inf"))
            out_i = torch.full((nq, k), -1, dtype=torch.long)
            for q in range(nq):
                j = 0
                for sc, r in zip(sl[q], il[q]):
                    if r < 0 or j >= k or not t._host_ok(t.rows.get(r)[2], checks):
                        continue
                    out_s[q, j], out_i[q, j] = sc, r
                    j += 1
            s, i = out_s.to(Q.device), out_i.to(Q.device)
        elif kk > k:
            s, i = s[:, :k], i[:, :k]
        return s.float(), self.global_ids(i)

    @guarded
    @torch.inference_mode()
    def search(self, Q: torch.Tensor, k: int, flt: dict | None = None, exact: bool = False):
        """This rank's queries Q [nq, d] -> global top-k (scores fp32, ids int64).  ``exact``: every shard
        scans all its rows (the ground truth recall is measured against) instead of the probed IVF lists."""
        g = self.group
        Q = Q.to(self.device, torch.bfloat16)
        if g.trivial:
            return self._local(Q, k, flt, exact)
        nq = Q.shape[0]
        sizes = g.all_gather(torch.tensor([nq], dtype=torch.int64, device=self.device)).view(-1)
        qmax = int(sizes.max())
        Qp = torch.zeros(qmax, Q.shape[1], dtype=Q.dtype, device=self.device)
        Qp[:nq] = Q
        Qall = g.all_gather(Qp).view(g.size * qmax, -1)  # C4
        s, i = self._local(Qall, k, flt, exact)
        kk = s.shape[1]
        packed = torch.empty(g.size * qmax, kk, 2, dtype=torch.int64, device=self.device)
        packed[..., 0] = i
        packed[..., 1] = s.view(torch.int32).to(torch.int64)
        recv = g.all_to_all(packed.view(g.size, qmax, kk, 2))  # C3: [shard, my query, k, 2]
        ids = recv[..., 0]
        sc = recv[..., 1].to(torch.int32).view(torch.float32)
        if Q.is_cuda and merge_fits(g.size, kk, 0, k):  # device merge: query q's lists are rows q + j*qmax
            ms, mi = merge_partials(sc.reshape(-1, kk).contiguous(), ids.reshape(-1, kk).contiguous(), k, qmax,
                                    cnt=g.size, affine=(qmax, 0, qmax))
            return ms[:nq], mi[:nq]
        ids = ids.permute(1, 0, 2).reshape(qmax, -1)[:nq]
        sc = sc.permute(1, 0, 2).reshape(qmax, -1)[:nq]
        sc = torch.where(ids >= 0, sc, torch.full_like(sc, float("-inf")))
        top, sel = sc.topk(min(k, sc.shape[1]), dim=1)
        return top, ids.gather(1, sel)
