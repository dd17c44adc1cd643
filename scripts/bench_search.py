"""Search latency of the product IVF table (index/store.py) on an idle GPU:
10M x 1024 bf16 rows, nlist 4096, nprobe 32, batches of 8 / 64 queries,
unfiltered and with the namespace / repo filters fused in the scan.  Reports
per-stage device times (coarse top-nprobe, probe plan, list scan, merge)
from CUDA events and the end-to-end wall time of ``ShardedIndex.search`` +
``.cpu()``.

usage: python scripts/bench_search.py [--rows 10000000] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.index.sharded import ShardedIndex  # noqa: E402
from githubrepostorag_amd.ops import topk as T  # noqa: E402
from githubrepostorag_amd.utils import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--nlist", type=int, default=4096)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    corpus = synthetic.SyntheticCorpus(args.rows, seed=7)
    X = synthetic.clustered_vectors(args.rows, args.dim, seed=1000, device=dev)
    idx = ShardedIndex(args.dim, None, dev, kind="ivf", nlist=args.nlist, nprobe=args.nprobe)
    t0 = time.perf_counter()
    idx.build_corpus(corpus, X, seed=7)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    t = idx.table
    out = {"rows": args.rows, "build_s": round(build_s, 2)}
    for nq in (8, 64):
        Q = X[torch.randint(0, args.rows, (nq,), device=dev)].float()
        Q = Q + 0.02 * torch.randn_like(Q) / args.dim ** 0.5
        for name, flt in (("nofilter", None), ("namespace", {"namespace": corpus.namespace}),
                          ("repo", {"repo": corpus.repo_name(3)})):
            for _ in range(3):
                idx.search(Q, 10, flt)[1].cpu()
            walls = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                a = time.perf_counter()
                idx.search(Q, 10, flt)[1].cpu()
                walls.append((time.perf_counter() - a) * 1e3)
            # stage breakdown (device events)
            q = Q.to(torch.bfloat16)
            pc = t.predicates(flt)
            preds = pc[0]
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            ev[0].record()
            _, lists = T.score_topk(t.centroids, q, args.nprobe)
            ev[1].record()
            rows, wq, cand = T.ivf_plan(lists, t.offsets, t.nlist)
            ev[2].record()
            ps, pi = T.score_topk_work(t.vectors, q, 10, rows, wq, 1, preds=preds, bitmap=t.live, row_ids=t.slot_row)
            ev[3].record()
            L = T.num_waves() * 10
            T.merge_partials(ps.view(-1, L), pi.view(-1, L), 10, nq, cand=cand, cnt=args.nprobe)
            ev[4].record()
            torch.cuda.synchronize()
            st = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(4)]
            out[f"nq{nq}_{name}"] = {"wall_ms_p50": round(statistics.median(walls), 3),
                                     "coarse_us": st[0], "plan_us": st[1], "scan_us": st[2], "merge_us": st[3]}
            print(json.dumps({f"nq{nq}_{name}": out[f"nq{nq}_{name}"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
