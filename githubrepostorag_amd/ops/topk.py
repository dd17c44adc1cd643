"""Fused cosine-score + filter + top-k (vector index hot path)."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from ._lib import call, lib, ptr

OP_EQ, OP_BITAND = 1, 2
MAX_FILTERS = 4
MAX_K = 32


@dataclass
class Predicate:
    column: torch.Tensor  # int32 [N] dictionary-encoded (or bitset) column
    value: int
    op: int = OP_EQ


def _mask_ref(n, preds, bitmap, device, row0=0):
    m = torch.ones(n, dtype=torch.bool, device=device)
    for p in preds or []:
        c = p.column[row0:row0 + n]
        m &= (c == p.value) if p.op == OP_EQ else ((c & p.value) != 0)
    if bitmap is not None:
        idx = torch.arange(row0, row0 + n, device=device)
        m &= ((bitmap[idx >> 5].long() >> (idx & 31)) & 1).bool()
    return m


def score_topk_ref(X, Q, k, preds=None, bitmap=None, row_ids=None, chunk=1 << 20, qpred=None):
    nq, N = Q.shape[0], X.shape[0]
    best_s = torch.full((nq, 0), float("-inf"), device=Q.device)
    best_i = torch.zeros((nq, 0), dtype=torch.long, device=Q.device)
    qf = Q.float()
    for r0 in range(0, N, chunk):
        xs = X[r0:r0 + chunk].float()
        s = qf @ xs.T
        m = _mask_ref(xs.shape[0], preds, bitmap, Q.device, r0)
        s = s.masked_fill(~m[None, :], float("-inf"))
        if qpred is not None:
            cols, sel, vals = qpred
            for qi in range(nq):
                c = int(sel[qi])
                if c >= 0:
                    s[qi] = s[qi].masked_fill(cols[c][r0:r0 + xs.shape[0]] != int(vals[qi]), float("-inf"))
        ids = torch.arange(r0, r0 + xs.shape[0], device=Q.device)
        best_s = torch.cat([best_s, s], 1)
        best_i = torch.cat([best_i, ids[None, :].expand(nq, -1)], 1)
        kk = min(k, best_s.shape[1])
        best_s, sel = best_s.topk(kk, dim=1)
        best_i = best_i.gather(1, sel)
    if best_s.shape[1] < k:
        pad = k - best_s.shape[1]
        best_s = torch.cat([best_s, torch.full((nq, pad), float("-inf"), device=Q.device)], 1)
        best_i = torch.cat([best_i, torch.full((nq, pad), -1, dtype=torch.long, device=Q.device)], 1)
    best_i = torch.where(torch.isinf(best_s), torch.full_like(best_i, -1), best_i)
    if row_ids is not None:
        best_i = torch.where(best_i >= 0, row_ids[best_i.clamp_min(0)], best_i)
    return best_s, best_i


def _filter_args(preds):
    preds = list(preds or [])
    if len(preds) > MAX_FILTERS:
        raise ValueError(f"at most {MAX_FILTERS} fused predicates")
    cols = (ctypes.c_void_p * MAX_FILTERS)()
    vals = (ctypes.c_int32 * MAX_FILTERS)()
    ops = (ctypes.c_int32 * MAX_FILTERS)()
    for i, p in enumerate(preds):
        cols[i] = p.column.data_ptr()
        vals[i] = int(p.value)
        ops[i] = int(p.op)
    return cols, vals, ops, len(preds)


def _qpred_args(qpred):
    """qpred = (columns: list[int32 tensor], colsel int32 [nq], vals int32 [nq])"""
    arr = (ctypes.c_void_p * 8)()
    if qpred is None:
        return arr, 0, None, None
    cols, sel, vals = qpred
    if len(cols) > 8:
        raise ValueError("at most 8 per-query predicate columns")
    for i, c in enumerate(cols):
        arr[i] = c.data_ptr()
    # return the tensors (not raw pointers) so they outlive the launch call
    return arr, len(cols), sel.to(torch.int32).contiguous(), vals.to(torch.int32).contiguous()


def _kmax(k):
    if k <= 16:
        return 16
    if k <= 32:
        return 32
    raise ValueError("k > 32")


def _nqt_for(nq, d, kmax):
    if kmax == 32:
        return 1 if nq <= 16 else 2
    if nq <= 16:
        return 1
    if nq <= 32 or d > 512:
        return 2
    return 4


def num_waves() -> int:
    return lib().grag_topk_num_waves()


def score_topk(X: torch.Tensor, Q: torch.Tensor, k: int, preds=None, bitmap=None, row_ids=None,
               row_begin: int = 0, row_end: int | None = None, qpred=None):
    """Top-k rows of X [N, d] (bf16, L2-normalised) by dot product with each
    query Q [nq, d].  Returns (scores fp32 [nq, k], ids int64 [nq, k]); ids are
    -1 where fewer than k rows pass the filters."""
    N = X.shape[0] if row_end is None else row_end
    nq = Q.shape[0]
    if not X.is_cuda or k > MAX_K:
        if row_begin or row_end is not None:
            raise NotImplementedError("row ranges on the reference path")
        return score_topk_ref(X, Q, k, preds, bitmap, row_ids, qpred=qpred)
    d = X.shape[1]
    if nq == 0 or N <= row_begin:
        return (torch.full((nq, k), float("-inf"), device=X.device),
                torch.full((nq, k), -1, dtype=torch.long, device=X.device))
    kmax = _kmax(k)
    nqt = _nqt_for(nq, d, kmax)
    nqtiles = (nq + nqt * 16 - 1) // (nqt * 16)
    rows = N - row_begin
    target = max(1, 1024 // nqtiles)
    rows_per_wg = max(128, -(-rows // target))
    rows_per_wg = -(-rows_per_wg // 16) * 16
    nchunks = -(-rows // rows_per_wg)
    nw = num_waves()
    slots = nqtiles * nchunks * nqt * 16 * nw
    out_s = torch.empty(slots * k, dtype=torch.float32, device=X.device)
    out_i = torch.empty(slots * k, dtype=torch.int64, device=X.device)
    cols, vals, ops, nf = _filter_args(preds)
    qc, nqc, qsel, qval = _qpred_args(qpred)
    Q = Q.contiguous()
    call("grag_score_topk_flat", ptr(X), row_begin, N, rows_per_wg, d, ptr(Q), nq, k, nqt, kmax,
         cols, vals, ops, nf, ptr(bitmap), ptr(row_ids), qc, nqc, ptr(qsel), ptr(qval), ptr(out_s), ptr(out_i))
    s = out_s.view(nqtiles, nchunks, nqt * 16, nw * k).permute(0, 2, 1, 3).reshape(nqtiles * nqt * 16, -1)[:nq]
    i = out_i.view(nqtiles, nchunks, nqt * 16, nw * k).permute(0, 2, 1, 3).reshape(nqtiles * nqt * 16, -1)[:nq]
    kk = min(k, s.shape[1])
    bs, sel = s.topk(kk, dim=1)
    bi = i.gather(1, sel)
    if kk < k:
        bs = torch.cat([bs, torch.full((nq, k - kk), float("-inf"), device=X.device)], 1)
        bi = torch.cat([bi, torch.full((nq, k - kk), -1, dtype=torch.long, device=X.device)], 1)
    return bs, bi


def score_topk_work(X, Q, k, work_rows: torch.Tensor, work_q: torch.Tensor, nqt: int, preds=None,
                    bitmap=None, row_ids=None, qpred=None):
    """IVF scan: work_rows int64 [W, 2] row ranges, work_q int32 [W, nqt*16]
    query ids (-1 = empty).  Returns raw partial lists (scores, ids) of shape
    [W, nqt*16, NWAVES*k]."""
    d = X.shape[1]
    kmax = _kmax(k)
    W = work_rows.shape[0]
    nw = num_waves()
    out_s = torch.empty(W * nqt * 16 * nw * k, dtype=torch.float32, device=X.device)
    out_i = torch.empty(W * nqt * 16 * nw * k, dtype=torch.int64, device=X.device)
    cols, vals, ops, nf = _filter_args(preds)
    qc, nqc, qsel, qval = _qpred_args(qpred)
    call("grag_score_topk_work", ptr(X), d, ptr(Q.contiguous()), Q.shape[0], k, nqt, kmax,
         ptr(work_rows), ptr(work_q), W, cols, vals, ops, nf, ptr(bitmap), ptr(row_ids), qc, nqc, ptr(qsel), ptr(qval),
         ptr(out_s), ptr(out_i))
    return out_s.view(W, nqt * 16, nw * k), out_i.view(W, nqt * 16, nw * k)


# ---------------------------------------------------------------- device-side merge / IVF plan / bitmap
MERGE_MAX_K = 16


def merge_partials(ps: torch.Tensor, pi: torch.Tensor, k: int, nq: int, cand: torch.Tensor | None = None,
                   cnt: int = 0, affine: tuple = (1, 0, 0), extra: tuple | None = None):
    """Final top-k per query from partial lists (``grag_topk_merge``): query q's
    candidate rows of ps/pi [R, L] are ``cand[q, :cnt]`` or the affine rows
    (q // G) * A + q % G + j * B; ``extra`` = (scores [nq, L2], ids [nq, L2])."""
    L = ps.shape[-1]
    G, A, B = affine
    out_s = torch.empty(nq, k, dtype=torch.float32, device=ps.device)
    out_i = torch.empty(nq, k, dtype=torch.int64, device=ps.device)
    es, ei = (None, None) if extra is None else (extra[0].contiguous(), extra[1].contiguous())
    L2 = 0 if extra is None else es.shape[1]
    call("grag_topk_merge", ptr(ps), ptr(pi), L, ptr(cand), cnt, G, A, B, ptr(es), ptr(ei), L2, nq, k,
         ptr(out_s), ptr(out_i))
    return out_s, out_i


def merge_fits(cnt: int, L: int, L2: int, k: int) -> bool:
    return k <= MERGE_MAX_K and cnt * L + L2 <= lib().grag_topk_merge_cap()


def ivf_plan(lists: torch.Tensor, offsets: torch.Tensor, nlist: int):
    """Coarse probe lists [nq, nprobe] int64 -> (work_rows [P, 2], work_q [P, 16], cand [nq, nprobe]),
    P = nq * nprobe (items past the real count are empty)."""
    nq, nprobe = lists.shape
    P = nq * nprobe
    dev = lists.device
    work_rows = torch.empty(P, 2, dtype=torch.int64, device=dev)
    work_q = torch.empty(P, 16, dtype=torch.int32, device=dev)
    cand = torch.empty(nq, nprobe, dtype=torch.int32, device=dev)
    call("grag_ivf_plan", ptr(lists.contiguous()), nq, nprobe, ptr(offsets), nlist, ptr(work_rows), ptr(work_q),
         ptr(cand))
    return work_rows, work_q, cand


def ivf_plan_fits(nq: int, nprobe: int) -> bool:
    return nq * nprobe <= lib().grag_ivf_plan_max_pairs()


def bitmap_update(bitmap: torch.Tensor, rows: torch.Tensor, alive: bool) -> None:
    """Set (alive) / clear live bits of rows (int64, device) in place."""
    if rows.numel() == 0:
        return
    if not bitmap.is_cuda:
        import numpy as np

        r = rows.long().cpu().numpy()
        words = bitmap.numpy().view(np.uint32)
        bits = (np.uint32(1) << (r & 31).astype(np.uint32)).astype(np.uint32)
        if alive:
            np.bitwise_or.at(words, r >> 5, bits)
        else:
            np.bitwise_and.at(words, r >> 5, ~bits)
        return
    call("grag_bitmap_update", ptr(bitmap), ptr(rows.to(torch.int64).contiguous()), rows.numel(), 1 if alive else 0)
