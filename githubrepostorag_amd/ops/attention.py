"""Attention ops over the paged KV cache (decoder) and packed QKV (encoder)."""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ._lib import call, ptr

import os

KV_TILE = 64  # keys per kernel tile; split lengths must be multiples of this
# decode kernel variant: 64-key tiles (nw code 1) or 32-key tiles (nw code 3,
# half the LDS ring -> more single-wave workgroups per CU)
# (scripts/microbench.py, B=64 ctx=1152: 64-key 42.3 us -> 32-key 36.7 us)
# GRAG_DECODE_STAGES: LDS ring depth of the 32-key kernel (2: nw 3; 3: nw 8; 4: nw 7 — NS - 1 tiles in flight
# per wave; csrc/kernels/attention.hip paged_decode_kernel)
_DEC_STAGES = int(os.environ.get("GRAG_DECODE_STAGES", "2"))
DECODE_NW = {64: 1, 32: {2: 3, 3: 8, 4: 7}[_DEC_STAGES]}[int(os.environ.get("GRAG_DECODE_TK", "32"))]
DECODE_RING_NW = {2: 3, 3: 8, 4: 7}  # stages -> nw code (microbench / A/B)
_DEC_AUTO = "GRAG_DECODE_STAGES" not in os.environ and os.environ.get("GRAG_DECODE_TK", "32") == "32"
# non-temporal K/V LDS-DMA loads (nt: the cache is read once per decode step; MI355X_MICROARCH 'nt-weights'):
# codes 11 / 12 are 3 / 8 with nt.  profiles/mb_decode_nt_r4.json: B512 ctx1100 206.4 -> 186.8 us (5.59 -> 6.18
# TB/s), B1024 413.7 -> 382.5, B256 113.3 -> 97.7, B176 ctx3000 (3 stages) 208.0 -> 197.0, B16 ctx6000 50.2 ->
# 48.0; grids under ~1.5K waves gain nothing (B64 ctx1152 x 5 parts: 35.8 vs 36.7, B1: equal) -> default there
DECODE_NT = {3: 11, 8: 12}
# round 6 (profiles/attn_sweep_r6.json, one box): nt pays from ~700 waves too -- B176 ctx1500 one part 94.6 ->
# 89.3 us, B256 134.8 -> 117.9 -- so the threshold moved down from 1536 waves
DECODE_NT_MIN_WAVES = int(os.environ.get("GRAG_DECODE_NT_MIN_WAVES", "512"))
# multi-part plans over >= this many (sequence x kv head) rows take the 3-stage ring: B192 ctx3000 (2 parts of
# 2048 keys) 222.7 -> 191.7 us, B128 ctx1500 (2 x 1024) 73.5 -> 67.8 (0: off)
DECODE_NS3_ROWS = int(os.environ.get("GRAG_DECODE_NS3_ROWS", "512"))
_DEC_NT = os.environ.get("GRAG_DECODE_NT", "auto")


# small-batch decode (csrc/kernels/attention.hip paged_decode_mw_kernel): codes 22 / 24 = 2 / 4 waves per
# (sequence, kv head, split), the splits merged in-launch by the last arriving workgroup.  Taken by the
# dispatch when sequences x kv heads <= DECODE_MW_ROWS (GRAG_DECODE_MW: 0 = off)
DECODE_MW = {22: 2, 24: 4}
DECODE_MW_CODE = int(os.environ.get("GRAG_DECODE_MW_CODE", "24"))
DECODE_MW_ROWS = int(os.environ.get("GRAG_DECODE_MW", "16"))
MW_SPLITS = int(os.environ.get("GRAG_DECODE_MW_SPLITS", "20"))  # target parts per sequence at B = 1


def decode_mw_plan(B: int, Hkv: int, max_ctx: int, max_model_len: int, force: bool = False) -> tuple[int, int] | None:
    """(nsplit, split_len) of the small-batch decode kernel, or None when the dispatch does not take it.
    Parts: the power of two (>= 128 keys: 4 waves x one 32-key tile) nearest in log2 to the context over
    MW_SPLITS / sqrt(B) parts -- the hipGraph-timed sweep's best cells (profiles/attn_sweep_r5_mw.json, 4-wave
    kernel): B1 1K / 4K / 11.6K -> 128 / 256 / 512 keys (11.1 / 15.5 / 25.6 us vs 14.9 / 25.5 / 38.0 for the
    single-wave kernel's best plan), B4 4K / 11.6K -> 512 / 1024 (19.0 / 32.3 vs 25.7 / 40.7).  nsplit counts
    parts up to max_model_len, so one captured graph serves a context range (empty parts exit at once)."""
    if not force and (not DECODE_MW_ROWS or B * Hkv > DECODE_MW_ROWS):
        return None
    import math

    per = max(1.0, max_ctx * math.sqrt(B) / MW_SPLITS)
    split_len = max(128, 1 << int(round(math.log2(per))))
    need = -(-max(1, max_ctx) // split_len)
    ns = 1
    while ns < need:
        ns *= 2
    return max(1, min(ns, -(-max_model_len // split_len))), split_len


def decode_counters(dev: torch.device) -> torch.Tensor:
    """The small-batch decode kernel's per-(sequence, kv head) tickets (zeroed once; every last arriver resets
    its word, so hipGraph replays need no memset).  Owned by the caller's workspace owner (ops/gemm.py
    WS.scratch: an engine's, so two engines' decodes on two streams never share a ticket word); allocate
    before any capture (LLMEngine does, under its owner)."""
    from .gemm import WS

    return WS.scratch("decode_tickets", torch.device(dev),
                      lambda d: torch.zeros(1 << 16, dtype=torch.int32, device=d))


def decode_variant(nsplit: int, split_len: int, waves: int | None = None) -> int:
    """Decode kernel per split plan (profiles/mb_decode_ring_r4.json, 32-key tiles): long-context decode
    (split-KV parts covering > 2048 keys: ingest's 3-6K-token prompts) keeps two tiles in flight per wave
    in a 3-stage ring (B176 ctx3000: 238.8 -> 207.8 us, B16 ctx6000: 53.5 -> 50.1 us); the serving
    batches (one part of ~1.1K keys, or 256-key parts) stay on the 2-stage ring, whose 5 waves per CU win
    there (B512 ctx1100: 207.8 vs 222.8 us, B64 ctx1152: 35.6 vs 40.7 us).  ``waves``: the launch's
    (sequence x kv-head x split) count; grids of >= DECODE_NT_MIN_WAVES load K/V non-temporally."""
    # round 5 (profiles/attn_sweep_r5_mw.json, same box): the 3-stage ring lost at B16 4K (45.2 vs 32.1 us at
    # 256-key parts) and tied elsewhere (B16 11.6K 78.0 vs 76.4, B176 1.5K 98.8 vs 96.5): 2 stages unless
    # GRAG_DECODE_STAGES asks (the round-4 auto rule is kept behind GRAG_DECODE_RING_AUTO=1)
    auto3 = _DEC_AUTO and os.environ.get("GRAG_DECODE_RING_AUTO") == "1"
    nw = DECODE_RING_NW[3] if auto3 and nsplit > 1 and nsplit * split_len > 2048 else DECODE_NW
    if (_DEC_AUTO and DECODE_NS3_ROWS and nsplit > 1 and waves is not None
            and waves // nsplit >= DECODE_NS3_ROWS):
        nw = DECODE_RING_NW[3]
    nt = _DEC_NT == "1" or (_DEC_NT == "auto" and waves is not None and waves >= DECODE_NT_MIN_WAVES)
    return DECODE_NT.get(nw, nw) if nt else nw


# prefill kernel: 8-wave LDS-DMA variant (nw code 5, head_dim 64/128) or the
# 4-wave register-staged kernel (nw code 4); GRAG_PREFILL_ATTN=v1 selects the latter
PREFILL_NW = 4 if os.environ.get("GRAG_PREFILL_ATTN", "v2") == "v1" else 5


@dataclass
class AttnMetadata:
    """Per-step attention metadata (device int32 tensors).

    q_start   [nseq+1]  cumulative query-token offsets
    ctx_len   [nseq]    total keys visible to each sequence (cached + new)
    block_tables [nseq, max_blocks]
    slot_mapping [T]    cache slot of every new token (-1 = padding)
    """

    q_start: torch.Tensor
    ctx_len: torch.Tensor
    block_tables: torch.Tensor
    slot_mapping: torch.Tensor
    max_q_len: int
    num_seqs: int
    num_tokens: int
    is_decode: bool = False
    num_splits: int = 1
    split_len: int = 1 << 30
    part_o: torch.Tensor | None = None
    part_ml: torch.Tensor | None = None
    extra: dict = field(default_factory=dict)
    # shared-prefix decode (prefix_groups / csrc/kernels/attention.hip paged_decode_prefix_kernel): a Cascade or
    # None.  The fp32 reference needs none of it (the same keys, attended in one pass)
    cascade: "Cascade | None" = None


@dataclass
class Cascade:
    """Decode rows grouped on a shared cached prefix (prefix_groups + cascade_layout).  pre_len [nseq] int32:
    keys the row's group shares (0 = none); pre_part [nseq] int32: the group's prefix-part length; items
    [n_items, 4] int32 (16-B aligned): (first row, end row, first key, end key) of each part of each group --
    the prefix kernel's work list, one workgroup per item and kv head (padding items (0, 0, 0, 0)); pre_o /
    pre_ml: fp32 workspaces of planes x nseq x Hq x (D | 2), plane = part index; rg: 16-row groups per wave of
    the prefix kernel (a group holds <= 16 * rg // G members)."""

    pre_len: torch.Tensor
    pre_part: torch.Tensor
    items: torch.Tensor
    planes: int
    pre_o: torch.Tensor
    pre_ml: torch.Tensor
    rg: int = 2


CASCADE_MIN_PART = int(os.environ.get("GRAG_CASCADE_MIN_PART", "256"))  # shortest prefix part (keys)
CASCADE_PARTS = int(os.environ.get("GRAG_CASCADE_PARTS", "4"))  # parts a group's prefix is cut into (at most)
CASCADE_MAX_PLANES = max(CASCADE_PARTS, 1)
CASCADE_RG = int(os.environ.get("GRAG_CASCADE_RG", "2"))
# when a decode window takes the shared-prefix path: its groups save at least CASCADE_MIN of the batch's K/V
# keys AND the prefix kernel gets >= CASCADE_MIN_WAVES waves (items x kv heads).  The prefix kernel runs
# ahead of the per-row kernel, so a thin prefix grid is a serial latency chain in front of it
# (profiles/mb_cascade_r6.json: B192, groups of 3 sharing 1536 keys: 105 -> 61 us; a third of B256's groups
# sharing: 122 -> 145 us; B64 fully shared, 352 prefix waves: 46 -> 53 us)
CASCADE_MIN = float(os.environ.get("GRAG_CASCADE_MIN", "0.3"))
CASCADE_MIN_WAVES = int(os.environ.get("GRAG_CASCADE_MIN_WAVES", "1024"))


def cascade_items(B: int) -> int:
    """Work-item slots of the prefix kernel for a batch of B rows (its grid: slots x kv heads)."""
    return max(8, min(2 * B, 1024))


def _up32(x: int) -> int:
    return -(-x // 32) * 32


def cascade_layout(pre, spans, n_items: int, parts: int = CASCADE_PARTS, min_part: int = CASCADE_MIN_PART):
    """Cut each group's P-key prefix into at most ``parts`` parts of max(min_part, ceil(P / parts) rounded up
    to 32) keys: one work item (group, part) each.  Returns (part [n] int32, items [n_items, 4] int32, items
    used).  A group that finds no slots left is dropped from the layout (its rows' pre set to 0: they attend
    to all their keys themselves)."""
    import numpy as np

    n = len(pre)
    part = np.zeros(n, dtype=np.int32)
    items = np.zeros((n_items, 4), dtype=np.int32)
    k = 0
    for a, b in spans:
        P = int(pre[a])
        pl = max(min_part, _up32(-(-P // parts)))
        cnt = -(-P // pl)
        if k + cnt > n_items:
            pre[a:b] = 0
            continue
        part[a:b] = pl
        for j in range(cnt):
            items[k] = (a, b, j * pl, min(P, (j + 1) * pl))
            k += 1
    return part, items, k


def prefix_groups(bt, L, bs: int, G: int, rg: int = CASCADE_RG, min_blocks: int = 8):
    """Group adjacent decode rows on a common leading run of KV block ids (the prefix cache hands every
    sequence of one cached prompt prefix the same blocks).  bt [n, W] int32 block table, L [n] each row's
    context length (keys, the current token's included).  Only whole blocks strictly before the current
    token's block count (that block is the row's own).  A group grows while its shared keys saved,
    (members - 1) x prefix, do not drop, up to 16 * rg // G members.  Returns (pre [n] int32, spans [(begin,
    end), ...] of the groups, saved keys) -- pre 0 for rows outside any group -- or None when none forms."""
    import numpy as np

    n = bt.shape[0]
    cap = (16 * rg) // G
    if n < 2 or cap < 2:
        return None
    full = (np.asarray(L, dtype=np.int64) - 1) // bs  # blocks wholly before each row's current position
    w = int(min(full.max(), bt.shape[1]))
    if w < min_blocks:
        return None
    eq = bt[1:, :w] == bt[:-1, :w]
    run = np.where(eq.all(1), w, eq.argmin(1))
    run = np.minimum(run, np.minimum(full[1:], full[:-1])).tolist()
    pre = np.zeros(n, dtype=np.int32)
    spans = []
    saved = 0
    i = 0
    while i < n - 1:
        P = run[i]
        if P < min_blocks:
            i += 1
            continue
        j = i + 1  # rows i..j share P blocks
        while j + 1 < n and j + 1 - i < cap:
            nP = min(P, run[j])
            if nP < min_blocks or nP * (j + 1 - i) < P * (j - i):  # the group's saved keys would drop
                break
            P = nP
            j += 1
        pre[i:j + 1] = P * bs
        spans.append((i, j + 1))
        saved += (j - i) * P * bs
        i = j + 1
    if not saved:
        return None
    return pre, spans, saved


def choose_splits(max_ctx: int, nseq: int, hkv: int, target_wgs: int = 1024, split_min: int = 256):
    """Split-KV plan for decode: enough workgroups to fill 256 CUs."""
    tiles = max(1, (max_ctx + KV_TILE - 1) // KV_TILE)
    base = max(1, nseq * hkv)
    want = max(1, min(tiles, (target_wgs + base - 1) // base))
    split_tiles = max(split_min // KV_TILE, (tiles + want - 1) // want)
    split_len = split_tiles * KV_TILE
    nsplit = (max_ctx + split_len - 1) // split_len
    return max(1, nsplit), split_len


def paged_attention_ref(q, k_cache, v_cache, meta: AttnMetadata, scale: float, causal: bool = True):
    """fp32 reference: q [T, Hq, D] -> out [T, Hq, D]."""
    T, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    out = torch.zeros(T, Hq, D, dtype=torch.float32, device=q.device)
    qs = meta.q_start.tolist()
    cl = meta.ctx_len.tolist()
    bt = meta.block_tables
    for s in range(meta.num_seqs):
        a, b = qs[s], qs[s + 1]
        ql, ctx = b - a, cl[s]
        if ql == 0:
            continue
        nblk = (ctx + BS - 1) // BS
        blocks = bt[s, :nblk].long()
        K = k_cache[blocks].permute(0, 2, 1, 3).reshape(-1, Hkv, D)[:ctx].float()
        V = v_cache[blocks].permute(0, 2, 1, 3).reshape(-1, Hkv, D)[:ctx].float()
        K = K.repeat_interleave(G, dim=1)
        V = V.repeat_interleave(G, dim=1)
        qq = q[a:b].float()
        sc = torch.einsum("phd,khd->hpk", qq, K) * scale
        if causal:
            pos = torch.arange(ctx - ql, ctx, device=q.device)[:, None]
            kk = torch.arange(ctx, device=q.device)[None, :]
            sc = sc.masked_fill((kk > pos)[None], float("-inf"))
        p = torch.softmax(sc, dim=-1)
        out[a:b] = torch.einsum("hpk,khd->phd", p, V)
    return out.to(q.dtype)


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, meta: AttnMetadata,
                    scale: float, causal: bool = True, out: torch.Tensor | None = None) -> torch.Tensor:
    """q [T, Hq, D] (token-major) -> out [T, Hq*D]."""
    dec = meta.extra.get("decode_rows")
    if dec is not None:  # mixed step: prefill rows [0, Tp) + one-token decode rows [Tp, T)
        Tp, dmeta = dec
        if out is None:
            out = torch.empty(q.shape[0], q.shape[1] * q.shape[2], dtype=q.dtype, device=q.device)
        pmeta = AttnMetadata(q_start=meta.q_start, ctx_len=meta.ctx_len, block_tables=meta.block_tables,
                             slot_mapping=meta.slot_mapping, max_q_len=meta.max_q_len, num_seqs=meta.num_seqs,
                             num_tokens=Tp)
        paged_attention(q[:Tp], k_cache, v_cache, pmeta, scale, causal, out=out[:Tp])
        paged_attention(q[Tp:], k_cache, v_cache, dmeta, scale, causal, out=out[Tp:])
        return out
    if not q.is_cuda:
        ref = paged_attention_ref(q, k_cache, v_cache, meta, scale, causal).reshape(q.shape[0], -1)
        if out is None:
            return ref
        out.copy_(ref)
        return out
    T, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    if out is None:
        out = torch.empty(T, Hq * D, dtype=q.dtype, device=q.device)
    nsplit = meta.num_splits if meta.is_decode else 1
    if meta.is_decode:
        nw = meta.extra.get("decode_nw")
        if nw is None:
            nw = decode_variant(nsplit, meta.split_len, meta.num_seqs * Hkv * nsplit)
            if DECODE_MW_ROWS and meta.num_seqs * Hkv <= DECODE_MW_ROWS:
                nw = DECODE_MW_CODE
        if nw in DECODE_MW and D in (64, 128) and Hq // Hkv <= 16 and BS % 16 == 0 \
                and (nsplit == 1 or meta.split_len % 32 == 0) and meta.num_seqs * Hkv <= (1 << 16):
            call("grag_paged_decode_mw", ptr(q), q.stride(0), ptr(k_cache), ptr(v_cache), ptr(out), out.stride(0),
                 ptr(meta.block_tables), meta.block_tables.stride(0), ptr(meta.q_start), ptr(meta.ctx_len),
                 meta.num_seqs, T, Hq, Hkv, D, BS, float(scale), nsplit, meta.split_len if nsplit > 1 else 0,
                 ptr(meta.part_o) if nsplit > 1 else None, ptr(meta.part_ml) if nsplit > 1 else None,
                 ptr(decode_counters(q.device)), DECODE_MW[nw], k_cache.shape[0])
            return out
        if nw in DECODE_MW:
            nw = decode_variant(nsplit, meta.split_len, meta.num_seqs * Hkv * nsplit)
        c = meta.cascade
        if c is not None:
            call("grag_paged_decode_cascade", ptr(q), q.stride(0), ptr(k_cache), ptr(v_cache), ptr(out),
                 out.stride(0), ptr(meta.block_tables), meta.block_tables.stride(0), ptr(meta.q_start),
                 ptr(meta.ctx_len), meta.num_seqs, T, Hq, Hkv, D, BS, float(scale), nsplit,
                 meta.split_len if nsplit > 1 else 0, ptr(meta.part_o) if nsplit > 1 else None,
                 ptr(meta.part_ml) if nsplit > 1 else None, nw, k_cache.shape[0], ptr(c.pre_len), ptr(c.pre_part),
                 ptr(c.items), c.items.numel() // 4, c.planes, ptr(c.pre_o), ptr(c.pre_ml), c.rg)
            return out
    else:
        nw = meta.extra.get("prefill_nw", PREFILL_NW)
        if nw in (5, 6) and D not in (64, 128):
            nw = 4
    call("grag_paged_attention", ptr(q), q.stride(0), ptr(k_cache), ptr(v_cache), ptr(out), out.stride(0),
         ptr(meta.block_tables), meta.block_tables.stride(0), ptr(meta.q_start), ptr(meta.ctx_len),
         meta.num_seqs, T, meta.max_q_len, Hq, Hkv, D, BS, float(scale), 1 if causal else 0, nsplit,
         meta.split_len if nsplit > 1 else 0, ptr(meta.part_o) if nsplit > 1 else None,
         ptr(meta.part_ml) if nsplit > 1 else None, nw, k_cache.shape[0])
    return out


# small-batch decode with the RoPE + KV-store pass folded into the attention launch (paged_decode_mw_kernel FR;
# GRAG_ROPE_FUSE=0: the separate qkv_rope_kvstore launch)
ROPE_FUSE = os.environ.get("GRAG_ROPE_FUSE", "1") != "0"


def paged_decode_mw_rope(qkv, bias, positions, cos_sin, k_cache, v_cache, meta: AttnMetadata, scale: float,
                         Hq: int, Hkv: int, D: int) -> torch.Tensor | None:
    """Decode attention straight from the qkv projection's deferred split-K planes (ops/gemm.py SplitKPartial):
    the kernel forms q with bias + NeoX RoPE in registers, folds the new token's key in from registers, and stores
    the new K / V to meta.slot_mapping's slots -- what ops/elementwise.qkv_rope_kvstore + paged_attention do in
    two launches (the small-kernel floor VERDICT r5 item 4 measured: RoPE 6.5 us of a B = 1 layer).  Returns
    out [T, Hq * D], or None when the small-batch decode kernel would not take this step (the caller then runs
    the two-launch path)."""
    from .gemm import SplitKPartial

    if not (ROPE_FUSE and isinstance(qkv, SplitKPartial) and qkv.device.type == "cuda" and cos_sin is not None
            and meta.is_decode and meta.cascade is None and "decode_rows" not in meta.extra):
        return None
    BS = k_cache.shape[2]
    nsplit = meta.num_splits
    nw = meta.extra.get("decode_nw")
    if nw is None and DECODE_MW_ROWS and meta.num_seqs * Hkv <= DECODE_MW_ROWS:
        nw = DECODE_MW_CODE
    if not (nw in DECODE_MW and D in (64, 128) and Hq // Hkv <= 16 and BS % 16 == 0 and qkv.N == (Hq + 2 * Hkv) * D
            and (nsplit == 1 or meta.split_len % 32 == 0) and meta.num_seqs * Hkv <= (1 << 16)
            and qkv.M == meta.num_tokens and meta.max_q_len == 1):
        return None
    out = torch.empty(qkv.M, Hq * D, dtype=qkv.dtype, device=qkv.device)
    call("grag_paged_decode_mw_rope", ptr(qkv.planes), qkv.S, ptr(bias), ptr(positions), ptr(cos_sin),
         ptr(meta.slot_mapping), ptr(k_cache), ptr(v_cache), ptr(out), out.stride(0), ptr(meta.block_tables),
         meta.block_tables.stride(0), ptr(meta.q_start), ptr(meta.ctx_len), meta.num_seqs, qkv.M, Hq, Hkv, D, BS,
         float(scale), nsplit, meta.split_len if nsplit > 1 else 0, ptr(meta.part_o) if nsplit > 1 else None,
         ptr(meta.part_ml) if nsplit > 1 else None, ptr(decode_counters(qkv.device)), DECODE_MW[nw],
         k_cache.shape[0], k_cache.shape[0] * BS, cos_sin.numel() // D)
    return out


def varlen_attention_ref(qkv, seq_start, H, D, scale, causal=False):
    T = qkv.shape[0]
    x = qkv.float().view(T, 3, H, D)
    out = torch.zeros(T, H, D, dtype=torch.float32, device=qkv.device)
    ss = seq_start.tolist()
    for s in range(len(ss) - 1):
        a, b = ss[s], ss[s + 1]
        if b <= a:
            continue
        q, k, v = x[a:b, 0], x[a:b, 1], x[a:b, 2]
        sc = torch.einsum("phd,khd->hpk", q, k) * scale
        if causal:
            L = b - a
            sc = sc.masked_fill(torch.ones(L, L, dtype=torch.bool, device=qkv.device).triu(1)[None], float("-inf"))
        out[a:b] = torch.einsum("hpk,khd->phd", torch.softmax(sc, -1), v)
    return out.reshape(T, H * D).to(qkv.dtype)


def varlen_attention(qkv: torch.Tensor, seq_start: torch.Tensor, seq_len: torch.Tensor, max_len: int,
                     H: int, D: int, scale: float, causal: bool = False) -> torch.Tensor:
    """Self-attention over packed QKV rows [T, 3*H*D] (encoder layers, no padding
    tokens computed) -> [T, H*D]."""
    if not qkv.is_cuda:
        return varlen_attention_ref(qkv, seq_start, H, D, scale, causal)
    T = qkv.shape[0]
    out = torch.empty(T, H * D, dtype=qkv.dtype, device=qkv.device)
    base = qkv.data_ptr()
    es = qkv.element_size()
    call("grag_varlen_attention", base, base + H * D * es, base + 2 * H * D * es, qkv.stride(0), ptr(out),
         out.stride(0), ptr(seq_start), ptr(seq_len), seq_len.numel(), max_len, H, H, D, float(scale),
         1 if causal else 0)
    return out
