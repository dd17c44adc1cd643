"""Fused sampler op + persistent per-slot sampler state."""
from __future__ import annotations

import numpy as np
import torch

from ._lib import call, lib, ptr


class SamplerState:
    """Per-slot sampling parameters, seen-token bitmaps and RNG counters kept
    on device so the decode step (forward + LM head + sampler) can be replayed
    from a captured hipGraph with no host round trip besides the token read."""

    def __init__(self, max_slots: int, vocab: int, device, seed: int = 0):
        self.max_slots = max_slots
        self.vocab = vocab
        self.words = (vocab + 31) // 32
        self.device = torch.device(device)
        self.seed = int(seed) & ((1 << 63) - 1)
        self.temperature = torch.ones(max_slots, dtype=torch.float32, device=device)
        self.top_p = torch.ones(max_slots, dtype=torch.float32, device=device)
        self.top_k = torch.zeros(max_slots, dtype=torch.int32, device=device)
        self.penalty = torch.ones(max_slots, dtype=torch.float32, device=device)
        self.seen = torch.zeros(max_slots, self.words, dtype=torch.int32, device=device)
        self.rng = torch.zeros(max_slots, dtype=torch.int64, device=device)
        self._ws = None  # device scratch of the multi-workgroup sampler (sized on first use)
        self._retired = []  # outgrown scratch stays alive: captured decode graphs still point at it
        # host mirror of which slots use top-k / top-p: the kernel chain only
        # launches the radix rounds some slot needs (decode graphs are keyed on it)
        self._uses_topk = [False] * max_slots
        self._uses_topp = [False] * max_slots

    rounds_override: int | None = None  # graph warm-up: capture for the rounds a workload WILL use

    @property
    def rounds(self) -> int:
        if self.rounds_override is not None:
            return self.rounds_override
        return (1 if any(self._uses_topk) else 0) | (2 if any(self._uses_topp) else 0)

    def workspace(self, rows: int) -> torch.Tensor:
        """Scratch for a ``rows``-row call of grag_sample; sized for the
        largest batch seen so far (at least 256 rows; the engine reserves its
        largest decode-graph bucket up front) and only grown outside hipGraph
        capture.  An outgrown buffer is retired, not freed: decode graphs
        captured at smaller buckets replay with its address (freeing it made a
        384-row graph, captured before a 448-row warm-up grew the scratch,
        fault on replay)."""
        need = int(lib().grag_sample_ws_floats(max(rows, 256), self.vocab))
        if self._ws is None or self._ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("sampler workspace must be sized before hipGraph capture")
            if self._ws is not None:
                self._retired.append(self._ws)
            self._ws = torch.empty(need, dtype=torch.float32, device=self.device)
        return self._ws

    def reset_slot(self, slot: int, temperature: float, top_p: float, top_k: int, penalty: float,
                   prompt_ids, seed: int | None = None) -> None:
        self.temperature[slot] = float(temperature)
        self.top_p[slot] = float(top_p)
        self.top_k[slot] = int(top_k)
        self.penalty[slot] = float(penalty)
        self.rng[slot] = int(seed) if seed is not None else 0
        sampled = temperature > 0
        self._uses_topk[slot] = sampled and 0 < int(top_k) < self.vocab
        self._uses_topp[slot] = sampled and float(top_p) < 1.0
        self.seen[slot].zero_()
        if penalty != 1.0 and len(prompt_ids):
            toks = torch.as_tensor(list(prompt_ids), dtype=torch.int32, device=self.device)
            mark_seen(self, toks, torch.full_like(toks, slot))


def reset_slots(state: SamplerState, entries) -> None:
    """``SamplerState.reset_slot`` for every sequence admitted in one engine step, batched: one upload of the
    sampling parameters, one index_copy per field, one seen-bit clear and one seen-bit scatter over all the
    prompts (a per-sequence reset costs about eight small launches each).
    entries: (slot, temperature, top_p, top_k, penalty, prompt_ids, seed) per sequence, distinct slots."""
    if len(entries) <= 1 or not state.temperature.is_cuda:
        for e in entries:
            state.reset_slot(*e)
        return
    dev = state.device
    fl = torch.tensor([[float(e[1]), float(e[2]), float(e[4])] for e in entries], dtype=torch.float32)
    it = torch.tensor([[e[0], int(e[3]), int(e[6]) if e[6] is not None else 0] for e in entries], dtype=torch.int64)
    fl, it = fl.pin_memory().to(dev, non_blocking=True), it.pin_memory().to(dev, non_blocking=True)
    idx = it[:, 0]
    state.temperature.index_copy_(0, idx, fl[:, 0])
    state.top_p.index_copy_(0, idx, fl[:, 1])
    state.penalty.index_copy_(0, idx, fl[:, 2])
    state.top_k.index_copy_(0, idx, it[:, 1].to(torch.int32))
    state.rng.index_copy_(0, idx, it[:, 2])
    state.seen.index_fill_(0, idx, 0)
    toks, sl, cnt = [], [], []
    for slot, temperature, top_p, top_k, penalty, prompt_ids, _ in entries:
        sampled = temperature > 0
        state._uses_topk[slot] = sampled and 0 < int(top_k) < state.vocab
        state._uses_topp[slot] = sampled and float(top_p) < 1.0
        if penalty != 1.0 and len(prompt_ids):
            toks.append(np.asarray(prompt_ids, dtype=np.int32))
            sl.append(slot)
            cnt.append(len(prompt_ids))
    if toks:
        # packed with numpy: a [2, N] list -> torch.tensor costs ~3x more at N = 8K prompt tokens
        packed = np.empty((2, sum(cnt)), dtype=np.int32)
        packed[0] = np.concatenate(toks)
        packed[1] = np.repeat(np.asarray(sl, dtype=np.int32), cnt)
        t = torch.from_numpy(packed).pin_memory().to(dev, non_blocking=True)
        mark_seen(state, t[0], t[1])


def mark_seen(state: SamplerState, tokens: torch.Tensor, slots: torch.Tensor) -> None:
    if not tokens.is_cuda:
        t = tokens.long()
        ok = (t >= 0) & (t < state.vocab)
        t, s = t[ok], slots.long()[ok]
        words = state.seen.view(torch.int32)
        for ti, si in zip(t.tolist(), s.tolist()):
            w = words[si, ti >> 5].item() | (1 << (ti & 31))
            words[si, ti >> 5] = w - (1 << 32) if w >= (1 << 31) else w
        return
    call("grag_mark_seen", ptr(tokens.to(torch.int32).contiguous()), ptr(slots.to(torch.int32).contiguous()),
         tokens.numel(), ptr(state.seen), state.words, state.vocab)


def _seen_mask(state, slot, V, device):
    words = state.seen[slot].long() & 0xFFFFFFFF
    idx = torch.arange(V, device=device)
    return ((words[idx >> 5] >> (idx & 31)) & 1).bool()


_M64 = (1 << 64) - 1


def _mix64(z):
    """splitmix64 finaliser (same constants as csrc/kernels/sampling.hip); z: uint64 ndarray."""
    import numpy as np

    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gumbel_noise(seed: int, counter: int, slot: int, V: int) -> torch.Tensor:
    """G_i = -log(-log u_i) from the kernel's counter-based hash of (seed,
    per-slot step counter, slot, token) — reproducible per request and equal
    on CPU and GPU."""
    import numpy as np

    with np.errstate(over="ignore"):
        inner = _mix64(np.asarray([(counter * 0x100000001B3 + slot) & _M64], dtype=np.uint64))
        base = _mix64(np.asarray([seed & _M64], dtype=np.uint64) ^ inner)
        h = _mix64(base + np.arange(V, dtype=np.uint64))
    u = ((h >> np.uint64(40)).astype(np.float64) + 0.5) * (1.0 / 16777216.0)
    return torch.from_numpy(-np.log(-np.log(u))).float()


def sample_ref(logits: torch.Tensor, state: SamplerState, slots: torch.Tensor, generator=None) -> torch.Tensor:
    """Reference sampler with the kernel's semantics and RNG stream (Gumbel-max
    over the kept tokens with the same counter-based noise); ``generator``
    switches to torch.multinomial for distribution tests."""
    B, V = logits.shape[0], state.vocab
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    for b in range(B):
        s = int(slots[b])
        x = logits[b, :V].float().clone()
        pen = float(state.penalty[s])
        if pen != 1.0:
            m = _seen_mask(state, s, V, logits.device)
            x = torch.where(m, torch.where(x > 0, x / pen, x * pen), x)
        t = float(state.temperature[s])
        if t <= 0:
            tok = int(torch.argmax(x))
        else:
            x = x / t
            k = int(state.top_k[s])
            keep = torch.ones(V, dtype=torch.bool, device=x.device)
            if 0 < k < V:
                thr = torch.topk(x, k).values[-1]
                keep &= x >= thr
            p = float(state.top_p[s])
            if p < 1.0:
                xs = torch.where(keep, x, torch.full_like(x, float("-inf")))
                probs = torch.softmax(xs, 0)
                sp, si = probs.sort(descending=True)
                csum = sp.cumsum(0)
                n = int((csum < p).sum()) + 1
                thr = x[si[min(n, V) - 1]]
                keep &= x >= thr
            xs = torch.where(keep, x, torch.full_like(x, float("-inf")))
            if generator is not None:
                tok = int(torch.multinomial(torch.softmax(xs, 0), 1, generator=generator))
            else:
                g = gumbel_noise(state.seed, int(state.rng[s]), s, V).to(xs.device)
                tok = int(torch.argmax(xs + g))
        out[b] = tok
        if True:  # the kernel always records the sampled token
            w = int(state.seen[s, tok >> 5]) & 0xFFFFFFFF
            w |= 1 << (tok & 31)
            state.seen[s, tok >> 5] = w - (1 << 32) if w >= (1 << 31) else w
        state.rng[s] += 1
    return out


def sample(logits: torch.Tensor, state: SamplerState, slots: torch.Tensor, out: torch.Tensor | None = None):
    """logits [B, >=V] (fp32 or bf16) -> sampled token ids int32 [B]."""
    if not logits.is_cuda:
        res = sample_ref(logits, state, slots)
        if out is not None:
            out.copy_(res)
            return out
        return res
    B = logits.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    dtype = 0 if logits.dtype == torch.float32 else 1
    call("grag_sample", ptr(logits), dtype, logits.stride(0), B, state.vocab, ptr(state.temperature),
         ptr(state.top_p), ptr(state.top_k), ptr(state.penalty), ptr(state.seen), state.words, ptr(state.rng),
         state.seed, ptr(slots), ptr(out), ptr(state.workspace(B)), state.rounds)
    return out


# ---------------------------------------------------------------------- vocab-parallel sampling (C2)
# Under TP the LM head is vocab-parallel: rank r holds logits of tokens [v0, v0 + Vs).  Round 2
# all-gathered the whole [B, V] logits every decode step (152064 x 2 B per row: at TP = 8 and 512
# rows, 136 MB into every rank per step) to run the sampler on the full row.  The sampler is
# decomposable instead: Gumbel-max over the kept set is a max over shards of shard-local maxima, and
# the only cross-shard state is the row max and the radix-select histograms of the top-k / top-p
# thresholds.  So each rank runs the kernel chain on its own columns and the group exchanges:
#   C2a  all-gather of [B, 2] (max, argmax) pairs            -> row max M (and greedy winners)
#   C2b  SUM all-reduce of a [B, 256] fp32 histogram per active radix round (<= 8; 4 for top-p)
#   C2c  all-gather of [B, 2] (Gumbel max, token) pairs      -> the sampled token
# = B x (16 W + 1 KB x rounds) bytes per step instead of B x 2 V bytes, and the same token on every
# rank (seen bitmaps and RNG counters stay replicated).  Tokens equal the TP = 1 sampler's up to the
# summation order of the histogram mass.

_QSCALE = 134217728.0  # 2^27, csrc/kernels/sampling.hip qkey
_DIGITS = ((28, 15), (20, 255), (12, 255), (4, 255))


def _adjusted_row(x: torch.Tensor, state: SamplerState, s: int, v0: int) -> torch.Tensor:
    """Penalty (seen tokens, by global id) then temperature, like the kernel's for_seg."""
    V = x.shape[0]
    pen = float(state.penalty[s])
    if pen != 1.0:
        words = state.seen[s].long() & 0xFFFFFFFF
        idx = torch.arange(v0, v0 + V, device=x.device)
        m = ((words[idx >> 5] >> (idx & 31)) & 1).bool()
        x = torch.where(m, torch.where(x > 0, x / pen, x * pen), x)
    t = float(state.temperature[s])
    return x if t <= 0 else x * (1.0 / t)


def _qkey(x: torch.Tensor, M: float) -> torch.Tensor:
    d = torch.clamp(M - x, 0.0, 32.0) * _QSCALE
    di = torch.where(d >= 4294967295.0, torch.full_like(d, -1.0), d).to(torch.float64).floor().to(torch.int64)
    return torch.where(di < 0, torch.zeros_like(di), 0xFFFFFFFF - di)


def _find_bin(hist: torch.Tensor, need: float) -> tuple[int, float]:
    """Highest bin whose inclusive suffix sum reaches ``need``; (bin, mass strictly above it)."""
    suffix = hist.flip(0).cumsum(0).flip(0)
    ok = (suffix >= need).nonzero()
    if ok.numel() == 0:  # rounding: the lowest bin
        return 0, float(suffix[0] - hist[0])
    b = int(ok.max())
    return b, float(suffix[b] - hist[b])


def sample_tp_ref(logits: torch.Tensor, state: SamplerState, slots: torch.Tensor, group, v0: int,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Host / CPU form of the vocab-parallel sampler (the kernel chain's semantics with the same
    collectives through ``group``: parallel.comm.Group).  logits [B, >= local columns]."""
    B, Vg = logits.shape[0], state.vocab
    Vl = max(0, min(logits.shape[1], Vg - v0))
    res = torch.empty(B, dtype=torch.int32)
    for b in range(B):
        s = int(slots[b])
        x = _adjusted_row(logits[b, :Vl].float(), state, s, v0)
        gid = torch.arange(v0, v0 + Vl)
        greedy = not float(state.temperature[s]) > 0
        if Vl:
            i = int(torch.argmax(x))
            pair = torch.tensor([float(x[i]), float(v0 + i)], dtype=torch.float64)
        else:
            pair = torch.tensor([float("-inf"), 2.0 ** 30], dtype=torch.float64)
        pairs = group.all_gather(pair)  # C2a
        M = float(pairs[:, 0].max())
        if greedy:
            best = max(range(pairs.shape[0]), key=lambda w: (float(pairs[w, 0]), -float(pairs[w, 1])))
            tok = int(pairs[best, 1])
        else:
            key = _qkey(x, M)
            k, p = int(state.top_k[s]), float(state.top_p[s])
            thr_k = 0
            if 0 < k < Vg:  # top-k rounds: counts
                prefix = pmask = 0
                need = float(k)
                for shift, mask in _DIGITS:
                    sel = (key & pmask) == prefix
                    h = torch.zeros(mask + 1, dtype=torch.float64)
                    h.index_add_(0, ((key[sel] >> shift) & mask), torch.ones(int(sel.sum()), dtype=torch.float64))
                    h = group.all_reduce_host(h)  # C2b
                    bn, above = _find_bin(h, need)
                    need -= above
                    prefix |= bn << shift
                    pmask |= mask << shift
                thr_k = prefix
            thr = thr_k
            if p < 1.0:  # top-p rounds: probability mass inside the top-k set
                prefix = pmask = 0
                w = torch.exp((x - M).double())
                need = None
                for shift, mask in _DIGITS:
                    sel = (key >= thr_k) & ((key & pmask) == prefix)
                    h = torch.zeros(mask + 1, dtype=torch.float64)
                    h.index_add_(0, ((key[sel] >> shift) & mask), w[sel])
                    h = group.all_reduce_host(h)  # C2b
                    if need is None:
                        need = p * float(h.sum())
                    bn, above = _find_bin(h, need)
                    need -= above
                    prefix |= bn << shift
                    pmask |= mask << shift
                thr = prefix
            keep = key >= thr
            if Vl and bool(keep.any()):
                g = gumbel_noise(state.seed, int(state.rng[s]), s, v0 + Vl)[v0:].to(x.device)
                z = torch.where(keep, x + g, torch.full_like(x, float("-inf")))
                i = int(torch.argmax(z))
                gp = torch.tensor([float(z[i]), float(gid[i])], dtype=torch.float64)
            else:
                gp = torch.tensor([float("-inf"), 2.0 ** 30], dtype=torch.float64)
            gps = group.all_gather(gp)  # C2c
            best = max(range(gps.shape[0]), key=lambda w: (float(gps[w, 0]), -float(gps[w, 1])))
            tok = int(gps[best, 1])
        if not 0 <= tok < Vg:
            tok = 0
        res[b] = tok
        wd = int(state.seen[s, tok >> 5]) & 0xFFFFFFFF
        wd |= 1 << (tok & 31)
        state.seen[s, tok >> 5] = wd - (1 << 32) if wd >= (1 << 31) else wd
        state.rng[s] += 1
    res = res.to(logits.device)
    if out is not None:
        out.copy_(res)
        return out
    return res


def sample_tp(logits: torch.Tensor, state: SamplerState, slots: torch.Tensor, group, v0: int,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """Vocab-parallel sampler: this rank's logits [B, >= local columns] of tokens [v0, ...) ->
    the same sampled ids int32 [B] on every rank of ``group`` (parallel.comm.Group)."""
    if group.trivial:
        return sample(logits, state, slots, out)
    if not logits.is_cuda:
        return sample_tp_ref(logits, state, slots, group, v0, out)
    B, Vg = logits.shape[0], state.vocab
    # a rank whose (8-aligned) vocab shard starts past the vocabulary holds no real columns: V = 0 makes
    # the kernel emit (-inf, sentinel) pairs and empty histograms for it
    Vl = max(0, min(logits.shape[1], Vg - v0))
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    dev = logits.device
    gmax = torch.empty(B, dtype=torch.float32, device=dev)
    ghist = torch.empty(B, 256, dtype=torch.float32, device=dev)
    pm = torch.empty(B, 2, dtype=torch.float32, device=dev)
    pg = torch.empty(B, 2, dtype=torch.float32, device=dev)
    dtype = 0 if logits.dtype == torch.float32 else 1
    ws = state.workspace(B)
    W = group.size

    def stage(st, r=0, r_prev=-1, j=0, pair_out=None, pmax=None, pgum=None):
        call("grag_sample_tp", st, ptr(logits), dtype, logits.stride(0), B, Vl, v0, Vg, ptr(state.temperature),
             ptr(state.top_p), ptr(state.top_k), ptr(state.penalty), ptr(state.seen), state.words,
             ptr(state.rng), state.seed, ptr(slots), ptr(out), ptr(ws), r, r_prev, j, ptr(gmax), ptr(ghist),
             ptr(pair_out), ptr(pmax), ptr(pgum), W)

    stage(0, pair_out=pm)
    pairs_max = group.all_gather(pm)  # C2a [W, B, 2]
    rounds = state.rounds
    r_prev, j = -1, 0
    for r in range(8):
        if not (rounds >> (r // 4)) & 1:
            continue
        stage(1, r, r_prev, j, pmax=pairs_max)
        group.all_reduce(ghist)  # C2b
        r_prev, j = r, j + 1
    stage(2, 0, r_prev, j, pair_out=pg, pmax=pairs_max)
    pairs_gum = group.all_gather(pg)  # C2c
    stage(3, pmax=pairs_max, pgum=pairs_gum)
    return out


def tp_sampling_bytes(rows: int, world: int, vocab: int, rounds: int) -> dict:
    """Bytes each rank receives per sampling call: vocab-parallel sampler vs a full-logit all-gather."""
    n_rounds = (4 if rounds & 1 else 0) + (4 if rounds & 2 else 0)
    shard = -(-vocab // world)
    return {"vocab_parallel": rows * (2 * 8 * (world - 1) + n_rounds * 256 * 4 * (world - 1) // world * 2),
            "logit_all_gather": rows * shard * 2 * (world - 1)}
