"""KV-cache manager (over the C++ block allocator) and the continuous-batching
scheduler.

Policy (what vLLM gave the reference at ``--max-num-seqs 4``, generalised):
* waiting requests are admitted FCFS while a sampler slot, token budget and
  KV blocks are available; long prompts are split into chunks
  (chunked prefill) so one request never blocks the batch;
* prompt prefixes already in the cache (same chained block hash) are reused
  instead of recomputed — the agent's repeated instructions and the ingest
  extractor prompts share long prefixes;
* when decode runs out of blocks the youngest running sequence is preempted
  (blocks freed, recomputed later);
* waiting requests carry a priority (SamplingParams.priority): critical-path
  requests (ingest roll-up summaries, interactive agent calls) are admitted
  ahead of bulk extractor waves, FCFS within a priority;
* in-step prefix sharing: a prefill item's full prompt blocks are registered in
  the prefix cache when it is SCHEDULED, so a prompt admitted later in the same
  step shares them (waves submit the summary / title / keyword prompts of one
  chunk together; without this every copy of the shared chunk would be
  prefilled).  Correct because each layer stores the whole step's K/V before
  its attention reads the cache; a step that fails unregisters them
  (``last_registered``).  (Round 3 deferred a prompt whose first 16 blocks
  matched one in flight by a step instead: prompts under 256 tokens, most
  extractor prompts, never qualified.)
"""
from __future__ import annotations

import collections
import threading

import numpy as np

from ..utils.runtime import rt
from .sequence import Sequence, SeqStatus


# requests someone waits on (EngineRunner.submit(interactive=True) raises them to this); below it is bulk work
INTERACTIVE_PRIORITY = 2


_ADAPTIVE_RESERVE = __import__("os").environ.get("GRAG_ADAPTIVE_RESERVE", "1") == "1"


def _order(seq) -> float:
    """A sequence's queue key within its priority (SamplingParams.order, else its arrival)."""
    o = seq.params.order
    return seq.arrival if o is None else o


def _before(other, pr: int, key: float) -> bool:
    """``other`` (already waiting) goes before a new request of priority ``pr`` and queue key ``key``."""
    op = other.params.priority
    return op > pr or (op == pr and _order(other) <= key)


class KVCacheManager:
    SCRATCH_BLOCK = 0  # never handed out: padding rows of graph-captured batches point here

    def __init__(self, num_blocks: int, block_size: int, enable_prefix_caching: bool = True):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.prefix_caching = enable_prefix_caching
        self._h = rt().grag_alloc_create(num_blocks, block_size)
        buf = np.zeros(1, dtype=np.int32)
        assert rt().grag_alloc_allocate(self._h, 1, buf.ctypes.data) == 0 and buf[0] == self.SCRATCH_BLOCK

    def __del__(self):
        try:
            rt().grag_alloc_destroy(self._h)
        except Exception:
            pass

    @property
    def num_free(self) -> int:
        return rt().grag_alloc_num_free(self._h)

    def usage(self) -> float:
        return 1.0 - self.num_free / max(1, self.num_blocks - 1)

    def stats(self) -> dict:
        out = np.zeros(3, dtype=np.int64)
        rt().grag_alloc_stats(self._h, out.ctypes.data)
        return {"prefix_hits": int(out[0]), "prefix_queries": int(out[1]), "cached_blocks": int(out[2])}

    def blocks_needed(self, seq: Sequence, upto: int) -> int:
        need = -(-upto // self.block_size)
        return max(0, need - len(seq.blocks))

    def ensure(self, seq: Sequence, upto: int) -> bool:
        n = self.blocks_needed(seq, upto)
        if n == 0:
            return True
        buf = np.zeros(n, dtype=np.int32)
        if rt().grag_alloc_allocate(self._h, n, buf.ctypes.data) != 0:
            return False
        seq.blocks.extend(buf.tolist())
        return True

    def match_prefix(self, seq: Sequence) -> int:
        """Reuse cached full blocks of the prompt (keeping >= 1 token to compute)."""
        if not self.prefix_caching or seq.blocks:
            return 0
        usable = (len(seq.prompt_ids) - 1) // self.block_size * self.block_size
        if usable <= 0:
            return 0
        toks = np.asarray(seq.prompt_ids[:usable], dtype=np.int32)
        nb = usable // self.block_size
        out = np.zeros(nb, dtype=np.int32)
        hashes = np.zeros(nb, dtype=np.uint64)
        m = rt().grag_alloc_match_prefix(self._h, toks.ctypes.data, usable, out.ctypes.data, hashes.ctypes.data)
        if m:
            seq.blocks = out[:m].tolist()
            seq.block_hashes = [int(h) for h in hashes[:m]]
            seq.num_computed = m * self.block_size
            seq.cached_prefix = seq.num_computed
        return m * self.block_size

    def register_full_blocks(self, seq: Sequence, upto: int | None = None) -> list[int]:
        """Register the prompt's full blocks below ``upto`` (default: the computed tokens) under their
        chained hashes; returns the newly registered block ids.  The scheduler registers a prefill item's
        blocks when it schedules it (``upto`` = the item's end): a later prompt admitted in the SAME step
        then shares them -- every layer stores the step's K/V for all its tokens before its attention
        reads the cache, so the sharer reads them after they are written."""
        if not self.prefix_caching:
            return []
        end = seq.num_computed if upto is None else upto
        full = min(end, len(seq.prompt_ids)) // self.block_size
        have = len(seq.block_hashes)
        if have >= full:
            return []
        bs = self.block_size
        parent = seq.block_hashes[-1] if seq.block_hashes else 0
        n = full - have  # one hashing call and one registration call for all the newly full blocks
        toks = np.asarray(seq.prompt_ids[have * bs:full * bs], dtype=np.int32)
        hashes = np.empty(n, dtype=np.uint64)
        rt().grag_hash_blocks(parent, toks.ctypes.data, n, bs, hashes.ctypes.data)
        blocks = np.asarray(seq.blocks[have:full], dtype=np.int32)
        rt().grag_alloc_register_many(self._h, blocks.ctypes.data, hashes.ctypes.data, n)
        seq.block_hashes.extend(int(h) for h in hashes)
        return blocks.tolist()

    def unregister(self, blocks: list[int]) -> None:
        """Forget the hashes of blocks registered for a step that failed before computing them."""
        if blocks:
            arr = np.asarray(blocks, dtype=np.int32)
            rt().grag_alloc_unregister(self._h, len(arr), arr.ctypes.data)

    def free(self, seq: Sequence) -> None:
        if seq.blocks:
            arr = np.asarray(seq.blocks, dtype=np.int32)
            rt().grag_alloc_free(self._h, len(arr), arr.ctypes.data)
        seq.blocks = []
        seq.block_hashes = []
        seq.num_computed = 0


class Scheduler:
    def __init__(self, kv: KVCacheManager, max_num_seqs: int, max_num_batched_tokens: int, max_model_len: int,
                 mixed_batches: bool = True, reserve_seqs: int = 0, reserve_tokens: int = 0):
        self.kv = kv
        # While interactive traffic is on (schedule() called with a bulk budget), bulk admissions leave this
        # many sequence slots and KV tokens for interactive arrivals: a query that finds the slots / blocks
        # taken by ingest waves waits through decode steps until some bulk sequence finishes (concurrent
        # ingest: 1.46 decode steps before a query's first token, bench concurrent_ingest r5)
        self.reserve_seqs = reserve_seqs
        self.reserve_blocks = -(-reserve_tokens // kv.block_size) if reserve_tokens else 0
        self.mixed_batches = mixed_batches
        self.max_num_seqs = max_num_seqs
        self.max_num_batched_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        # running sequences admitted with prompt tokens still to prefill (admission order): the chunked-prefill
        # pass walks these instead of every running sequence (a 512-row decode step has none)
        self.prefilling: list[Sequence] = []
        self.free_slots = list(range(max_num_seqs - 1, -1, -1))
        # interactive sequences holding a slot, and an EMA of their prompt blocks: the bulk reserve grows with
        # the interactive load (_ADAPTIVE_RESERVE), so bulk work cannot fill the slots / blocks live queries
        # are about to need
        self.n_interactive = 0
        self._int_blocks = 0.0
        self.lock = threading.Lock()
        self.num_preemptions = 0
        self.last_registered: list[int] = []  # prompt blocks registered by the last schedule() (rollback)

    def add(self, seq: Sequence) -> None:
        with self.lock:
            pr = seq.params.priority
            key = _order(seq)
            w = self.waiting
            if not w or _before(w[-1], pr, key):
                w.append(seq)
                return
            # insert after the last waiting request that goes first: higher priority, or the same priority
            # and an order key not above this one (FIFO among equal keys)
            i = len(w)
            while i > 0 and not _before(w[i - 1], pr, key):
                i -= 1
            w.insert(i, seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def _finish(self, seq: Sequence) -> None:
        if seq in self.prefilling:
            self.prefilling.remove(seq)
        self.kv.free(seq)
        if seq.slot >= 0 and seq.params.priority >= INTERACTIVE_PRIORITY:
            self.n_interactive -= 1
        if seq.slot >= 0:
            self.free_slots.append(seq.slot)
            seq.slot = -1
        seq.status = SeqStatus.FINISHED

    def finish(self, seq: Sequence) -> None:
        with self.lock:
            if seq in self.running:
                self.running.remove(seq)
            self._finish(seq)

    def reap_cancelled(self) -> list[Sequence]:
        out = []
        with self.lock:
            for s in list(self.waiting):
                if s.cancelled:
                    self.waiting.remove(s)
                    self._finish(s)
                    s.finish_reason = "abort"
                    out.append(s)
            for s in list(self.running):
                if s.cancelled:
                    self.running.remove(s)
                    self._finish(s)
                    s.finish_reason = "abort"
                    out.append(s)
        return out

    @staticmethod
    def prefill_target(seq: Sequence) -> int:
        return seq.total_len - (1 if seq.output_ids else 0)

    def _preempt_one(self, keep: Sequence) -> bool:
        victims = [s for s in self.running if s is not keep]
        if not victims:
            return False
        # lowest priority first (a bulk ingest sequence before an interactive query), newest within it (by the
        # queue key: an agent job's call carries its job's start, so the newest JOB gives its blocks back first)
        v = max(victims, key=lambda s: (-s.params.priority, _order(s)))
        self.running.remove(v)
        if v in self.prefilling:
            self.prefilling.remove(v)
        self.kv.free(v)
        if v.params.priority >= INTERACTIVE_PRIORITY:
            self.n_interactive -= 1
        self.free_slots.append(v.slot)
        v.slot = -1
        v.status = SeqStatus.WAITING
        v.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(v)
        return True

    def schedule(self, budget: int | None = None, bulk_budget: int | None = None):
        """Returns ("prefill", [(seq, start, end)]), ("mixed", prefill items then
        one-token decode items), ("decode", [(seq, pos, pos+1)]) or (None, []).
        ``budget``: this step's prefill token budget (default max_num_batched_tokens; the serving loop
        passes a smaller one while interactive arrivals queue, so one step never carries a burst's worth
        of prompts and the first of them reach their first token sooner).  ``bulk_budget``: of that, at most
        this many tokens for requests below INTERACTIVE_PRIORITY (ingest beside the serving loop: the step an
        arrival waits for stays short), and none in a step that carries an interactive prompt."""
        with self.lock:
            budget = min(budget or self.max_num_batched_tokens, self.max_num_batched_tokens)
            items = []
            admitted = []
            # the prompt blocks this step computes are registered as they are scheduled: later admissions of
            # the same step share them
            registered = []
            # continue partially prefilled running sequences (the ones whose prompt is done drop out here)
            if self.prefilling:
                self.prefilling = [q for q in self.prefilling if q.status == SeqStatus.RUNNING and q.is_prefill]
            # one merged order: chunks of prompts already in prefill and new admissions, higher priority first,
            # in-flight prompts first within a priority -- an interactive arrival (priority 2) takes this step's
            # budget ahead of the remaining chunks of a bulk ingest prompt admitted earlier
            pf = sorted(self.prefilling, key=lambda q: (-q.params.priority, _order(q))) if self.prefilling else []
            i = 0
            admit_ok = True
            bulk_left = bulk_budget if bulk_budget is not None else 1 << 30
            if bulk_budget is not None and (
                    (self.waiting and self.waiting[0].params.priority >= INTERACTIVE_PRIORITY)
                    or any(q.params.priority >= INTERACTIVE_PRIORITY for q in pf)):
                bulk_left = 0  # a step that carries an interactive prompt carries no bulk prefill: it stays short

            def cap(seq, n):  # the bulk share of this step's budget
                return n if seq.params.priority >= INTERACTIVE_PRIORITY else min(n, bulk_left)

            reserve = bulk_budget is not None  # interactive traffic: hold the reserve back from bulk admissions
            res_seqs, res_blocks = self.reserve_seqs, self.reserve_blocks
            if reserve and _ADAPTIVE_RESERVE and self.n_interactive:
                # half the live interactive load again on top: at 40 queries/s beside ingest ~100 queries are live
                # (128 decode steps each) and a fixed 16-slot reserve let bulk fill the rest -- a new query then
                # waited for some sequence to finish (concurrent-ingest TTFT p90 250-413 ms)
                res_seqs += self.n_interactive // 2
                res_blocks += int(self.n_interactive * self._int_blocks) // 2

            while budget > 0:
                can_admit = (admit_ok and self.waiting and self.free_slots
                             and len(self.running) < self.max_num_seqs)
                if i < len(pf) and (not can_admit or pf[i].params.priority >= self.waiting[0].params.priority):
                    seq = pf[i]
                    i += 1
                    out_ids = seq.output_ids
                    if seq.num_computed < len(seq.prompt_ids) + len(out_ids) - (1 if out_ids else 0):  # is_prefill
                        tgt = self.prefill_target(seq)
                        n = cap(seq, min(tgt - seq.num_computed, budget))
                        if n > 0 and self.kv.ensure(seq, seq.num_computed + n):
                            items.append((seq, seq.num_computed, seq.num_computed + n))
                            registered += self.kv.register_full_blocks(seq, upto=seq.num_computed + n)
                            budget -= n
                            if seq.params.priority < INTERACTIVE_PRIORITY:
                                bulk_left -= n
                    continue
                if not can_admit:
                    break
                seq = self.waiting[0]
                if seq.total_len >= self.max_model_len:
                    self.waiting.popleft()
                    seq.finish_reason = "length"
                    self._finish(seq)
                    admitted.append(("rejected", seq))
                    continue
                bulk = seq.params.priority < INTERACTIVE_PRIORITY
                if bulk and (bulk_left <= 0 or (reserve and len(self.running) >= self.max_num_seqs - res_seqs)):
                    admit_ok = False  # (waiting is priority-ordered: only bulk requests follow)
                    continue
                if not seq.blocks:
                    self.kv.match_prefix(seq)
                tgt = self.prefill_target(seq)
                n = cap(seq, min(tgt - seq.num_computed, budget))
                # decode watermark: an admission must leave one free block per running sequence, so the next
                # decode window's block-boundary crossings never preempt (admitting into the last free
                # blocks and preempting at the next decode step recomputes whole prompts: at 1024 agent jobs
                # on one GPU that thrash dominated, profiles/agent_saturation_r4.json)
                if self.running and self.kv.num_free - self.kv.blocks_needed(seq, seq.num_computed + max(n, 0)) \
                        < len(self.running) + 1 + (res_blocks if reserve and bulk else 0):
                    admit_ok = False
                    continue
                if n <= 0 or not self.kv.ensure(seq, seq.num_computed + n):
                    admit_ok = False
                    continue
                self.waiting.popleft()
                seq.slot = self.free_slots.pop()
                if not bulk:
                    self.n_interactive += 1
                    nb = -(-seq.total_len // self.kv.block_size)
                    self._int_blocks = nb if self._int_blocks == 0.0 else 0.9 * self._int_blocks + 0.1 * nb
                seq.status = SeqStatus.RUNNING
                self.running.append(seq)
                self.prefilling.append(seq)
                admitted.append(("admitted", seq))
                items.append((seq, seq.num_computed, seq.num_computed + n))
                registered += self.kv.register_full_blocks(seq, upto=seq.num_computed + n)
                budget -= n
                if seq.params.priority < INTERACTIVE_PRIORITY:
                    bulk_left -= n
            self.last_registered = registered
            self.last_admitted = [s for tag, s in admitted if tag == "admitted"]
            self.last_rejected = [s for tag, s in admitted if tag == "rejected"]
            if items:
                if self.mixed_batches:
                    # piggyback one decode token of every decode-ready sequence on
                    # this prefill step: the weights are streamed once for both
                    # (a separate decode step would stream all of them again)
                    n_pref = len(items)
                    taken = {id(it[0]) for it in items}
                    for seq in self.running:
                        if id(seq) in taken or seq.is_prefill or not seq.output_ids:
                            continue
                        L = seq.total_len
                        if self.kv.ensure(seq, L):
                            items.append((seq, L - 1, L))
                    if len(items) > n_pref:
                        return "mixed", items
                return "prefill", items
            # decode every running sequence (one new token each).  Fast path: every sequence holds, or can
            # take from the free list, the blocks for its next token -> no preemption (at 1-step windows about
            # 1/16 of the rows cross a block boundary every step; ensure is idempotent, so the slow path
            # below redoes the whole batch if the free list runs dry)
            bs = self.kv.block_size
            ensure = self.kv.ensure
            out = []
            for seq in self.running:
                out_ids = seq.output_ids
                L = len(seq.prompt_ids) + len(out_ids)
                if seq.num_computed < L - (1 if out_ids else 0):
                    continue
                if len(seq.blocks) * bs < L and not ensure(seq, L):
                    break
                out.append((seq, L - 1, L))
            else:
                return ("decode", out) if out else (None, [])
            out = []
            preempted = False
            running = SeqStatus.RUNNING
            for seq in list(self.running):
                if seq.status != running:  # preempted earlier in this loop
                    continue
                out_ids = seq.output_ids
                L = len(seq.prompt_ids) + len(out_ids)  # total_len / is_prefill inlined: 512-row hot loop
                if seq.num_computed < L - (1 if out_ids else 0):
                    continue
                if len(seq.blocks) * bs < L:
                    while not self.kv.ensure(seq, L):
                        if not self._preempt_one(seq):
                            break
                        preempted = True
                if seq.status == SeqStatus.RUNNING and len(seq.blocks) * bs >= L:
                    out.append((seq, L - 1, L))
            if preempted:  # drop anything preempted meanwhile
                out = [it for it in out if it[0].status == SeqStatus.RUNNING]
            if out:
                return "decode", out
            return None, []
