"""In-process LLM engine: continuous batching over the paged KV cache,
chunked prefill, prefix caching, fused sampler and hipGraph-captured decode.

Replaces the reference's external vLLM container (helm/templates/
qwen-deployment.yaml:20-71, ``--max-num-seqs 4 --max-model-len 11712``) with
an engine that lives in the worker process next to the index and encoder.

Decode runs in multi-step windows: K in {1, 2, 4, 8} consecutive decode steps
(embed -> 28 layers -> LM head -> sampler, K times, each step's sampled ids
feeding the next step's embedding gather on device) are captured per
(batch bucket, split plan, K) into one ``torch.cuda.CUDAGraph`` (a hipGraph
on ROCm).  The host builds the positions / slot mapping / context lengths of
all K steps at once (KV blocks are reserved K tokens ahead), issues one H2D
copy of a packed int32 control buffer, one replay and one D2H copy of the
K x B sampled ids, so the per-token host work (scheduling, detokenising,
stop checks) is amortised over K steps and the GPU is not left idle between
tokens.  Tokens sampled after a sequence hit EOS/stop inside a window are
discarded.
"""
from __future__ import annotations

import contextlib

import logging
import threading
import time
import uuid
from dataclasses import dataclass

import numpy as np
import torch

from ..ops.attention import (CASCADE_MAX_PLANES, CASCADE_MIN, CASCADE_MIN_WAVES, CASCADE_RG, KV_TILE, AttnMetadata, Cascade,
                             cascade_items, cascade_layout, prefix_groups)
from ..ops._lib import check_device_errors
from ..ops.gemm import WS
from ..ops.sampling import SamplerState, reset_slots, sample, sample_tp
from .scheduler import KVCacheManager, Scheduler
from .sequence import Completion, SamplingParams, Sequence, SeqStatus
from ..utils.gpu_guard import gpu_guard, gpu_shared, no_gc
from .tokenizer import IncrementalDetokenizer

log = logging.getLogger(__name__)
_TP_SAMPLER = __import__("os").environ.get("GRAG_TP_SAMPLER", "shard")


class PromptTooLongError(ValueError):
    """A prompt that leaves no room for one generated token within max_model_len."""

    def __init__(self, n_prompt: int, max_model_len: int):
        super().__init__(f"This model's maximum context length is {max_model_len} tokens. However, your prompt has "
                         f"{n_prompt} tokens. Please reduce the length of the messages.")
        self.n_prompt, self.max_model_len = n_prompt, max_model_len


@dataclass
class EngineConfig:
    max_num_seqs: int = 64
    max_num_batched_tokens: int = 16384
    max_model_len: int = 11712  # reference --max-model-len (helm/values.yaml:74)
    block_size: int = 16
    num_blocks: int | None = None
    kv_cache_gb: float | None = None
    gpu_memory_fraction: float = 0.5
    enable_prefix_caching: bool = True
    use_cuda_graph: bool = True
    graph_batch_sizes: tuple = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512)
    decode_window: int = 8  # max decode steps per graph replay (power of two)
    # decode tokens ride along in prefill steps (one weight pass for both).  Off by
    # default: measured on the headline bench the odd GEMM M (4096 + live rows)
    # misses the tuned library solutions and costs more than the saved decode steps
    mixed_batches: bool = False
    seed: int = 0
    # slots / KV tokens bulk (below interactive priority) admissions leave free while interactive traffic is on
    # (engine/scheduler.py Scheduler reserve): a query beside ingest waves is admitted at the next step
    interactive_reserve_seqs: int = 16
    interactive_reserve_tokens: int = 16384
    # shared-prefix decode attention (ops/attention.prefix_groups, csrc/kernels/attention.hip
    # paged_decode_prefix_kernel): decode rows that share cached prompt blocks read them once per group
    cascade_decode: bool = __import__("os").environ.get("GRAG_CASCADE", "1") == "1"


_SPLIT_MID = int(__import__("os").environ.get("GRAG_DECODE_SPLIT_128", "1024"))


def _split_len_for(batch: int) -> int:
    """Keys per split-KV part of the decode attention (flash-decoding) for a batch size.  Small batches
    need splits to put enough waves on the CUs (B64 ctx1152: split 256 36.7 us < split 512 38.0 us); from
    ~200 live sequences (x 4 KV heads) the batch alone fills the chip, and long parts win by dropping the
    combine pass and the partial round trip: B512 ctx1100 251 -> 233 / 225 / 210 us at parts of 512 /
    1024 / 2048 keys, B256 ctx1100 125 -> 105 us at 2048 (profiles/mb_decode_splits_r3.json).  The part
    length still caps one wave's keys, so a long sequence among short ones is split."""
    if batch >= 160:  # B176 ctx1500: one 2048-key part 96.5 us vs 256-key parts 121.2 (profiles/attn_sweep_r5_mw.json)
        return 32 * KV_TILE
    if batch >= 128:  # B128 ctx1500: 2 x 1024 keys 67.8 us vs one 2048-key part 87.7 (profiles/attn_sweep_r6.json)
        return _SPLIT_MID
    if batch >= 8:
        return 4 * KV_TILE
    return 2 * KV_TILE


def _decode_plan(model, B: int, max_ctx: int, max_model_len: int, graph: bool = True) -> tuple[int, int]:
    """(nsplit, split_len) of the decode attention for a batch of B sequences: the small-batch kernel's plan
    (ops/attention.decode_mw_plan) when it takes the batch, else split parts of _split_len_for(B) keys
    (graphs: a power-of-two split count, so one capture serves a range of contexts)."""
    from ..ops.attention import decode_mw_plan

    mw = decode_mw_plan(B, getattr(model, "hkv", 1), max_ctx, max_model_len) if model.device.type == "cuda" else None
    if mw is not None:
        return mw
    split_len = _split_len_for(B)
    need = -(-max_ctx // split_len)
    if graph:
        return min(_pow2_at_least(need), -(-max_model_len // split_len)), split_len
    return max(1, need), split_len


# prefix-sharing decode rows side by side (GRAG_DECODE_GROUP_ROWS=1): off by default -- the shared blocks
# already come from the Infinity Cache in any row order (profiles/mb_shared_prefix_r6.json)
_GROUP_ROWS = __import__("os").environ.get("GRAG_DECODE_GROUP_ROWS", "0") == "1"


_CASCADE_PROBE = 7  # block index probed for prefix sharing (ops/attention.prefix_groups min_blocks - 1)


def _prefix_blocks(s) -> list:
    return s.blocks[:32]


def _pow2_at_least(n: int) -> int:
    p = 1
    while p < n:
        p *= 2
    return p


def _ctrl_layout(B: int, width: int, K: int = 1) -> dict:
    """Offsets (int32 elements) and shapes of the decode control buffer for a K-step window of B rows:
    ids[B] | pos[K,B] | slot[K,B] | ctx[K,B] | sampler slots[B] | q_start[B+1] | pre[B] | part[B] | (pad to
    16 B) items[NI,4] | block table[B,width].  pre / part / items: the shared-prefix decode layout
    (ops/attention.cascade_layout; NI = cascade_items(B)); zeros when the window does not take it."""
    lay = {}
    o = 0
    for name, shape in (("ids", (B,)), ("pos", (K, B)), ("slot", (K, B)), ("ctx", (K, B)), ("slots", (B,)),
                        ("qs", (B + 1,)), ("pre", (B,)), ("part", (B,)), ("items", (cascade_items(B), 4)),
                        ("bt", (B, width))):
        if name == "items":
            o += -o % 4  # int4 loads in the prefix kernel
        lay[name] = (o, shape)
        o += int(np.prod(shape))
    lay["size"] = o + 4  # room for the pad of a buffer whose base is 16-B aligned
    return lay


class _DecodeGraph:
    def __init__(self, graph, out_tokens, batch, nsplit, split_len, steps):
        self.graph = graph
        self.out_tokens = out_tokens  # [steps, batch] int32
        self.batch = batch
        self.nsplit = nsplit
        self.split_len = split_len
        self.steps = steps


class LLMEngine:
    def __init__(self, model, tokenizer, config: EngineConfig | None = None):
        self.model = model
        self.tok = tokenizer
        self.cfg = config or EngineConfig()
        self.device = model.device
        self.on_gpu = self.device.type == "cuda"
        cfg = self.cfg
        cfg.max_model_len = min(cfg.max_model_len, model.cfg.max_position)
        bs = cfg.block_size
        nblocks = cfg.num_blocks or self._plan_blocks()
        self.kv = KVCacheManager(nblocks, bs, cfg.enable_prefix_caching)
        self.kv_caches = model.allocate_kv_cache(nblocks, bs)
        self.sched = Scheduler(self.kv, cfg.max_num_seqs, cfg.max_num_batched_tokens, cfg.max_model_len,
                               mixed_batches=cfg.mixed_batches,
                               reserve_seqs=min(cfg.interactive_reserve_seqs, cfg.max_num_seqs // 4),
                               reserve_tokens=min(cfg.interactive_reserve_tokens, nblocks * bs // 8))
        self.scratch_slot = cfg.max_num_seqs
        self.sampler = SamplerState(cfg.max_num_seqs + 1, model.cfg.vocab_size, self.device, seed=cfg.seed)
        self.max_blocks_per_seq = -(-cfg.max_model_len // bs)
        self._seqs: dict[str, Sequence] = {}
        self._graphs: dict[tuple, _DecodeGraph] = {}
        self._graph_pool = None
        self._static = None
        self._cascade_plan = 0
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "prefill_s": 0.0, "decode_s": 0.0, "steps": 0,
                      "graph_replays": 0, "graph_captures": 0, "decode_steps": 0, "decode_wait_s": 0.0,
                      "step_s": 0.0, "mixed_steps": 0,
                      # host-side time by section (the GPU idles whenever one of these outlasts the queued work)
                      "host_sched_s": 0.0, "host_prefill_prep_s": 0.0, "host_prefill_launch_s": 0.0,
                      "host_prefill_sample_s": 0.0, "host_prefill_post_s": 0.0, "host_decode_prep_s": 0.0,
                      "host_decode_post_s": 0.0, "capture_s": 0.0,
                      # prompt tokens submitted / taken from the prefix cache at admission (the rest is prefill)
                      "prompt_tokens": 0, "prefix_hit_tokens": 0,
                      # shared-prefix decode: windows that took it, rows in groups, K/V keys not re-read (of
                      # decode_keys: the context keys of the batches it was considered for)
                      "cascade_windows": 0, "cascade_rows": 0, "cascade_saved_keys": 0, "decode_keys": 0}
        # optional per-step timeline (a list; None = off): (t_start, kind, rows, tokens, seconds) per step,
        # kind "prefill" / "decode" / "mixed" / "capture" — the ingest critical-path trace reads it
        self.trace: list | None = None
        self._eos = set(getattr(tokenizer, "eos_token_ids", set()))
        self._lock = threading.RLock()
        # split-K / stream-K workspaces of this engine's steps and graphs (ops/gemm.py WS.owned_by): owned by
        # the engine, whichever thread steps it
        self._ws: dict = {}
        max_split = -(-cfg.max_model_len // KV_TILE)
        self._max_b = max(cfg.graph_batch_sizes) if cfg.use_cuda_graph else cfg.max_num_seqs
        self._max_b = max(self._max_b, cfg.max_num_seqs)
        self.stream = None
        if self.on_gpu:
            hq, d = model.hq, model.head_dim
            self._part_o = torch.empty(max_split * self._max_b * hq * d, dtype=torch.float32, device=self.device)
            self._part_ml = torch.empty(max_split * self._max_b * hq * 2, dtype=torch.float32, device=self.device)
            if cfg.cascade_decode:  # prefix parts of the shared-prefix decode
                npl = CASCADE_MAX_PLANES
                self._pre_o = torch.empty(npl * self._max_b * hq * d, dtype=torch.float32, device=self.device)
                self._pre_ml = torch.empty(npl * self._max_b * hq * 2, dtype=torch.float32, device=self.device)
            # sampler scratch for the largest decode batch up front: graphs captured later all see one buffer
            self.sampler.workspace(self._max_b)
            from ..ops.attention import decode_counters  # small-batch decode tickets: before any capture
            from ..ops.gemm import fold_ws
            from ..ops.norm import norm_ws

            with WS.owned_by(self._ws):  # this engine's own ticket words (ops/gemm.py WS.scratch)
                decode_counters(self.device)
                norm_ws(self.device)
                fold_ws(self.device)
            # kernels report out-of-range index inputs (block tables, slots, token ids, tickets) to a
            # host-mapped block instead of faulting; every step's host read checks it (_read_host)
            from ..ops._lib import bind_error_guard, lib

            lib()
            bind_error_guard(self.device.index if self.device.index is not None else torch.cuda.current_device())
            # the engine's own (non-default) stream: retrieval / API threads issue their copies and syncs
            # on other streams; with the engine on the legacy default stream their runtime calls stalled
            # the engine thread (profiles/timeline_r2_*.txt).  Weights and the KV cache were written on
            # the default stream: drain it once before the first engine launch.
            torch.cuda.synchronize(self.device)
            self.stream = torch.cuda.Stream(self.device)

    # ------------------------------------------------------------------ setup
    def _plan_blocks(self) -> int:
        cfg = self.cfg
        per_block = self.model.kv_bytes_per_block(cfg.block_size)
        want_tokens = cfg.max_num_seqs * cfg.max_model_len
        want = -(-want_tokens // cfg.block_size) + 1
        if self.device.type != "cuda":
            return min(want, 4096)
        if cfg.kv_cache_gb:
            cap = int(cfg.kv_cache_gb * (1 << 30) // per_block)
        else:
            free, _ = torch.cuda.mem_get_info(self.device)
            cap = int(free * cfg.gpu_memory_fraction // per_block)
        n = max(64, min(want, cap))
        # replicated TP scheduling needs bit-identical admission/preemption on
        # every rank, hence the same block pool: take the group minimum
        return self.model.tp.min_int(n, self.device)

    # ------------------------------------------------------------------ API
    def add_request(self, prompt, params: SamplingParams | None = None, req_id: str | None = None,
                    on_token=None) -> str:
        params = params or SamplingParams()
        ids = self.tok.encode(prompt) if isinstance(prompt, str) else list(prompt)
        if not ids:
            ids = [self.tok.pad_token_id] if hasattr(self.tok, "pad_token_id") else [0]
        if len(ids) >= self.cfg.max_model_len:
            # rejected like vLLM's server does (helm/templates/qwen-deployment.yaml:30-31 --max-model-len):
            # never cut silently here.  Callers that own the prompt's structure fit it first (agent/llm.py
            # EngineLLM keeps the head and the answer cue); the OpenAI endpoints answer HTTP 400.
            raise PromptTooLongError(len(ids), self.cfg.max_model_len)
        req_id = req_id or uuid.uuid4().hex
        seq = Sequence(req_id, ids, params, on_token=on_token)
        with self._lock:
            self._seqs[req_id] = seq
            self.stats["prompt_tokens"] += len(ids)
        self.sched.add(seq)
        return req_id

    def abort(self, req_id: str) -> None:
        seq = self._seqs.get(req_id)
        if seq is not None:
            seq.cancelled = True

    def has_unfinished(self) -> bool:
        return self.sched.has_work()

    def has_pending_prefill(self) -> bool:
        """Admitted or waiting requests whose prompt is not fully prefilled yet."""
        sch = self.sched
        return bool(sch.waiting) or any(s.is_prefill for s in sch.running)

    def get(self, req_id: str) -> Sequence | None:
        return self._seqs.get(req_id)

    def pop(self, req_id: str) -> Sequence | None:
        with self._lock:
            return self._seqs.pop(req_id, None)

    def generate(self, prompts, params: SamplingParams | list | None = None) -> list[Completion]:
        if isinstance(params, list):
            ids = [self.add_request(p, sp) for p, sp in zip(prompts, params)]
        else:
            ids = [self.add_request(p, params) for p in prompts]
        while self.has_unfinished():
            self.step()
        return [self.completion(self.pop(r)) for r in ids]

    def completion(self, seq: Sequence) -> Completion:
        return Completion(seq.req_id, seq.text, list(seq.output_ids), seq.finish_reason, len(seq.prompt_ids),
                          seq.ttft, None if seq.finish_time is None else seq.finish_time - seq.arrival,
                          seq.cached_prefix, seq.first_token_time)

    # ------------------------------------------------------------------ step
    def step(self, max_window: int | None = None, prefill_budget: int | None = None,
             bulk_budget: int | None = None) -> list[Sequence]:
        """Run one scheduler step; returns sequences that finished in it.
        ``max_window`` caps the decode window (tokens per sequence this step); ``prefill_budget`` caps this
        step's prefill tokens (Scheduler.schedule)."""
        t0 = time.perf_counter()
        try:
            # shared capture guard for the whole step (utils/gpu_guard.py): the step's host reads sync, and
            # a sync while another thread captures (the embedder's query-bucket graphs) breaks that capture
            with self._on_stream(), WS.owned_by(self._ws), (gpu_shared() if self.on_gpu else contextlib.nullcontext()):
                return self._step(max_window, prefill_budget, bulk_budget)
        finally:
            self.stats["step_s"] += time.perf_counter() - t0

    def _on_stream(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    @torch.inference_mode()
    def _step(self, max_window: int | None = None, prefill_budget: int | None = None,
              bulk_budget: int | None = None) -> list[Sequence]:
        th = time.perf_counter()
        finished = self.sched.reap_cancelled()
        for s in finished:
            self._notify(s, None, True)
        kind, items = self.sched.schedule(prefill_budget, bulk_budget)
        for s in getattr(self.sched, "last_rejected", []):
            s.finish_time = time.perf_counter()
            self._notify(s, None, True)
            finished.append(s)
        adm = getattr(self.sched, "last_admitted", [])
        if adm:
            self.stats["prefix_hit_tokens"] += sum(s.cached_prefix for s in adm)
            reset_slots(self.sampler, [(s.slot, s.params.temperature, s.params.top_p, s.params.top_k,
                                        s.params.repetition_penalty, s.all_ids, s.params.seed) for s in adm])
        self.stats["host_sched_s"] += time.perf_counter() - th
        if not items:
            return finished
        self.stats["steps"] += 1
        trace = self.trace  # another thread may switch tracing on or off mid-step: the step's own view
        t0 = time.perf_counter() if trace is not None else 0.0
        tok0 = self.stats["prefill_tokens"] + self.stats["decode_tokens"]
        if kind in ("prefill", "mixed"):
            try:
                finished += self._run_prefill(items)
            except BaseException:
                # the step's prompt blocks were registered when scheduled (in-step prefix sharing): never let
                # the cache serve blocks this failed step may not have written
                bad = list(getattr(self.sched, "last_registered", []))
                self.kv.unregister(bad)
                self._rollback_prefill(items, set(bad))
                raise
        else:
            finished += self._run_decode([s for s, _, _ in items], max_window)
        if trace is not None:
            trace.append((t0, kind, len(items), self.stats["prefill_tokens"] + self.stats["decode_tokens"] - tok0,
                          time.perf_counter() - t0))
        return finished

    def _rollback_prefill(self, items, bad: set) -> None:
        """Undo a failed prefill step's effect on its sequences, so a caller that keeps stepping never
        attends over K/V the step did not write: a sequence whose already-computed prefix includes a
        block registered (and so possibly matched) in this step restarts its prefill from scratch; every
        other prefill item is reset to where the step started, its hash chain cut back to the blocks
        computed before it (the step's blocks are registered again once they are really computed)."""
        bs = self.cfg.block_size
        for seq, a, b in items:
            if not seq.is_prefill and b - a == 1 and seq.output_ids:
                continue  # a decode row riding in a mixed step
            if bad and any(blk in bad for blk in seq.blocks[: -(-a // bs)]):
                self.kv.free(seq)
                seq.cached_prefix = 0
                continue
            seq.num_computed = min(seq.num_computed, a)
            del seq.block_hashes[a // bs:]

    # ------------------------------------------------------------------ helpers
    def _slots_of(self, seq: Sequence, start: int, end: int) -> np.ndarray:
        bs = self.cfg.block_size
        pos = np.arange(start, end)
        blocks = np.asarray(seq.blocks, dtype=np.int64)
        return (blocks[pos // bs] * bs + pos % bs).astype(np.int32)

    def _block_table(self, seqs, width: int) -> np.ndarray:
        bt = np.zeros((len(seqs), width), dtype=np.int32)
        for i, s in enumerate(seqs):
            n = min(len(s.blocks), width)
            bt[i, :n] = s.blocks[:n]
        return bt

    def _read_host(self, t: torch.Tensor) -> np.ndarray:
        """Device int tensor -> host numpy through a persistent pinned buffer (a non-blocking copy and an
        event wait that releases the GIL).  A pageable .cpu() is staged by the runtime through a shared
        bounce buffer, where it queued behind other threads' copies (retrieval) while the GPU idled."""
        if not self.on_gpu:
            return t.cpu().numpy()
        n = t.numel()
        buf = getattr(self, "_pinned_out", None)
        if buf is None or buf.numel() < n or buf.dtype != t.dtype:
            buf = self._pinned_out = torch.empty(max(n, 4096), dtype=t.dtype, pin_memory=True)
            self._pinned_ev = torch.cuda.Event()
        dst = buf[:n].view(t.shape)
        dst.copy_(t, non_blocking=True)
        self._pinned_ev.record()
        self._pinned_ev.synchronize()
        check_device_errors("engine step")
        return dst.numpy().copy()

    def _to_dev(self, arr: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(arr)
        if self.on_gpu:
            return t.pin_memory().to(self.device, non_blocking=True)
        return t

    # ------------------------------------------------------------------ prefill
    def _run_prefill(self, items) -> list[Sequence]:
        n_pref = next((i for i, (s, a, b) in enumerate(items) if b - a == 1 and s.output_ids and a == s.total_len - 1),
                      len(items))
        if 0 < n_pref < len(items):
            return self._run_mixed(items[:n_pref], [s for s, _, _ in items[n_pref:]])
        t0 = time.perf_counter()
        seqs = [s for s, _, _ in items]
        ids, pos, slots, q_start, ctx = [], [], [], [0], []
        for s, a, b in items:
            ids.append(np.asarray(s.all_ids[a:b], dtype=np.int32))
            pos.append(np.arange(a, b, dtype=np.int32))
            slots.append(self._slots_of(s, a, b))
            q_start.append(q_start[-1] + (b - a))
            ctx.append(b)
        # rows to sample: the last token of every chunk that completes its prompt.  Uploaded with the step's
        # inputs: a separate pageable upload after the forward is a synchronous copy queued behind it, which
        # held the host until the forward finished and left the GPU idle while the LM head and sampler launched
        samp = [i for i, (s, a, b) in enumerate(items) if b == s.total_len]
        width = max(len(s.blocks) for s in seqs)
        packed = np.concatenate([np.concatenate(ids), np.concatenate(pos), np.concatenate(slots),
                                 np.asarray(q_start, dtype=np.int32), np.asarray(ctx, dtype=np.int32),
                                 self._block_table(seqs, width).reshape(-1),
                                 np.asarray([q_start[i + 1] - 1 for i in samp], dtype=np.int32),
                                 np.asarray([items[i][0].slot for i in samp], dtype=np.int32)])
        dev = self._to_dev(packed)
        th = time.perf_counter()
        self.stats["host_prefill_prep_s"] += th - t0
        T, n = q_start[-1], len(seqs)
        o = 0
        d_ids = dev[o:o + T]; o += T
        d_pos = dev[o:o + T]; o += T
        d_slot = dev[o:o + T]; o += T
        d_qs = dev[o:o + n + 1]; o += n + 1
        d_ctx = dev[o:o + n]; o += n
        d_bt = dev[o:o + n * width].view(n, width); o += n * width
        d_rows = dev[o:o + len(samp)]; o += len(samp)
        d_samp_slots = dev[o:o + len(samp)]
        meta = AttnMetadata(q_start=d_qs, ctx_len=d_ctx, block_tables=d_bt, slot_mapping=d_slot,
                            max_q_len=max(b - a for _, a, b in items), num_seqs=n, num_tokens=T)
        hidden = self.model.forward(d_ids, d_pos, meta, self.kv_caches)
        tp = self.model.tp
        if samp:  # LM head + sampler queued right behind the forward
            toks_d = self._sample(hidden.index_select(0, d_rows), d_samp_slots)
            tp.stage_health()
        t1 = time.perf_counter()
        self.stats["host_prefill_launch_s"] += t1 - th
        for s, a, b in items:  # host bookkeeping while the GPU runs
            s.num_computed = b
            self.kv.register_full_blocks(s)
        finished = []
        if samp:
            toks = self._read_host(toks_d).reshape(-1).tolist()
            tp.check_health()
            now = time.perf_counter()
            self.stats["host_prefill_sample_s"] += now - t1
            for i, t in zip(samp, toks):
                s = items[i][0]
                if self._append(s, int(t), now):
                    finished.append(s)
            self.stats["host_prefill_post_s"] += time.perf_counter() - now
        self.stats["prefill_tokens"] += T
        self.stats["prefill_s"] += time.perf_counter() - t0
        return finished

    def _run_mixed(self, pitems, dseqs) -> list[Sequence]:
        """One step of prefill chunks plus one decode token for every decode-ready sequence (stall-free
        batching): the decode rows ride in the prefill step's GEMMs (M = prefill tokens + decode rows,
        run at the prefill schedule's MFMA rate instead of a separate weight-streaming decode step) and
        their attention runs on the split-KV decode kernel.  Inputs go up as one packed int32 buffer: the
        prefill part built per chunk, the decode part from the per-slot block table (_decode_inputs)."""
        t0 = time.perf_counter()
        bs = self.cfg.block_size
        n_pref, n_dec = len(pitems), len(dseqs)
        ids, pos, slots, q_start, ctx = [], [], [], [0], []
        for s, a, b in pitems:
            ids.append(np.asarray(s.all_ids[a:b], dtype=np.int32))
            pos.append(np.arange(a, b, dtype=np.int32))
            slots.append(self._slots_of(s, a, b))
            q_start.append(q_start[-1] + (b - a))
            ctx.append(b)
        Tp = q_start[-1]
        T = Tp + n_dec
        pseqs = [s for s, _, _ in pitems]
        wp = max(len(s.blocks) for s in pseqs)
        max_ctx = max(s.total_len for s in dseqs)
        wd = -(-max_ctx // bs)
        dec = self._decode_inputs(dseqs, n_dec, wd, 1)
        lay = _ctrl_layout(n_dec, wd, 1)

        def part(name):
            o, shape = lay[name]
            return dec[o:o + int(np.prod(shape))]

        d_ids, d_pos, d_slot, d_ctx, d_samp, d_bt = (part(k) for k in ("ids", "pos", "slot", "ctx", "slots", "bt"))
        # rows to sample: the last token of every prefill chunk that completes its prompt, then every decode row
        done = [i for i, (s, a, b) in enumerate(pitems) if b == s.total_len]
        samp_rows = np.concatenate([np.asarray([q_start[i + 1] - 1 for i in done], dtype=np.int32),
                                    np.arange(Tp, T, dtype=np.int32)])
        samp_slots = np.concatenate([np.asarray([pseqs[i].slot for i in done], dtype=np.int32), d_samp])
        packed = np.concatenate([
            *ids, d_ids, *pos, d_pos, *slots, d_slot,                       # [T] x 3
            np.asarray(q_start, dtype=np.int32), np.asarray(ctx, dtype=np.int32),
            self._block_table(pseqs, wp).reshape(-1),                       # prefill chunks
            np.arange(n_dec + 1, dtype=np.int32), d_ctx, d_bt,              # decode rows
            samp_rows, samp_slots])
        dev = self._to_dev(packed)
        th = time.perf_counter()
        self.stats["host_prefill_prep_s"] += th - t0
        o = 0
        t_ids = dev[o:o + T]; o += T
        t_pos = dev[o:o + T]; o += T
        t_slot = dev[o:o + T]; o += T
        p_qs = dev[o:o + n_pref + 1]; o += n_pref + 1
        p_ctx = dev[o:o + n_pref]; o += n_pref
        p_bt = dev[o:o + n_pref * wp].view(n_pref, wp); o += n_pref * wp
        q_qs = dev[o:o + n_dec + 1]; o += n_dec + 1
        q_ctx = dev[o:o + n_dec]; o += n_dec
        q_bt = dev[o:o + n_dec * wd].view(n_dec, wd); o += n_dec * wd
        ns = len(samp_rows)
        t_rows = dev[o:o + ns]; o += ns
        t_samp = dev[o:o + ns]
        nsplit, split_len = _decode_plan(self.model, n_dec, max_ctx, self.cfg.max_model_len, graph=False)
        hq, dh = self.model.hq, self.model.head_dim
        meta = AttnMetadata(q_start=p_qs, ctx_len=p_ctx, block_tables=p_bt, slot_mapping=t_slot,
                            max_q_len=max(b - a for _, a, b in pitems), num_seqs=n_pref, num_tokens=Tp)
        meta.extra["decode_rows"] = (Tp, AttnMetadata(
            q_start=q_qs, ctx_len=q_ctx, block_tables=q_bt, slot_mapping=t_slot[Tp:], max_q_len=1, num_seqs=n_dec,
            num_tokens=n_dec, is_decode=True, num_splits=nsplit, split_len=split_len,
            part_o=self._part_o[: nsplit * n_dec * hq * dh] if self.on_gpu else None,
            part_ml=self._part_ml[: nsplit * n_dec * hq * 2] if self.on_gpu else None))
        hidden = self.model.forward(t_ids, t_pos, meta, self.kv_caches)
        toks_d = self._sample(hidden.index_select(0, t_rows), t_samp)
        t1 = time.perf_counter()
        self.stats["host_prefill_launch_s"] += t1 - th
        tp = self.model.tp
        tp.stage_health()
        toks = self._read_host(toks_d).reshape(-1).tolist()
        tp.check_health()
        now = time.perf_counter()
        self.stats["host_prefill_sample_s"] += now - t1
        finished = []
        for s, a, b in pitems:
            s.num_computed = b
            self.kv.register_full_blocks(s)
        k = 0
        for i in done:
            s = pseqs[i]
            if self._append(s, int(toks[k]), now):
                finished.append(s)
            k += 1
        for s in dseqs:
            if s.finish_reason is None and s.status == SeqStatus.RUNNING:
                s.num_computed = s.total_len
                if self._append(s, int(toks[k]), now):
                    finished.append(s)
            k += 1
        self.stats["host_prefill_post_s"] += time.perf_counter() - now
        self.stats["prefill_tokens"] += Tp
        self.stats["decode_tokens"] += n_dec
        self.stats["mixed_steps"] += 1
        self.stats["prefill_s"] += time.perf_counter() - t0
        return finished

    # ------------------------------------------------------------------ decode
    @staticmethod
    def _last_id(s: Sequence) -> int:
        return s.output_ids[-1] if s.output_ids else s.prompt_ids[-1]

    def _decode_inputs(self, seqs, B: int, width: int, K: int = 1, groups: bool = False) -> np.ndarray:
        """Packed int32 control buffer for a K-step decode window:
        ids[B] | pos[K,B] | slot[K,B] | ctx[K,B] | sampler slots[B] | q_start[B+1] | pre[B] | groups[B//2,2] |
        block table[B,width].  Rows >= len(seqs) are padding (scratch slot, slot mapping -1).  pre / groups:
        the shared-prefix decode layout (ops/attention.prefix_groups) when ``groups`` and the batch's rows
        share enough cached prefix (self._cascade_plan is then 1), else zeros."""
        n = len(seqs)
        bs = self.cfg.block_size
        lay = _ctrl_layout(B, width, K)
        buf = np.zeros(lay["size"], dtype=np.int32)

        def part(name):
            o, shape = lay[name]
            return buf[o:o + int(np.prod(shape))].reshape(shape)

        ids, pos, slot, ctx, sl, qs, bt = (part(k) for k in ("ids", "pos", "slot", "ctx", "slots", "qs", "bt"))
        qs[:] = np.arange(B + 1, dtype=np.int32)
        self._cascade_plan = 0
        ids[n:] = 0
        pos[:, n:] = 0
        slot[:, n:] = -1
        ctx[:, n:] = 1
        sl[n:] = self.scratch_slot
        if n:
            # block-table rows come from a per-slot table kept across steps: a running sequence only
            # appends to its block list (KVCacheManager.ensure extends in place; free / prefix match
            # install a new list), so a step writes just the new tail, a full row when the slot's list
            # object changed, and the batch is one row gather
            tab, owner, have = self._slot_block_table()
            tw = tab.shape[1]
            rows_l, ids_l, len_l = [0] * n, [0] * n, [0] * n  # one pass over the rows (1024-row steps)
            for i, s in enumerate(seqs):
                r = s.slot
                b = s.blocks
                nb = len(b)
                if nb > tw:
                    nb = tw
                h = have[r]
                if owner[r] is not b or h > nb:
                    tab[r, :nb] = b[:nb]
                    owner[r] = b
                    have[r] = nb
                elif h < nb:
                    tab[r, h:nb] = b[h:nb]
                    have[r] = nb
                out = s.output_ids
                pr = s.prompt_ids
                rows_l[i] = r
                ids_l[i] = out[-1] if out else pr[-1]
                len_l[i] = len(pr) + len(out)
            rows = np.asarray(rows_l, dtype=np.int64)
            bt[:n] = tab[rows, :width] if width <= tw else np.pad(tab[rows], ((0, 0), (0, width - tw)))
            ids[:n] = ids_l
            sl[:n] = rows_l
            L = np.asarray(len_l, dtype=np.int64)
            p = L[None, :] - 1 + np.arange(K, dtype=np.int64)[:, None]  # [K, n]
            pos[:, :n] = p
            ctx[:, :n] = p + 1
            slot[:, :n] = bt[np.arange(n)[None, :], p // bs].astype(np.int64) * bs + p % bs
            if groups and n >= 4:
                self._plan_cascade(bt[:n], L, part("pre"), part("part"), part("items"))
        return buf

    def _plan_cascade(self, bt, L, pre, part, items) -> None:
        """Fill the shared-prefix layout of one decode window when its groups save at least CASCADE_MIN of
        the batch's K/V keys (a group's prefix is read once instead of once per member)."""
        total = int(L.sum())
        self.stats["decode_keys"] += total
        r = prefix_groups(bt, L, self.cfg.block_size, self.model.hq // max(1, self.model.hkv), CASCADE_RG)
        if r is None:
            return
        p, spans, saved = r
        if saved < CASCADE_MIN * total:
            return
        pl, it, used = cascade_layout(p, spans, items.shape[0])
        if used * max(1, self.model.hkv) < CASCADE_MIN_WAVES:
            return
        pre[: len(p)] = p
        part[: len(pl)] = pl
        items[:] = it
        self._cascade_plan = 1
        self.stats["cascade_windows"] += 1
        self.stats["cascade_rows"] += sum(b - a for a, b in spans)
        self.stats["cascade_saved_keys"] += saved

    def _slot_block_table(self):
        """(table [slots, max blocks], row owner, row length) behind _decode_inputs."""
        t = getattr(self, "_sbt", None)
        if t is None:
            rows = self.cfg.max_num_seqs + 1
            t = self._sbt = (np.zeros((rows, self.max_blocks_per_seq + 1), dtype=np.int32), [None] * rows,
                             [0] * rows)
        return t

    def _views(self, buf: torch.Tensor, B: int, width: int, K: int = 1):
        lay = _ctrl_layout(B, width, K)
        lay.pop("size")
        return {name: buf[o:o + int(np.prod(shape))].view(*shape) for name, (o, shape) in lay.items()}

    def _decode_forward(self, v, B, nsplit, split_len, out_tokens, K: int = 1, npre: int = 0):
        """K chained decode steps; step j > 0 embeds the ids step j-1 sampled (on device).  npre: 1 = the
        shared-prefix decode over v["pre"] / v["part"] / v["items"]."""
        hq, d = self.model.hq, self.model.head_dim
        part_o = self._part_o[: nsplit * B * hq * d] if self.on_gpu else None
        part_ml = self._part_ml[: nsplit * B * hq * 2] if self.on_gpu else None
        cas = None
        if npre:
            npl = CASCADE_MAX_PLANES
            cas = Cascade(pre_len=v["pre"], pre_part=v["part"], items=v["items"], planes=npl,
                          pre_o=self._pre_o[: npl * B * hq * d] if self.on_gpu else None,
                          pre_ml=self._pre_ml[: npl * B * hq * 2] if self.on_gpu else None, rg=CASCADE_RG)
        for j in range(K):
            ids = v["ids"] if j == 0 else out_tokens[j - 1]
            meta = AttnMetadata(q_start=v["qs"], ctx_len=v["ctx"][j], block_tables=v["bt"], slot_mapping=v["slot"][j],
                                max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True, num_splits=nsplit,
                                split_len=split_len, part_o=part_o, part_ml=part_ml, cascade=cas)
            hidden = self.model.forward(ids, v["pos"][j], meta, self.kv_caches)
            self._sample(hidden, v["slots"], out=out_tokens[j])
        return out_tokens

    def _sample(self, hidden: torch.Tensor, slots: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """LM head + sampler.  Under TP the vocab-parallel sampler runs on this rank's logit shard
        (ops/sampling.sample_tp: small (max, histogram, winner) exchanges instead of a full-logit
        all-gather); GRAG_TP_SAMPLER=gather keeps the gather for A/B."""
        m = self.model
        if m.tp.trivial or not hasattr(m, "local_logits") or _TP_SAMPLER == "gather":
            return sample(m.compute_logits(hidden), self.sampler, slots, out=out)
        return sample_tp(m.local_logits(hidden), self.sampler, slots, m.tp, m.vocab0, out=out)

    def _window(self, seqs, cap: int | None = None) -> int:
        """Largest power-of-two window <= decode_window that no sequence's
        max_tokens / max_model_len cuts short and whose KV blocks fit."""
        K = max(1, self.cfg.decode_window if cap is None else min(cap, self.cfg.decode_window))
        if K == 1:  # nothing to cut short (a 1-step window is what the scheduler already reserved for)
            return 1
        for s in seqs:
            K = min(K, s.params.max_tokens - len(s.output_ids), self.cfg.max_model_len - s.total_len)
        K = max(1, K)
        while K & (K - 1):
            K &= K - 1
        if K > 1:
            for s in seqs:
                if not self.kv.ensure(s, s.total_len + K - 1):
                    return 1
        return K

    def _run_decode(self, seqs, max_window: int | None = None) -> list[Sequence]:
        t0 = time.perf_counter()
        n = len(seqs)
        casc = False
        probe = None
        if self.cfg.cascade_decode and n >= 8:
            # the prefix cache hands out one block id per (content, prefix) chain, so two rows holding the same
            # id at block index k share their first k + 1 blocks.  Probe at the index a group's prefix must
            # reach for the window to save CASCADE_MIN of its keys (at least min_blocks): a batch whose rows
            # share only a short system prompt is not sorted and grouped every window
            k = max(_CASCADE_PROBE, int(CASCADE_MIN * sum(s.total_len for s in seqs) / (n * self.cfg.block_size)))
            probe = [s.blocks[k] for s in seqs if len(s.blocks) > k]
        if probe and len(set(probe)) < len(probe):
            # some rows share a cached prompt prefix (ingest's summary / title / keyword calls of one chunk, an
            # agent job's calls over the same documents): rows side by side by leading block ids, so the
            # shared-prefix decode (ops/attention.prefix_groups) can group adjacent rows
            seqs = sorted(seqs, key=_prefix_blocks)
            casc = True
        elif _GROUP_ROWS and n >= 32:
            # rows that share a cached prompt prefix side by side: with the decode kernel's XCD placement
            # (csrc/kernels/attention.hip g_decode_xcd) their shared K/V blocks are read on one XCD at about
            # the same time and come from its L2 for all but the first
            seqs = sorted(seqs, key=_prefix_blocks)
        # under TP the graphs hold the decode's collectives (one-shot IPC all-reduce, RCCL logits gather);
        # replicated scheduling makes every TP rank pick, capture and replay the same graph in lockstep
        use_graph = (self.on_gpu and self.cfg.use_cuda_graph and n <= max(self.cfg.graph_batch_sizes)
                     and getattr(self.model.tp, "capturable", True))  # gloo-staged TP collectives: eager decode
        K = self._window(seqs, max_window) if use_graph else 1
        max_ctx = max(len(s.prompt_ids) + len(s.output_ids) for s in seqs) + K - 1
        if use_graph:
            width = self.max_blocks_per_seq
            B = next(b for b in self.cfg.graph_batch_sizes if b >= n)
            nsplit, split_len = _decode_plan(self.model, B, max_ctx, self.cfg.max_model_len)
            packed = self._decode_inputs(seqs, B, width, K, groups=casc)
            npre = self._cascade_plan
            g = self._graphs.get((B, nsplit, split_len, K, self.sampler.rounds, npre))
            if g is None:
                g = self._capture(B, nsplit, split_len, K, npre)
            self._static_host[: packed.size] = torch.from_numpy(packed)
            self._static_dev[: packed.size].copy_(self._static_host[: packed.size], non_blocking=True)
            g.graph.replay()
            tw = time.perf_counter()
            self.stats["host_decode_prep_s"] += tw - t0
            self.model.tp.stage_health()
            toks = self._read_host(g.out_tokens[:K, :n])
            self.model.tp.check_health()
            self.stats["decode_wait_s"] += time.perf_counter() - tw
            self.stats["graph_replays"] += 1
        else:
            nsplit, split_len = _decode_plan(self.model, n, max_ctx, self.cfg.max_model_len, graph=False)
            width = max(len(s.blocks) for s in seqs)
            dev = self._to_dev(self._decode_inputs(seqs, n, width, 1, groups=casc))
            out = torch.empty(1, n, dtype=torch.int32, device=self.device)
            out = self._decode_forward(self._views(dev, n, width, 1), n, nsplit, split_len, out, 1,
                                       npre=self._cascade_plan)
            self.model.tp.stage_health()
            toks = out.cpu().numpy()
            check_device_errors("engine step")
            self.model.tp.check_health()
        now = time.perf_counter()
        finished = []
        # fast path for sequences nobody watches per token (no stream consumer, no stop strings / ids) and
        # no EOS stop in this window: the window's tokens are appended in one extend, and only the token
        # that ends the sequence goes through _append (finish + detokenize)
        cols = toks[:K, :n].T.tolist()
        eos, mml = self._eos, self.cfg.max_model_len
        slow = []
        ntok = 0
        running = SeqStatus.RUNNING
        for i, s in enumerate(seqs):
            if s.finish_reason is not None or s.status is not running:
                continue
            p = s.params
            c = cols[i]
            if (s.on_token is not None or p.stop or p.stop_token_ids
                    or (not p.ignore_eos and eos and not eos.isdisjoint(c))):
                slow.append(i)
                continue
            out = s.output_ids
            lo = len(out)
            L = len(s.prompt_ids) + lo
            left = p.max_tokens - lo  # tokens until max_tokens / max_model_len end the sequence
            if mml - L < left:
                left = mml - L
            if left <= 0:
                slow.append(i)
                continue
            if s.first_token_time is None:
                s.first_token_time = now
            if left <= K:  # the window's token `left` ends the sequence: it goes through _append
                out.extend(c[:left - 1])
                s.num_computed = L + left - 1
                if self._append(s, c[left - 1], now):
                    finished.append(s)
                ntok += left
            else:
                out.extend(c)
                s.num_computed = L + K - 1
                ntok += K
        self.stats["decode_tokens"] += ntok
        if slow:
            live = [seqs[i] for i in slow]
            for j in range(K):
                nxt = []
                for s, i in zip(live, slow):
                    if s.finish_reason is not None or s.status != SeqStatus.RUNNING:
                        continue
                    s.num_computed = s.total_len
                    if self._append(s, int(toks[j, i]), now):
                        finished.append(s)
                    else:
                        nxt.append((s, i))
                self.stats["decode_tokens"] += len(live)
                if not nxt:
                    break
                live, slow = [s for s, _ in nxt], [i for _, i in nxt]
        self.stats["decode_steps"] += K
        self.stats["decode_s"] += now - t0
        self.stats["host_decode_post_s"] += time.perf_counter() - now
        return finished

    def _ensure_static(self):
        if self._static is None:
            W = self.max_blocks_per_seq
            Kmax = max(1, self.cfg.decode_window)
            size = _ctrl_layout(self._max_b, W, Kmax)["size"]
            self._static_dev = torch.zeros(size, dtype=torch.int32, device=self.device)
            self._static_host = torch.zeros(size, dtype=torch.int32).pin_memory()
            self._static = True
            self._graph_pool = torch.cuda.graph_pool_handle()

    def _capture(self, B, nsplit, split_len, K=1, npre=0) -> _DecodeGraph:
        with WS.owned_by(self._ws):
            return self._capture_ws(B, nsplit, split_len, K, npre)

    def _capture_ws(self, B, nsplit, split_len, K=1, npre=0) -> _DecodeGraph:
        t0 = time.perf_counter()
        try:
            # The eager warm-up step of the shape runs real TP collectives (all-reduces, the sampler's
            # exchanges): it runs under the SHARED guard.  Only the capture itself -- local work, its
            # collectives are recorded, not run -- holds the guard exclusively.  An exclusive section that
            # waited on a peer rank could deadlock against a retrieval thread holding the shared guard in a
            # cross-rank search collective on either rank.
            with gpu_shared():
                prep = self._capture_prepare(B, nsplit, split_len, K, npre)
            with gpu_guard():  # no other thread may sync / allocate while the capture is open
                return self._capture_locked(B, nsplit, split_len, K, prep, npre)
        finally:
            dt = time.perf_counter() - t0
            self.stats["capture_s"] += dt
            if self.trace is not None:
                self.trace.append((t0, "capture", B, K, dt))

    def _capture_prepare(self, B, nsplit, split_len, K=1, npre=0):
        self._ensure_static()
        W = self.max_blocks_per_seq
        # a benign batch: every row is a padding row (scratch block, scratch slot)
        dummy = self._decode_inputs([], B, W, K)
        self._static_dev[: dummy.size].copy_(torch.from_numpy(dummy))
        v = self._views(self._static_dev, B, W, K)
        out = torch.zeros(K, B, dtype=torch.int32, device=self.device)
        rng_save = self.sampler.rng.clone()
        seen_save = self.sampler.seen[self.scratch_slot].clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # one warm-up step of this shape (every window step has the same shapes)
            self._decode_forward(v, B, nsplit, split_len, out, 1, npre)
        torch.cuda.current_stream().wait_stream(s)
        return v, out, rng_save, seen_save

    def _capture_locked(self, B, nsplit, split_len, K, prep, npre=0) -> _DecodeGraph:
        v, out, rng_save, seen_save = prep
        graph = torch.cuda.CUDAGraph()
        # thread_local: API / retrieval threads keep launching (and syncing) on
        # their own streams while the engine thread captures
        with no_gc(), torch.cuda.graph(graph, pool=self._graph_pool, capture_error_mode="thread_local"):
            self._decode_forward(v, B, nsplit, split_len, out, K, npre)
        torch.cuda.synchronize()
        self.sampler.rng.copy_(rng_save)
        self.sampler.seen[self.scratch_slot].copy_(seen_save)
        g = _DecodeGraph(graph, out, B, nsplit, split_len, K)
        # the sampler's launch chain depends on which sampling features live slots use
        self._graphs[(B, nsplit, split_len, K, self.sampler.rounds, npre)] = g
        self.stats["graph_captures"] += 1
        return g

    @torch.inference_mode()
    def warmup_graphs(self, batch_sizes=None, max_ctx=2048, windows=(1,), params: SamplingParams | None = None,
                      cascade=(False,)) -> int:
        """Capture the decode graphs a workload will replay ahead of time
        (batch buckets x decode windows K, split plan of ``max_ctx``) so no
        capture lands inside a latency-sensitive step.  Keyed on the
        sampler's current launch chain: call it once requests with the
        serving sampling parameters have been admitted.  Returns the number
        of graphs captured.  ``max_ctx`` may be a list (one split plan per context length).  ``params``:
        capture for the sampler launch chain these sampling parameters select (top-k / top-p rounds)
        instead of the live slots' (e.g. an ingest engine warmed before its first request).  ``cascade``:
        which decode variants to capture: False = the plain graph, True = the shared-prefix decode's (batches of
        >= 8 rows only)."""
        if not (self.on_gpu and self.cfg.use_cuda_graph and getattr(self.model.tp, "capturable", True)):
            return 0
        prev = self.sampler.rounds_override
        if params is not None:
            sampled = params.temperature > 0
            self.sampler.rounds_override = ((1 if sampled and 0 < params.top_k < self.sampler.vocab else 0)
                                            | (2 if sampled and params.top_p < 1.0 else 0))
        try:
            with self._on_stream():
                n = 0
                for mc in (max_ctx if isinstance(max_ctx, (list, tuple)) else [max_ctx]):
                    n += self._warmup_graphs(batch_sizes, mc, windows, cascade)
                return n
        finally:
            self.sampler.rounds_override = prev

    def _warmup_graphs(self, batch_sizes, max_ctx, windows, cascade=(False,)) -> int:
        n = 0
        parts = [int(c) for c in cascade if not c or self.cfg.cascade_decode]
        for B in batch_sizes or self.cfg.graph_batch_sizes:
            nsplit, split_len = _decode_plan(self.model, B, max_ctx, self.cfg.max_model_len)
            for K in windows:
                if K > max(1, self.cfg.decode_window):
                    continue
                for npre in parts:
                    if npre and B < 8:
                        continue
                    if (B, nsplit, split_len, K, self.sampler.rounds, npre) not in self._graphs:
                        self._capture(B, nsplit, split_len, K, npre)
                        n += 1
        return n

    # ------------------------------------------------------------------ outputs
    def _append(self, s: Sequence, tok: int, now: float) -> bool:
        if s.first_token_time is None:
            s.first_token_time = now
        s.output_ids.append(tok)
        p = s.params
        reason = None
        if not p.ignore_eos and tok in self._eos and len(s.output_ids) > p.min_tokens:
            reason = "stop"
        elif tok in p.stop_token_ids:
            reason = "stop"
        elif len(s.output_ids) >= p.max_tokens:
            reason = "length"
        elif s.total_len >= self.cfg.max_model_len:
            reason = "length"
        if s.on_token is None and not p.stop:
            # nobody reads the text before the end (no stream consumer, no stop strings): detokenize once
            # at finish instead of per token (~2 us x 512 rows of host time per decode step)
            if reason is not None:
                ids = s.output_ids[:-1] if reason == "stop" and tok in self._eos else s.output_ids
                s.text = self._detok_all(ids)
                s.finish_reason = reason
                s.finish_time = now
                self.sched.finish(s)
                return True
            return False
        if s.detok is None:
            s.detok = IncrementalDetokenizer(self.tok)
        delta = ""
        if reason != "stop" or tok not in self._eos:
            delta = s.detok.push(tok)
        if reason is not None:
            delta += s.detok.flush()
        s.text += delta
        if p.stop and reason is None:
            for st in p.stop:
                idx = s.text.find(st, max(0, len(s.text) - len(delta) - len(st)))
                if idx >= 0:
                    s.text = s.text[:idx]
                    reason = "stop"
                    break
        if reason is not None:
            s.finish_reason = reason
            s.finish_time = now
            self.sched.finish(s)
        self._notify(s, delta, reason is not None)
        return reason is not None

    def _detok_all(self, ids) -> str:
        """The text IncrementalDetokenizer would have produced for ``ids`` (same bytes, same decoder)."""
        tb = getattr(self.tok, "token_bytes", None)
        if tb is None:
            return "".join(self.tok.decode([t]) for t in ids)
        return b"".join(tb(t) for t in ids).decode("utf-8", errors="replace")

    def _notify(self, s: Sequence, delta, finished: bool) -> None:
        if s.on_token is not None:
            try:
                s.on_token(s, delta, finished)
            except Exception:  # a slow/broken consumer must never kill the engine loop
                log.exception("on_token callback failed for %s", s.req_id)
