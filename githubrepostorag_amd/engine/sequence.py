"""Requests, sampling parameters and per-sequence state."""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field
from typing import Callable


@dataclass
class SamplingParams:
    """OpenAI/vLLM-style knobs.  Reference defaults: worker temperature 0.4,
    top_p 0.8, repetition_penalty 1.2, max 4096 tokens
    (rag_worker/src/worker/services/qwen_llm.py:107-113); ingest temperature
    0.5, top_p 0.9, max 2048 (ingest/src/app/llm_init.py:108-114)."""

    max_tokens: int = 256
    temperature: float = 0.4
    top_p: float = 0.8
    top_k: int = 0
    repetition_penalty: float = 1.0
    stop: list[str] = field(default_factory=list)
    stop_token_ids: list[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: int | None = None
    min_tokens: int = 0
    priority: int = 0  # higher is admitted first (critical-path requests ahead of bulk waves)
    # queue key within a priority, lower first (None: the request's arrival).  An agent job's calls carry the
    # job's start time, so an older job's next call is admitted and prefilled before newer jobs' calls
    order: float | None = None


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


@dataclass(eq=False)  # identity semantics: the scheduler's list membership tests must not
class Sequence:      # compare every field (that cost ~150 ms per step at 192 live sequences)
    req_id: str
    prompt_ids: list[int]
    params: SamplingParams
    on_token: Callable | None = None
    output_ids: list[int] = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    slot: int = -1
    blocks: list[int] = field(default_factory=list)
    block_hashes: list[int] = field(default_factory=list)
    num_computed: int = 0  # tokens whose KV is in the cache
    cached_prefix: int = 0  # tokens reused from the prefix cache
    finish_reason: str | None = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: float | None = None
    finish_time: float | None = None
    text: str = ""
    cancelled: bool = False
    num_preemptions: int = 0
    detok: object = None  # tokenizer.IncrementalDetokenizer, created on the first output token

    @property
    def all_ids(self) -> list[int]:
        return self.prompt_ids + self.output_ids

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def is_prefill(self) -> bool:
        # KV missing for some token other than the newest sampled one
        return self.num_computed < self.total_len - (1 if self.output_ids else 0)

    @property
    def ttft(self) -> float | None:
        return None if self.first_token_time is None else self.first_token_time - self.arrival


@dataclass
class Completion:
    req_id: str
    text: str
    token_ids: list[int]
    finish_reason: str | None
    prompt_tokens: int
    ttft_s: float | None
    latency_s: float | None
    cached_tokens: int = 0
    first_token_at: float | None = None  # time.perf_counter() stamp of the first generated token
