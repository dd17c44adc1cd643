"""LLM clients with the reference's ``complete(prompt) -> .text`` contract.

* ``EngineLLM`` — in-process client of the GPU engine (no HTTP hop, no 60 s
  socket timeout): chat-templates the prompt (user turn; optional system
  turn), applies the worker's sampling defaults (temperature 0.4, top_p 0.8,
  repetition_penalty 1.2 — rag_worker/src/worker/services/qwen_llm.py:107-113)
  or the ingest ones (system "metadata writer" prompt, temperature 0.5,
  top_p 0.9, ``enable_thinking=False`` when ALLOW_THINKING=false —
  ingest/src/app/llm_init.py:27-33,108-120), cleans selector answers
  (qwen_llm.py:41-102) and sanitises chain-of-thought / role markers
  (llm_init.py:36-48).  Failures are retried (bounded) and then surface as
  ``"Error: ..."`` text exactly like the reference (errors become content,
  SURVEY §2.11 quirk 8) — but are also counted in metrics and flagged on the
  response object.
* ``HTTPLLM`` — the same contract against any OpenAI-compatible endpoint
  (this package's own /v1/chat/completions or an external server).
* ``MeteredLLM`` — Prometheus wrapper (worker.py:73-88).
* ``ScriptedLLM`` — deterministic fake for tests / fault injection.
"""
from __future__ import annotations

import json
import logging
import re
import time
from dataclasses import dataclass
from typing import Callable

from ..engine.sequence import SamplingParams
from . import prompts

log = logging.getLogger(__name__)


@dataclass
class CompletionResponse:
    text: str
    error: bool = False
    ttft_s: float | None = None
    tokens: int = 0


_COT_PATTERNS = [
    r"(?is)<think>.*?</think>",
    r"(?im)^(assistant|system|user)\s*:\s*\d*\s*",
    r"(?im)^(okay|alright|let me|i need to|thinking|hmm)[^\n]*\n",
]


def sanitize(text: str) -> str:
    s = text or ""
    for pat in _COT_PATTERNS:
        s = re.sub(pat, "", s)
    s = re.sub(r"(?i)^\s*(final answer|summary)\s*:\s*", "", s.strip())
    return s.strip()


_SELECTOR_MARKERS = ("choice 1:", "choice 2:", "choice 3:", "choice 4:", "select one of the following",
                     "choose from the following options", "pick the best option")


def is_selector_prompt(prompt: str) -> bool:
    pl = prompt.lower()
    return any(m in pl for m in _SELECTOR_MARKERS)


def clean_selector_response(text: str) -> str:
    """Coerce a router/selector reply to a bare choice digit (qwen_llm.py:56-102)."""
    if not text:
        return "1"
    lines, seen = [], set()
    for ln in text.split("\n"):
        s = ln.strip()
        if s and s not in seen:
            lines.append(s)
            seen.add(s)
            if len(lines) >= 3:
                break
    t = "\n".join(lines)
    m = re.findall(r'\{"choice":\s*(\d+)(?:,\s*"reason":[^}]*)?\}', t)
    if m:
        return m[0]
    m = re.findall(r"\b([1-4])\b", t)
    if m:
        return m[0]
    try:
        parsed = json.loads(re.sub(r"^[{\[]+", "[", re.sub(r"]}]+$", "]", t)))
        if isinstance(parsed, list) and parsed and isinstance(parsed[0], dict) and "choice" in parsed[0]:
            return str(parsed[0]["choice"])
    except Exception:
        pass
    return "1"


class EngineLLM:
    WORKER = dict(temperature=0.4, top_p=0.8, repetition_penalty=1.2)
    INGEST = dict(temperature=0.5, top_p=0.9, repetition_penalty=1.0)

    def __init__(self, runner, tokenizer, max_tokens: int = 4096, mode: str = "worker",
                 allow_thinking: bool = True, timeout_s: float = 300.0, retries: int = 1,
                 stop: list[str] | None = None):
        self.runner = runner
        self.tok = tokenizer
        self.max_tokens = max_tokens
        self.mode = mode
        self.defaults = dict(self.WORKER if mode == "worker" else self.INGEST)
        self.allow_thinking = allow_thinking
        self.timeout_s = timeout_s
        self.retries = retries
        self.stop = stop or []

    def _messages(self, prompt: str) -> list[dict]:
        if self.mode == "ingest":
            return [{"role": "system", "content": prompts.METADATA_WRITER_SYSTEM},
                    {"role": "user", "content": prompt}]
        return [{"role": "user", "content": prompt}]

    def params(self, **kw) -> SamplingParams:
        d = dict(self.defaults)
        for k in ("temperature", "top_p", "repetition_penalty", "top_k", "seed", "priority", "order"):
            if kw.get(k) is not None:
                d[k] = kw[k]
        mt = kw.get("max_tokens") or kw.get("max_completion_tokens") or self.max_tokens
        return SamplingParams(max_tokens=int(mt), stop=list(kw.get("stop") or self.stop),
                              ignore_eos=bool(kw.get("ignore_eos", False)), **d)

    def fit(self, ids: list[int], max_tokens: int) -> list[int]:
        """Prompt ids that fit the engine's max_model_len with room to generate: an over-long prompt loses
        the MIDDLE of its text (the agent's prompts are system + question, then the retrieved context
        blocks, then the answer cue; ingest prompts are an instruction, then the material) — the head and
        the answer cue / chat-template tail are kept.  Counted in grag_llm_prompt_truncations_total."""
        eng = getattr(self.runner, "engine", None)
        mml = getattr(getattr(eng, "cfg", None), "max_model_len", None)
        if not mml:
            return ids
        reserve = max(1, min(int(max_tokens), max(16, mml // 8)))
        budget = mml - reserve
        if len(ids) <= budget:
            return ids
        tail = min(64, budget // 4)
        log.warning("prompt of %d tokens cut to %d (max_model_len %d, %d reserved to generate): middle "
                    "context dropped", len(ids), budget, mml, reserve)
        from ..service import metrics as M

        M.PROMPT_TRUNCATIONS.inc()
        return ids[:budget - tail] + ids[len(ids) - tail:]

    def _post(self, prompt: str, out: str) -> str:
        if self.mode == "ingest":
            return sanitize(out) or "No response generated"
        if is_selector_prompt(prompt):
            return clean_selector_response(out)
        return out

    def complete_many(self, prompt_list: list[str], **kw) -> list[CompletionResponse]:
        """A wave of independent completions (ingest extractors, roll-ups): tokenised here, in the
        caller's thread, and submitted to the engine together — no thread per call, no tokenising on
        the engine thread — then awaited; failed items are retried as one smaller wave."""
        sp = self.params(**kw)
        ids = [self.fit(self.tok.encode(self.tok.apply_chat_template(self._messages(p), True,
                                                                     None if self.allow_thinking else False)),
                        sp.max_tokens)
               for p in prompt_list]
        out: list[CompletionResponse | None] = [None] * len(prompt_list)
        todo = list(range(len(prompt_list)))
        for attempt in range(self.retries + 1):
            hs = [(i, self.runner.submit(ids[i], sp, interactive=self.mode != "ingest")) for i in todo]
            failed = []
            for i, h in hs:
                try:
                    c = h.wait(self.timeout_s)
                    out[i] = CompletionResponse(self._post(prompt_list[i], c.text), False, c.ttft_s, len(c.token_ids))
                except Exception as e:
                    log.warning("LLM call failed (attempt %d): %s", attempt + 1, e)
                    h.cancel()
                    out[i] = CompletionResponse(f"Error: {e}", True)
                    failed.append(i)
            todo = failed
            if not todo:
                break
        return out

    def complete(self, prompt: str, on_token: Callable[[str], None] | None = None, **kw) -> CompletionResponse:
        text = self.tok.apply_chat_template(self._messages(prompt), True,
                                            None if self.allow_thinking else False)
        sp = self.params(**kw)
        text = self.fit(self.tok.encode(text), sp.max_tokens)  # token ids, within max_model_len
        cancel_check = kw.get("cancel_check")
        err = None
        for attempt in range(self.retries + 1):
            try:
                if cancel_check is None:
                    c = self.runner.generate(text, sp, on_token=on_token, timeout=self.timeout_s)
                else:  # poll the job's cancel flag so a cancel aborts mid-decode
                    h = self.runner.submit(text, sp, on_token=on_token, interactive=self.mode != "ingest")
                    t_end = time.monotonic() + self.timeout_s
                    while not h.done.wait(0.05):
                        if cancel_check() or time.monotonic() > t_end:
                            h.cancel()
                            h.done.wait(5.0)
                            if cancel_check():
                                from .graph_agent import Cancelled

                                raise Cancelled()
                            raise TimeoutError("generation timed out")
                    c = h.wait(0)
                return CompletionResponse(self._post(prompt, c.text), False, c.ttft_s, len(c.token_ids))
            except Exception as e:  # bounded retry, then the reference's "errors become content"
                if type(e).__name__ == "Cancelled":
                    raise
                err = e
                log.warning("LLM call failed (attempt %d): %s", attempt + 1, e)
                time.sleep(0.05 * (attempt + 1))
        return CompletionResponse(f"Error: {err}", True)

    CANCEL_POLL_S = 0.25  # acomplete: how often a waiting call checks its job's cancel flag

    async def acomplete(self, prompt: str, on_token: Callable[[str], None] | None = None,
                        **kw) -> CompletionResponse:
        """``complete`` for a coroutine: the request is submitted to the engine runner and its completion
        awaited as a future (set from the engine / streamer thread), so a waiting call holds no thread."""
        import asyncio

        loop = asyncio.get_running_loop()
        text = self.tok.apply_chat_template(self._messages(prompt), True,
                                            None if self.allow_thinking else False)
        sp = self.params(**kw)
        ids = self.fit(self.tok.encode(text), sp.max_tokens)
        cancel_check = kw.get("cancel_check")
        err = None

        def _resolve(fut, h):
            if not fut.done():
                fut.set_result(h)

        for attempt in range(self.retries + 1):
            h = None
            try:
                fut = loop.create_future()
                h = self.runner.submit(ids, sp, on_token=on_token, interactive=self.mode != "ingest")
                h.add_done_callback(lambda hh, fut=fut: loop.call_soon_threadsafe(_resolve, fut, hh))
                t_end = loop.time() + self.timeout_s
                while not fut.done():
                    wait = max(0.0, t_end - loop.time())
                    if cancel_check is not None:
                        wait = min(wait, self.CANCEL_POLL_S)
                    await asyncio.wait({fut}, timeout=wait)
                    if fut.done():
                        break
                    if (cancel_check is not None and cancel_check()) or loop.time() >= t_end:
                        h.cancel()
                        if cancel_check is not None and cancel_check():
                            from .graph_agent import Cancelled

                            raise Cancelled()
                        raise TimeoutError("generation timed out")
                c = h.wait(0)
                return CompletionResponse(self._post(prompt, c.text), False, c.ttft_s, len(c.token_ids))
            except asyncio.CancelledError:
                if h is not None:
                    h.cancel()
                raise
            except Exception as e:  # bounded retry, then the reference's "errors become content"
                if type(e).__name__ == "Cancelled":
                    raise
                err = e
                log.warning("LLM call failed (attempt %d): %s", attempt + 1, e)
                await asyncio.sleep(0.05 * (attempt + 1))
        return CompletionResponse(f"Error: {err}", True)

    def stream_complete(self, prompt: str, **kw):
        yield self.complete(prompt, **kw)


class HTTPLLM:
    """OpenAI-compatible HTTP client (the reference's only transport)."""

    def __init__(self, endpoint: str, model: str, max_tokens: int = 4096, mode: str = "worker",
                 timeout_s: float = 60.0, allow_thinking: bool = True):
        self.endpoint = endpoint.rstrip("/")
        self.model = model
        self.max_tokens = max_tokens
        self.mode = mode
        self.timeout_s = timeout_s
        self.allow_thinking = allow_thinking

    def complete(self, prompt: str, **kw) -> CompletionResponse:
        import requests

        msgs = [{"role": "user", "content": prompt}]
        if self.mode == "ingest":
            msgs.insert(0, {"role": "system", "content": prompts.METADATA_WRITER_SYSTEM})
        base = EngineLLM.WORKER if self.mode == "worker" else EngineLLM.INGEST
        payload = {"model": self.model, "messages": msgs,
                   "max_completion_tokens": kw.get("max_tokens", self.max_tokens),
                   "temperature": kw.get("temperature", base["temperature"]),
                   "top_p": kw.get("top_p", base["top_p"])}
        if self.mode == "worker":
            payload["repetition_penalty"] = kw.get("repetition_penalty", base["repetition_penalty"])
        if not self.allow_thinking:
            payload["chat_template_kwargs"] = {"enable_thinking": False}
        try:
            r = requests.post(f"{self.endpoint}/v1/chat/completions", json=payload, timeout=self.timeout_s)
            r.raise_for_status()
            text = ((r.json().get("choices") or [{}])[0].get("message") or {}).get("content", "") or ""
            if self.mode == "ingest":
                text = sanitize(text) or "No response generated"
            elif is_selector_prompt(prompt):
                text = clean_selector_response(text)
            return CompletionResponse(text)
        except Exception as e:
            return CompletionResponse(f"Error: {e}", True)


class MeteredLLM:
    def __init__(self, base):
        self._base = base
        if hasattr(base, "acomplete"):
            self.acomplete = self._acomplete

    async def _acomplete(self, prompt: str, **kw) -> CompletionResponse:
        from ..service import metrics as M

        t0 = time.perf_counter()
        try:
            out = await self._base.acomplete(prompt, **kw)
        except Exception:
            M.WORKER_LLM_DURATION.observe(time.perf_counter() - t0)
            M.WORKER_LLM_CALLS_TOTAL.labels(result="error").inc()
            raise
        M.WORKER_LLM_DURATION.observe(time.perf_counter() - t0)
        M.WORKER_LLM_CALLS_TOTAL.labels(result="error" if getattr(out, "error", False) else "ok").inc()
        return out

    def complete(self, prompt: str, **kw) -> CompletionResponse:
        from ..service import metrics as M

        t0 = time.perf_counter()
        try:
            out = self._base.complete(prompt, **kw)
        except Exception:
            M.WORKER_LLM_DURATION.observe(time.perf_counter() - t0)
            M.WORKER_LLM_CALLS_TOTAL.labels(result="error").inc()
            raise
        M.WORKER_LLM_DURATION.observe(time.perf_counter() - t0)
        M.WORKER_LLM_CALLS_TOTAL.labels(result="error" if getattr(out, "error", False) else "ok").inc()
        return out

    def __getattr__(self, name):
        return getattr(self._base, name)


class ScriptedLLM:
    """Returns scripted replies: a list (consumed in order, last one repeats),
    a dict of {substring: reply}, or a callable(prompt) -> reply.  A reply that
    is an Exception instance is raised (fault injection)."""

    def __init__(self, script):
        self.script = script
        self.calls: list[str] = []

    def complete(self, prompt: str, on_token=None, **kw) -> CompletionResponse:
        self.calls.append(prompt)
        s = self.script
        if callable(s):
            r = s(prompt)
        elif isinstance(s, dict):
            r = next((v for k, v in s.items() if k in prompt), "")
        else:
            r = s[min(len(self.calls) - 1, len(s) - 1)] if s else ""
        if isinstance(r, BaseException):
            raise r
        if on_token is not None and r:
            for w in r.split(" "):
                on_token(w + " ")
        return CompletionResponse(r)
