"""API contracts (rag_shared/models.py:6-14)."""
from __future__ import annotations

from typing import Any, Optional

from pydantic import BaseModel, Field


class QueryRequest(BaseModel):
    query: str
    top_k: Optional[int] = 5
    repo_name: Optional[str] = None
    # accepted by the reference worker (worker.py:106-107) but never sent by its API
    force_level: Optional[str] = None
    namespace: Optional[str] = None


class RAGResponse(BaseModel):
    answer: str
    sources: Optional[list[dict[str, Any]]] = None


class ChatMessage(BaseModel):
    role: str
    content: str


class ChatCompletionRequest(BaseModel):
    """OpenAI /v1/chat/completions body as the reference clients send it
    (qwen_llm.py:107-113, llm_init.py:108-120)."""

    model: Optional[str] = None
    messages: list[ChatMessage]
    max_tokens: Optional[int] = None
    max_completion_tokens: Optional[int] = None
    temperature: Optional[float] = 0.7
    top_p: Optional[float] = 1.0
    top_k: Optional[int] = 0
    repetition_penalty: Optional[float] = 1.0
    stop: Optional[list[str] | str] = None
    stream: Optional[bool] = False
    seed: Optional[int] = None
    chat_template_kwargs: Optional[dict[str, Any]] = Field(default=None)


class CompletionRequest(BaseModel):
    model: Optional[str] = None
    prompt: str
    max_tokens: Optional[int] = 256
    temperature: Optional[float] = 0.7
    top_p: Optional[float] = 1.0
    stop: Optional[list[str] | str] = None


class EmbeddingRequest(BaseModel):
    model: Optional[str] = None
    input: list[str] | str
