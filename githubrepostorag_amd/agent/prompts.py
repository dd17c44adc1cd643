"""Prompt inventory.  The wording follows the reference's
prompts so a real Qwen checkpoint behaves the same way; each builder cites
the reference location it mirrors."""
from __future__ import annotations

import json

SCOPE_EXAMPLE = '{"scope":"package","filters":{"repo":"payments","module":"messaging","topics":"activemq"}}'


def plan_scope(question: str) -> str:
    # rag_worker/src/worker/services/agent_graph.py:207-212
    sys = ("Choose the best search scope for a codebase question. "
           "Return JSON: {scope: project|package|file|code, filters?:{repo?,module?,topics?}}")
    return f"{sys}\nQuestion: {question}\nExample: {SCOPE_EXAMPLE}\nJSON:"


def expand_query(question: str, repo: str | None, scope: str | None) -> str:
    # agent_graph.py:108-125
    sys = ("Generate 3-4 semantically related search queries for a codebase question. "
           "Focus on technical synonyms, related concepts, and different ways to express the same need. "
           'Return JSON array of strings: ["query1", "query2", "query3"]')
    ctx = ""
    if repo:
        ctx += f" Repository: {repo}"
    if scope:
        ctx += f" Scope: {scope}"
    return (f"{sys}\n\nOriginal question: {question}{ctx}\n\n"
            "Examples for 'authentication cache':\n"
            '["OAuth2 configuration caching", "security settings cache mechanism", '
            '"Spring Security cache authentication", "authentication token caching"]\n\n'
            "JSON array:")


JUDGE_RUBRIC = ("Judge if the retrieved content is semantically relevant and sufficient to answer the question. "
                "Consider both metadata relevance AND content preview relevance. Return JSON: "
                "{coverage:0..1, needs_more:boolean, suggest_filters?:{repo?,module?,topics?}, "
                "stage_down?: 'package'|'file'|'code'|null, rewrite?:string, semantic_match:boolean}")


def context_prefix(blocks: list[str]) -> str:
    """The job's retrieved documents as one text block that the judge, synthesize and synthesize-retry
    prompts all START with, so the engine's prefix cache computes their KV once per retrieval and the later
    calls prefill only their own instruction + question (shared prefixes)."""
    return "Context:\n" + "\n\n".join(blocks) + "\n\n"


def judge(question: str, context_quality: str, inventory: list[dict], blocks: list[str] | None = None) -> str:
    # agent_graph.py:325-341 (same rubric and fields).  With ``blocks`` the top documents lead the prompt as
    # the shared context prefix (their inventory entries then point at their block instead of repeating a
    # preview of the same text)
    body = (f"{JUDGE_RUBRIC}\n\nQuestion: {question}\nContext quality: {context_quality}\n"
            f"Retrieved items: {json.dumps(inventory, ensure_ascii=False)}\nJSON:")
    return context_prefix(blocks) + body if blocks else body


def rewrite(base_query: str, context: str) -> str:
    # agent_graph.py:417-421
    extra = f" Context: {context}" if context else ""
    return (f"Rewrite this codebase question to be more specific and searchable: '{base_query}'{extra}"
            "\nReturn only the rewritten question, no explanation:")


SYNTH_OVERVIEW = ("You are a senior developer assistant. Use the provided context blocks to give a comprehensive "
                  "answer. Cite sources as [1], [2], etc. Synthesize information across blocks when relevant. "
                  "If the question asks for an overview of available projects/repositories, describe what you see "
                  "in the context.")
SYNTH_SPECIFIC = ("You are a senior developer assistant. Answer using the provided context blocks. "
                  "Cite blocks as [1], [2]. If the specific information needed is not in the context, "
                  "say so clearly and suggest looking in specific repos/modules that might contain the answer.")
SYNTH_RETRY = ("You are a helpful developer assistant. The user is asking about available projects. "
               "Use the context provided to describe the projects you can see. Don't be overly conservative - "
               "if you have project descriptions, share them! Cite sources as [1], [2].")


def synthesize(system: str, question: str, blocks: list[str], shared_prefix: bool = False) -> str:
    # agent_graph.py:467-476 / 485-488: the same system text, question, numbered context blocks and answer
    # cue; the context blocks come first (context_prefix) so this call reuses the judge's KV of them and the
    # retry reuses this one's.  shared_prefix=False: the reference's order (system, question, context)
    if not shared_prefix:
        return f"{system}\n\nQuestion: {question}\n\nContext:\n" + "\n\n".join(blocks) + "\n\nAnswer:"
    return context_prefix(blocks) + f"{system}\n\nQuestion: {question}\n\nAnswer:"


# ---- ingest prompts -------------------------------------------------------
METADATA_WRITER_SYSTEM = (  # ingest/src/app/llm_init.py:27-33
    "You are a metadata writer for an indexing pipeline. "
    "Return ONLY the final answer requested by the prompt. "
    "Do not include internal reasoning, prefaces, apologies, or meta-commentary. "
    "No headings, no role tags. Output just the final text.")


def summary_extract(context: str) -> str:
    # LlamaIndex SummaryExtractor default template
    return f"Here is the content of the section:\n{context}\n\nSummarize the key topics and entities of the section. \nSummary: "


def keyword_extract(context: str, n: int = 10) -> str:
    # LlamaIndex KeywordExtractor default template
    return f"{context}. Give {n} unique keywords for this document. Format as comma separated. Keywords: "


def title_candidate(context: str) -> str:
    # LlamaIndex TitleExtractor node template
    return (f"Context: {context}. Give a title that summarizes all of the unique entities, titles or themes "
            "found in the context. Title: ")


def title_combine(candidates: list[str]) -> str:
    # LlamaIndex TitleExtractor combine template
    return (f"{', '.join(candidates)}. Based on the above candidate titles and content, what is the comprehensive "
            "title for this document? Title: ")


def readme_quality(readme: str) -> str:
    # ingest/src/app/catalog/catalog_builder.py:13-22
    return ("\nEvaluate if this README provides useful information for understanding what this software project does.\n"
            "A good README should explain the purpose, functionality, or architecture of the project.\n"
            "A bad README contains only stubs, todos, boilerplate, or very minimal information.\n\n"
            f"README content:\n{readme[:1000]}...\n\n"
            'Respond with only "GOOD" if the README is useful for understanding the project, or "BAD" if it\'s just '
            "a stub/placeholder or does not provide enough information.\n")


def catalog_from_summaries(repo: str, tech: str, summaries: str) -> str:
    # catalog_builder.py:165-187
    return ("\nBased on these code-level summaries, create a comprehensive project catalog entry that explains:\n\n"
            "1. **Purpose & Functionality**: What this software component does\n"
            "2. **Architecture & Design**: Key architectural patterns and components\n"
            "3. **Technology Stack**: Technologies and frameworks used\n"
            "4. **Integration Points**: How it connects to other services/systems\n"
            "5. **Key Features**: Main capabilities and functionality\n\n"
            f"Repository: {repo}\nDetected Technologies: {tech}\n\nCode Summaries:\n{summaries}\n\n"
            "Create a clear, structured catalog entry in markdown format that would help an AI agent understand:\n"
            "- What this component is responsible for\n- How it fits into a larger system architecture\n"
            "- What other components might need to be updated when this changes\n- Key entry points and interfaces\n\n"
            "Focus on architectural understanding rather than implementation details.\n")


def file_summary(path: str) -> str:
    # hierarchy_summary_service.py:32-37
    return ("You are creating a high-level FILE SUMMARY for developers and retrieval.\n"
            f"Path: {path}\n"
            "Summarize responsibilities, main APIs/entry points, external dependencies, and debugging gotchas.\n"
            "Avoid boilerplate; keep it under ~200–300 words.")


def file_summary_prompt(path: str, content: str) -> str:
    """The FILE SUMMARY roll-up call (hierarchy_summary_service.py:32-38: instruction + "\n\n" + the file's
    chunks) with the same instruction and content, the content FIRST and in the extractors' section form:
    a single-chunk file's prompt then starts with exactly the token prefix of that chunk's summary / title
    / keyword prompts (``summary_extract``), so the engine's prefix cache computes the file text once for
    all four calls (content first so ingest prompts share a KV prefix)."""
    return f"Here is the content of the section:\n{content}\n\n{file_summary(path)}"


def module_summary(module: str, repo: str) -> str:
    # hierarchy_summary_service.py:112-116
    return (f"MODULE SUMMARY for '{module}' in repo {repo}.\n"
            "Aggregate responsibilities, key subcomponents, boundaries, external integrations, and ops pitfalls.\n"
            "Produce a concise overview appropriate for routing debugging and how-to questions.")


def repo_overview(repo: str) -> str:
    # hierarchy_summary_service.py:172-176
    return (f"REPO OVERVIEW for {repo}:\n"
            "Provide purpose, primary services/modules, tech stack, data stores/queues, deployment/runtime, "
            "and the most common user asks. Be concise and actionable.")
