"""GraphAgent state machine with scripted LLMs and in-memory retrievers
(reference: rag_worker/src/worker/services/agent_graph.py; tests mirror its
node semantics: plan fallback, judge stage-down, rewrite, expansion,
conservative-answer retry, cancellation, token streaming)."""
import json

import pytest

from githubrepostorag_amd.agent.graph_agent import (Cancelled, GraphAgent, doc_to_source, extract_repo_hint,
                                                    looks_codey, score_of)
from githubrepostorag_amd.agent.llm import ScriptedLLM, clean_selector_response, is_selector_prompt, sanitize
from githubrepostorag_amd.retrieval.graph import Document


class FakeRetriever:
    def __init__(self, docs):
        self.docs = docs
        self.calls = []

    def invoke(self, q, filter=None):
        self.calls.append((q, dict(filter or {})))
        return list(self.docs)


def _doc(i, text="x" * 80, **md):
    return Document(text, {"repo": "payments", "module": "core", "file_path": f"f{i}.py",
                           "_similarity_score": 1.0 - 0.1 * i, **md})


def _retrievers(n=4):
    return {s: FakeRetriever([_doc(i) for i in range(n)]) for s in ("project", "package", "file", "code")}


def _router(plan=None, judge=None, answer="The answer is [1].", expand='["q1", "q2"]', rewrite="a sharper question"):
    def reply(p):
        if p.startswith("Choose the best search scope"):
            return plan if plan is not None else json.dumps({"scope": "package", "filters": {"module": "core"}})
        if "Judge if the retrieved" in p:
            return judge if judge is not None else json.dumps({"coverage": 0.9, "needs_more": False})
        if p.startswith("Generate 3-4"):
            return expand
        if p.startswith("Rewrite this"):
            return rewrite
        return answer
    return reply


def test_happy_path_scope_and_filters():
    rs = _retrievers()
    agent = GraphAgent(ScriptedLLM(_router()), rs, namespace="default")
    out = agent.run("How does the payments service publish events?")
    assert out["scope"] == "package"
    assert out["answer"] == "The answer is [1]."
    assert len(out["sources"]) == 4 and out["sources"][0]["metadata"]["file_name"] == "f0.py"
    q, flt = rs["package"].calls[0]
    assert flt["namespace"] == "default" and flt["module"] == "core"
    stages = [t["stage"] for t in out["debug"]["turns"]]
    assert stages == ["plan", "retrieve", "judge"]


def test_plan_parse_failure_falls_back_on_codey_heuristic():
    agent = GraphAgent(ScriptedLLM(_router(plan="not json")), _retrievers())
    assert agent.run("Why does this method throw a NullPointerException?")["scope"] == "code"
    agent = GraphAgent(ScriptedLLM(_router(plan="garbage")), _retrievers())
    assert agent.run("Give me an overview of the projects")["scope"] == "project"


def test_force_level_and_repo_hint():
    agent = GraphAgent(ScriptedLLM(_router()), _retrievers())
    assert agent.run("anything", force_level="file")["scope"] == "file"
    assert extract_repo_hint("look at repo:billing-api please") in ("billing-api", None)


def test_repo_name_pins_filter_and_top_k_caps_docs():
    """QueryRequest.repo_name / top_k (accepted but ignored by the reference)
    pin the repo filter against the planner's and judge's suggestions and cap
    the retrieved documents."""
    plan = json.dumps({"scope": "code", "filters": {"repo": "other-repo"}})
    judges = iter([json.dumps({"coverage": 0.1, "needs_more": True, "suggest_filters": {"repo": "x"}}),
                   json.dumps({"coverage": 0.9, "needs_more": False})])
    rs = _retrievers(n=6)

    def reply(p):
        return next(judges) if "Judge if the retrieved" in p else _router(plan=plan)(p)

    out = GraphAgent(ScriptedLLM(reply), rs).run("where is the retry loop?", repo="payments", top_k=2)
    assert rs["code"].calls and all(f["repo"] == "payments" for _, f in rs["code"].calls)
    assert len(out["sources"]) == 2


def test_judge_stage_down_and_rewrite_loop():
    judges = iter([json.dumps({"coverage": 0.1, "needs_more": True, "stage_down": "file"}),
                   json.dumps({"coverage": 0.9, "needs_more": False})])

    def reply(p):
        if "Judge if the retrieved" in p:
            return next(judges)
        return _router()(p)

    rs = _retrievers()
    agent = GraphAgent(ScriptedLLM(reply), rs, max_iters=3)
    out = agent.run("where is retry configured?")
    assert out["scope"] == "file"
    stages = [t["stage"] for t in out["debug"]["turns"]]
    assert stages.count("retrieve") == 2 and "rewrite" in stages
    assert rs["file"].calls and rs["file"].calls[0][0] == "a sharper question"


def test_judge_failure_fallback_stages_down_from_project():
    rs = _retrievers()
    agent = GraphAgent(ScriptedLLM(_router(plan='{"scope":"project"}', judge="???")), rs, max_iters=2)
    out = agent.run("overview of the projects")
    turns = out["debug"]["turns"]
    judges = [t["decision"] for t in turns if t["stage"] == "judge"]
    assert [j["stage_down"] for j in judges] == ["package", "file"]  # project -> package -> file
    assert out["scope"] == "file"


def test_expansion_when_few_hits():
    rs = {s: FakeRetriever([_doc(0)]) for s in ("project", "package", "file", "code")}
    seq = {"n": 0}

    class Growing(FakeRetriever):
        def invoke(self, q, filter=None):
            seq["n"] += 1
            return [_doc(seq["n"], text=f"doc {seq['n']} " * 20)]

    rs["package"] = Growing([])
    agent = GraphAgent(ScriptedLLM(_router()), rs, router_top_k=5)
    out = agent.run("how is auth done?")
    assert len(out["sources"]) == 3  # original + 2 expansions
    expansion_turn = out["debug"]["turns"][1]
    assert expansion_turn["original_hits"] == 1 and expansion_turn["hits"] == 3


def test_expansion_parse_failure_uses_keyword_fallback():
    agent = GraphAgent(ScriptedLLM(_router(expand="nope")), {})
    from githubrepostorag_amd.agent.graph_agent import RunContext

    assert agent._expand("cache config for login", {}, RunContext(None, None, None)) == [
        "authentication mechanism", "security configuration", "OAuth2 setup"]


def test_conservative_answer_retry():
    answers = iter(["There is not enough information to say.", "Projects: payments [1]."])

    def reply(p):
        if ("You are a senior" in p or "You are a helpful" in p):
            return next(answers)
        return _router()(p)

    agent = GraphAgent(ScriptedLLM(reply), _retrievers())
    out = agent.run("Tell me about the projects you have")
    assert out["answer"] == "Projects: payments [1]."


def test_cancel_stops_run():
    flag = {"c": False}

    def reply(p):
        if "Judge if the retrieved" in p:
            flag["c"] = True
        return _router()(p)

    agent = GraphAgent(ScriptedLLM(reply), _retrievers())
    with pytest.raises(Cancelled):
        agent.run("q", cancel_check=lambda: flag["c"])


def test_answer_tokens_stream_and_progress():
    toks, prog = [], []
    agent = GraphAgent(ScriptedLLM(_router(answer="alpha beta gamma")), _retrievers())
    agent.run("q", progress_cb=prog.append, on_answer_token=toks.append)
    assert "".join(toks).split() == ["alpha", "beta", "gamma"]
    assert [p["stage"] for p in prog][:2] == ["plan", "retrieve"] and prog[-1]["stage"] == "synthesize"


def test_llm_error_becomes_answer_text():
    def reply(p):
        if ("You are a senior" in p or "You are a helpful" in p):
            raise RuntimeError("boom")
        return _router()(p)

    out = GraphAgent(ScriptedLLM(reply), _retrievers()).run("q")
    assert out["answer"].startswith("(LLM error)")


def test_helpers():
    assert looks_codey("stacktrace in class Foo")
    assert not looks_codey("what projects exist")
    d = _doc(0)
    assert score_of(d) == pytest.approx(1.0)
    s = doc_to_source(1, d)
    assert s["metadata"]["file_path"] == "f0.py" and s["metadata"]["file_name"] == "f0.py" and s["block"] == 1
    assert sanitize("<think>hidden</think>visible") == "visible"
    assert is_selector_prompt("Select one of the following:\nChoice 1: a\nChoice 2: b")
    assert not is_selector_prompt("Choose the best search scope for x")
    assert clean_selector_response('{"choice": 3, "reason": "x"}') == "3"
    assert clean_selector_response("I pick 2 because") == "2"
    assert clean_selector_response("") == "1"


def _arun(agent, q, **kw):
    import asyncio
    import concurrent.futures

    with concurrent.futures.ThreadPoolExecutor(2) as ex:
        return asyncio.run(agent.arun(q, search_executor=ex, **kw))


@pytest.mark.parametrize("judge", [None, json.dumps({"coverage": 0.1, "needs_more": True, "stage_down": "file"})])
def test_async_driver_matches_sync(judge):
    """GraphAgent.arun (coroutine driver: LLM calls awaited or on the executor, searches on the executor)
    walks the same nodes and returns the same result as the thread-per-job ``run``."""
    def make():
        return GraphAgent(ScriptedLLM(_router(judge=judge)), _retrievers(), namespace="default")

    want = make().run("How does the payments service publish events?")
    got = _arun(make(), "How does the payments service publish events?")
    assert got["answer"] == want["answer"] and got["scope"] == want["scope"]
    assert [t["stage"] for t in got["debug"]["turns"]] == [t["stage"] for t in want["debug"]["turns"]]
    assert got["sources"] == want["sources"]


def test_async_driver_llm_errors_and_cancel():
    """Node-level fallbacks see errors raised by awaited calls (thrown back into the node generator), and a
    cancel check stops the coroutine with Cancelled."""
    class ALLM:  # an LLM with acomplete: the plan call fails, the rest answer
        def __init__(self):
            self.calls = 0

        async def acomplete(self, prompt, **kw):
            self.calls += 1
            if prompt.startswith("Choose the best search scope"):
                raise RuntimeError("boom")
            return ScriptedLLM(_router()).complete(prompt, **kw)

    llm = ALLM()
    out = _arun(GraphAgent(llm, _retrievers()), "Why does this method throw a NullPointerException?")
    assert out["scope"] == "code" and out["answer"] == "The answer is [1]." and llm.calls >= 3
    with pytest.raises(Cancelled):
        _arun(GraphAgent(ALLM(), _retrievers()), "q", cancel_check=lambda: True)


def test_shared_context_layout_opt_in():
    """GRAG_AGENT_SHARED_CONTEXT / shared_context=True: synthesize and its retry start with the same context
    blocks (prompts.context_prefix), so the retry reuses the synthesize call's KV; the synthesize call runs
    at SYNTH_PRIORITY (ahead of other jobs' plan / judge prefills)."""
    from githubrepostorag_amd.agent import prompts
    from githubrepostorag_amd.agent.graph_agent import SYNTH_PRIORITY

    seen = []

    class Rec(ScriptedLLM):
        def complete(self, prompt, **kw):
            seen.append((prompt, kw.get("priority")))
            return super().complete(prompt, **kw)

    rs = _retrievers(5)
    agent = GraphAgent(Rec(_router(answer="there is insufficient context")), rs, shared_context=True)
    agent.run("How does the payments service publish events?")
    synth = [(p, pr) for p, pr in seen if "You are a senior" in p or "You are a helpful" in p]
    assert len(synth) == 2 and all(pr == SYNTH_PRIORITY for _, pr in synth)
    pre = synth[0][0][: synth[0][0].index("You are")]
    assert pre.startswith("Context:\n[1] repo=payments") and synth[1][0].startswith(pre)
    assert prompts.context_prefix(["a", "b"]) == "Context:\na\n\nb\n\n"
