#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): RAG queries/sec + p50 TTFT with
Qwen2-7B over a 10M-vector index, plus ingest docs/sec.

Config (BASELINE config 3): Qwen2-7B TP=1 per GPU + bge-large-en-v1.5 encoder,
10M x 1024-d IVF index sharded data-parallel over the N GPUs, per-shard top-k
merged with one RCCL all-gather over xGMI.  Weights are random-init of the
real architectures; data is synthetic (no network): clustered unit vectors for
the index, generated code/prose chunk texts addressed by row id, generated
questions.

One timed step = one batch of B RAG queries per GPU, end to end:
  encode questions (bge-large, HIP encoder) -> sharded IVF search
  (fused score+top-k kernels + all-gather merge) -> prompt from the top-5
  blocks (reference synthesize(), agent_graph.py:448-476) -> Qwen2-7B
  prefill + decode of gen_len tokens with the reference worker's sampling
  (temperature 0.4, top_p 0.8, repetition_penalty 1.2; qwen_llm.py:107-113).
The server runs at saturation with a continuous arrival stream: queries
arrive in groups of u = B/A (`--arrival-groups` A), and U = D*A groups are in
flight at once (`--inflight` D batches' worth), staggered by gen_len/U
generated tokens (a fill phase before the warmup sets this up).  One step =
A times {a group of u queries arrives (embed + search + prompt) and is handed
to the engine; the engine runs until the OLDEST in-flight group has all
gen_len tokens}.  Exactly B queries complete per step and every timed step
does the same work (B queries' retrieval + prefill, gen_len/U decode tokens
per in-flight group per sub-step).  The engine prefills new arrivals first
(chunked prefill), then decodes all live sequences in one batch (decode is
weight-bandwidth bound, so D*B rows cost little more than B).
--inflight 1 --arrival-groups 1 is the closed-batch mode (submit B, finish B).
Scaling is weak (B queries per GPU fixed).  `value` = total queries/s over
all ranks (B * N / max-over-ranks step time).  p50 TTFT = submission -> first
generated token per query (over the queries completed in the timed steps).  The ingest phase (split -> LLM summary+keywords ->
embed -> index upsert over a synthetic repo) runs after the timed steps and is
reported separately as ingest_docs_per_s.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import statistics
import sys
import time


# BASELINE.json configs as flag presets (explicit flags still win: the preset only fills defaults).
#   c1  plumbing floor, no GPU: tiny synthetic corpus, MiniLM-L6 encoder on CPU, brute-force (flat) cosine,
#       GPT-2-small greedy answers (reference default encoder: rag_shared/config.py:24)
#   c2  Qwen2-1.5B + bge-base, 1M-vector brute-force cosine-GEMM index, one MI355X bf16
#   c3  Qwen2-7B TP=1 + bge-large, 10M-vector IVF sharded DP=N (the headline; the flag defaults)
#   c4  Qwen2-72B TP=8 + 100M-vector index, concurrent ingest + query (needs the 8-GPU node)
#   c5  3-round refinement loop on Qwen2-7B: the agent phase is the measured workload (jobs/s, SSE TTFT)
PRESETS = {
    "c1": dict(model="gpt2", encoder="all-minilm-l6-v2", index_kind="flat", index_size=20_000, batch=8,
               prompt_len=256, gen_len=32, inflight=2, arrival_groups=2, greedy=1, cpu=1, ingest_files=8,
               ingest_ref_cap_files=0, ingest_seqs=16, agent_jobs=16, agent_concurrency=4, agent_synth_len=32,
               agent_gen_len=16, steps=2, warmup=1),
    "c2": dict(model="qwen2-1.5b", encoder="bge-base-en-v1.5", index_kind="flat", index_size=1_000_000),
    "c3": dict(),
    "c4": dict(model="qwen2-72b", tp=8, index_size=100_000_000, nlist=16384, nprobe=64),
    "c5": dict(agent_jobs=512, agent_concurrency=256, agent_synth_len=256),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default=None, choices=sorted(PRESETS),
                    help="a BASELINE.json config (c1..c5, see PRESETS); explicit flags override its values")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="qwen2-7b")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree of the decoder (BASELINE config 4: qwen2-72b --tp 8); "
                         "TP peers serve the same queries in lockstep, DP = world / tp")
    ap.add_argument("--encoder", default="bge-large-en-v1.5")
    ap.add_argument("--index-size", type=int, default=10_000_000)
    ap.add_argument("--index-kind", default="ivf", choices=["ivf", "flat"])
    ap.add_argument("--nlist", type=int, default=4096)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--batch", type=int, default=64, help="queries per GPU per step")
    ap.add_argument("--inflight", type=int, default=16,
                    help="batches' worth of queries in flight (1 = closed batch).  Default 16 = 1024 live sequences; "
                         "same-box sweep (profiles/sweep_inflight_r3b.txt): D 8 -> 69.0-69.3, 12 -> 71.4-71.9, "
                         "16 -> 71.9-72.4 queries/s at the same p50 TTFT (86-87 ms)")
    ap.add_argument("--arrival-groups", type=int, default=8, help="queries of a step arrive in this many groups")
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--top-k", type=int, default=10)
    ap.add_argument("--ingest-files", type=int, default=192, help="source files in the synthetic repo to ingest")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--ingest-ref-cap-files", type=int, default=32,
                    help="second ingest pass at the reference's one 2048-token cap for every LLM call "
                         "(ingest/src/app/llm_init.py:56) over this many files: ingest_docs_per_s_ref_cap (0: skip)")
    ap.add_argument("--ingest-ref-cap", type=int, default=2048, help="the cap of that pass (tests shrink it)")
    ap.add_argument("--ingest-seqs", type=int, default=256, help="concurrent sequences of the ingest engine")
    ap.add_argument("--ingest-multi", default="auto",
                    help="RxF: R synthetic repos of F files through ingest_many, all at once on one engine "
                         "(auto: 8x48 on a GPU, 2x2 on the host; 0: skip)")
    ap.add_argument("--ingest-mixed", type=int, default=0,
                    help="1: the ingest engine piggybacks decode tokens on prefill steps (mixed batches)")
    ap.add_argument("--mixed", type=int, default=0,
                    help="1: stall-free batching in the serving engine: every prefill step also carries one decode "
                         "token of every decode-ready sequence (decode rows run in the prefill GEMMs)")
    ap.add_argument("--max-batched-tokens", type=int, default=16384,
                    help="prefill token budget per engine step (smaller: arrivals prefilled in chunks over "
                         "several mixed steps)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--switch-interval", type=float, default=0.0005,
                    help="Python GIL switch interval (s; 0 keeps Python's 5 ms): the engine thread re-takes the GIL "
                         "quickly when the retrieval prefetch thread runs Python.  Same-box A/B, 2 rounds: 5 ms "
                         "71.8 / 69.8, 0.5 ms 72.0 / 73.3, 2 ms 68.5 / 73.4 queries/s (profiles/ab_switch_r3.txt)")
    ap.add_argument("--prefetch", type=int, default=1,
                    help="1: the next group's retrieval overlaps engine steps on a helper thread")
    ap.add_argument("--agent-jobs", type=int, default=256,
                    help="end-to-end phase: agent-loop jobs through POST /rag/jobs + SSE over real HTTP "
                         "(0 disables); secondary fields e2e_ttft_p50_ms / p90 / agent_jobs_per_s")
    ap.add_argument("--agent-concurrency", type=int, default=64)
    ap.add_argument("--agent-slots", type=int, default=256,
                    help="jobs a replica runs at once (WORKER_MAX_JOBS); offered concurrency above it waits in "
                         "the front door's FIFO queue (profiles/agent_saturation_r4.json: one thread per running "
                         "job, throughput collapses past ~256 on one GPU: 11.6 -> 8.4 -> 3.1 jobs/s at 256 / 512 "
                         "/ 1024 running jobs)")
    ap.add_argument("--agent-gen-len", type=int, default=32,
                    help="token cap of the agent's plan / expand / judge / rewrite calls (JSON or one line)")
    ap.add_argument("--agent-synth-len", type=int, default=256, help="token cap of the agent's synthesize call")
    ap.add_argument("--quant", default="none", choices=["none", "w4"],
                    help="w4: AWQ-format W4A16 decoder weights (group-128 scales + zero points, the reference's "
                         "precision: helm/values.yaml:67) on the decode GEMMs; reported as its own config line")
    ap.add_argument("--gc-freeze", type=int, default=1,
                    help="1: gc.freeze() the setup objects before the timed steps (serving does the same at startup)")
    ap.add_argument("--pysample", type=float, default=0.0,
                    help="ms between stack samples of the engine thread over the timed steps (0: off; diagnostics)")
    ap.add_argument("--arrival-cap", type=int, default=1,
                    help="1: the harness caps the decode window to one step while an arrival's retrieval is in "
                         "flight (an admission policy of this bench loop; the serving runner paces its windows by the "
                         "arrival rate instead, GRAG_ARRIVAL_WINDOW=auto).  Reported as ttft_admission_policy")
    ap.add_argument("--greedy", type=int, default=0,
                    help="1: greedy answers (temperature 0; BASELINE config 1) instead of the reference worker's "
                         "temperature 0.4 / top_p 0.8 / repetition_penalty 1.2")
    ap.add_argument("--cpu", type=int, default=0, help="1: run on the host even if a GPU is visible (config 1)")
    ap.add_argument("--kv-cache-gb", type=float, default=None,
                    help="KV pool of the serving engine in GiB (default: half the free HBM); several ranks "
                         "sharing one GPU (a rehearsal) split the card with it")
    ap.add_argument("--ingest-kv-gb", type=float, default=None, help="KV pool of the ingest engine in GiB")
    ap.add_argument("--agent-sweep", default="",
                    help="comma list of agent concurrencies (per GPU) to sweep after the agent phase: "
                         "agent_saturation in the JSON (jobs/s and SSE first-token p50 at each)")
    ap.add_argument("--serving-steps", type=int, default=-1,
                    help="timed steps of the same workload through the SERVING loop (engine/runner.py "
                         "EngineRunner thread, arrivals submitted from the retrieval thread under the runner's "
                         "admission hint): serving_runner in the JSON.  -1: --steps; 0: skip")
    ap.add_argument("--interactive-prefill", type=int, default=4096,
                    help="serving loop: prefill tokens per engine step while interactive arrivals are pending "
                         "(EngineRunner interactive_prefill; 0: the engine's --max-batched-tokens)")
    ap.add_argument("--serving-open-load", default="0.5,0.9",
                    help="after the closed loop: open-loop Poisson arrivals of query groups at these fractions of "
                         "the closed loop's throughput through the same serving loop (serving_runner.open_loop: "
                         "TTFT p50 / p90 at each load; empty: skip)")
    ap.add_argument("--bulk-prefill", type=int, default=512,
                    help="of --interactive-prefill, the prefill tokens per step bulk work (ingest) may take while "
                         "interactive arrivals keep coming (EngineRunner bulk_prefill; 0: no separate cap)")
    ap.add_argument("--heartbeat", type=float, default=0.0,
                    help="seconds between rank 0's progress lines (engine step counters); 0: none")
    ap.add_argument("--low-load", type=int, default=1,
                    help="1: the reference's own regime (vLLM --max-num-seqs 4 --max-model-len 11712): single-prompt "
                         "TTFT at 1K / 4K / 11.6K tokens, decode TPOT at 1 / 4 / 16 live sequences x those contexts "
                         "(engine/probe.py), and agent jobs at concurrency 1 and 4: low_load in the JSON")
    ap.add_argument("--concurrent-ingest", type=int, default=1,
                    help="1: after the ingest phase, ingest the synthetic repo again on ONE engine that also serves "
                         "open-loop query arrivals at 50 %% of the serving loop's rate (BASELINE config 4's concurrent "
                         "ingest + query streams on one server): concurrent_ingest in the JSON")
    ap.add_argument("--recall-queries", type=int, default=64,
                    help="queries per rank for recall@top-k of the IVF search vs an exact scan of every shard "
                         "(index_recall; 0: skip)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.preset:
        explicit = {a.split("=", 1)[0].lstrip("-").replace("-", "_") for a in sys.argv[1:] if a.startswith("--")}
        for k, v in PRESETS[args.preset].items():
            if k not in explicit:
                setattr(args, k, v)
    return args


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start N rank processes
    of this same script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* in their env), forward rank 0's stdout, wait for all of them and
    return the worst exit status.  This parent imports nothing that touches
    the GPU (no torch) and never execs: the ranks are children.  If one rank
    fails the others are terminated (by pid) so the job cannot hang."""
    import signal
    import subprocess

    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port,
                   GRAG_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in live:  # a failed rank leaves its peers blocked in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.switch_interval > 0:
        sys.setswitchinterval(args.switch_interval)
    if os.environ.get("GRAG_DUMP_STACKS_AFTER"):  # debugging a stuck rank: every thread's stack, once
        import faulthandler

        # every N seconds (GRAG_DUMP_STACKS_REPEAT=1) or once
        faulthandler.dump_traceback_later(float(os.environ["GRAG_DUMP_STACKS_AFTER"]), exit=False,
                                          repeat=os.environ.get("GRAG_DUMP_STACKS_REPEAT") == "1")
    if args.cpu:  # before torch initialises HIP: this process never touches a GPU
        os.environ["HIP_VISIBLE_DEVICES"] = ""
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
    import torch

    from githubrepostorag_amd.parallel import comm

    info = comm.init_distributed()
    rank, world = info.rank, info.world_size
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = torch.device("cuda", info.local_rank) if torch.cuda.is_available() else torch.device("cpu")
    group = comm.world_group()
    tp = max(1, args.tp)
    tp_group = dp_group = None
    dp_rank, dp_size = rank, world
    if tp > 1:
        # TP groups of consecutive ranks; every rank of a group runs the same
        # arrivals (seeded by its DP rank) and steps its shard of the engine in
        # lockstep (deterministic scheduler + identical sampling seeds).  An
        # arrival is admitted at the same engine step on every TP rank: its
        # "retrieval done" flag is agreed over the TP group (MIN) each step.
        from githubrepostorag_amd.parallel.custom_ar import enable_for_group

        tp_group, dp_group = comm.make_tp_dp_groups(tp)
        if dev.type == "cuda":
            enable_for_group(tp_group, dev)
        dp_rank, dp_size = rank // tp, world // tp
    if world > 1:
        # the index (C6 k-means, C4 query all-gather, C3 top-k all-to-all) on a communicator of its
        # own: the prefetch thread's search collectives then never share one with the engine's
        # TP all-reduces or the main thread's barriers
        import torch.distributed as dist

        group = comm.Group(list(range(world)), pg=dist.new_group(list(range(world))))

    from githubrepostorag_amd.embed.service import Embedder
    from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.engine.tokenizer import load_tokenizer
    from githubrepostorag_amd.index.sharded import ShardedIndex
    from githubrepostorag_amd.models import build_decoder
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.utils import synthetic

    def log(*a):
        if rank == 0:
            print("[bench]", *a, file=sys.stderr, flush=True)

    t_setup = time.perf_counter()
    dcfg = decoder_config(args.model)
    model = build_decoder(dcfg, device=dev, seed=1, tp=tp_group,  # Qwen2 or GPT-2 by the config's arch
                          **({} if dev.type == "cuda" else {"dtype": torch.float32}))
    if args.quant == "w4" and not hasattr(model, "quantize_w4"):
        raise SystemExit(f"--quant w4 needs a Qwen2 decoder, not {dcfg.arch}")
    w4_bytes = model.quantize_w4() if args.quant == "w4" else 0
    if w4_bytes:
        log(f"W4A16 decode weights: {w4_bytes / 1e9:.2f} GB packed (+ bf16 copy of the same values for prefill)")
    tok = load_tokenizer(None, dcfg.vocab_size)
    emb = Embedder.from_name(args.encoder, device=dev, seed=2)
    log(f"models ready {time.perf_counter() - t_setup:.1f}s  decoder={model.param_bytes() / 1e9:.1f} GB")

    # ---- index shard: N / world rows of d-dim clustered vectors
    n_local = args.index_size // world + (1 if rank < args.index_size % world else 0)
    t0 = time.perf_counter()
    # one corpus: the same cluster centres on every shard, each rank's own draws around them
    X = synthetic.clustered_vectors(n_local, emb.dim, seed=1000 + rank, device=dev, center_seed=1000)
    # the product table (index/store.py) per shard: IVF lists + metadata filter columns; the
    # corpus rows (row id, chunk text, repo/module/file metadata) are a deterministic recipe
    corpus = synthetic.SyntheticCorpus(args.index_size, seed=7)
    index = ShardedIndex(emb.dim, group, dev, kind=args.index_kind, nlist=args.nlist, nprobe=args.nprobe)
    index.build_corpus(corpus, X, seed=7)
    del X
    torch.cuda.synchronize() if dev.type == "cuda" else None
    log(f"index shard ready: {n_local} rows ({args.index_kind}) in {time.perf_counter() - t0:.1f}s")

    max_len = args.prompt_len + args.gen_len + 64
    if args.agent_jobs > 0:  # the agent phase's synthesize prompts carry 5 context blocks
        max_len = max(max_len, 4096)
    max_len = min(max_len, dcfg.max_position)  # GPT-2: 1024 positions
    D = max(1, min(args.inflight, args.gen_len))
    A = max(1, min(args.arrival_groups, args.batch, max(1, args.gen_len // D)))
    while args.batch % A:
        A -= 1
    U = D * A  # groups in flight
    u = args.batch // A  # queries per group
    live = max(args.batch * D, 8)
    gsizes = EngineConfig.graph_batch_sizes
    if live > max(gsizes):  # deeper pipelines: decode graphs up to the live-sequence count, 128-row buckets
        gsizes = tuple(sorted({*gsizes, *range(max(gsizes) + 128, live + 127, 128)}))
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=live, max_num_batched_tokens=args.max_batched_tokens,
                                             mixed_batches=bool(args.mixed), kv_cache_gb=args.kv_cache_gb,
                                             max_model_len=max_len, use_cuda_graph=not args.no_graph,
                                             seed=dp_rank, graph_batch_sizes=gsizes))
    if args.heartbeat > 0 and rank == 0:
        import threading

        # a line every --heartbeat seconds from rank 0 (engine step counters): long multi-rank rehearsals
        # (Qwen2-72B at TP=8 over gloo on one card) show progress between phase lines
        import weakref

        eng_ref = weakref.ref(eng)  # the phases free the serving engine later (del eng): no strong reference here

        def _beat():
            t_hb = time.perf_counter()
            while True:
                time.sleep(args.heartbeat)
                e = eng_ref()
                if e is None:
                    return
                st = dict(e.stats)
                del e
                print(f"[bench] alive {time.perf_counter() - t_hb:.0f} s: engine steps {st['steps']}, prefill "
                      f"tokens {st['prefill_tokens']}, decode tokens {st['decode_tokens']}", file=sys.stderr, flush=True)
        threading.Thread(target=_beat, name="bench-heartbeat", daemon=True).start()
    sp = (SamplingParams(max_tokens=args.gen_len, temperature=0.0, ignore_eos=True) if args.greedy else
          SamplingParams(max_tokens=args.gen_len, temperature=0.4, top_p=0.8, repetition_penalty=1.2,
                         ignore_eos=True))
    sys_prompt = ("You are a senior developer assistant. Answer using the provided context blocks. "
                  "Cite blocks as [1], [2]. If the specific information needed is not in the context, "
                  "say so clearly and suggest looking in specific repos/modules that might contain the answer.")

    # row texts: the index's body_blob column (the reference stores chunk text
    # next to the vector, vector_write_service.py:166-198) — the corpus rows of a
    # pool generated once here, so the timed loop does a lookup, not text generation
    text_pool = [corpus.text(i) for i in range(4096)]

    def row_block(d: int) -> tuple[str, dict]:
        return text_pool[d % len(text_pool)], corpus.meta(d)

    qcounter = [dp_rank * 1_000_000]
    phase = {"embed": 0.0, "search": 0.0, "prompt": 0.0, "generate": 0.0}

    # The engine is stepped from this thread between arrivals: a thread per
    # engine (engine/runner.py, as in the service) measured slower here
    # (prefill fragmented by per-request hand-off, shorter decode windows).
    inflight = collections.deque()  # groups, oldest first: (request ids, submission time)

    from concurrent.futures import ThreadPoolExecutor

    from githubrepostorag_amd.utils.gpu_guard import gpu_shared, side_stream

    # the end of every prompt (answer cue + assistant turn), kept when the context is cut to --prompt-len
    tail_ids = tok.encode(tok.apply_chat_template([{"role": "user", "content": "\n\nAnswer:"}])
                          .split("\n\nAnswer:", 1)[1])
    tail_ids = tok.encode("\n\nAnswer:") + tail_ids

    def prepare(B: int | None = None):
        """Retrieve + build prompts for the next group of B (default u) RAG queries (the
        group's arrival time is when its retrieval starts).  B = 0 (a DP rank with no arrivals in a
        lockstep retrieval round of the serving loop) still joins the sharded search's collectives."""
        B = u if B is None else B
        with side_stream(dev):  # off the engine's stream: the .cpu() waits only for the search
            t_sub = time.perf_counter()
            qs = [synthetic.question(qcounter[0] + i) for i in range(B)]
            qcounter[0] += B
            qv = emb.embed_queries(qs) if B else torch.zeros(0, emb.dim, dtype=torch.bfloat16, device=dev)
            t_e = time.perf_counter()
            # every reference retrieval carries the namespace filter (agent_graph.py:249): fused in the scan
            with gpu_shared():  # the .cpu() is a host sync: never inside another thread's graph capture
                scores, ids = index.search(qv, args.top_k, {"namespace": corpus.namespace})
                ids = ids.cpu().tolist()
            t_s = time.perf_counter()
        prompts = []
        for q, row in zip(qs, ids):
            blocks = []
            for j, d in enumerate([x for x in row if x >= 0][:5]):
                text, md = row_block(d)
                blocks.append(f"[{j + 1}] repo={md['repo']} module={md['module']} file={md['file_path']}\n{text}")
            text = tok.apply_chat_template([{"role": "user", "content": f"{sys_prompt}\n\nQuestion: {q}\n\n"
                                             "Context:\n" + "\n\n".join(blocks) + "\n\nAnswer:"}])
            pid = tok.encode(text)
            if len(pid) < args.prompt_len:  # pad short prompts by repeating the context
                pid = (pid * (args.prompt_len // max(1, len(pid)) + 1))[: args.prompt_len]
            else:  # keep system + question + the leading context, cut the rest, keep the answer cue
                pid = pid[: args.prompt_len - len(tail_ids)] + tail_ids
            prompts.append(pid)
        t_p = time.perf_counter()
        return prompts, t_sub, (("embed", t_e - t_sub), ("search", t_s - t_e), ("prompt", t_p - t_s))

    # --prefetch: a new group's retrieval (embed + search + prompt) runs on a
    # helper thread (side stream) while this thread keeps stepping the engine;
    # the group is admitted at the first engine step after its prompts are
    # ready, as a continuous-batching server admits arrivals.  Only one thread
    # issues collectives at a time: every arrival is admitted (its future
    # joined) before the sub-step ends, so barriers never overlap a search.
    pool = ThreadPoolExecutor(1, thread_name_prefix="prefetch") if args.prefetch else None

    def admit(nxt):
        t0 = time.perf_counter()
        prompts, t_sub, ph = nxt
        inflight.append(([eng.add_request(p, sp) for p in prompts], t_sub))
        phase["admit"] = phase.get("admit", 0.0) + time.perf_counter() - t0
        for k, v in ph:
            phase[k] += v

    def submit():
        """A new group of u RAG queries arrives; retrieve + prompt it, hand it to the engine."""
        admit(prepare())

    def run_until(rids, ntok, arrival=None):
        """Step the engine until every request in ``rids`` has ``ntok`` tokens
        (decode windows capped so no sequence runs past that target),
        admitting the ``arrival`` future's group as soon as it is ready."""
        t0 = time.perf_counter()

        def ready(fut):  # TP: every rank of the group admits the arrival at the same engine step
            if tp_group is None or tp_group.trivial:
                return fut.done()
            return bool(tp_group.min_int(1 if fut.done() else 0, dev))

        while True:
            have = min(len(eng.get(r).output_ids) for r in rids)
            if have >= ntok:
                # stall-free batching: the sub-step also finishes its arrivals' prefill (chunks ride with one
                # decode token of every live sequence), so every sub-step does one group's prefill work
                if not (args.mixed and (arrival is not None or eng.has_pending_prefill())):
                    break
            cap = max(1, ntok - have)
            arrived = arrival is not None and ready(arrival)
            if arrival is not None and not arrived and args.arrival_cap:
                # an arrival's retrieval is in flight: one decode step per replay, so the engine looks
                # for its prompts every ~step instead of every window (TTFT no longer depends on
                # whether retrieval beats a multi-step window)
                cap = 1
            if arrived:
                admit(arrival.result())
                arrival = None
            eng.step(max_window=cap)
        if arrival is not None:
            admit(arrival.result())
        phase["generate"] += time.perf_counter() - t0

    def run_step():
        """A groups arrive, the A oldest complete; returns the completed queries' TTFTs (s)."""
        ttft = []
        for _ in range(A):
            arrival = None
            if pool is not None and inflight:
                arrival = pool.submit(prepare)
            else:
                submit()
            rids, t_sub = inflight.popleft()
            run_until(rids, args.gen_len, arrival)
            for r in rids:
                s = eng.pop(r)
                ttft.append(s.first_token_time - t_sub)
                assert len(s.output_ids) == args.gen_len, (len(s.output_ids), s.finish_reason)
        return ttft

    # pipeline fill: U-1 groups staggered by s = (gen_len - 1) / U decode tokens (rounded
    # cumulatively).  Steady state: a group gets its first token from prefill and s decode tokens in
    # each of the U sub-steps it is in flight (its arrival's included), 1 + U s = gen_len; so before
    # a sub-step the in-flight ages are 1 + s j, j = 1..U-1.  Each fill round decodes s tokens for
    # every group: the newest (1 token after its prefill) is run to 1 + s.  Every timed step then
    # decodes about B (gen_len - 1) tokens (reported as steady_state_decode_ratio ~ 1.0).
    S = (args.gen_len - 1) / U
    for k in range(U - 1):
        submit()
        d = max(1, round((k + 1) * S) - round(k * S))
        run_until(inflight[-1][0], 1 + d)

    # capture the decode graphs of the steady state now (batch buckets the
    # live count can reach x every decode window), not inside a timed step
    if dev.type == "cuda" and not args.no_graph:
        buckets = eng.cfg.graph_batch_sizes
        lo = next((b for b in buckets if b >= (U - 1) * u), buckets[-1])
        hi = next((b for b in buckets if b >= (U + 1) * u), buckets[-1])
        t0 = time.perf_counter()
        ncap = eng.warmup_graphs([b for b in buckets if lo <= b <= hi], args.prompt_len + args.gen_len,
                                 windows=(1, 2, 4, 8))
        log(f"captured {ncap} decode graphs in {time.perf_counter() - t0:.1f}s")
    log(f"warmup ({U} groups of {u} queries in flight)")
    for _ in range(args.warmup):
        run_step()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    for k in phase:  # phase breakdown over the timed steps only
        phase[k] = 0.0
    # long-lived setup objects (corpus tables, tokenizer tables, index metadata) leave the cyclic GC's
    # generations: a gen-2 pass over them runs in whichever thread triggers it, holding the GIL, and the
    # engine thread cannot launch meanwhile
    import gc
    gc.collect()
    if args.gc_freeze:
        gc.freeze()
    gc_ms = collections.Counter()
    gc_t0 = {}

    def _gc_cb(phase_, info):
        if phase_ == "start":
            gc_t0["t"] = time.perf_counter()
        elif "t" in gc_t0:
            gc_ms[info.get("generation", -1)] += (time.perf_counter() - gc_t0.pop("t")) * 1000
    gc.callbacks.append(_gc_cb)
    stats0 = dict(eng.stats)
    sampler = None
    if args.pysample:  # diagnostics: where the engine thread spends the timed steps
        from githubrepostorag_amd.utils.pysample import StackSampler
        sampler = StackSampler(interval=args.pysample / 1000.0, depth=4, all_threads=True).start()
    mark = os.environ.get("GRAG_TRACE_MARK") == "1" and dev.type == "cuda"
    if mark:  # a float64 fill kernel on the engine's stream marks the timed window in a kernel trace
        with torch.cuda.stream(eng.stream):
            torch.full((1,), 7.0, dtype=torch.float64, device=dev)
    t_start = time.perf_counter()
    phase["admit"] = 0.0
    ttfts = []
    for _ in range(args.steps):
        ttfts += run_step()
    if mark:
        with torch.cuda.stream(eng.stream):
            torch.full((1,), 7.0, dtype=torch.float64, device=dev)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if sampler is not None:
        sampler.stop()
        for share, where in sampler.top(30):
            log(f"pysample {share:7.4f}  {where}")
        for share, where in sampler.top_other(40):
            log(f"pysample-other {share:7.4f}  {where}")
    stats1 = dict(eng.stats)
    gc.callbacks.remove(_gc_cb)
    comm.barrier()
    elapsed = time.perf_counter() - t_start
    phase_timed = dict(phase)
    ttfts_all = [ttfts]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tt = torch.tensor(ttfts, dtype=torch.float64, device=dev)
        ttfts_all = group.all_gather(tt).cpu().tolist()
    elapsed = float(t.item())
    total_q = args.batch * args.steps * dp_size
    qps = total_q / elapsed
    p50 = statistics.median([x for r in ttfts_all for x in r]) * 1000.0
    ms_step = elapsed / args.steps * 1000.0

    while inflight:  # drain the pipeline (untimed)
        rids, _ = inflight.popleft()
        run_until(rids, args.gen_len)
        for r in rids:
            eng.pop(r)
    log(f"harness loop: {qps:.3f} queries/s, p50 TTFT {p50:.1f} ms, {ms_step:.1f} ms/step")

    # ---- index quality next to index speed: recall@k of the filtered IVF search (the timed loop's nprobe and
    # its neighbours) against an exact scan of every shard, on fresh queries (all ranks: the search is collective)
    recall = None
    if args.recall_queries > 0 and args.index_kind == "ivf":
        qs = [synthetic.question(77_000_000 + dp_rank * 10_000 + i) for i in range(args.recall_queries)]
        with side_stream(dev):
            qv = emb.embed_queries(qs)
            npbs = sorted({max(1, args.nprobe // 2), args.nprobe, 2 * args.nprobe, 4 * args.nprobe})
            recall = index.recall(qv, args.top_k, {"namespace": corpus.namespace}, nprobes=npbs)
        at = {r["nprobe"]: r["recall_at_k"] for r in recall["by_nprobe"]}
        recall["recall_at_10" if args.top_k == 10 else f"recall_at_{args.top_k}"] = at.get(args.nprobe)
        log(f"recall@{args.top_k} vs exact scan ({args.recall_queries} queries/rank): "
            + ", ".join(f"nprobe {r['nprobe']}: {r['recall_at_k']} ({r['search_ms']} ms)" for r in recall["by_nprobe"])
            + f"; exact scan {recall['exact_scan_ms']} ms")
    eng_stats = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()}

    # ---- the same workload through the serving loop (reported next to the harness numbers)
    serving_res = None
    n_srv = args.steps if args.serving_steps < 0 else args.serving_steps
    if n_srv > 0 and pool is not None:
        serving_res = serving_runner_phase(args, eng, prepare, sp, U, u, A, S, n_srv, dev, dp_size, group,
                                           world, log, tp_group)
    if pool is not None:
        pool.shutdown(wait=True)
    log("per-step phases (ms, timed steps): " + ", ".join(f"{k}={v / args.steps * 1000:.1f}"
                                                           for k, v in phase_timed.items()))
    timed_engine = {k: round((v - stats0.get(k, 0)) / args.steps, 4) for k, v in stats1.items()
                    if isinstance(v, (int, float))}

    # ---- end-to-end phase (reported separately): the reference's job path over real HTTP --
    # uvicorn serving service/api.py on 127.0.0.1, jobs through the queue + worker + GraphAgent
    # (plan / retrieve / judge / rewrite / synthesize, SSE token streaming) on this engine,
    # encoder and the 10M-row IVF chunk table (namespace filter fused in the scan)
    agent_res = None
    if args.agent_jobs > 0:
        agent_res = agent_phase(args, rank, world, dev, eng, tok, emb, index, corpus, log, tp_group, dp_size)
        if agent_res is not None:
            agent_res["agent_jobs_per_s"] = agent_res["jobs_per_s"]
            log(f"agent e2e: {agent_res['jobs_per_s']} jobs/s ({agent_res.get('steady_jobs_per_s')} steady), "
                f"e2e TTFT p50 {agent_res['e2e_ttft_p50_ms']} ms p90 {agent_res['e2e_ttft_p90_ms']} ms, "
                f"errors {agent_res['errors']}")

    # ---- the reference's own operating regime (one user, <= 4 sequences, up to 11.7K context)
    low_load = None
    if args.low_load and dev.type == "cuda" and tp == 1:
        from githubrepostorag_amd.engine.probe import run_low_load

        low_load = run_low_load(model, tok, kv_cache_gb=12.0, use_graph=not args.no_graph, log=log)
        if agent_res is not None:
            low_load["agent"] = agent_res.pop("low_concurrency", None)

    # ---- ingest phase (reported separately)
    ingest_dps = None
    ingest_stages = None
    ingest_ref = None
    if not args.no_ingest and args.ingest_files > 0:
        from githubrepostorag_amd.ingest.bench_ingest import run_ingest_bench

        del eng  # release the serving engine's KV cache; ingest builds a long-context engine
        # the engine (and its decode graphs) may sit in reference cycles frozen out of the GC's reach before
        # the timed steps: collect them now, before the ingest engine captures its graphs
        gc.unfreeze()
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        comm.barrier()
        n_docs, secs, ingest_stages = run_ingest_bench(model, tok, emb, args.ingest_files, seed=dp_rank,
                                                       max_num_seqs=args.ingest_seqs, use_graph=not args.no_graph,
                                                       mixed_batches=bool(args.ingest_mixed), tp=tp_group,
                                                       kv_cache_gb=args.ingest_kv_gb,
                                                       max_model_len=min(8192, dcfg.max_position))
        tt = torch.tensor([secs], dtype=torch.float64, device=dev)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ingest_dps = n_docs * dp_size / float(tt.item())  # one ingest per DP replica (TP peers share it)
        log(f"ingest: {n_docs} docs/rank in {float(tt.item()):.2f}s")
        if args.ingest_ref_cap_files > 0:
            n2, secs2, st2 = run_ingest_bench(model, tok, emb, args.ingest_ref_cap_files, seed=1000 + dp_rank,
                                              max_num_seqs=args.ingest_seqs, use_graph=not args.no_graph,
                                              mixed_batches=bool(args.ingest_mixed), tp=tp_group, token_cap=args.ingest_ref_cap,
                                              max_model_len=min(11712, dcfg.max_position), kv_cache_gb=args.ingest_kv_gb)
            tt2 = torch.tensor([secs2], dtype=torch.float64, device=dev)
            if world > 1:
                import torch.distributed as dist

                dist.all_reduce(tt2, op=dist.ReduceOp.MAX)
            ingest_ref = {"docs_per_s": round(n2 * dp_size / float(tt2.item()), 3), "files": n2,
                          "seconds": round(float(tt2.item()), 2), "token_cap": args.ingest_ref_cap, "max_model_len": 11712,
                          "decode_tokens": (st2.get("engine") or {}).get("decode_tokens"),
                          "llm_calls": st2.get("llm_calls")}
            log(f"ingest at a {args.ingest_ref_cap}-token cap on every call: {n2} docs/rank in {float(tt2.item()):.2f}s")

    ingest_multi = None
    spec = args.ingest_multi
    if spec == "auto":
        spec = "8x48" if dev.type == "cuda" else "2x2"
    if not args.no_ingest and spec not in ("0", "", "none") and tp == 1:
        from githubrepostorag_amd.ingest.bench_ingest import run_ingest_multi

        nr, nf = (int(x) for x in spec.lower().split("x"))
        comm.barrier()
        ingest_multi = run_ingest_multi(model, tok, emb, nr, nf, seed=dp_rank, max_num_seqs=args.ingest_seqs,
                                        use_graph=not args.no_graph, kv_cache_gb=args.ingest_kv_gb,
                                        max_model_len=min(8192, dcfg.max_position))
        tm = torch.tensor([ingest_multi["seconds"]], dtype=torch.float64, device=dev)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        ingest_multi["docs_per_s"] = round(ingest_multi["docs"] * dp_size / float(tm.item()), 3)
        log(f"multi-repo ingest ({nr} repos x {nf} files, ingest_many at once): {ingest_multi['docs_per_s']} docs/s")

    concurrent = None
    if (args.concurrent_ingest and not args.no_ingest and args.ingest_files > 0 and tp == 1 and serving_res
            and serving_res.get("open_loop")):
        base = next((o for o in serving_res["open_loop"] if abs(o["load"] - 0.5) < 1e-6), serving_res["open_loop"][0])
        concurrent = concurrent_phase(args, model, tok, emb, prepare, sp, u, dev, group, world, dp_rank, base, log)

    if rank == 0:
        # headline loop: the product's serving loop (EngineRunner, per-query arrivals; under TP the leader's
        # runner with its peers mirroring): its closed-loop queries/s is `value`, its TTFT is the open-loop
        # TTFT at the highest load <= 90 % of that rate (BASELINE: POST -> first token of a server at a set
        # load); the harness loop is kept as harness_loop (and is the headline with --serving-steps 0)
        harness = {"value": round(qps, 3), "p50_ttft_ms": round(p50, 2), "ms_per_step": round(ms_step, 2),
                   "steps": args.steps, "warmup": args.warmup,
                   "ttft_admission_policy": ("decode window capped to 1 step while an arrival's retrieval is in flight"
                                             if args.arrival_cap else "uncapped decode windows"),
                   "loop": "bench.py run_step: deterministic pipeline stepping the engine from the main thread, "
                           "groups of u queries admitted together"}
        srv = serving_res
        ol = [o for o in (srv or {}).get("open_loop") or [] if o["load"] <= 0.9 + 1e-9]
        ttft_src = max(ol, key=lambda o: o["load"]) if ol else None
        head_qps = srv["value"] if srv else qps
        head_ms = srv["ms_per_step"] if srv else ms_step
        head_p50 = ttft_src["p50_ttft_ms"] if ttft_src else (srv["p50_ttft_ms"] if srv else p50)
        res = {
            "metric": "RAG queries/sec + p50 TTFT (Qwen2-7B, 10M-vec index); ingest docs/sec",
            "value": round(head_qps, 3),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head_ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp32" if dev.type != "cuda" else "bf16") if args.quant == "none" else
                     "w4a16 (AWQ format, group 128) decode / bf16 prefill",
            "data": "synthetic (random-init weights, clustered synthetic vectors, generated chunk texts/questions)",
            "p50_ttft_ms": round(head_p50, 2),
            "p90_ttft_ms": ttft_src["p90_ttft_ms"] if ttft_src else (srv["p90_ttft_ms"] if srv else None),
            "headline_loop": (
                f"serving loop (engine/runner.py EngineRunner, per-query arrivals): value = closed-loop queries/s "
                f"over {args.steps} timed steps of {args.batch} completions per GPU after one pipeline turnover; "
                + (f"TTFT = arrival -> first token under open-loop Poisson arrivals at {ttft_src['load']:.0%} of that "
                   f"rate ({ttft_src['offered_queries_per_s']} queries/s per GPU)" if ttft_src else
                   "TTFT = arrival -> first token in the closed loop")) if srv else
                "harness loop (bench.py run_step; the serving loop runs at TP = 1 only)",
            "harness_loop": harness,
            "ingest_docs_per_s": None if ingest_dps is None else round(ingest_dps, 3),
            "ingest_docs_per_s_ref_cap": None if ingest_ref is None else ingest_ref["docs_per_s"],
            "config": {
                "preset": args.preset or "c3",
                "model": f"{args.model} TP={tp} + {args.encoder}, {args.index_size}-vec {args.index_kind} index "
                         f"(nlist={args.nlist}, nprobe={args.nprobe}) sharded dp{world}",
                "sampling": "greedy" if args.greedy else "temperature 0.4, top_p 0.8, repetition_penalty 1.2",
                "device": dev.type,
                "global_batch": args.batch * dp_size,
                "inflight_batches": D,
                "mixed_batches": bool(args.mixed),
                "max_batched_tokens": args.max_batched_tokens,
                "arrival_groups": A,
                "concurrent_seqs": args.batch * D * dp_size,
                "seq_len": args.prompt_len,
                "gen_len": args.gen_len,
                "top_k": args.top_k,
                "parallelism": f"tp{tp}dp{dp_size}" if tp > 1 else f"dp{world}",
                **({"quant": "w4a16 awq-format (round-to-nearest group-128 codes of the random-init weights)",
                    "decode_weight_gb": round(w4_bytes / 1e9, 3)} if args.quant == "w4" else {}),
            },
            "engine": eng_stats,
            "engine_per_timed_step": timed_engine,
            # timed decode tokens / (completed queries x (gen_len - 1)): ~1.0 when the timed steps did the
            # steady state's decode work (no backlog from the fill drained or built inside the timed region)
            "steady_state_decode_ratio": round(timed_engine.get("decode_tokens", 0) * dp_size * args.steps
                                               / max(1, total_q * (args.gen_len - 1)), 3),
            "phase_ms_per_step": {k: round(v / args.steps * 1000, 2) for k, v in phase_timed.items()},
            "gc_pause_ms_per_step": {f"gen{k}": round(v / args.steps, 2) for k, v in sorted(gc_ms.items())},
            "main_thread_ms_per_step": {"engine_step": round(timed_engine.get("step_s", 0) * 1000, 2),
                                        "engine_prefill": round(timed_engine.get("prefill_s", 0) * 1000, 2),
                                        "engine_decode": round(timed_engine.get("decode_s", 0) * 1000, 2)},
            "retrieval_prefetch": bool(args.prefetch),
            # TP: bytes each rank receives per 512-row decode sampling step
            "tp_sampler_bytes_per_decode_step": None if tp == 1 else __import__(
                "githubrepostorag_amd.ops.sampling", fromlist=["x"]).tp_sampling_bytes(
                args.batch * D, tp, dcfg.vocab_size, 2),
            "serving_runner": serving_res,
            "ingest_stage_s": ingest_stages,
            "ingest_ref_cap": ingest_ref,
            # several repositories through ingest_many at once on one engine (the next repo's extractor waves
            # fill a repo's roll-up tail); ingest_docs_per_s above is one repository at a time
            "ingest_multi_repo": ingest_multi,
            "e2e_ttft_p50_ms": None if agent_res is None else agent_res["e2e_ttft_p50_ms"],
            "e2e_ttft_p90_ms": None if agent_res is None else agent_res["e2e_ttft_p90_ms"],
            "agent_jobs_per_s": None if agent_res is None else agent_res["agent_jobs_per_s"],
            "agent_steady_jobs_per_s": None if agent_res is None else agent_res.get("steady_jobs_per_s"),
            "agent_saturation": None if agent_res is None else agent_res.get("agent_saturation"),
            "agent_e2e": agent_res,
            "low_load": low_load,
            "index_recall": recall,
            "concurrent_ingest": concurrent,
            "recall_at_10": None if recall is None else recall.get("recall_at_10"),
            # the two operating points the headline combines, side by side: the closed loop's saturating rate
            # with its own TTFT, and each open-loop level's achieved rate with its TTFT
            "operating_points": ([{"loop": "closed (saturating)", "queries_per_s": srv["value"],
                                   "ttft_p50_ms": srv["p50_ttft_ms"], "ttft_p90_ms": srv["p90_ttft_ms"]}]
                                 + [{"loop": f"open, Poisson at {o['load']:.0%}",
                                     "queries_per_s": round(o["achieved_queries_per_s"] * dp_size, 3),
                                     "ttft_p50_ms": o["p50_ttft_ms"], "ttft_p90_ms": o["p90_ttft_ms"]}
                                    for o in srv.get("open_loop") or []]) if srv else None,
            # kernels' out-of-range index reports over the whole run (csrc/kernels/common.h index guard): the
            # engine raises on the first at its next step, so a clean run reports 0
            "device_index_reports": __import__("githubrepostorag_amd.ops._lib", fromlist=["x"]).device_errors()[2],
        }
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


class _ArrivalPump:
    """Per-query arrivals of the serving loop.  ``arrive()`` stamps a query's POST time; one thread takes
    the queries that have arrived (up to u) into one retrieval micro-batch (embed + filtered sharded search
    + prompt) under the runner's admission hint and submits every prompt on its own, as a server's request
    handlers do (each query is admitted by the engine when its own prompt is ready, not with a group).
    DP > 1: the sharded search is a collective, so the ranks' pumps run lockstep rounds -- a (queries,
    stop) all-gather first; a round no rank has queries for is skipped; a rank with none joins the search
    with an empty batch; the pumps exit together once every rank asks to stop."""

    def __init__(self, runner, prepare, sp, u, group, dev, tick: float = 0.002, follower: bool = False):
        import queue
        import threading

        self.runner, self.prepare, self.sp, self.u, self.group, self.dev, self.tick = \
            runner, prepare, sp, u, group, dev, tick
        # a TP follower rank: no arrivals of its own (its TP leader submits, its engine mirrors the leader's
        # steps); it joins every retrieval round's search collectives with an empty batch, never holds a
        # barrier back, and stops when every rank has asked to
        self.follower = follower
        self.q = collections.deque()
        self.cv = threading.Condition()
        self.done = queue.SimpleQueue()  # (handle, t_arrival, t_submitted) per completed query
        self.stop_req = False
        self.taken = 0      # arrivals taken into a retrieval micro-batch (each completes once submitted)
        self.submitted = 0
        self.abs_times = []  # (submitted, first token) perf_counter stamps of the completions taken by get()
        self.batches = []    # queries per retrieval micro-batch
        self.retrieval = []  # per micro-batch: first arrival -> prompts submitted (s)
        self.error = None
        self.sync_req = follower
        self.stop_req = follower
        self.sync_ev = threading.Event()
        self.th = threading.Thread(target=self._run, name="bench-pump", daemon=True)
        self.th.start()

    def arrive(self, n: int = 1) -> None:
        t = time.perf_counter()
        with self.cv:
            self.q.extend([t] * n)
            self.cv.notify()

    def queued(self) -> int:
        with self.cv:
            return len(self.q)

    def _take(self):
        with self.cv:
            if not self.q and not self.stop_req:
                self.cv.wait(0.05 if self.group is None else self.tick)
            n = min(len(self.q), self.u)
            self.taken += n
            return [self.q.popleft() for _ in range(n)], self.stop_req, self.sync_req

    def _run(self):
        import torch

        from githubrepostorag_amd.utils.gpu_guard import side_stream

        try:
            while True:
                ts, stop, sync = self._take()
                if self.group is not None:
                    with side_stream(self.dev):  # off the engine's stream, as the search itself
                        f = self.group.all_gather(torch.tensor([len(ts), int(stop), int(sync)], dtype=torch.int64,
                                                               device=self.dev)).view(-1, 3).cpu()
                    if int(f[:, 2].min()) == 1:  # every rank is at barrier(): release them together
                        with self.cv:
                            self.sync_req = self.follower
                        self.sync_ev.set()
                    if int(f[:, 1].min()) == 1:
                        return
                    if int(f[:, 0].max()) == 0:
                        continue
                else:
                    if sync:
                        with self.cv:
                            self.sync_req = False
                        self.sync_ev.set()
                    if stop and not ts:
                        return
                    if not ts:
                        continue
                with self.runner.arrival():
                    prompts, _, _ = self.prepare(len(ts))
                    hs = [self.runner.submit(p, self.sp) for p in prompts]
                t_in = time.perf_counter()
                self.submitted += len(hs)
                if ts:
                    self.batches.append(len(ts))
                    self.retrieval.append(t_in - ts[0])
                for h, t0 in zip(hs, ts):
                    h.add_done_callback(lambda h, t0=t0, t_in=t_in: self.done.put((h, t0, t_in)))
        except BaseException as e:  # surfaced by the phase's waits
            self.error = e
            self.done.put(None)

    def join_follower(self, timeout: float = 3600.0) -> None:
        """A follower's pump: serve the rounds until every rank has stopped."""
        self.th.join(timeout=timeout)
        if self.error is not None:
            raise RuntimeError("serving phase: follower pump failed") from self.error

    def barrier(self, timeout: float = 600.0) -> None:
        """A barrier of all ranks' main threads taken inside the pumps' round stream (the pump is the only
        thread issuing collectives while it runs: a world barrier beside its rounds could interleave two
        communicators differently on different ranks)."""
        self.sync_ev.clear()
        with self.cv:
            self.sync_req = True
            self.cv.notify()
        if not self.sync_ev.wait(timeout):
            raise TimeoutError("serving phase: barrier timed out")

    def get(self, timeout: float = 600.0):
        import queue

        try:
            item = self.done.get(timeout=timeout)
        except queue.Empty:
            raise TimeoutError(f"serving phase: no completion for {timeout:.0f} s") from None
        if item is None:
            raise RuntimeError("serving phase: arrival pump failed") from self.error
        h, t0, t_in = item
        c = h.wait(0)  # a failed request raises here
        self.abs_times.append((t_in, c.first_token_at))
        return c.first_token_at - t0, c.first_token_at - t_in

    def drain_and_stop(self, completed: int, timeout: float = 600.0) -> int:
        """Wait for every arrival to be retrieved and completed (``completed`` = completions consumed so
        far), then stop the pump (all ranks together).  Returns the completions consumed here."""
        n = 0
        t_end = time.perf_counter() + timeout
        while self.queued() or completed + n < self.taken:
            if self.error is not None:
                break
            if time.perf_counter() > t_end:
                raise TimeoutError("serving phase: drain timed out")
            try:
                self.get(timeout=1.0)
                n += 1
            except TimeoutError:
                pass
        with self.cv:
            self.stop_req = True
            self.cv.notify()
        self.th.join(timeout=timeout)
        if self.error is not None:
            raise RuntimeError("serving phase: arrival pump failed") from self.error
        return n


def serving_runner_phase(args, eng, prepare, sp, U, u, A, S, steps, dev, dp_size, group, world, log, tp_group=None):
    """The headline workload through the product's serving loop: the engine steps on its own EngineRunner
    thread (engine/runner.py, as ``serve`` runs it); queries arrive ONE AT A TIME (a POST each) and go
    through a retrieval micro-batcher (_ArrivalPump: the queries that arrived meanwhile, up to u, share one
    embed + sharded search) and are submitted one by one.  Closed loop at the harness's concurrency (U x u
    live queries; each completion is replaced by a new arrival at once); the fill submits u queries every S
    decode steps, so completions are spread over the pipeline as in the harness.  Timed: ``steps`` x B
    completions per rank after one untimed turnover of the pipeline; qps = completed queries / wall time
    (max over ranks); TTFT = arrival -> first token.  Then ``--serving-open-load``: Poisson arrivals of
    single queries at fractions of the closed loop's rate (``open_loop``) -- the TTFT a server sees at a set
    load.  ``--interactive-prefill`` caps the prefill tokens per step while arrivals are pending.
    TP > 1: the TP leader's runner takes the arrivals and every TP peer's runner mirrors its engine steps
    (engine/runner.py follow); the peers' pumps join each retrieval round's sharded search with no queries."""
    import torch

    from githubrepostorag_amd.engine.runner import EngineRunner
    from githubrepostorag_amd.parallel import comm

    B = u * A
    pg = group if world > 1 else None
    if dev.type == "cuda" and not args.no_graph and os.environ.get("GRAG_SERVING_WARMUP", "1") != "0":
        # the loop fills from an empty engine, so its first steps meet small decode buckets / split plans and
        # 1..u-query encoder buckets the harness never used: capture them here, outside the timed window (every
        # rank runs this in the same order: the sharded search and TP captures are collective).  Not
        # load-bearing for correctness: GRAG_SERVING_WARMUP=0 leaves every capture to the runner / retrieval
        # threads while the other one works (the round-5 fault's setting; the workspaces those threads' kernels
        # use are owned per engine / embedder / thread and the index guard reports bad indices)
        hi = next((b for b in eng.cfg.graph_batch_sizes if b >= (U + 1) * u), eng.cfg.graph_batch_sizes[-1])
        ctxs = sorted({args.prompt_len + k for k in range(1, args.gen_len + 2, 32)} | {args.prompt_len + args.gen_len})
        n_cap = eng.warmup_graphs([b for b in eng.cfg.graph_batch_sizes if b <= hi], ctxs, windows=(1, 2, 4, 8),
                                  params=sp)
        for n in range(1, u + 1):
            prepare(n)
        log(f"serving loop: {n_cap} more decode graphs and the 1-{u}-query retrieval buckets warmed")
    runner = EngineRunner(eng, watchdog_s=0, interactive_prefill=args.interactive_prefill,
                          bulk_prefill=args.bulk_prefill, tp=tp_group)
    res_open = []
    loads = [float(x) for x in str(args.serving_open_load).split(",") if x.strip()]
    if not runner.leader:
        try:  # the closed loop's pump, then one per open-loop level, each followed by the leaders' barrier
            for _ in range(1 + len(loads)):
                _ArrivalPump(runner, prepare, sp, u, pg, dev, follower=True).join_follower()
                comm.barrier()
        finally:
            runner.shutdown()
        t = torch.tensor([0.0], dtype=torch.float64, device=dev)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            comm.world_group().all_gather(torch.full((steps * B,), float("nan"), dtype=torch.float64, device=dev))
        return None
    try:
        pump = _ArrivalPump(runner, prepare, sp, u, pg, dev)
        d0 = eng.stats["decode_steps"]
        for k in range(U):  # fill: u queries every S decode steps
            pump.arrive(u)
            want = d0 + round((k + 1) * S)
            t0 = time.perf_counter()
            while eng.stats["decode_steps"] < want and time.perf_counter() - t0 < 120:
                time.sleep(0.0002)

        def complete(n: int, replace: bool = True) -> tuple[list, list]:
            tt, te = [], []
            while len(tt) < n:
                a, b = pump.get()
                tt.append(a)
                te.append(b)
                if replace:
                    pump.arrive(1)
            return tt, te

        complete(U * u)  # one full turnover of the pipeline (untimed)
        pump.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t_start = time.perf_counter()
        dec0 = eng.stats["decode_tokens"]
        nb0, nr0 = len(pump.batches), len(pump.retrieval)
        eng.trace = []  # engine steps of the timed window (kind, rows, tokens, seconds)
        ttfts, engs = complete(steps * B)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        pump.barrier()
        elapsed = time.perf_counter() - t_start
        dec1 = eng.stats["decode_tokens"]
        trace, eng.trace = eng.trace, None
        batches, retr = pump.batches[nb0:], pump.retrieval[nr0:]
        pump.drain_and_stop(completed=U * u + steps * B)
        comm.barrier()
        n_open = max(4 * B, min(steps * B, 768))  # arrivals per load level (bounds the bench's wall time)
        for load in loads:
            res_open.append({"load": load, **_open_loop(runner, prepare, sp, u, pg, dev, load * B * steps / elapsed,
                                                         n_open)})
            comm.barrier()
    finally:
        runner.shutdown()
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    allt = [ttfts]
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        allt = comm.world_group().all_gather(torch.tensor(ttfts, dtype=torch.float64, device=dev)).cpu().tolist()
    elapsed = float(t.item())
    qps = B * steps * dp_size / elapsed
    flat = sorted(x for r in allt for x in r if x == x)  # TP peers send NaN rows
    p50 = statistics.median(flat) * 1000.0
    p90 = flat[min(len(flat) - 1, int(0.9 * len(flat)))] * 1000.0
    log(f"serving loop (EngineRunner, per-query arrivals): {qps:.3f} queries/s, closed-loop TTFT p50 {p50:.1f} ms")
    for o in res_open:
        log(f"serving loop, open-loop Poisson arrivals at {o['offered_queries_per_s']} queries/s ({o['load']:.0%} "
            f"of the closed loop): TTFT p50 {o['p50_ttft_ms']} ms, p90 {o['p90_ttft_ms']} ms")
    return {"value": round(qps, 3), "p50_ttft_ms": round(p50, 2), "p90_ttft_ms": round(p90, 2), "steps": steps,
            "ms_per_step": round(elapsed / steps * 1000.0, 2),
            # TTFT = queueing for a retrieval micro-batch + retrieval (embed + search + prompt) + engine admission
            # and prefill; the retrieval micro-batches and the submit -> first token part (this rank)
            "retrieval_batch_mean": round(statistics.mean(batches), 2) if batches else None,
            "retrieval_p50_ms": round(statistics.median(retr) * 1000.0, 2) if retr else None,
            "submit_to_first_token_p50_ms": round(statistics.median(engs) * 1000.0, 2) if engs else None,
            "engine_steps": _trace_summary(trace),
            "open_loop": res_open,
            # decode tokens the engine produced in the timed window / what the completed queries needed:
            # ~1.0 when the window was the pipeline's steady state (no backlog built or drained in it)
            "steady_state_decode_ratio": round((dec1 - dec0) / max(1, B * steps * (args.gen_len - 1)), 3),
            "arrival_window": os.environ.get("GRAG_ARRIVAL_WINDOW", "auto"),
            "interactive_prefill_tokens": args.interactive_prefill or None,
            "bulk_prefill_tokens": args.bulk_prefill or None,
            "loop": "engine/runner.py EngineRunner thread (free-running; decode replays paced by the arrival rate: "
                    "engine/runner.py _window); per-query arrivals through a retrieval micro-batcher "
                    "(_ArrivalPump), each prompt submitted on its own; closed loop at the harness's concurrency"}


def _open_loop(runner, prepare, sp, u, pg, dev, rate: float, n: int) -> dict:
    """n single-query arrivals at Poisson times (``rate`` queries/s on this rank) through a fresh pump;
    TTFT p50 / p90 and the achieved completion rate."""
    import random

    import torch.distributed as dist

    rng = random.Random(4321 + (dist.get_rank() if dist.is_available() and dist.is_initialized() else 0))
    pump = _ArrivalPump(runner, prepare, sp, u, pg, dev)
    t0 = time.perf_counter()
    due = t0
    for _ in range(n):
        due += rng.expovariate(rate)
        dt = due - time.perf_counter()
        if dt > 0:
            time.sleep(dt)
        pump.arrive(1)
    t_last = time.perf_counter()
    tt = []
    while len(tt) < n:
        tt.append(pump.get()[0])
    t_done = time.perf_counter()
    pump.drain_and_stop(completed=n)
    tt.sort()
    return {"offered_queries_per_s": round(rate, 3), "queries": n,
            "achieved_queries_per_s": round(n / (t_done - t0), 3), "arrival_window_s": round(t_last - t0, 2),
            "retrieval_batch_mean": round(statistics.mean(pump.batches), 2) if pump.batches else None,
            "p50_ttft_ms": round(1000 * tt[len(tt) // 2], 2),
            "p90_ttft_ms": round(1000 * tt[min(len(tt) - 1, int(0.9 * len(tt)))], 2)}


def concurrent_phase(args, model, tok, emb, prepare, sp, u, dev, group, world, dp_rank, base, log) -> dict:
    """BASELINE config 4's second half on one GPU: the ingest pipeline (bulk waves + roll-ups, the same
    synthetic repo as the ingest phase) and open-loop query arrivals at the serving loop's ``base`` load
    share ONE engine (one EngineRunner), as the reference's single vLLM server takes both
    (helm/templates/qwen-deployment.yaml:32-33).  Queries are admitted ahead of ingest work (priority 2 vs the
    roll-ups' 1 and the waves' 0) and cap the prefill per step while they arrive (interactive_prefill).
    Reports ingest docs/s and query TTFT p50 / p90 next to the ingest-free numbers (``base``)."""
    import dataclasses
    import random
    import threading

    import torch
    import torch.distributed as dist

    from githubrepostorag_amd.agent.llm import EngineLLM
    from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
    from githubrepostorag_amd.engine.runner import EngineRunner
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.ingest.bench_ingest import run_ingest_bench
    from githubrepostorag_amd.parallel import comm

    seqs = args.ingest_seqs + 256
    sizes = tuple(sorted({*EngineConfig.graph_batch_sizes, *range(256, seqs + 1, 128), seqs}))
    mml = min(8192, model.cfg.max_position)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=seqs, max_num_batched_tokens=16384, max_model_len=mml,
                                             use_cuda_graph=not args.no_graph and dev.type == "cuda",
                                             seed=dp_rank, kv_cache_gb=args.ingest_kv_gb,
                                             graph_batch_sizes=tuple(b for b in sizes if b <= seqs)))
    q_sp = dataclasses.replace(sp, priority=2)
    if dev.type == "cuda" and not args.no_graph:
        t0 = time.perf_counter()
        n = eng.warmup_graphs(max_ctx=[c for c in (2048, 4096, mml) if c <= mml], windows=(1, 2, 4, 8),
                              params=SamplingParams(temperature=EngineLLM.INGEST["temperature"],
                                                    top_p=EngineLLM.INGEST["top_p"]),
                              cascade=(False, True))
        n += eng.warmup_graphs(max_ctx=[2048, 4096], windows=(1, 2, 4, 8), params=q_sp)
        log(f"concurrent phase: {n} decode graphs captured in {time.perf_counter() - t0:.1f}s")
    runner = EngineRunner(eng, watchdog_s=0, interactive_prefill=args.interactive_prefill,
                          bulk_prefill=args.bulk_prefill)
    pg = group if world > 1 else None
    rate = base["offered_queries_per_s"]
    out = {}
    try:
        done = threading.Event()

        def ingest():
            try:
                out["ingest"] = run_ingest_bench(model, tok, emb, args.ingest_files, seed=dp_rank, runner=runner)
            finally:
                done.set()

        pump = _ArrivalPump(runner, prepare, q_sp, u, pg, dev)
        comm.barrier()
        eng.trace = []  # the engine steps of the concurrent window (kind, rows, tokens, seconds)
        th = threading.Thread(target=ingest, name="bench-concurrent-ingest", daemon=True)
        rng = random.Random(8642 + (dist.get_rank() if dist.is_available() and dist.is_initialized() else 0))
        t0 = time.perf_counter()
        th.start()
        due, n = t0, 0
        while not done.is_set():
            due += rng.expovariate(rate)
            dt = due - time.perf_counter()
            if dt > 0 and done.wait(dt):
                break
            pump.arrive(1)
            n += 1
        t_ing = time.perf_counter() - t0
        th.join()
        got = [pump.get() for _ in range(n)]
        tt, te = [g[0] for g in got], sorted(g[1] for g in got)
        retr = sorted(pump.retrieval)
        abs_times = list(pump.abs_times)
        pump.drain_and_stop(completed=n)
    finally:
        runner.shutdown()
        trace, eng.trace = eng.trace, None
        del eng
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    docs, secs, st = out["ingest"]
    if os.environ.get("GRAG_DUMP_TRACE"):  # the raw step trace + each query's (submitted, first token) stamps
        with open(os.environ["GRAG_DUMP_TRACE"], "w") as f:
            json.dump({"trace": [list(t) for t in trace or []], "abs_times": abs_times,
                       "ttft": [g[0] for g in got], "submit_to_first": [g[1] for g in got]}, f)
    tt.sort()
    p50 = 1000 * tt[len(tt) // 2] if tt else None
    p90 = 1000 * tt[min(len(tt) - 1, int(0.9 * len(tt)))] if tt else None
    res = {"ingest_docs_per_s": round(docs / secs, 3), "ingest_seconds": round(secs, 2), "files": docs,
           "queries": n, "offered_queries_per_s": round(rate, 3), "achieved_queries_per_s": round(n / t_ing, 3),
           "p50_ttft_ms": None if p50 is None else round(p50, 2), "p90_ttft_ms": None if p90 is None else round(p90, 2),
           "ingest_free": {"load": base["load"], "p50_ttft_ms": base["p50_ttft_ms"], "p90_ttft_ms": base["p90_ttft_ms"]},
           "ttft_p50_vs_ingest_free": None if p50 is None else round(p50 / base["p50_ttft_ms"], 3),
           # TTFT = retrieval (embed + search + prompt, on the GPU beside the engine) + submit -> first token
           "retrieval_p50_ms": round(1000 * retr[len(retr) // 2], 2) if retr else None,
           "submit_to_first_token_p50_ms": round(1000 * te[len(te) // 2], 2) if te else None,
           "engine": (st or {}).get("engine"),
           "engine_steps": _trace_summary(trace),
           "submit_to_first_token_anatomy": _wait_anatomy(trace, abs_times),
           "setup": "one LLMEngine + EngineRunner (max_model_len 8192) shared by the ingest pipeline and the "
                    "serving loop's per-query arrivals (Poisson at the ingest-free open loop's load, until the "
                    "ingest ends); queries at priority 2, ingest roll-ups 1, extractor waves 0"}
    log(f"concurrent ingest + queries: ingest {res['ingest_docs_per_s']} docs/s, {n} queries at {rate:.1f}/s, TTFT "
        f"p50 {res['p50_ttft_ms']} ms (ingest-free {base['p50_ttft_ms']} ms), p90 {res['p90_ttft_ms']} ms")
    return res


def _wait_anatomy(trace, abs_times) -> dict:
    """Where a query's submit -> first token goes, from the engine trace: the rest of the step in flight when
    it was submitted, and the steps that started before its first token (its own prefill step included),
    by kind.  Medians over the queries."""
    steps = sorted((t[0], t[1], t[4]) for t in trace or [] if t[1] in ("prefill", "mixed", "decode"))
    if not steps or not abs_times:
        return {}
    import bisect

    starts = [t for t, _, _ in steps]
    inflight, n_steps, kinds = [], [], collections.Counter()
    for t_in, t_first in abs_times:
        i = bisect.bisect_left(starts, t_in)
        if i > 0 and starts[i - 1] + steps[i - 1][2] > t_in:
            inflight.append(starts[i - 1] + steps[i - 1][2] - t_in)
        else:
            inflight.append(0.0)
        j = bisect.bisect_left(starts, t_first)
        n_steps.append(j - i)
        for _, kind, _ in steps[i:j]:
            kinds[kind] += 1
    inflight.sort()
    n_steps.sort()
    nq = len(abs_times)
    return {"inflight_step_rest_p50_ms": round(1000 * inflight[nq // 2], 2),
            "steps_started_before_first_token_p50": n_steps[nq // 2],
            "steps_started_per_query_by_kind": {k: round(v / nq, 2) for k, v in kinds.items()}}


def _trace_summary(trace) -> dict:
    """Engine steps of a window (LLMEngine.trace records): count, mean rows / tokens / ms per kind."""
    out = {}
    for kind in ("prefill", "mixed", "decode"):
        st = [t for t in trace or [] if t[1] == kind]
        if st:
            out[kind] = {"steps": len(st), "mean_rows": round(sum(t[2] for t in st) / len(st), 1),
                         "mean_tokens": round(sum(t[3] for t in st) / len(st), 1),
                         "mean_ms": round(1000 * sum(t[4] for t in st) / len(st), 2)}
    return out


def _scope_tables(store, emb, corpus, rank, world, dev):
    """This rank's shard of the project / package / file summary tables next to the chunk table
    (synthetic hierarchy rows, utils/synthetic.scope_rows; random unit vectors: the corpus is
    synthetic), rows owned by crc32(row_id) mod world as the sharded store routes them."""
    import torch

    from githubrepostorag_amd.index.sharded_store import shard_of
    from githubrepostorag_amd.utils import synthetic

    for scope in ("repo", "module", "file"):
        ids, texts, metas = synthetic.scope_rows(corpus, scope)
        keep = [i for i, r in enumerate(ids) if shard_of(r, world) == rank]
        g = torch.Generator(device="cpu").manual_seed(4242 + rank * 7 + len(scope))
        v = torch.nn.functional.normalize(torch.randn(len(keep), emb.dim, generator=g), dim=1)
        store.table(scope).upsert([ids[i] for i in keep], [texts[i] for i in keep], v.to(dev),
                                  [metas[i] for i in keep])


def agent_phase(args, rank, world, dev, eng, tok, emb, index, corpus, log, tp_group=None, dp_size=1):
    """POST /rag/jobs -> SSE over real HTTP: ``--agent-jobs`` agent jobs per GPU at
    ``--agent-concurrency`` per GPU, over all four scope tables (10M-row chunk table + project /
    package / file summary tables).  N > 1: one front door on rank 0 (service/cluster.py) over a
    replica on every rank; each replica holds its shard of every table and every retrieval round
    fans out through the hub (index/sharded_store.py), as ``serve --replicas N`` runs.  Under TP
    the group's TP rank 0 runs the jobs (its engine runner leads, the peers follow in lockstep) and
    every other rank joins as a shard-only replica (capacity 0) that answers the index rounds for
    its shard of the chunk table."""
    import threading

    from githubrepostorag_amd.agent.llm import EngineLLM, MeteredLLM
    from githubrepostorag_amd.config import Settings
    from githubrepostorag_amd.engine.runner import EngineRunner
    from githubrepostorag_amd.index.store import VectorStore
    from githubrepostorag_amd.service.api import APIState, create_app
    from githubrepostorag_amd.service.e2e import run_e2e
    from githubrepostorag_amd.service.runtime import RAGRuntime
    from githubrepostorag_amd.utils import synthetic

    conc = args.agent_concurrency
    levels = [int(x) for x in args.agent_sweep.split(",") if x.strip()]
    # a replica's job slots: the largest concurrency it will be driven at, capped at --agent-slots (the rest queue)
    slots = min(max([conc, *levels]), max(1, args.agent_slots))
    s = Settings(qwen_model=args.model, embed_model=args.encoder, qwen_max_output=args.agent_gen_len,
                 synth_max_tokens=args.agent_synth_len, worker_max_jobs=slots, max_rag_attempts=3,
                 default_namespace=corpus.namespace, job_timeout_s=1800, llm_retries=0, stream_tokens=True,
                 index_kind=args.index_kind, nlist=args.nlist, nprobe=args.nprobe, embed_batch_window_ms=1.0,
                 data_dir=None, seed=rank)
    store = VectorStore(emb.dim, dev)
    store.tables["chunk"] = index.table
    _scope_tables(store, emb, corpus, rank, world, dev)
    tp = tp_group if tp_group is not None and not tp_group.trivial else None
    runner = EngineRunner(eng, watchdog_s=600, tp=tp)
    leader = runner.leader
    llm = MeteredLLM(EngineLLM(runner, tok, max_tokens=args.agent_gen_len, timeout_s=1800, retries=0)) \
        if leader else None
    rt = RAGRuntime(s, device=str(dev), llm=llm, embedder=emb, store=store, build_engine=False)
    rt.engine, rt.runner = eng, runner
    import logging

    logging.getLogger("githubrepostorag_amd.agent").setLevel(logging.ERROR)  # random weights: parse fallbacks
    n_jobs, n_conc = args.agent_jobs * dp_size, conc * dp_size
    q0 = 50_000_000

    def mix(i):  # half code questions (code scope), half project overviews (project -> package -> file)
        return synthetic.code_question(q0 + i) if i % 2 == 0 else synthetic.overview_question(q0 + i, corpus)

    warm = [mix(500_000 + i) for i in range(min(n_conc, 16 * world))]
    qs = [mix(i) for i in range(n_jobs)]
    # saturation sweep: 2 x concurrency jobs per level (>= 64), fresh questions for each
    sweep = []
    for j, c in enumerate(levels):
        n = max(64, 2 * c) * dp_size
        sweep.append(([mix(10_000_000 * (j + 1) + i) for i in range(n)], c * dp_size))
    # the reference's regime: one user (concurrency 1) and vLLM's 4 sequences (concurrency 4), few jobs each
    low = [(4, 1), (8, 4)] if (args.low_load and world == 1) else []
    for j, (n, c) in enumerate(low):
        sweep.append(([mix(90_000_000 + 1000 * j + i) for i in range(n)], c))
    res = None
    try:
        if world == 1:
            res = run_e2e(create_app(APIState(runtime=rt)), qs, n_conc, warmup=warm, sweep=sweep,
                          stats_fn=lambda: {**eng.stats, "preemptions": eng.sched.num_preemptions})
        else:
            import torch.distributed as dist

            from githubrepostorag_amd.service.cluster import ClusterRuntimeView, ReplicaHub, run_replica
            from githubrepostorag_amd.service.events import EventLog

            hub = None
            obj = [None]
            if rank == 0:
                events = EventLog()
                hub = ReplicaHub(events, job_timeout=1800.0)
                obj = [(tuple(hub.address), hub.authkey)]
            dist.broadcast_object_list(obj, src=0)
            addr, key = obj[0]
            rgroup = None
            if os.environ.get("GRAG_SHARD_TRANSPORT", "collective") == "collective":
                # the replicas' shard rounds as lockstep collectives (service/collective.py: RCCL over xGMI, the
                # score exchange a device all-gather) on a communicator of their own; GRAG_SHARD_TRANSPORT=mesh
                # keeps the socket mesh
                from githubrepostorag_amd.parallel import comm

                rgroup = comm.Group(list(range(world)), pg=dist.new_group(list(range(world))))
            th = threading.Thread(target=run_replica, args=(rt, addr, key, rank),
                                  kwargs={"shards": world, "capacity": slots if leader else 0, "group": rgroup},
                                  name="bench-replica", daemon=True)
            th.start()
            if rank == 0:
                t0 = time.time()
                while hub.live_count() < world:
                    if time.time() - t0 > 300:
                        raise RuntimeError(f"only {hub.live_count()} of {world} replicas connected")
                    time.sleep(0.05)
                state = APIState(runtime=ClusterRuntimeView(hub, s), queue=hub.queue, events=events,
                                 flags=hub.flags)
                try:
                    res = run_e2e(create_app(state), qs, n_conc, warmup=warm, sweep=sweep)
                    res["replicas"] = hub.health()["replicas"]
                finally:
                    hub.close()  # replicas return from run_replica
            th.join(timeout=120)
            if leader:
                runner.shutdown()  # TP: stops the followers' lockstep loops
            else:
                runner.join(timeout=600)
            dist.barrier()
    finally:
        runner.shutdown()
        emb.close()  # the runtime turned on query-embedding batching for this phase
        st = getattr(rt.store, "close", None)
        if st is not None and rt.store is not store:
            st()
    if res is None:
        return None
    if low and res.get("agent_saturation"):
        curve = res["agent_saturation"]
        res["low_concurrency"] = [{k: v for k, v in r.items() if k != "engine"} for r in curve[len(levels):]]
        res["agent_saturation"] = curve[:len(levels)] or None
    res["concurrency"] = n_conc
    res["worker_slots_per_replica"] = slots
    res["llm_token_cap"] = args.agent_gen_len
    res["synthesize_token_cap"] = args.agent_synth_len
    res["tables"] = {"chunk": {"rows": corpus.n, "index": index.table.index_kind},
                     **{sc: {"rows_this_shard": store.table(sc).count()} for sc in ("repo", "module", "file")}}
    res["question_mix"] = "1/2 code (code scope), 1/2 project overview (project -> package -> file)"
    res["front_door"] = "single process" if world == 1 else (
        f"front door + {world} sharded replicas" if tp is None else
        f"front door + {dp_size} TP-{tp.size} job replicas + {world - dp_size} shard-only replicas, {world} shards")
    return res


if __name__ == "__main__":
    main()
