"""The capture guard (utils/gpu_guard.py): shared sections run together, a capture (exclusive) runs alone,
and a thread inside a shared section -- the engine thread for its whole step -- can take the capture
guard for a lazy capture without deadlocking against another thread doing the same."""
import threading
import time

from githubrepostorag_amd.utils.gpu_guard import _CaptureGuard


def _run(threads, timeout=10.0):
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
    assert not any(t.is_alive() for t in threads), "guard deadlocked"


def test_shared_sections_overlap_and_exclusive_runs_alone():
    g = _CaptureGuard()
    inside = []
    peak = [0, 0]  # readers at once, readers seen during a writer
    lock = threading.Lock()

    def reader():
        for _ in range(50):
            with g.shared():
                with lock:
                    inside.append("r")
                    peak[0] = max(peak[0], inside.count("r"))
                    peak[1] += "w" in inside
                time.sleep(0.0005)
                with lock:
                    inside.remove("r")

    def writer():
        for _ in range(20):
            with g.exclusive():
                with lock:
                    assert not inside, inside
                    inside.append("w")
                time.sleep(0.0005)
                with lock:
                    inside.remove("w")

    _run([threading.Thread(target=reader) for _ in range(3)] + [threading.Thread(target=writer)])
    assert peak[1] == 0


def test_upgrade_from_shared_section():
    """Two threads each inside a shared section take the capture guard (the engine thread's lazy decode
    capture, a retrieval thread's encoder-bucket capture): both finish, never together, and each is back
    in its shared section afterwards (a third thread's capture still excludes it)."""
    g = _CaptureGuard()
    state = {"writers": 0, "max": 0, "back": 0}
    lock = threading.Lock()

    def upgrader():
        for _ in range(30):
            with g.shared():
                with g.exclusive():
                    with lock:
                        state["writers"] += 1
                        state["max"] = max(state["max"], state["writers"])
                    time.sleep(0.0003)
                    with lock:
                        state["writers"] -= 1
                with g.shared():  # re-entrant after the upgrade
                    pass
                with lock:
                    state["back"] += g._readers >= 1

    _run([threading.Thread(target=upgrader) for _ in range(2)])
    assert state["max"] == 1
    assert state["back"] == 60
    assert g._readers == 0 and g._writer is None and g._waiting == 0


def test_writer_waits_for_a_shared_step():
    g = _CaptureGuard()
    order = []
    in_step = threading.Event()

    def step():
        with g.shared():
            in_step.set()
            time.sleep(0.05)
            order.append("step done")

    def capture():
        in_step.wait()
        with g.exclusive():
            order.append("capture")

    _run([threading.Thread(target=step), threading.Thread(target=capture)])
    assert order == ["step done", "capture"]


def _lazy_capture_beside_search(rank, world):
    """One rank of test_lazy_capture_during_cross_rank_search_does_not_deadlock: the engine thread steps
    under the shared guard with a TP collective per step and, at a rank-dependent step, runs the engine's
    real capture path (LLMEngine._capture_ws: warm-up step with its TP collective, then the exclusive
    capture); the retrieval thread runs a cross-rank search collective on another group inside the shared
    guard, as the bench's pump and the service's shard rounds do."""
    import torch
    import torch.distributed as dist

    from githubrepostorag_amd.engine.llm_engine import LLMEngine
    from githubrepostorag_amd.utils.gpu_guard import gpu_shared

    tp = dist.new_group(list(range(world)))
    idx = dist.new_group(list(range(world)))
    captured = []

    class FakeEngine:
        stats = {"capture_s": 0.0}
        trace = None

        def _capture_prepare(self, B, nsplit, split_len, K, npre=0):
            t = torch.ones(1)
            dist.all_reduce(t, group=tp)  # the warm-up step's TP all-reduce
            return t

        def _capture_locked(self, B, nsplit, split_len, K, prep, npre=0):
            time.sleep(0.01)  # the capture itself: local work only
            captured.append(B)
            return None

    eng = FakeEngine()
    errors = []

    def engine():
        try:
            for i in range(40):
                with gpu_shared():  # LLMEngine.step holds the guard shared
                    t = torch.ones(1)
                    dist.all_reduce(t, group=tp)
                    if i in (7 + 5 * rank, 20):  # lazy captures at steps that differ between the ranks
                        LLMEngine._capture_ws(eng, 8 + i, 1, 128, 1)
        except BaseException as e:
            errors.append(e)

    def pump():
        try:
            for _ in range(60):
                with gpu_shared():  # a sharded search: collective inside the shared section
                    t = torch.ones(4)
                    dist.all_reduce(t, group=idx)
                time.sleep(0.001 * (1 + rank))
        except BaseException as e:
            errors.append(e)

    th = [threading.Thread(target=engine), threading.Thread(target=pump)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    if any(t.is_alive() for t in th):
        return "deadlock"
    if errors:
        raise errors[0]
    return len(captured)


def test_lazy_capture_during_cross_rank_search_does_not_deadlock():
    """a lazy decode capture used to run its eager warm-up step (real TP collectives) inside the
    exclusive guard, while the retrieval thread held the shared guard across a cross-rank search; two
    ranks could then wait on each other for ever.  The warm-up now runs under the shared guard, the
    exclusive section is local."""
    from tests.dist_utils import run_ranks

    assert run_ranks(_lazy_capture_beside_search, 2, timeout=150) == [2, 2]
