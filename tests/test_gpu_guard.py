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
