"""Multi-process CPU harness for the distributed paths (gloo backend,
127.0.0.1 rendezvous): ``run_ranks(fn, world, *args)`` spawns ``world``
processes that each call ``fn(rank, world, *args)`` after init_distributed and
returns the list of per-rank results (pickled through a queue)."""
from __future__ import annotations

import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, q):
    try:
        os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        import torch.distributed as dist

        from githubrepostorag_amd.parallel import comm

        comm.init_distributed(backend="gloo", timeout_s=120)
        try:
            q.put((rank, fn(rank, world, *args), None))
        finally:
            dist.destroy_process_group()
    except Exception:  # surfaced in the parent
        q.put((rank, None, traceback.format_exc()))


def run_ranks(fn, world: int, *args, timeout: float = 240.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [None] * world
    errs = []
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=timeout)
            out[rank] = res
            if err:
                errs.append(f"rank {rank}:\n{err}")
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errs:
        raise AssertionError("\n".join(errs))
    return out
