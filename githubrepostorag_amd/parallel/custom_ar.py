"""One-shot all-reduce over IPC-mapped peer buffers (csrc/kernels/allreduce.hip).

SURVEY §2.8 C1: the TP all-reduce after o_proj / down_proj is latency-bound at
decode ([B, hidden] bf16: 7 KB per row for Qwen2-7B, 16 KB for 72B).  xGMI is
point-to-point (7 links per MI355X), so a ring all-reduce pays 2(W-1)
dependent hops on one link per direction; the one-shot kernel has every rank
read all W-1 peers' copies directly — all links at once, one signal round.
Large messages (prefill) stay on RCCL.

Setup (collective over the TP group): every rank allocates one uncached
region (flags + two data slots), exports it with hipIpcGetMemHandle, the
64-byte handles are all-gathered through torch.distributed (any backend),
and every rank opens its peers' regions.  A self-check against the process
group's all-reduce runs before the communicator is used.

``IpcAllReduce.simulated(W, device)`` builds W "ranks" inside one process
(no IPC) — the kernel protocol (epochs, double buffering, flags) is tested
on one GPU by running the W ranks' launches concurrently on W streams.
"""
from __future__ import annotations

import ctypes
import logging
import os

import torch

from ..ops._lib import check, lib, ptr

log = logging.getLogger(__name__)

P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
_SIGS = {
    "grag_ar_data_offset": ([], L), "grag_ar_region_bytes": ([L], L), "grag_ar_alloc": ([L, P], I),
    "grag_ar_free": ([P], I), "grag_ar_get_handle": ([P, P], I), "grag_ar_handle_size": ([], I),
    "grag_ar_open_handle": ([P, P], I), "grag_ar_close_handle": ([P], I),
    "grag_ar_oneshot": ([P, I, I, P, P, L, L, P, P, I, L, P], I),
    "grag_ar_oneshot_op": ([P, I, I, I, P, P, L, L, P, P, I, L, P], I),
}
OP_SUM_F32, OP_GATHER = 1, 2
MAX_RANKS = 8


def _fn(name):
    f = getattr(lib(), name)
    args, res = _SIGS[name]
    f.argtypes, f.restype = args, res
    return f


def _alloc(nbytes: int) -> int:
    p = ctypes.c_void_p()
    check(_fn("grag_ar_alloc")(nbytes, ctypes.byref(p)), "grag_ar_alloc")
    return p.value


TIMEOUT_S = float(os.environ.get("GRAG_AR_TIMEOUT_S", "5"))  # a peer slower than this fails the exchange
TICKS_PER_S = 100_000_000  # s_memrealtime: 100 MHz


class IpcAllReduce:
    def __init__(self, regions: list[int], rank: int, device, slot_bytes: int, owned: list[int],
                 opened: list[int], grid: int = 64, timeout_s: float | None = None):
        self.regions = regions
        self.W = len(regions)
        self.rank = rank
        self.device = torch.device(device)
        self.slot_bytes = slot_bytes
        self.grid = grid
        # the kernel's wait bound in s_memrealtime ticks (csrc/kernels/allreduce.hip: wall time, then the
        # error word is set and the step raises CommError -> the TP group detaches to RCCL together)
        self.spin_max = int((TIMEOUT_S if timeout_s is None else timeout_s) * TICKS_PER_S)
        self._owned, self._opened = owned, opened
        self._arr = (ctypes.c_void_p * self.W)(*regions)
        self.epochs = torch.zeros(grid, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # host mirror of `err`, refreshed asynchronously once per engine step
        # (stage_error_check) and read after the step's token sync (raise_if_failed)
        self._host_err = torch.zeros(1, dtype=torch.int32, pin_memory=self.device.type == "cuda")

    # ------------------------------------------------------------------ setup
    @classmethod
    def create(cls, pg, rank: int, world: int, device, slot_bytes: int = 8 << 20, grid: int = 64):
        """Collective over ``pg`` (torch.distributed group): allocate, export,
        exchange and open the IPC regions of all ``world`` ranks."""
        import torch.distributed as dist

        assert 1 < world <= MAX_RANKS
        region_bytes = int(_fn("grag_ar_region_bytes")(slot_bytes))
        base = _alloc(region_bytes)
        hs = int(_fn("grag_ar_handle_size")())
        buf = ctypes.create_string_buffer(hs)
        check(_fn("grag_ar_get_handle")(base, buf), "grag_ar_get_handle")
        handles = [None] * world
        dist.all_gather_object(handles, bytes(buf.raw), group=pg)
        regions, opened = [], []
        for r, h in enumerate(handles):
            if r == rank:
                regions.append(base)
                continue
            p = ctypes.c_void_p()
            check(_fn("grag_ar_open_handle")(ctypes.create_string_buffer(h, hs), ctypes.byref(p)),
                  "grag_ar_open_handle")
            regions.append(p.value)
            opened.append(p.value)
        dist.barrier(group=pg)
        return cls(regions, rank, device, slot_bytes, [base], opened, grid)

    @classmethod
    def simulated(cls, world: int, device, slot_bytes: int = 1 << 20, grid: int = 64) -> list["IpcAllReduce"]:
        """W communicators over W regions of ONE process (no IPC): rank r's
        launches must run concurrently with the others' (separate streams)."""
        region_bytes = int(_fn("grag_ar_region_bytes")(slot_bytes))
        regions = [_alloc(region_bytes) for _ in range(world)]
        comms = [cls(regions, r, device, slot_bytes, [], [], grid) for r in range(world)]
        comms[0]._owned = list(regions)  # one owner frees them all
        return comms

    def close(self) -> None:
        for p in self._opened:
            _fn("grag_ar_close_handle")(p)
        for p in self._owned:
            _fn("grag_ar_free")(p)
        self._opened, self._owned = [], []

    # ------------------------------------------------------------------ op
    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
                and t.numel() * 2 <= self.slot_bytes)

    def all_reduce(self, t: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """Sum over ranks (in place by default); bf16, contiguous, <= slot_bytes."""
        if not self.fits(t):
            raise ValueError("tensor does not fit the one-shot all-reduce buffer")
        out = t if out is None else out
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = _fn("grag_ar_oneshot")(self._arr, self.W, self.rank, ptr(t), ptr(out), t.numel(), self.slot_bytes,
                                    ptr(self.epochs), ptr(self.err), self.grid, self.spin_max, s.cuda_stream)
        check(rc, "grag_ar_oneshot")
        return out

    def fits_bytes(self, t: torch.Tensor) -> bool:
        nb = t.numel() * t.element_size()
        return t.is_cuda and t.is_contiguous() and nb % 16 == 0 and 0 < nb <= self.slot_bytes

    def all_reduce_f32(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        """fp32 sum over ranks, in place (rank-order accumulation: bit-identical on every rank)."""
        if t.dtype != torch.float32 or not self.fits_bytes(t):
            raise ValueError("tensor does not fit the one-shot fp32 all-reduce")
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = _fn("grag_ar_oneshot_op")(self._arr, self.W, self.rank, OP_SUM_F32, ptr(t), ptr(t),
                                       t.numel() * 4, self.slot_bytes, ptr(self.epochs), ptr(self.err), self.grid,
                                       self.spin_max, s.cuda_stream)
        check(rc, "grag_ar_oneshot_op(sum_f32)")
        return t

    def all_gather(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        """[...] -> [W, ...] (rank order), any dtype; the bytes per rank a multiple of 16."""
        if not self.fits_bytes(t):
            raise ValueError("tensor does not fit the one-shot all-gather")
        out = torch.empty((self.W, *t.shape), dtype=t.dtype, device=t.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = _fn("grag_ar_oneshot_op")(self._arr, self.W, self.rank, OP_GATHER, ptr(t), ptr(out),
                                       t.numel() * t.element_size(), self.slot_bytes, ptr(self.epochs),
                                       ptr(self.err), self.grid, self.spin_max, s.cuda_stream)
        check(rc, "grag_ar_oneshot_op(gather)")
        return out

    def failed(self) -> bool:
        return bool(self.err.item())

    # A spin that times out inside the kernel sets `err` and leaves `out`
    # holding only the local partial sum, so a stalled peer must surface as an
    # error, not as silently wrong logits.  The engine queues the err copy
    # before its per-step token sync and checks it right after (no extra sync).
    def stage_error_check(self, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):
            self._host_err.copy_(self.err, non_blocking=True)

    def raise_if_failed(self) -> None:
        """Call after the stream that ran stage_error_check() was synchronised."""
        if int(self._host_err[0]) != 0:
            raise CommError(f"one-shot all-reduce timed out waiting for a peer (rank {self.rank} of {self.W}); "
                            "outputs of this step are invalid")

    def reset_error(self) -> None:
        self.err.zero_()
        self._host_err.zero_()


class CommError(RuntimeError):
    """A collective failed on device (peer stalled / timed out)."""


def enable_for_group(group, device) -> IpcAllReduce | None:
    """Attach a one-shot all-reduce to a TP ``parallel.comm.Group`` on GPU
    (GRAG_CUSTOM_AR=0 disables).  Verified against the group's RCCL
    all-reduce before use; any failure leaves the group on RCCL."""
    if group.trivial or os.environ.get("GRAG_CUSTOM_AR", "1") == "0" or group.size > MAX_RANKS:
        return None
    dev = torch.device(device)
    if dev.type != "cuda":
        return None
    import torch.distributed as dist

    # ranks sharing ONE device (a single-GPU rehearsal of a TP group): W spinning exchange kernels from W
    # processes on one card depend on the hardware scheduler mapping every process's queue at once; past
    # GRAG_CUSTOM_AR_SHARED_MAX ranks per device (default 2: the tested TP=2 rehearsal) the group stays on
    # its process-group collectives.  One process per GPU (the 8-GPU node) is unaffected.
    p = torch.cuda.get_device_properties(dev)
    ident = f"{p.pci_domain_id}:{p.pci_bus_id}:{p.pci_device_id}:{p.uuid}"
    ids = [None] * group.size
    dist.all_gather_object(ids, ident, group=group.pg)
    shared = max(ids.count(i) for i in ids)
    if shared > int(os.environ.get("GRAG_CUSTOM_AR_SHARED_MAX", "2")):
        log.warning("%d TP ranks share one device: one-shot all-reduce off (process-group collectives)", shared)
        return None
    try:
        ar = IpcAllReduce.create(group.pg, group.rank, group.size, dev)
        g = torch.Generator(device=dev).manual_seed(1234 + group.rank)
        x = torch.randn(4096, generator=g, device=dev).to(torch.bfloat16)
        cdev = group.ctrl_device(dev)  # RCCL: on the GPU; gloo (shared-GPU rehearsal): on the host
        ref = x.float().to(cdev)
        dist.all_reduce(ref, group=group.pg)
        got = ar.all_reduce(x.clone())
        # the sampler's exchanges: fp32 sum and all-gather over the same communicator
        y = torch.arange(64, dtype=torch.float32, device=dev) + group.rank
        ys = ar.all_reduce_f32(y.clone())
        yg = ar.all_gather(y)
        want_s = sum(torch.arange(64, dtype=torch.float32) + r for r in range(group.size))
        good = (not ar.failed() and torch.allclose(got.float().cpu(), ref.cpu(), atol=0.1, rtol=0.02)
                and torch.equal(ys.cpu(), want_s)
                and all(torch.equal(yg[r].cpu(), torch.arange(64, dtype=torch.float32) + r) for r in range(group.size)))
        ok = torch.tensor([1 if good else 0], device=cdev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group.pg)
        if int(ok.item()) != 1:
            log.warning("one-shot all-reduce self-check failed; staying on RCCL")
            ar.close()
            return None
        group.custom_ar = ar
        return ar
    except Exception as e:  # IPC unavailable (e.g. legacy IPC mode): RCCL only
        log.warning("one-shot all-reduce unavailable (%s); staying on RCCL", e)
        return None
