"""Process groups and collectives.

One process per GPU; ``torch.distributed`` with backend ``"nccl"`` is RCCL on
ROCm (collectives over xGMI), ``"gloo"`` is the CPU fallback used by the
multi-process CPU tests.  The reference has no collectives at all (SURVEY
§2.8); the ones here are introduced by the MI355X design:

* C1  TP all-reduce of row-parallel projections (Qwen2 o_proj / down_proj)
* C2  TP all-gather of vocab-parallel LM-head logits
* C3  DP all-gather of per-shard top-k lists for the sharded vector index
* C5  all-gather of scalar counts (ingest id assignment)
* C6  all-reduce of k-means centroid sums/counts (IVF training across shards)

xGMI is point-to-point (7 links per GPU), so small latency-bound messages
(decode all-reduce [B, hidden], top-k lists of a few KB) are issued as single
fused collectives per step rather than many small ones.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


_INFO = DistInfo()


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def init_distributed(backend: str | None = None, timeout_s: int = 600) -> DistInfo:
    """Initialise the default process group from torchrun-style env vars.
    Single-process runs get a trivial DistInfo and no process group."""
    global _INFO
    rank, world, local = env_world()
    if world <= 1:
        _INFO = DistInfo(0, 1, local, "none")
        if torch.cuda.is_available():
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        return _INFO
    if backend is None:
        # GRAG_DIST_BACKEND=gloo: rehearse a multi-rank run with every rank on one shared GPU (RCCL refuses
        # two ranks on one device); ranks then map to devices local % device_count
        backend = os.environ.get("GRAG_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
    if backend != "nccl" and torch.cuda.is_available():
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
    _INFO = DistInfo(rank, world, local, backend)
    return _INFO


def info() -> DistInfo:
    return _INFO


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if _INFO.backend == "nccl":
            dist.barrier(device_ids=[_INFO.local_rank])
        else:
            dist.barrier()


class Group:
    """A (possibly trivial) communicator over a subset of ranks."""

    def __init__(self, ranks: list[int] | None = None, pg=None):
        self.ranks = ranks or [0]
        self.pg = pg
        self.size = len(self.ranks)
        me = _INFO.rank
        self.rank = self.ranks.index(me) if me in self.ranks else 0

    @property
    def trivial(self) -> bool:
        return self.size == 1

    custom_ar = None  # parallel.custom_ar.IpcAllReduce: one-shot xGMI all-reduce for small messages

    @property
    def capturable(self) -> bool:
        """Whether this group's decode-time collectives can live inside a hipGraph: RCCL or the one-shot IPC
        kernels can; gloo (host-staged, the shared-GPU rehearsal) cannot."""
        return self.trivial or self.custom_ar is not None or _INFO.backend == "nccl"

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """C1: small bf16 messages (decode [B, hidden]) and small fp32 ones (the
        TP sampler's histograms) take the one-shot IPC all-reduce when attached;
        everything else goes to RCCL / gloo."""
        if not self.trivial:
            ar = self.custom_ar
            if ar is not None:
                if ar.fits(t):
                    return ar.all_reduce(t)
                if t.dtype == torch.float32 and ar.fits_bytes(t):
                    return ar.all_reduce_f32(t)
            _gloo_staged(lambda x: dist.all_reduce(x, group=self.pg), t)
        return t

    def stage_health(self) -> None:
        """Queue the device-side error word of the attached one-shot all-reduce
        for readback (before the engine's per-step token sync)."""
        ar = self.custom_ar
        if ar is not None:
            ar.stage_error_check()

    def check_health(self) -> None:
        """After the step's sync: raise ``CommError`` if a one-shot all-reduce
        of this step timed out on a peer.  The detach is NOT decided here: one
        rank's error word says nothing about its peers, and a rank that went
        back to RCCL alone would meet its peers' IPC kernels in the next
        collective.  The engine runner counts the error in its next control
        all-reduce and every rank calls ``detach_custom_ar`` at that same
        iteration (engine/runner.py)."""
        ar = self.custom_ar
        if ar is not None:
            ar.raise_if_failed()

    def detach_custom_ar(self) -> bool:
        """Leave the one-shot all-reduce for RCCL (every rank of the group at the
        same iteration; decode graphs that captured the IPC kernel must be
        dropped by the caller).  The IPC regions stay mapped: graphs or peers
        may still hold their addresses until they are gone."""
        ar = self.custom_ar
        if ar is None:
            return False
        ar.reset_error()
        self.custom_ar = None
        return True

    def ctrl_device(self, device=None):
        """Where a small control tensor of this group lives (RCCL: the GPU, gloo: the host)."""
        if device is not None and torch.device(device).type == "cuda" and _INFO.backend == "nccl":
            return torch.device(device)
        return torch.device("cpu")

    def agree(self, ok: bool, device=None) -> bool:
        """All ranks learn whether every rank's step succeeded (MIN all-reduce
        of a status word; RCCL needs it on the GPU, gloo on the host)."""
        return bool(self.min_int(1 if ok else 0, device))

    def min_int(self, v: int, device=None) -> int:
        """Group-wide minimum of a host integer (e.g. the planned KV block count:
        replicated scheduling needs identical pools on every TP rank)."""
        if self.trivial:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.ctrl_device(device))
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.pg)
        return int(t.item())

    def all_reduce_host(self, t: torch.Tensor, device=None) -> torch.Tensor:
        """SUM of a small host tensor over the group (through the GPU under RCCL)."""
        if self.trivial:
            return t
        x = t.to(self.ctrl_device(device))
        dist.all_reduce(x, group=self.pg)
        return x.cpu()

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[...] -> [size, ...] (one collective)."""
        if self.trivial:
            return t.unsqueeze(0)
        ar = self.custom_ar
        if ar is not None and t.is_cuda:  # C2 small exchanges: one-shot IPC gather (capturable)
            src = t.contiguous()
            nb = src.numel() * src.element_size()
            if nb % 16 == 0 and ar.fits_bytes(src):
                return ar.all_gather(src)
            nbp = -(-nb // 16) * 16
            if 0 < nbp <= ar.slot_bytes:  # odd sizes (e.g. [1, 2] fp32): padded to 16-byte vectors
                pad = torch.zeros(nbp, dtype=torch.uint8, device=t.device)
                pad[:nb] = src.view(-1).view(torch.uint8)
                g = ar.all_gather(pad)[:, :nb].contiguous()
                return g.view(t.dtype).view(self.size, *t.shape)
        # flat concatenated form: the only layout both RCCL and gloo accept
        src = t.contiguous().view(-1)
        if _INFO.backend == "gloo" and src.is_cuda:  # shared-GPU rehearsal: gloo works on host tensors
            out = torch.empty(self.size * src.numel(), dtype=t.dtype)
            dist.all_gather_into_tensor(out, src.cpu(), group=self.pg)
            return out.to(t.device).view(self.size, *t.shape)
        out = torch.empty(self.size * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, src, group=self.pg)
        return out.view(self.size, *t.shape)

    def all_gather_topk(self, scores: torch.Tensor, ids: torch.Tensor, k: int):
        """C3: merge per-shard top-k lists.  scores fp32 [nq, k], ids int64
        [nq, k] (already global ids) -> global top-k.  Packs both into one
        fp64-sized buffer so the merge is a single all-gather."""
        if self.trivial:
            return scores, ids
        nq = scores.shape[0]
        packed = torch.empty(nq, k, 2, dtype=torch.int64, device=scores.device)
        packed[..., 0] = ids
        packed[..., 1] = scores.float().view(torch.int32).to(torch.int64)
        g = self.all_gather(packed)  # [W, nq, k, 2]
        all_ids = g[..., 0].permute(1, 0, 2).reshape(nq, -1)
        all_s = g[..., 1].to(torch.int32).view(torch.float32).permute(1, 0, 2).reshape(nq, -1)
        s, sel = all_s.topk(min(k, all_s.shape[1]), dim=1)
        return s, all_ids.gather(1, sel)

    def all_to_all(self, t: torch.Tensor) -> torch.Tensor:
        """[size, ...] -> [size, ...]: slice j goes to local rank j; slice i of
        the result came from local rank i (one all_to_all_single)."""
        if self.trivial:
            return t
        if _INFO.backend == "gloo" and t.is_cuda:  # shared-GPU rehearsal: gloo works on host tensors
            h = t.contiguous().cpu()
            out = torch.empty_like(h)
            dist.all_to_all_single(out.view(-1), h.view(-1), group=self.pg)
            return out.to(t.device)
        out = torch.empty_like(t)
        dist.all_to_all_single(out.view(-1), t.contiguous().view(-1), group=self.pg)
        return out

    def broadcast(self, t: torch.Tensor, src_local: int = 0) -> torch.Tensor:
        if not self.trivial:
            _gloo_staged(lambda x: dist.broadcast(x, src=self.ranks[src_local], group=self.pg), t)
        return t


def _gloo_staged(op, t: torch.Tensor) -> None:
    """Run an in-place collective ``op`` on ``t``; under gloo a GPU tensor goes through a host copy
    (the shared-GPU rehearsal: several ranks on one card, where RCCL refuses duplicate devices)."""
    if _INFO.backend == "gloo" and t.is_cuda:
        h = t.cpu()
        op(h)
        t.copy_(h)
    else:
        op(t)


def world_group() -> Group:
    if not _INFO.is_distributed:
        return Group([0])
    return Group(list(range(_INFO.world_size)), pg=dist.group.WORLD)


def make_tp_dp_groups(tp: int) -> tuple[Group, Group]:
    """Split the world into TP groups of `tp` consecutive ranks (share one
    xGMI-connected node) and DP groups of the ranks with the same TP rank.
    Every rank must call this (new_group is collective)."""
    W = _INFO.world_size
    if W == 1:
        return Group([0]), Group([0])
    assert W % tp == 0, f"world {W} not divisible by tp {tp}"
    my_tp = my_dp = None
    for s in range(0, W, tp):
        ranks = list(range(s, s + tp))
        pg = dist.new_group(ranks) if tp > 1 else None
        if _INFO.rank in ranks:
            my_tp = Group(ranks, pg)
    for r in range(tp):
        ranks = list(range(r, W, tp))
        pg = dist.new_group(ranks) if len(ranks) > 1 else None
        if _INFO.rank in ranks:
            my_dp = Group(ranks, pg)
    return my_tp, my_dp
