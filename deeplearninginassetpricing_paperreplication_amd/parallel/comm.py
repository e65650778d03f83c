"""Process-group plumbing for the multi-GPU drivers (one process per GPU).

``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm: collectives run over xGMI between
the GPUs of a node. Every message of this workload is small (KB-MB: weights [T, N] per model,
metric tables), so the drivers issue ONE collective per payload (a padded all-gather of a
stacked tensor), never one per model. Without a GPU (tests, CPU plumbing) the same code runs
on ``gloo``.

Launch: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m <driver> ...``; a driver
calls ``init()`` and gets a ``Dist`` context (single-process when WORLD_SIZE is unset).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as tdist


@dataclass
class Dist:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def active(self) -> bool:
        return self.world > 1 and tdist.is_available() and tdist.is_initialized()

    def comm_device(self) -> torch.device:
        """Where collective buffers must live (RCCL: the rank's GPU; gloo: host)."""
        return self.device if self.backend == "nccl" else torch.device("cpu")


def init(backend: Optional[str] = None, timeout_s: float = 600.0, use_gpu: Optional[bool] = None) -> Dist:
    """Initialise from torchrun-style env vars. ``timeout_s`` bounds every collective, so a
    rank that died turns into an error on its peers instead of a hang."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if use_gpu and os.environ.get("DLAP_SHARE_GPU", "0") == "1":
        # rehearsal of a multi-rank job on fewer GPUs (with DLAP_DIST_BACKEND=gloo: RCCL
        # refuses two ranks on one device)
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    if world <= 1:
        return Dist(0, 1, 0, "none", dev)
    backend = backend or os.environ.get("DLAP_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not tdist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        tdist.init_process_group(**kw)
    return Dist(rank, world, local, backend, dev)


def shutdown(d: Dist):
    if d.active:
        tdist.barrier()
        tdist.destroy_process_group()


def shard(n: int, rank: int, world: int) -> List[int]:
    """Round-robin item indices of ``rank`` (9 seeds over 8 ranks: rank 0 gets 2)."""
    return list(range(rank, n, world))


def barrier(d: Dist):
    if d.active:
        tdist.barrier()


def assign_lpt(costs: Sequence[float], world: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of items with the given costs to ``world``
    ranks: items in decreasing cost (ties by index) each go to the least-loaded rank (ties by
    rank). Deterministic, so every rank computes the same table without a collective. Each
    rank's list is in increasing item order."""
    load = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda k: (-float(costs[k]), k)):
        r = min(range(world), key=lambda q: (load[q], q))
        out[r].append(i)
        load[r] += float(costs[i])
    return [sorted(x) for x in out]


def all_gather_rows(d: Dist, local: np.ndarray, n_total: int, owner_index: Sequence[int],
                    assignment: Optional[Sequence[Sequence[int]]] = None) -> np.ndarray:
    """Gather per-item rows from all ranks into item order.

    ``local`` is [n_local, ...] for the items ``owner_index`` of this rank; ``assignment``
    (per rank, the item indices it owns; default the round-robin ``shard``) tells where every
    rank's rows go. Returns [n_total, ...] on every rank. One padded all-gather of a single
    stacked tensor (plus nothing else: counts follow from the assignment).
    """
    local = np.ascontiguousarray(local)
    if not d.active:
        out = np.empty((n_total,) + local.shape[1:], local.dtype)
        out[list(owner_index)] = local
        return out
    owners = [list(a) for a in assignment] if assignment is not None else \
        [shard(n_total, r, d.world) for r in range(d.world)]
    per = [len(x) for x in owners]
    cap = max(per)
    pad = np.zeros((cap,) + local.shape[1:], local.dtype)
    pad[:len(local)] = local
    dev = d.comm_device()
    t = torch.from_numpy(pad).to(dev)
    bufs = torch.empty((d.world * cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    tdist.all_gather_into_tensor(bufs, t)          # concatenated along dim 0 (RCCL and gloo)
    g = bufs.cpu().numpy().reshape((d.world, cap) + local.shape[1:])
    out = np.empty((n_total,) + local.shape[1:], local.dtype)
    for r in range(d.world):
        idx = owners[r]
        out[idx] = g[r, :len(idx)]
    return out


def all_gather_rows_tensor(d: Dist, local: torch.Tensor, n_total: int, owner_index: Sequence[int],
                           assignment: Optional[Sequence[Sequence[int]]] = None) -> torch.Tensor:
    """``all_gather_rows`` for a torch tensor that stays on the collective device (the rank's
    GPU under RCCL): the result [n_total, ...] is not copied to the host."""
    dev = d.comm_device() if d.active else local.device
    local = local.to(dev).contiguous()
    if not d.active:
        out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
        out[list(owner_index)] = local
        return out
    owners = [list(a) for a in assignment] if assignment is not None else \
        [shard(n_total, r, d.world) for r in range(d.world)]
    cap = max(len(x) for x in owners)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[:len(local)] = local
    bufs = torch.empty((d.world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    tdist.all_gather_into_tensor(bufs, pad)
    g = bufs.reshape((d.world, cap) + tuple(local.shape[1:]))
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    for r in range(d.world):
        if owners[r]:
            out[owners[r]] = g[r, :len(owners[r])]
    return out


def broadcast_arrays(d: Dist, arrays: Optional[dict], src: int = 0, as_tensors: bool = False) -> dict:
    """Broadcast a dict of numpy arrays from ``src`` (e.g. a panel read once from disk): one
    metadata object broadcast, then one tensor broadcast per array. ``as_tensors`` returns the
    received tensors where they landed (the rank's GPU under RCCL: no host copy on the peers)."""
    if not d.active:
        if as_tensors and arrays is not None:
            return {k: torch.as_tensor(np.ascontiguousarray(v)).to(d.comm_device()) for k, v in arrays.items()}
        return arrays
    meta = [None]
    if d.rank == src:
        meta = [{k: (v.shape, str(v.dtype)) for k, v in arrays.items()}]
    tdist.broadcast_object_list(meta, src=src)
    dev = d.comm_device()
    out = {}
    for k, (shape, dt) in meta[0].items():
        if d.rank == src:
            t = torch.from_numpy(np.ascontiguousarray(arrays[k])).to(dev)
        else:
            t = torch.empty(shape, dtype=torch.from_numpy(np.empty(0, np.dtype(dt))).dtype, device=dev)
        tdist.broadcast(t, src=src)
        out[k] = t if as_tensors else t.cpu().numpy()
    return out


def broadcast_batches(d: Dist, batches: Optional[dict], src: int = 0) -> dict:
    """Split dicts ``{split: {key: array/tensor}}`` held on ``src`` only, delivered to every
    rank as tensors on its collective device: one metadata broadcast, then one RCCL broadcast
    per array over xGMI. A tensor already on ``src``'s collective device (a panel generated or
    loaded on its GPU) is broadcast in place -- no host round trip on any rank."""
    if not d.active:
        return batches
    meta = [None]
    if d.rank == src:
        meta = [{f"{sp}/{k}": (tuple(v.shape), str(v.dtype).replace("torch.", "") if isinstance(v, torch.Tensor)
                               else str(np.asarray(v).dtype))
                 for sp, b in batches.items() for k, v in b.items() if v is not None}]
    tdist.broadcast_object_list(meta, src=src)
    dev = d.comm_device()
    out: dict = {}
    for key, (shape, dt) in meta[0].items():
        sp, k = key.split("/", 1)
        if d.rank == src:
            v = batches[sp][k]
            t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
            t = t.to(dev).contiguous()
        else:
            tdt = getattr(torch, dt) if hasattr(torch, dt) else torch.from_numpy(np.empty(0, np.dtype(dt))).dtype
            t = torch.empty(shape, dtype=tdt, device=dev)
        tdist.broadcast(t, src=src)
        out.setdefault(sp, {})[k] = t
    return out
