"""Multi-GPU self-play: one process per GPU, games sharded by id, and one
exchange -- an all-gather of the finished games' (s, pi, z) records -- over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the
CPU tests).

Sharding: rank r, slot s plays game ids  r*n_slots + s + g*(world*n_slots),
g = 0, 1, ...  -- disjoint across ranks, identical to a single-GPU run of the
same ids (every game's RNG streams depend only on its id).
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from .boards import RECORD_DTYPE


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def local_device():
    """GPU of this rank: LOCAL_RANK (one process per GPU).  GZ_DIST_SAME_DEVICE=1 puts
    every rank on GPU 0 -- a rehearsal of the multi-rank path on a one-GPU box, with
    GZ_DIST_BACKEND=gloo (RCCL refuses two ranks on one device)."""
    if os.environ.get("GZ_DIST_SAME_DEVICE") == "1":
        return 0
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env vars (no-op for WORLD_SIZE=1).
    Backend: `backend`, else GZ_DIST_BACKEND, else nccl (= RCCL) with a GPU, gloo without."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 or dist.is_initialized():
        return world()
    if backend is None:
        backend = os.environ.get("GZ_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device())
    dist.init_process_group(backend=backend)
    return world()


def shard_ids(rank, world_size, n_slots):
    """(game_id_base, game_id_stride) for SelfPlayEngine on this rank."""
    return rank * n_slots, world_size * n_slots


def all_gather_records(rec_bytes, count, group=None):
    """All-gather variable-length record buffers.

    rec_bytes: uint8 tensor (device for nccl, cpu for gloo) holding >= count
    records of RECORD_DTYPE.  Returns one uint8 tensor with every rank's
    records, rank-major.  Two collectives: the counts, then the padded payload
    (all_gather_into_tensor).
    """
    rank, ws = world()
    item = RECORD_DTYPE.itemsize
    dev = rec_bytes.device
    if ws == 1:
        return rec_bytes[: count * item]
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    cnts = torch.zeros(ws, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(cnts, cnt, group=group)
    counts = [int(x) for x in cnts.cpu()]
    mx = max(counts)
    send = torch.zeros(max(1, mx) * item, dtype=torch.uint8, device=dev)
    if count:
        send[: count * item] = rec_bytes[: count * item]
    recv = torch.zeros(ws * send.numel(), dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(recv, send, group=group)
    parts = [recv[r * send.numel(): r * send.numel() + counts[r] * item] for r in range(ws)]
    return torch.cat(parts)


def to_records(t):
    return np.frombuffer(t.cpu().numpy().tobytes(), RECORD_DTYPE)
