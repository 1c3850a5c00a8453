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


class RecordExchange:
    """Per-step all-gather of finished games' records with no host synchronisation.

    The engine leaves each step's records in a buffer of ``record_cap`` rows with
    the count on the device (``SelfPlayEngine.d_counters``).  ``push`` appends them
    to a device-resident outbox ring (rows past the count go to a dummy row, so
    the copy has a fixed shape); ``exchange`` all-gathers the oldest
    ``min(pending, chunk)`` rows of every rank as a fixed ``chunk``-row payload plus
    the per-rank counts (two ``all_gather_into_tensor`` calls, RCCL over xGMI) and
    advances the ring.  Nothing reads a count on the host, so a step never waits
    for the GPU; records a burst leaves behind go out in later steps.  ``chunk`` ~
    2x the mean records per step (one record per ply: n_slots x plies_per_step)
    bounds the per-step payload instead of padding to the worst case
    (record_cap = n_slots x 200 rows).  ``overflow`` counts records that found
    the ring full (0 unless the consumer falls behind by a whole ring).
    """

    def __init__(self, record_cap, chunk, device, capacity=None, group=None):
        self.item = RECORD_DTYPE.itemsize
        self.record_cap, self.chunk = int(record_cap), int(chunk)
        self.R = int(capacity) if capacity else self.record_cap + 4 * self.chunk
        self.group = group
        self.rank, self.ws = world()
        dev = torch.device(device)
        self.box = torch.zeros((self.R + 1, self.item), dtype=torch.uint8, device=dev)  # row R = dummy
        self.head = torch.zeros(1, dtype=torch.int64, device=dev)
        self.tail = torch.zeros(1, dtype=torch.int64, device=dev)
        self.overflow = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ar_cap = torch.arange(self.record_cap, dtype=torch.int64, device=dev)
        self.ar_chunk = torch.arange(self.chunk, dtype=torch.int64, device=dev)
        self.recv = torch.zeros((self.ws, self.chunk, self.item), dtype=torch.uint8, device=dev)
        self.recv_counts = torch.zeros(self.ws, dtype=torch.int64, device=dev)

    def push(self, rec_bytes, d_count):
        """Append the first d_count (device int tensor, 1 element) of the record
        rows in rec_bytes (uint8, record_cap x 80 bytes or more) to the outbox."""
        n = d_count.reshape(1).to(torch.int64).clamp(0, self.record_cap)
        free = self.R - (self.tail - self.head)
        k = torch.minimum(n, free)
        self.overflow += n - k
        pos = torch.where(self.ar_cap < k, (self.tail + self.ar_cap) % self.R, self.R)
        src = rec_bytes[: self.record_cap * self.item].view(self.record_cap, self.item)
        self.box.index_copy_(0, pos, src)
        self.tail += k

    def exchange(self):
        """All-gather one chunk per rank -> (recv uint8 [ws, chunk, 80], counts int64 [ws]),
        both on the device; rank r's valid rows are recv[r, :counts[r]]."""
        cnt = torch.minimum(self.tail - self.head, torch.full_like(self.head, self.chunk))
        pos = torch.where(self.ar_chunk < cnt, (self.head + self.ar_chunk) % self.R, self.R)
        # zero padding rows (the dummy row is scratch); a multiply, not a masked
        # assignment, which would synchronise on the mask's nonzero count
        send = self.box.index_select(0, pos) * (self.ar_chunk < cnt).to(torch.uint8)[:, None]
        if self.ws > 1:
            dist.all_gather_into_tensor(self.recv.view(-1), send.view(-1), group=self.group)
            dist.all_gather_into_tensor(self.recv_counts, cnt, group=self.group)
        else:
            self.recv[0].copy_(send)
            self.recv_counts.copy_(cnt)
        self.head += cnt
        return self.recv, self.recv_counts

    def pending(self):
        """Records pushed but not yet exchanged (device tensor)."""
        return self.tail - self.head


def chunks_to_records(recv, counts):
    """Host view of one exchange: every rank's valid rows, rank-major (synchronises)."""
    c = counts.cpu().numpy()
    raw = recv.cpu().numpy()
    return np.concatenate([np.frombuffer(raw[r, : int(c[r])].tobytes(), RECORD_DTYPE) for r in range(len(c))])


def to_records(t):
    return np.frombuffer(t.cpu().numpy().tobytes(), RECORD_DTYPE)
