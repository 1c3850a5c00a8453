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

    def __init__(self, record_cap, chunk, device, capacity=None, group=None, max_push=None):
        self.item = RECORD_DTYPE.itemsize
        self.record_cap, self.chunk = int(record_cap), int(chunk)
        # rows a push copies (a fixed shape): every row of the engine's buffer by
        # default (lossless); a bound below that counts the excess as overflow
        self.max_push = min(self.record_cap, int(max_push)) if max_push else self.record_cap
        self.R = int(capacity) if capacity else self.max_push + 4 * self.chunk
        self.group = group
        self.rank, self.ws = world()
        dev = torch.device(device)
        # rows R .. R + max_push - 1: scratch for the copied rows past the count (one
        # row each, so the fixed-shape copy never piles writes onto one row)
        self.box = torch.zeros((self.R + self.max_push, self.item), dtype=torch.uint8, device=dev)
        self.head = torch.zeros(1, dtype=torch.int64, device=dev)
        self.tail = torch.zeros(1, dtype=torch.int64, device=dev)
        self.overflow = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ar_cap = torch.arange(self.max_push, dtype=torch.int64, device=dev)
        self.ar_chunk = torch.arange(self.chunk, dtype=torch.int64, device=dev)
        self.recv = torch.zeros((self.ws, self.chunk, self.item), dtype=torch.uint8, device=dev)
        self.recv_counts = torch.zeros(self.ws, dtype=torch.int64, device=dev)

    def push(self, rec_bytes, d_count):
        """Append the first d_count (device int tensor, 1 element) of the record
        rows in rec_bytes (uint8, record_cap x 80 bytes or more) to the outbox."""
        n = d_count.reshape(1).to(torch.int64).clamp(0, self.record_cap)
        free = self.R - (self.tail - self.head)
        k = torch.minimum(torch.minimum(n, free), torch.full_like(n, self.max_push))
        self.overflow += n - k
        pos = torch.where(self.ar_cap < k, (self.tail + self.ar_cap) % self.R, self.R + self.ar_cap)
        src = rec_bytes[: self.max_push * self.item].view(self.max_push, self.item)
        self.box.index_copy_(0, pos, src)
        self.tail += k

    def exchange(self):
        """All-gather one chunk per rank -> (recv uint8 [ws, chunk, 80], counts int64 [ws]),
        both on the device; rank r's valid rows are recv[r, :counts[r]].  The two tensors
        are this object's own buffers, overwritten by the next exchange(): consume them
        (ReplayCollector.absorb, chunks_to_records) or clone them before then."""
        cnt = torch.minimum(self.tail - self.head, torch.full_like(self.head, self.chunk))
        pos = torch.where(self.ar_chunk < cnt, (self.head + self.ar_chunk) % self.R, self.R + self.ar_chunk % self.max_push)
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


class ReplayCollector:
    """Every rank's copy of one self-play iteration's replay, built on the device from
    the per-step RecordExchange chunks.  ``absorb`` itself never synchronises; its
    caller decides when to read ``games`` (training.selfplay_device reads it once per
    step, in the same device-to-host copy as the engine's counters and the loss
    counters).

    ``absorb`` appends the rows of all ranks whose game id lies in [id_lo, id_hi) --
    the iteration's games; the engines' continuous refill plays on past them and
    those rows are dropped -- to a device buffer and counts the finished games (one
    ply-0 row per game).  With ``per_rank`` = G, a row sent by rank r is kept only
    if its id lies in rank r's own share [id_lo + r G, id_lo + (r + 1) G): an
    engine refills a slot with id + n_slots, so rank r's refill games carry rank
    r + 1's ids (the same games, replayed from the same id-keyed RNG streams) and
    must not be counted twice.  Every rank absorbs the same chunks, so every rank's
    buffer, count and finish decision agree without another collective.
    ``records`` sorts the rows by (game id, ply): the union of the ranks' games in
    id order, which is the order the reference's replay has (training.py:377-395:
    games in play order, each game's plies in order)."""

    def __init__(self, capacity, id_lo, id_hi, device, per_rank=None):
        self.item = RECORD_DTYPE.itemsize
        self.cap = int(capacity)
        self.id_lo, self.id_hi = int(id_lo), int(id_hi)
        self.per_rank = int(per_rank) if per_rank else None
        dev = torch.device(device)
        self.buf = torch.zeros((self.cap + 1, self.item), dtype=torch.uint8, device=dev)  # row cap = dummy
        self.n = torch.zeros(1, dtype=torch.int64, device=dev)
        self.games = torch.zeros(1, dtype=torch.int64, device=dev)
        self.dropped = torch.zeros(1, dtype=torch.int64, device=dev)

    def absorb(self, recv, counts):
        ws, chunk, item = recv.shape
        rows = recv.reshape(ws * chunk, item)
        gid = rows[:, 64:72].contiguous().view(torch.int64).reshape(-1)
        ply = rows[:, 72:74].contiguous().view(torch.int16).reshape(-1)
        valid = (torch.arange(chunk, device=recv.device)[None, :] < counts[:, None]).reshape(-1)
        if self.per_rank:
            lo = self.id_lo + self.per_rank * torch.arange(ws, device=recv.device, dtype=torch.int64)
            lo = lo.repeat_interleave(chunk)
            keep = valid & (gid >= lo) & (gid < torch.clamp(lo + self.per_rank, max=self.id_hi))
        else:
            keep = valid & (gid >= self.id_lo) & (gid < self.id_hi)
        k = keep.to(torch.int64)
        pos = self.n + torch.cumsum(k, 0) - 1
        ok = keep & (pos < self.cap)
        self.dropped += (keep & ~ok).to(torch.int64).sum()
        self.buf.index_copy_(0, torch.where(ok, pos, torch.full_like(pos, self.cap)), rows)
        self.n += ok.to(torch.int64).sum()
        self.games += (ok & (ply == 0)).to(torch.int64).sum()

    def records(self):
        """Device uint8 rows [n, 80] sorted by (game id, ply), and n (synchronises)."""
        n = int(self.n.item())
        rows = self.buf[:n]
        gid = rows[:, 64:72].contiguous().view(torch.int64).reshape(-1)
        ply = rows[:, 72:74].contiguous().view(torch.int16).reshape(-1).to(torch.int64)
        order = torch.argsort(gid * 1024 + ply, stable=True)
        return rows.index_select(0, order), n


def chunks_to_records(recv, counts):
    """Host view of one exchange: every rank's valid rows, rank-major (synchronises)."""
    c = counts.cpu().numpy()
    raw = recv.cpu().numpy()
    return np.concatenate([np.frombuffer(raw[r, : int(c[r])].tobytes(), RECORD_DTYPE) for r in range(len(c))])


def to_records(t):
    return np.frombuffer(t.cpu().numpy().tobytes(), RECORD_DTYPE)
