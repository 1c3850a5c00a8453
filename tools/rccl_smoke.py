#!/usr/bin/env python3
"""RCCL sanity check on one GPU box: the bench's multi-GPU collectives (the record
exchange's all_gather_into_tensor of fixed-size chunks + counts, the ReplayCollector,
the max-over-ranks barrier / all_reduce) through torch.distributed's "nccl" backend
(RCCL on ROCm) with every rank of this node -- run under torch.distributed.run with
--nproc-per-node = the GPUs available (1 on the development box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gzero import boards  # noqa: E402
from gzero.dist import RecordExchange, ReplayCollector  # noqa: E402


def main():
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl")  # (init_from_env skips a world of 1; here RCCL itself is the point)
    rank, ws = dist.get_rank(), dist.get_world_size()
    assert dist.get_backend() == "nccl", dist.get_backend()
    dev = torch.device("cuda", torch.cuda.current_device())
    cap, chunk = 64, 8
    ex = RecordExchange(cap, chunk, "cuda", capacity=4096)
    col = ReplayCollector(ws * 3 * 225, 0, 3 * ws, "cuda")
    for step in range(6):
        n = 5 if step < 3 else 0
        rec = np.zeros(cap, boards.RECORD_DTYPE)
        rec["game_id"][:n] = rank * 3 + (step % 3)
        rec["ply"][:n] = np.arange(n)
        ex.push(torch.from_numpy(rec.view(np.uint8).copy()).to(dev), torch.tensor([n], dtype=torch.int32, device=dev))
        col.absorb(*ex.exchange())
    rows, cnt = col.records()
    t = torch.tensor([float(rank)], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    torch.cuda.synchronize()
    if rank == 0:
        print(f"rccl ok: world {ws}, {int(cnt)} records collected (want {ws * 15}), overflow {int(ex.overflow.item())}, "
              f"max rank {int(t.item())}")
    assert int(cnt) == ws * 15 and int(ex.overflow.item()) == 0
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
