"""world_size-2 gloo run of the tuple all-gather used by multi-GPU self-play
(the only collective on the path).  CPU only."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gzero import boards
from gzero.dist import all_gather_records, shard_ids, to_records


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    n = 3 + 2 * rank  # ragged: ranks finish different numbers of records
    rec = np.zeros(n, boards.RECORD_DTYPE)
    base, stride = shard_ids(rank, ws, 4)
    rec["game_id"] = base + np.arange(n)
    rec["move"] = rank * 100 + np.arange(n)
    rec["z"] = 1 - 2 * (np.arange(n) % 2)
    t = torch.from_numpy(rec.view(np.uint8).copy())
    out = to_records(all_gather_records(t, n))
    empty = to_records(all_gather_records(torch.zeros(0, dtype=torch.uint8), 0))
    q.put((rank, out.tobytes(), len(empty), stride))
    dist.destroy_process_group()


def test_all_gather_records_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    outs = {r: np.frombuffer(b, boards.RECORD_DTYPE) for r, b, _, _ in res}
    assert outs[0].tobytes() == outs[1].tobytes()
    g = outs[0]
    assert len(g) == 3 + 5
    assert list(g["game_id"][:3]) == [0, 1, 2] and list(g["game_id"][3:]) == [4, 5, 6, 7, 8]
    assert list(g["move"][3:]) == [100, 101, 102, 103, 104]
    assert all(n == 0 for _, _, n, _ in res)
    assert all(s == 8 for _, _, _, s in res)


def test_shards_disjoint():
    ids = set()
    for r in range(8):
        base, stride = shard_ids(r, 8, 16)
        for s in range(16):
            for g in range(5):
                gid = base + s + g * stride
                assert gid not in ids
                ids.add(gid)
