"""world_size-2 gloo run of the tuple all-gather used by multi-GPU self-play
(the only collective on the path).  CPU only."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gzero import boards
from gzero.dist import RecordExchange, ReplayCollector, all_gather_records, chunks_to_records, shard_ids, to_records


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


CAP, CHUNK = 12, 5
# records finished per step by each rank: bursts above the chunk, empty steps
BURSTS = {0: [3, 12, 0, 7, 0, 0, 0, 0], 1: [0, 5, 11, 1, 0, 0, 0, 0]}


def _exchange_worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    ex = RecordExchange(CAP, CHUNK, "cpu")
    serial = 0
    got = []
    for n in BURSTS[rank]:
        rec = np.zeros(CAP, boards.RECORD_DTYPE)
        rec["game_id"] = rank * 1000 + serial + np.arange(CAP)  # rows past n are junk the exchange must skip
        rec["move"] = -7
        rec["move"][:n] = rank
        serial += n
        ex.push(torch.from_numpy(rec.view(np.uint8).copy()), torch.tensor([n], dtype=torch.int32))
        recv, counts = ex.exchange()
        assert recv.shape == (ws, CHUNK, 80) and counts.shape == (ws,)
        got.append(chunks_to_records(recv, counts))
    q.put((rank, np.concatenate(got).tobytes(), int(ex.pending().item()), int(ex.overflow.item())))
    dist.destroy_process_group()


def test_record_exchange_world2():
    """Fixed-size per-step exchange: every record arrives exactly once, in order,
    bursts above the chunk carry over to later steps, padding rows never leak."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    outs = {r: np.frombuffer(b, boards.RECORD_DTYPE) for r, b, _, _ in res}
    assert outs[0].tobytes() == outs[1].tobytes()
    g = outs[0]
    assert (g["move"] >= 0).all()
    for r in range(2):
        ids = g["game_id"][g["move"] == r]
        assert list(ids) == [r * 1000 + i for i in range(sum(BURSTS[r]))]
    assert all(pend == 0 and ovf == 0 for _, _, pend, ovf in res)


def test_record_exchange_overflow_counts():
    ex = RecordExchange(4, 2, "cpu", capacity=6)
    rec = torch.zeros(4 * 80, dtype=torch.uint8)
    for _ in range(3):
        ex.push(rec, torch.tensor([4]))
    assert int(ex.pending().item()) == 6 and int(ex.overflow.item()) == 6
    ex.exchange()
    assert int(ex.pending().item()) == 4


# training.run_iteration's collector (training.selfplay_device) under world size 2:
# each rank's "engine" finishes games in bursts, plies of a game arriving together,
# game ids past the iteration's range keep coming (continuous refill) and must be
# dropped; every rank must end with the union of both ranks' games, sorted by
# (game id, ply), and stop after the same number of exchanges.
G_PER_RANK = 5


def _games_of(rank):
    """(game id, plies) this rank's engine finishes, in finishing order: its 5 games
    of the iteration (ids 10 + 5 rank + i, iteration base 10), then its slots'
    refill games, which follow the engine's real stride (id + n_slots, n_slots = 5):
    rank 0's refills carry rank 1's ids 15..19 -- other plies, other moves, never to
    be collected -- and rank 1's run past 20."""
    rng = np.random.default_rng(rank)
    own = list(10 + G_PER_RANK * rank + rng.permutation(G_PER_RANK))
    refill = [10 + G_PER_RANK * (rank + 1) + k for k in range(G_PER_RANK)] + [30 + rank]
    return [(int(g), int(rng.integers(1, 30))) for g in own + refill]


def _move_of(rank, gid, ply):
    return (gid * 7 + ply + 100 * (gid // G_PER_RANK - 2 != rank)) % 225


def _collector_worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    games = _games_of(rank)
    cap = 64
    ex = RecordExchange(cap, 8, "cpu", capacity=4096)  # chunk < a game: its plies span exchanges
    col = ReplayCollector(ws * G_PER_RANK * 225, 10, 10 + ws * G_PER_RANK, "cpu", per_rank=G_PER_RANK)
    k = steps = 0
    while True:
        rows = []
        for _ in range(1 + (steps + rank) % 2):  # 1 or 2 games finish per step
            if k < len(games):
                gid, plies = games[k]
                k += 1
                r = np.zeros(plies, boards.RECORD_DTYPE)
                r["game_id"], r["ply"] = gid, np.arange(plies)[::-1]  # plies in any order
                r["move"] = [_move_of(rank, gid, p) for p in np.arange(plies)[::-1]]
                rows.append(r)
        rec = np.concatenate(rows) if rows else np.zeros(0, boards.RECORD_DTYPE)
        buf = np.zeros(cap, boards.RECORD_DTYPE)
        buf[: len(rec)] = rec
        ex.push(torch.from_numpy(buf.view(np.uint8).copy()), torch.tensor([len(rec)], dtype=torch.int32))
        col.absorb(*ex.exchange())
        steps += 1
        if int(col.games.item()) >= ws * G_PER_RANK:
            break
    while True:  # drain the outboxes as training.selfplay_device does
        recv, cnt = ex.exchange()
        col.absorb(recv, cnt)
        if int(cnt.sum().item()) == 0:
            break
    rows_t, n = col.records()
    q.put((rank, rows_t.numpy().tobytes(), steps, int(ex.overflow.item()), int(col.dropped.item())))
    dist.destroy_process_group()


def test_replay_collector_world2_is_the_union_of_the_ranks_games():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_collector_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (b, st, ov, dr) for r, b, st, ov, dr in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    assert res[0][1] == res[1][1]  # the same number of exchanges
    assert all(v[2] == 0 and v[3] == 0 for v in res.values())
    got = {r: np.frombuffer(v[0], boards.RECORD_DTYPE) for r, v in res.items()}
    assert got[0].tobytes() == got[1].tobytes()
    want = []
    for r in range(2):
        for gid, plies in _games_of(r):
            if 10 + G_PER_RANK * r <= gid < 10 + G_PER_RANK * (r + 1):  # the rank's own share
                want += [(gid, p, _move_of(r, gid, p)) for p in range(plies)]
    want.sort()
    g = got[0]
    assert [(int(a), int(b), int(c)) for a, b, c in zip(g["game_id"], g["ply"], g["move"])] == want
    # every game exactly once: one ply-0 row per id, no (id, ply) twice
    assert len(set(zip(g["game_id"].tolist(), g["ply"].tolist()))) == len(g)
    assert sorted(g["game_id"][g["ply"] == 0].tolist()) == list(range(10, 20))


# training.main under world size 2: rank 0 alone runs the arena (which draws from
# the global RNGs) and the ranks' own val_loss values could drift; every rank must
# still draw the same random / torch / numpy numbers and stop at the same iteration.
VAL = {0: [1.0, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0], 1: [1.0, 0.5, 0.4, 0.3, 0.2, 0.1, 0.05]}


def _main_worker(rank, ws, port, q, tmp):
    import random
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    os.chdir(tmp)
    import neural_network
    import training
    from gzero import train as gtrain
    draws = []

    def fake_iteration(model, trainer, it, *a, **k):
        draws.append((random.random(), float(torch.rand(1)), float(np.random.rand())))
        return {"iteration": it, "records": 10, "val_loss": VAL[rank][it - 1]}

    def fake_arena(*a, **k):  # the real arena builds AIs / planners / models: all draw
        random.random(), random.getrandbits(64), torch.rand(7), np.random.rand(3)
        return {"win_rate": 0.5}

    real_model = neural_network.GomokuModel
    neural_network.GomokuModel = lambda *a, **k: real_model(*a, **dict(k, device="cpu"))
    gtrain.DeviceTrainer = lambda model: None
    training.run_iteration = fake_iteration
    training.evaluate_model = fake_arena
    hist = training.main(iterations=7, games_per_iteration=1, seed=5, models_dir=os.path.join(tmp, f"m{rank}"))
    q.put((rank, len(hist), draws))
    dist.destroy_process_group()


def test_training_main_ranks_stay_in_step(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_main_worker, args=(r, 2, port, q, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (n, d) for r, n, d in (q.get(timeout=180) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    # rank 0's losses: improve at iterations 1-2, then 3 without improvement -> stop after 5
    assert res[0][0] == res[1][0] == 5
    assert res[0][1] == res[1][1], (res[0][1], res[1][1])


def test_bench_self_launches_n_ranks_stub():
    """`bench.py --gpus 2` without torchrun's env starts the 2 ranks itself (a child
    torch.distributed.run) and relays rank 0's line: n_gpus 2, the backend and both
    ranks' devices (--stub: the plumbing without GPU work, gloo)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GZ_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--stub", "--steps", "3",
                        "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["stub"] is True
    d = out["distributed"]
    assert d["backend"] == "gloo" and d["world_size"] == 2
    assert d["launch"] == "self-launched torch.distributed.run"
    assert [x["rank"] for x in d["ranks"]] == [0, 1] and [x["local_rank"] for x in d["ranks"]] == [0, 1]


def test_bench_self_launch_fails_when_a_rank_fails():
    """A rank that exits non-zero after the rendezvous makes the self-launched
    `bench.py --gpus 2` exit non-zero and print no JSON line (the driver must never
    read a partial run as a result)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GZ_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--stub", "--steps", "3",
                        "--warmup", "1", "--stub-fail-rank", "1"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode != 0, (r.returncode, r.stderr[-2000:])
    assert not [s for s in r.stdout.splitlines() if s.startswith("{")], r.stdout


def _loss_worker(rank, ws, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    import training
    # only rank 1 lost records (its outbox overflowed); rank 0 dropped one in its engine
    overflow = torch.tensor([7 if rank == 1 else 0])
    drops = torch.tensor([1 if rank == 0 else 0])
    lost = training.collective_losses([overflow, drops], ws)
    q.put((rank, lost.tolist()))
    dist.destroy_process_group()


def test_selfplay_loss_counters_are_collective():
    """a loss counter that only one rank sees must reach every rank in the
    same step (else that rank raises alone and the others block in the next all-gather)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_loss_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert got[0] == got[1] == [7, 1]
