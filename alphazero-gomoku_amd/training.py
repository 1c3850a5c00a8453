"""Drop-in ``training`` module (reference: training.py:38-537).

Self-play collection is the hot path:

* ``play_one_game(ai_black, ai_white, ...)`` keeps the reference's
  one-game-at-a-time interface (training.py:141-218): each ply is one GPU
  search through ``AlphaZeroGomokuAI.get_move``.
* ``selfplay(n_games, ...)`` is the batched form the engine is built for:
  thousands of concurrent games on the device (``gzero.selfplay``), returning
  the same ``SimpleReplay`` fields.

The dataset / augmentation / SGD helpers follow the reference's definitions
(including its 8-fold augmentation, whose index map disagrees with the plane
rotation for k = 1, 3 -- kept by default, ``fix_labels=True`` corrects it).
"""
import random
import re
import time
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import Dataset

from gomoku_board import GomokuBoard

# ---------------------------------------------------------------- augmentation


def _transform_planes(planes: np.ndarray, k_rot: int, flip: bool) -> np.ndarray:
    x = np.rot90(planes, k=k_rot % 4, axes=(1, 2))  # counter-clockwise (training.py:44-51)
    if flip:
        x = np.flip(x, axis=2)
    return x.copy()


def _transform_index(idx: int, k_rot: int, flip: bool, n: int = 15, fix_labels: bool = False) -> int:
    r, c = divmod(idx, n)
    for _ in range(k_rot % 4):
        # reference (training.py:53-61) rotates the label clockwise; fixed mode
        # rotates it counter-clockwise like the planes
        r, c = (n - 1 - c, r) if fix_labels else (c, n - 1 - r)
    if flip:
        c = n - 1 - c
    return r * n + c


def augment_sample(planes: np.ndarray, move_idx: int, fix_labels: bool = False) -> List[Tuple[np.ndarray, int]]:
    return [(_transform_planes(planes, k, f), _transform_index(move_idx, k, f, fix_labels=fix_labels))
            for k in range(4) for f in (False, True)]


# ---------------------------------------------------------------- replay


class SimpleReplay:
    """(s, pi, z) buffer of training.py:77-97."""

    def __init__(self):
        self.states: List[np.ndarray] = []
        self.move_indices: List[int] = []
        self.players: List[int] = []
        self.outcomes: List[int] = []

    def add(self, planes: np.ndarray, move_idx: int, player: int):
        self.states.append(planes.astype(np.float32))
        self.move_indices.append(int(move_idx))
        self.players.append(int(player))

    def finalize_with_winner(self, winner: Optional[int]):
        for p in self.players[len(self.outcomes):]:
            self.outcomes.append(0 if winner is None else (1 if p == winner else -1))

    def extend_records(self, recs):
        """Append device records (gzero.boards.RECORD_DTYPE, z already final)."""
        from gzero.selfplay import records_to_replay
        planes, mv, pl, z = records_to_replay(recs)
        self.states.extend(list(planes))
        self.move_indices.extend(int(x) for x in mv)
        self.players.extend(int(x) for x in pl)
        self.outcomes.extend(int(x) for x in z)

    def __len__(self) -> int:
        return len(self.states)


class GomokuSelfPlayDataset(Dataset):
    """training.py:104-134: every sample plus 8 symmetries of a random subset."""

    def __init__(self, replay: SimpleReplay, use_augmentation: bool = True, augment_ratio: float = 0.5,
                 fix_labels: bool = False):
        n = len(replay)
        self.samples = [(replay.states[i], replay.move_indices[i], float(replay.outcomes[i])) for i in range(n)]
        if use_augmentation and n > 0:
            for i in random.sample(range(n), k=max(1, int(n * augment_ratio))):
                v = float(replay.outcomes[i])
                for x, y in augment_sample(replay.states[i], replay.move_indices[i], fix_labels):
                    self.samples.append((x, y, v))

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        planes, move_idx, value = self.samples[idx]
        return (torch.from_numpy(planes), torch.tensor(move_idx, dtype=torch.long),
                torch.tensor([value], dtype=torch.float32))


# ---------------------------------------------------------------- self-play


def _is_device_failure(e: BaseException) -> bool:
    """Errors that must not be papered over with a random move: the engine is
    missing or a HIP call failed (a dead GPU would otherwise silently turn
    self-play into random-move training data)."""
    from gzero._lib import GzeroError, GzeroUnavailable
    if isinstance(e, (GzeroUnavailable, GzeroError)):
        return True
    # whole words only: "relationship" / "ownership" in an AI-logic error must
    # still fall back to a random move as the reference does
    return isinstance(e, RuntimeError) and _DEVICE_ERR.search(str(e)) is not None


_DEVICE_ERR = re.compile(r"\b(?:HIP|hip|CUDA|cuda)\b|\b(?:hip|cuda)[A-Z]\w*|device-side")


def play_one_game(ai_black, ai_white, step_timeout: float = 10.0,
                  game_timeout: float = 300.0) -> Tuple[SimpleReplay, int]:
    """One game between two AIs (training.py:141-218); timeouts and AI-logic
    exceptions fall back to a random move as in the reference, device failures
    (GzeroUnavailable, GzeroError, HIP runtime errors) propagate.  Each call is
    a new game for both AIs: their random streams move to a fresh game id
    (AlphaZeroGomokuAI.new_game), as the reference's global ``random`` would."""
    for ai in (ai_black, ai_white):
        if hasattr(ai, "new_game"):
            ai.new_game()
    board = GomokuBoard()
    buf = SimpleReplay()
    t_game = time.time()
    while not board.game_over:
        if time.time() - t_game > game_timeout:
            break
        player = board.current_player
        ai = ai_black if player == GomokuBoard.BLACK else ai_white
        t0 = time.time()
        try:
            move = ai.get_move(board)
            if time.time() - t0 > step_timeout:
                valid = board.get_valid_moves()
                if not valid:
                    break
                move = random.choice(valid)
        except Exception as e:  # training.py:191-198
            if _is_device_failure(e):
                raise
            valid = board.get_valid_moves()
            if not valid:
                break
            move = random.choice(valid)
        if move is None:
            break
        buf.add(board.get_board_tensor(), move[0] * board.BOARD_SIZE + move[1], player)
        board.make_move(move[0], move[1])
    buf.finalize_with_winner(board.winner)
    return buf, board.get_move_count()


def selfplay(n_games: int, num_simulations: int = 200, difficulty: str = "medium", beta: float = 0.2,
             seed: int = 0, n_slots: int = 4096, game_id_base: int = 0, model=None,
             plies_per_step: int = 16, planner_steps: int = 0, planner=None,
             pv_mode: str = "tree") -> Tuple[SimpleReplay, dict]:
    """Play game ids [game_id_base, game_id_base + n_games) concurrently on the GPU.

    With ``model`` (a GomokuModel) the policy-value network is evaluated on every
    node the searches create, as the reference does -- by default incrementally
    (``pv_mode="tree"``: each root's children and grandchildren recompute only the
    windows their stone changes, outputs bit-identical; f16x3 models only, at most
    4 plies per step to bound its workspace).  ``planner_steps > 0`` adds
    BG-planner plies to every rollout (the reference's default AI, planner_steps=5);
    ``planner`` is the BGPlannerAI whose nets they use (a fresh one if None)."""
    from gzero.selfplay import SelfPlayEngine
    c_puct, expl = {"easy": (1.4, 0.2), "medium": (1.6, 0.05), "hard": (1.8, 0.01)}[difficulty]
    slots = min(n_slots, n_games)
    gnw = None
    if planner_steps:
        if planner is None:
            from bg_planner import BGPlannerAI
            planner = BGPlannerAI(1, difficulty)
        gnw = planner.device_weights()
    pvw = model.device_weights() if model is not None else None
    tree = pv_mode == "tree" and pvw is not None and pvw.precision == "f16x3"
    eng = SelfPlayEngine(n_slots=slots, num_simulations=num_simulations, c_puct=c_puct, exploration=expl,
                         beta=beta, seed=seed, pv_weights=pvw,
                         plies_per_step=min(plies_per_step, 4) if tree else plies_per_step,
                         game_id_base=game_id_base, planner_steps=planner_steps,
                         planner_difficulty=difficulty, gn_weights=gnw, pv_mode="tree" if tree else "full")
    replay = SimpleReplay()
    done = {}
    moves = 0
    t0 = time.time()
    while len(done) < n_games:
        eng.step()
        c = eng.counters()
        moves += int(c["moves"])
        recs = eng.records()
        recs = recs[recs["game_id"] < game_id_base + n_games]
        for gid in np.unique(recs["game_id"]):
            if int(gid) not in done:
                g = recs[recs["game_id"] == gid]
                done[int(gid)] = g[np.argsort(g["ply"])]
    slices = {}
    for gid in sorted(done):
        slices[gid] = (len(replay), len(done[gid]))
        replay.extend_records(done[gid])
    return replay, {"games": len(done), "moves_played": moves, "seconds": time.time() - t0,
                    "game_slices": slices}


def selfplay_device(n_games: int, id_lo: int, id_hi: int, num_simulations: int = 200, difficulty: str = "medium",
                    beta: float = 0.2, seed: int = 0, n_slots: int = 4096, game_id_base: int = 0, model=None,
                    plies_per_step: int = 16, planner_steps: int = 0, planner=None, pv_mode: str = "tree",
                    compact: bool = True):
    """training.run_iteration's self-play on every rank: this rank plays game ids
    [game_id_base, game_id_base + n_games) as ``selfplay`` does, and each step's
    finished games go through the sync-free RecordExchange (one all-gather per step,
    RCCL) into a ReplayCollector, so every rank ends with the rows of ALL ranks'
    games in [id_lo, id_hi), sorted by (game id, ply), on the device -- each game
    once: rank r's rows count only for rank r's own ids.  compact=True: a slot whose
    games are done goes idle instead of starting the next id (game_id_end), and after
    every step the active slots move to the front, so that the next step runs only
    those (the games and rows are the same; the refill games a slot would otherwise
    play while the last games finish -- rank r + 1's ids, discarded -- are not
    played).  compact=False: continuous refill.  One host synchronisation per step
    reads the played moves, the finished-game count, the active slots and every loss
    counter (exchange overflow, collector drops, engine record drops: any of them
    raises at once).  The loop
    ends when every one of those games has arrived (the count every rank computes
    from the same chunks, so the ranks stop together), or raises after a bound on
    the steps the games can take.
    Returns (device uint8 rows [n, 80], n, stats)."""
    from gzero import dist as gdist
    from gzero.selfplay import SelfPlayEngine
    rank, ws = gdist.world()
    c_puct, expl = {"easy": (1.4, 0.2), "medium": (1.6, 0.05), "hard": (1.8, 0.01)}[difficulty]
    slots = min(n_slots, n_games)
    gnw = None
    if planner_steps:
        if planner is None:
            from bg_planner import BGPlannerAI
            planner = BGPlannerAI(1, difficulty)
        gnw = planner.device_weights()
    pvw = model.device_weights() if model is not None else None
    tree = pv_mode == "tree" and pvw is not None and pvw.precision == "f16x3"
    eng = SelfPlayEngine(n_slots=slots, num_simulations=num_simulations, c_puct=c_puct, exploration=expl,
                         beta=beta, seed=seed, pv_weights=pvw,
                         plies_per_step=min(plies_per_step, 4) if tree else plies_per_step,
                         game_id_base=game_id_base, planner_steps=planner_steps,
                         planner_difficulty=difficulty, gn_weights=gnw, pv_mode="tree" if tree else "full",
                         game_id_end=game_id_base + n_games if compact else None)
    # a chunk of a quarter of the engine's record buffer: a game's records leave the
    # outbox in one or a few steps even when many games end together
    ex = gdist.RecordExchange(eng.record_cap, max(2 * eng.n_slots * eng.plies_per_step, eng.record_cap // 4), "cuda")
    want = id_hi - id_lo
    if want != ws * n_games or game_id_base != id_lo + rank * n_games:
        raise ValueError(f"selfplay_device: rank {rank} must play ids [id_lo + rank * n_games, +n_games) of "
                         f"[id_lo, id_hi) (got game_id_base {game_id_base}, id_lo {id_lo}, id_hi {id_hi}, "
                         f"n_games {n_games}, {ws} ranks)")
    # rank r keeps only its own share from rank r's rows: with continuous refill its
    # slots' refill games (id + n_slots) run into rank r + 1's ids
    col = gdist.ReplayCollector(want * _MAX_GAME_RECORDS, id_lo, id_hi, "cuda", per_rank=n_games)
    moves = steps = 0
    # a slot plays ceil(n_games / slots) games of <= 200 plies: past that bound a
    # lost ply-0 row would otherwise keep every rank stepping forever
    max_steps = (-(-n_games // slots) + 1) * 200 // eng.plies_per_step + 8
    t0 = time.time()
    while True:
        eng.step()
        ex.push(eng.d_records, eng.d_counters[0:4].view(torch.int32))
        col.absorb(*ex.exchange())
        steps += 1
        # this rank's own losses (outbox overflow, engine record drops) made collective
        # before anyone reads them: a rank that raised alone would leave the others
        # blocked in the next exchange (col.dropped comes from the gathered chunks and
        # is the same on every rank already)
        lost = collective_losses([ex.overflow, eng.d_counters[0:16].view(torch.int32)[2:3]], ws)
        parts = [eng.d_counters.view(torch.int64)[2:3], col.games, lost[0:1], col.dropped, lost[1:2]]
        if compact:
            parts.append(eng.compact().to(torch.int64))
        # the step's one host synchronisation: moves, finished games, active slots and
        # every loss counter
        c = torch.cat(parts).cpu().tolist()
        moves += int(c[0])
        if compact:
            eng.n_active = int(c[5])
        if c[2] or c[3] or c[4]:
            raise RuntimeError(f"selfplay_device: records lost (exchange overflow {c[2]}, collector {c[3]}, "
                               f"engine buffer {c[4]}; max over ranks)")
        if c[1] >= want:  # every game's first record is in
            break
        if steps >= max_steps:
            raise RuntimeError(f"selfplay_device: {c[1]} of {want} games after {steps} steps")
    # drain: the outboxes may still hold later plies of those games; an exchange in
    # which every rank sent nothing means every outbox is empty (all ranks see the
    # same counts, so they stop together)
    while True:
        recv, cnt = ex.exchange()
        col.absorb(recv, cnt)
        if int(cnt.sum().item()) == 0:
            break
    rows, n = col.records()
    if int(ex.overflow.item()) or int(col.dropped.item()):
        raise RuntimeError(f"selfplay_device: {int(ex.overflow.item())} records overflowed the exchange, "
                           f"{int(col.dropped.item())} the collector")
    return rows, n, {"games": want, "moves_played": moves, "steps": steps, "seconds": time.time() - t0}


_MAX_GAME_RECORDS = 225  # a game has at most 225 plies (one record each)


def collective_losses(counters, ws):
    """selfplay_device's per-rank loss counters (one-element device tensors),
    concatenated and MAX-all-reduced over the `ws` ranks (no host synchronisation), so
    every rank sees the same values in the step's one host read and all raise together."""
    lost = torch.cat([c.reshape(1).to(torch.int64) for c in counters])
    if ws > 1:
        torch.distributed.all_reduce(lost, op=torch.distributed.ReduceOp.MAX)
    return lost


# ---------------------------------------------------------------- arena (training.py:221-270)


class RandomAgent:
    """evaluate_model's opponent when there is no baseline: random.choice(valid),
    drawn from the (seed, game_id, ply, 0) stream."""

    def __init__(self, seed: int = 0, game_id: int = 0):
        self.seed, self.game_id = int(seed), int(game_id)

    def get_move(self, board: GomokuBoard):
        from gzero import rng
        v = board.get_valid_moves()
        if not v:
            return None
        return rng.Stream(rng.stream_key(self.seed, self.game_id, board.get_move_count(), 0)).choice(v)


def evaluate_model(current, baseline, device=None, games: int = 8, eval_difficulty: str = "easy",
                   eval_num_sim: int = 60, eval_plans: int = 2, seed: Optional[int] = None,
                   return_games: bool = False, alternate: bool = True, seeds: Optional[Tuple[int, int]] = None,
                   game_id_base: int = 0):
    """training.py:221-270 with all ``games`` played at once: every ply, the games
    whose side to move belongs to the same agent are searched in ONE batched GPU
    call (AlphaZeroGomokuAI.get_moves).  As in the reference the evaluated model
    alternates colours (black in even games), its AI uses ``eval_num_sim``
    simulations only when there is no baseline (otherwise the difficulty's own
    count; the baseline's AI uses ``eval_num_sim``), both with ``eval_plans``
    planner plies, and a missing move ends the game as a draw.  Game g draws from
    the streams of (seed_a / seed_b, g): the result equals playing the games one
    by one with per-game AIs of those seeds and ``game_id = g``.  ``alternate=False``
    keeps the evaluated model on black in every game -- what training.main's six
    ``evaluate_model(..., games=1)`` calls amount to (training.py:484-492).
    ``seeds`` = (seed_a, seed_b) overrides the pair derived from ``seed``; game g
    uses game id ``game_id_base + g`` (tests/golden arena fixture: one seed for
    both sides, as the reference's single global stream)."""
    from ai_agent import AlphaZeroGomokuAI
    seed = random.getrandbits(64) if seed is None else int(seed)
    seed_a, seed_b = seed, (seed * 0x9E3779B97F4A7C15 + 1) & ((1 << 64) - 1)
    if seeds is not None:
        seed_a, seed_b = int(seeds[0]), int(seeds[1])
    gid = [int(game_id_base) + g for g in range(games)]
    # one AI object per (agent, colour): the colour is the AI's player in the search
    ai_a, ai_b = {}, {}
    for color in (GomokuBoard.BLACK, GomokuBoard.WHITE):
        a = AlphaZeroGomokuAI(color, difficulty=eval_difficulty, planner_steps=eval_plans, seed=seed_a)
        a.model = current
        if baseline is None:
            a.params = dict(a.params, num_simulations=eval_num_sim)
            b = RandomAgent(seed_b)
        else:
            b = AlphaZeroGomokuAI(color, difficulty=eval_difficulty, planner_steps=eval_plans, seed=seed_b)
            b.params = dict(b.params, num_simulations=eval_num_sim)
            b.model = baseline
        ai_a[color], ai_b[color] = a, b
    boards = [GomokuBoard() for _ in range(games)]
    color_a = [GomokuBoard.BLACK if (g % 2 == 0 or not alternate) else GomokuBoard.WHITE for g in range(games)]
    active = list(range(games))
    moves = [[] for _ in range(games)]
    plies = [[] for _ in range(games)]  # per move: the search's (predicts, main_draws, sim_draws)
    while active:
        groups = {}
        for g in active:
            cp = boards[g].current_player
            who = "a" if cp == color_a[g] else "b"
            groups.setdefault((who, cp), []).append(g)
        stopped = set()
        for (who, cp), gs in groups.items():
            agent = (ai_a if who == "a" else ai_b)[cp]
            if isinstance(agent, RandomAgent):
                mv = [RandomAgent(agent.seed, gid[g]).get_move(boards[g]) for g in gs]
                st = [None] * len(gs)
            else:
                mv = agent.get_moves([boards[g] for g in gs], [gid[g] for g in gs])
                st = agent.last_batch_stats
            for g, m, s in zip(gs, mv, st):
                if m is None:
                    stopped.add(g)
                    continue
                boards[g].make_move(*m)
                moves[g].append(m[0] * 15 + m[1])
                plies[g].append(s)
        active = [g for g in active if g not in stopped and not boards[g].game_over]
    wins = sum(1 for g in range(games) if boards[g].winner is not None and boards[g].winner == color_a[g])
    draws = sum(1 for g in range(games) if boards[g].winner is None)
    losses = games - wins - draws
    out = {"wins": wins, "losses": losses, "draws": draws, "win_rate": wins / max(1, games)}
    if return_games:
        out["games"] = [{"moves": moves[g], "winner": boards[g].winner, "color_a": color_a[g], "plies": plies[g]}
                        for g in range(games)]
        out["seeds"] = (seed_a, seed_b)
    return out


# ---------------------------------------------------------------- SGD (training.py:277-337)


def train_epoch(model, loader, optimizer, device, grad_clip: float = 1.0, epoch_index: int = 1,
                num_epochs: int = 1) -> float:
    model.train_mode()
    ce, mse = nn.CrossEntropyLoss(), nn.MSELoss()
    total, batches = 0.0, 0
    for x, y_p, y_v in loader:
        x, y_p, y_v = x.to(device), y_p.to(device), y_v.to(device)
        optimizer.zero_grad()
        logits, v = model.model(x)
        loss = ce(logits, y_p) + mse(v, y_v)
        loss.backward()
        if grad_clip is not None and grad_clip > 0:
            nn.utils.clip_grad_norm_(model.model.parameters(), grad_clip)
        optimizer.step()
        total += float(loss.item())
        batches += 1
    return total / max(1, batches)


def validate_epoch(model, loader, device, epoch_index: int = 1, num_epochs: int = 1) -> float:
    model.eval_mode()
    ce, mse = nn.CrossEntropyLoss(), nn.MSELoss()
    total, batches = 0.0, 0
    with torch.no_grad():
        for x, y_p, y_v in loader:
            x, y_p, y_v = x.to(device), y_p.to(device), y_v.to(device)
            logits, v = model.model(x)
            total += float((ce(logits, y_p) + mse(v, y_v)).item())
            batches += 1
    return total / max(1, batches)


# ---------------------------------------------------------------- training.main (training.py:361-537)


def _render_bar(pct: float, width: int = 20) -> str:
    k = int(round(max(0.0, min(1.0, pct)) * width))
    return "[" + "#" * k + "-" * (width - k) + "]"


def _fmt_duration(seconds: float) -> str:
    seconds = int(max(0, seconds))
    h, r = divmod(seconds, 3600)
    m, s = divmod(r, 60)
    return f"{h}h{m:02d}m{s:02d}s" if h else (f"{m}m{s:02d}s" if m else f"{s}s")


def run_iteration(model, trainer, it: int, games_per_iteration: int = 10, num_simulations: int = 200,
                  difficulty: str = "medium", beta: float = 0.2, planner_steps: int = 5, seed: int = 0,
                  train_split: float = 0.9, batch_size: int = 128, epochs: int = 2, augment_ratio: float = 0.35,
                  planner=None, verbose: bool = True) -> dict:
    """One iteration of training.main on the device (training.py:399-480):
    self-play of ``games_per_iteration`` games per rank (ids sharded by rank,
    records all-gathered so every rank holds the same replay), the dataset with
    35 % 8-fold augmentation, a 90/10 split drawn from ``random``, ``epochs``
    epochs of the data-parallel SGD step and the StepLR step."""
    from gzero import dist as gdist
    from gzero.train import DeviceDataset
    rank, ws = gdist.world()
    t0 = time.time()
    id_lo = it * ws * games_per_iteration
    replay_base = id_lo + rank * games_per_iteration
    # every rank's records reach every rank step by step (RecordExchange), sorted by
    # game id at the end: the same replay on every rank, in the reference's game order
    d, n_rec, st = selfplay_device(games_per_iteration, id_lo, id_lo + ws * games_per_iteration,
                                   num_simulations=num_simulations, difficulty=difficulty, beta=beta, seed=seed,
                                   game_id_base=replay_base, model=model, planner_steps=planner_steps,
                                   planner=planner)
    d = d.reshape(-1)
    moves = torch.tensor([float(st["moves_played"])], dtype=torch.float64, device="cuda")
    if ws > 1:
        import torch.distributed as tdist
        tdist.all_reduce(moves)
    t1 = time.time()
    out = {"iteration": it, "records": n_rec, "selfplay_s": t1 - t0, "moves_played": int(moves.item())}
    if n_rec == 0:
        return dict(out, skipped=True)
    ds = DeviceDataset(d, use_augmentation=True, augment_ratio=augment_ratio, n_records=n_rec)
    if len(ds) < 8:  # training.py:431-433
        return dict(out, skipped=True)
    n = len(ds)
    idx = list(range(n))
    random.shuffle(idx)
    split = int(n * train_split)
    tr_idx = torch.tensor(idx[:split], dtype=torch.int64, device="cuda")
    va_idx = torch.tensor(idx[split:], dtype=torch.int64, device="cuda")
    tl, vl = [], []
    t_tr = t_va = 0.0
    t_ds = time.time() - t1
    for ep in range(epochs):
        ta = time.time()
        tl.append(trainer.train_epoch(ds, batch_size, indices=tr_idx))
        tb = time.time()
        vl.append(trainer.validate_epoch(ds, batch_size, indices=va_idx))
        t_tr += tb - ta
        t_va += time.time() - tb
        if verbose and rank == 0:
            print(f"    ├── 模型训练: {_render_bar((ep + 1) / epochs, 12)} epoch {ep + 1}/{epochs} "
                  f"train {tl[-1]:.3f} val {vl[-1]:.3f}")
    trainer.step_scheduler()
    model.eval_mode()
    t2 = time.time()
    return dict(out, samples=n, train_loss=float(np.mean(tl)), val_loss=float(np.mean(vl)), sgd_s=t2 - t1,
                sgd_parts_s={"dataset_split": round(t_ds, 4), "train_epochs": round(t_tr, 4),
                             "validation": round(t_va, 4)})


def _rng_isolated(fn, *a, **k):
    """Run fn (rank 0's arena) without moving the global random / numpy / torch
    RNGs: the arena builds AIs, planners and models that draw from them, and every
    rank must keep drawing the same dataset subset, split and loader order."""
    py, npst = random.getstate(), np.random.get_state()
    devices = [torch.cuda.current_device()] if torch.cuda.is_available() else []
    with torch.random.fork_rng(devices=devices):
        try:
            return fn(*a, **k)
        finally:
            random.setstate(py)
            np.random.set_state(npst)


def _broadcast_int(x: int) -> int:
    """Rank 0's value of x on every rank (identity for one process)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(x)
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
    dist.broadcast(t, 0)
    return int(t.item())


def main(iterations: int = 6, games_per_iteration: int = 10, seed: Optional[int] = None, models_dir: str = "models",
         num_simulations: int = 200, planner_steps: int = 5, eval_games: int = 6):
    """training.main (training.py:361-537) on the MI355X engine: same loop, the
    same hyper-parameters (Adam 8e-4 / wd 1e-5, StepLR(2, 0.85), clip 0.8,
    batch 128, 2 epochs, 35 % augmentation, 90/10 split, patience 3, 6 arena
    games) and the same checkpoint names.  Under torchrun every rank plays its
    own games and trains data-parallel (gzero.train.DeviceTrainer)."""
    import math
    import os
    from gzero import dist as gdist
    from gzero.train import DeviceTrainer
    from neural_network import GomokuModel
    rank, ws = gdist.init_from_env()
    seed = int(seed if seed is not None else 20240101)
    random.seed(seed)  # every rank draws the same dataset / split / shuffles
    np.random.seed(seed % (1 << 32))
    torch.manual_seed(seed)
    if rank == 0:
        os.makedirs(models_dir, exist_ok=True)
    model = GomokuModel(model_path=None, board_size=15, device="cuda")
    trainer = DeviceTrainer(model)
    best_val, patience, patience_count = math.inf, 3, 0
    best_snapshot = None
    t0 = time.time()
    history = []
    for it in range(1, iterations + 1):
        res = run_iteration(model, trainer, it, games_per_iteration, num_simulations=num_simulations,
                            planner_steps=planner_steps, seed=seed, verbose=rank == 0)
        if res.get("skipped"):
            if rank == 0:
                print("自我对弈样本过少，跳过本轮训练。")
            continue
        if rank == 0:
            model.save_model(os.path.join(models_dir, f"alphazero_gomoku_iter_{it}.pth"))
        # rank 0's decision on every rank (val_loss is already the same global value
        # everywhere -- DeviceTrainer.validate_epoch all-reduces it -- so this only
        # guards the early stop and the torch-RNG use of the snapshot against drift)
        improved = bool(_broadcast_int(int(res["val_loss"] < best_val)))
        if improved:
            best_val, patience_count = res["val_loss"], 0
            best_path = os.path.join(models_dir, "alphazero_gomoku_best.pth")
            if rank == 0:
                model.save_model(best_path)
            best_snapshot = GomokuModel(board_size=15, device="cuda")
            best_snapshot.model.load_state_dict(model.model.state_dict())
            best_snapshot.eval_mode()
        else:
            patience_count += 1
        stats = _rng_isolated(evaluate_model, model, best_snapshot, games=eval_games, seed=seed + it,
                              alternate=False) if rank == 0 else {}
        res.update(eval=stats, elapsed=time.time() - t0)
        history.append(res)
        if rank == 0:
            pct = it / iterations
            print(f"📊 {_render_bar(pct)} {int(pct * 100)}% | {_fmt_duration(res['elapsed'])} | "
                  f"records {res['records']} | loss {res['val_loss']:.3f} | win rate "
                  f"{100.0 * stats.get('win_rate', 0.0):.1f}%")
        if patience_count >= patience:
            if rank == 0:
                print("触发早停条件，结束训练。")
            break
    if rank == 0:
        model.save_model(os.path.join(models_dir, "alphazero_gomoku_final.pth"))
    return history


if __name__ == "__main__":
    main()
