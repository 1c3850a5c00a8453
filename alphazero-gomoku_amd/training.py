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


def play_one_game(ai_black, ai_white, step_timeout: float = 10.0,
                  game_timeout: float = 300.0) -> Tuple[SimpleReplay, int]:
    """One game between two AIs (training.py:141-218); timeouts fall back to a random move."""
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
        except Exception:  # training.py:191-198
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
             plies_per_step: int = 16, planner_steps: int = 0, planner=None) -> Tuple[SimpleReplay, dict]:
    """Play game ids [game_id_base, game_id_base + n_games) concurrently on the GPU.

    With ``model`` (a GomokuModel) the policy-value network is evaluated on every
    node the searches create, as the reference does.  ``planner_steps > 0`` adds
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
    eng = SelfPlayEngine(n_slots=slots, num_simulations=num_simulations, c_puct=c_puct, exploration=expl,
                         beta=beta, seed=seed, pv_weights=model.device_weights() if model is not None else None,
                         plies_per_step=plies_per_step, game_id_base=game_id_base, planner_steps=planner_steps,
                         planner_difficulty=difficulty, gn_weights=gnw)
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
