"""Drop-in ``neural_network`` module (reference: neural_network.py:74-382).

``GomokuModel`` keeps the reference's interface: ``.model`` is the torch
``nn.Module`` (parameter names identical to ``AlphaZeroGomokuNet``, so
``.pth`` checkpoints are interchangeable and training code calls
``model.model(x)`` as before), ``predict`` / ``get_move_probabilities`` /
``save_model`` / ``load_model`` / ``auto_save_model`` / ``train_mode`` /
``eval_mode``.  ``predict`` runs on the MI355X policy-value kernel
(``gz_pv_forward``); the packed weights are refreshed whenever the torch
parameters change.  There is no CPU inference path.
"""
import logging
import os
from typing import Optional, Tuple

import numpy as np
import torch

from gzero import weights as _w

AlphaZeroGomokuNet = _w.PolicyValueNet
ResidualBlock = _w._Block


class GomokuModel:
    def __init__(self, model_path: Optional[str] = None, board_size: int = 15, device: str = "cpu",
                 precision: str = "f16x3"):
        self.board_size = board_size
        self.model_path = model_path
        self.device = torch.device(device)
        self.precision = precision
        self.logger = logging.getLogger(__name__)
        self.model = AlphaZeroGomokuNet(board_size)
        self.model.to(self.device)
        self.model.eval()
        self._packed = None
        self._packed_key = None
        # auto-load order of the reference (neural_network.py:189-212): path, best, newest
        if model_path and os.path.exists(model_path):
            self.load_model(model_path)
        elif os.path.exists("models/alphazero_gomoku_best.pth"):
            self.load_model("models/alphazero_gomoku_best.pth")
        else:
            latest = self._find_latest_model()
            if latest:
                self.load_model(latest)

    # ---- device weights ---------------------------------------------------
    def _param_key(self):
        return tuple((p.data_ptr(), p._version) for p in self.model.state_dict().values())

    def device_weights(self):
        """Packed weights on the GPU, repacked after any parameter change."""
        from gzero.device import PVWeights
        key = self._param_key()
        if self._packed is None or key != self._packed_key:
            # packed on the device (the host packer's numpy took ~0.5 s per repack)
            self._packed = PVWeights(_w.pack_pv_weights_torch(self.model.state_dict(), "cuda"),
                                     precision=self.precision)
            self._packed_key = key
        return self._packed

    # ---- inference (neural_network.py:214-252) ------------------------------
    def predict_batch(self, cells) -> Tuple[np.ndarray, np.ndarray]:
        """[n, 225] cells (0/1/2) -> (softmax policy [n, 225] float32, value [n] float32)."""
        from gzero import boards, device
        cells = np.asarray(cells).reshape(-1, 225)
        bl, wh = boards.cells_to_words(cells)
        _, v, pr = device.pv_forward(self.device_weights(), boards.leaf_words(bl, wh))
        return pr, v

    def predict(self, board_state: np.ndarray) -> Tuple[np.ndarray, float]:
        board_state = np.asarray(board_state)
        if board_state.ndim == 2:
            cells = board_state.reshape(1, -1)
        else:  # (3, 15, 15) planes: black, white, empty
            cells = (board_state[0] > 0.5).astype(np.int8) + 2 * (board_state[1] > 0.5).astype(np.int8)
            cells = cells.reshape(1, -1)
        pr, v = self.predict_batch(cells)
        return pr[0], float(v[0])

    def _softmax(self, x: np.ndarray, temperature: float = 1.0) -> np.ndarray:
        x = x / temperature
        e = np.exp(x - np.max(x))
        return e / np.sum(e)

    def get_move_probabilities(self, board_state: np.ndarray, valid_moves: list) -> np.ndarray:
        policy, _ = self.predict(board_state)
        probs = np.array([policy[r * self.board_size + c] for r, c in valid_moves], dtype=np.float64)
        s = probs.sum()
        return probs / s if s > 0 else probs

    # ---- checkpoints (neural_network.py:270-352) -----------------------------
    def _find_latest_model(self) -> Optional[str]:
        if not os.path.isdir("models"):
            return None
        files = [os.path.join("models", f) for f in os.listdir("models")
                 if f.startswith("alphazero_gomoku_") and f.endswith(".pth")]
        return max(files, key=os.path.getmtime) if files else None

    def save_model(self, filepath: str):
        d = os.path.dirname(filepath)
        if d:
            os.makedirs(d, exist_ok=True)
        torch.save({"model_state_dict": self.model.state_dict(), "model_type": "alphazero_gomoku",
                    "board_size": self.board_size, "device": str(self.device)}, filepath)

    def load_model(self, filepath: str) -> bool:
        if not os.path.exists(filepath):
            self.logger.warning(f"Model file not found: {filepath}")
            return False
        try:
            ckpt = torch.load(filepath, map_location=self.device, weights_only=True)
            missing, unexpected = self.model.load_state_dict(ckpt["model_state_dict"], strict=False)
            self.model.eval()
            if missing or unexpected:
                self.logger.warning(f"Loaded with mismatches. missing={len(missing)}, unexpected={len(unexpected)}")
            return True
        except Exception as e:  # the reference reports failure rather than raising
            self.logger.warning(f"Failed to load model: {e}")
            return False

    def auto_save_model(self, iteration: int = None, suffix: str = ""):
        os.makedirs("models", exist_ok=True)
        name = f"alphazero_gomoku_iter_{iteration}{suffix}.pth" if iteration is not None \
            else f"alphazero_gomoku_auto{suffix}.pth"
        path = os.path.join("models", name)
        self.save_model(path)
        return path

    def train_mode(self):
        self.model.train()

    def eval_mode(self):
        self.model.eval()


def create_pretrained_model(board_size: int = 15) -> GomokuModel:
    path = f"models/pretrained_gomoku_{board_size}x{board_size}.pth"
    return GomokuModel(path if os.path.exists(path) else None, board_size)


def test_model():
    """Module smoke check, as the reference's (neural_network.py:385-424): predict on a
    board with one centre stone, the masked move probabilities, and a save/load round
    trip through models/test_model.pth (removed afterwards).  Needs the GPU engine."""
    model = GomokuModel()
    board_state = np.zeros((15, 15), dtype=int)
    board_state[7, 7] = 1
    policy, value = model.predict(board_state)
    print("policy", policy.shape, "sum", float(np.sum(policy)), "| value", value)
    print("move probabilities", model.get_move_probabilities(board_state, [(7, 6), (7, 8), (6, 7), (8, 7)]))
    path = "models/test_model.pth"
    model.save_model(path)
    print("reloaded:", GomokuModel().load_model(path))
    if os.path.exists(path):
        os.remove(path)
    print("GomokuModel smoke check done")


if __name__ == "__main__":
    test_model()
