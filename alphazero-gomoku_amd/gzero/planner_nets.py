"""BG-Planner networks (reference: bg_planner.py:22-78): ``GraphNet`` and
``OpponentDQN`` with the reference's parameter names, deterministic
initialisation, and packing into the device blob of ``csrc/gz_gnet.h``.

GraphNet: embed conv3x3 3->64, then 4 x [conv3x3 64->64 + ReLU, conv1x1 64->64
+ ReLU], policy head conv1x1 64->2 -> flatten -> Linear 450->225 (logits).
OpponentDQN: Linear 675->256, ReLU, Linear 256->256, ReLU, Linear 256->225.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .weights import pack_mfma_b

N = 15
POS = N * N
HID = 64
DQN_H = 256


class GraphNet(nn.Module):
    def __init__(self, board_size=N, in_channels=3, hidden_dim=HID, num_layers=4):
        super().__init__()
        self.board_size = board_size
        self.hidden_dim = hidden_dim
        self.embed = nn.Conv2d(in_channels, hidden_dim, 3, padding=1)
        layers = []
        for _ in range(num_layers):
            layers.append(nn.Conv2d(hidden_dim, hidden_dim, 3, padding=1))
            layers.append(nn.Conv2d(hidden_dim, hidden_dim, 1))
        self.layers = nn.ModuleList(layers)
        self.policy_head = nn.Sequential(nn.Conv2d(hidden_dim, 2, 1), nn.Flatten(),
                                         nn.Linear(2 * board_size * board_size, board_size * board_size))

    def forward(self, x):
        h = F.relu(self.embed(x))
        for i in range(0, len(self.layers), 2):
            h = F.relu(self.layers[i](h))
            h = F.relu(self.layers[i + 1](h))
        return self.policy_head(h)


class OpponentDQN(nn.Module):
    def __init__(self, board_size=N, in_channels=3, hidden=DQN_H):
        super().__init__()
        self.board_size = board_size
        self.net = nn.Sequential(nn.Linear(in_channels * board_size * board_size, hidden), nn.ReLU(),
                                 nn.Linear(hidden, hidden), nn.ReLU(),
                                 nn.Linear(hidden, board_size * board_size))

    def forward(self, planes):
        return self.net(planes.view(planes.size(0), -1))


def _uniform_init(module, rng):
    """Uniform(+-1/sqrt(fan_in)) for every weight and bias, from numpy's rng."""
    sd = {}
    for name, t in module.state_dict().items():
        shape = tuple(t.shape)
        owner = name.rsplit(".", 1)[0]
        w = module.state_dict()[owner + ".weight"]
        fan_in = int(np.prod(w.shape[1:]))
        bound = 1.0 / np.sqrt(fan_in)
        sd[name] = torch.from_numpy(rng.uniform(-bound, bound, shape).astype(np.float32))
    return sd


def init_graphnet_state(seed=0):
    return _uniform_init(GraphNet(), np.random.default_rng(seed))


def init_dqn_state(seed=1):
    return _uniform_init(OpponentDQN(), np.random.default_rng(seed))


# ---------------------------------------------------------------- blob layout (mirror of csrc/gz_gnet.h)
K3 = 9 * HID   # 576: k = tap*64 + cin
GE_W = 0                               # embed [28][64] (k = tap*3 + cin, row 27 zero)
GE_B = GE_W + 28 * HID
GL0 = GE_B + HID                       # 8 layers: W then bias
GL_W3 = K3 * HID                       # 3x3 layer weights [576][64]
GL_W1 = HID * HID                      # 1x1 layer weights [64][64]


def _layer_off(i):
    off = GL0
    for j in range(i):
        off += (GL_W3 if j % 2 == 0 else GL_W1) + HID
    return off


GP_W = _layer_off(8)                   # policy conv [2][64]
GP_B = GP_W + 2 * HID                  # [2] (+2)
GF_WT = GP_B + 4                       # policy fc [450][225]
GF_B = GF_WT + 450 * POS               # [225] (+3)
D0_WT = GF_B + 228                     # dqn fc0 [675][256]
D0_B = D0_WT + 3 * POS * DQN_H
D1_WT = D0_B + DQN_H                   # [256][256]
D1_B = D1_WT + DQN_H * DQN_H
D2_WT = D1_B + DQN_H                   # [256][225]
D2_B = D2_WT + DQN_H * POS             # [225] (+3)
GH_E = (D2_B + 228 + 3) & ~3           # fp16 embed A fragments: hi [4][64][8], lo
GH_L0 = GH_E + 4 * 64 * 8              # fp16 layer fragments, hi then lo per layer
GH_KS3, GH_KS1 = 18, 2                 # 32-deep k-steps of a 3x3 / 1x1 layer


def _h_layer_off(i):
    off = GH_L0
    for j in range(i):
        off += (GH_KS3 if j % 2 == 0 else GH_KS1) * 4 * 64 * 8  # hi + lo halves = floats
    return off


# DQN fc0 restated for one-hot inputs: fc0(x) = base + sum over stones of the
# (black - empty) or (white - empty) row, base = bias + sum of the empty rows
D0_BASE = _h_layer_off(8)              # [256]
D0_DELTA = D0_BASE + DQN_H             # [450][256]: rows 0..224 black - empty, 225..449 white - empty
GF_P = D0_DELTA + 450 * DQN_H          # batched heads, MFMA B-fragment order (weights.pack_mfma_b)
D0_P = GF_P + 29 * 15 * 256
D1_P = D0_P + 29 * 16 * 256
D2_P = D1_P + 16 * 16 * 256
GN_TOTAL = D2_P + 16 * 15 * 256
GN_MACS = POS * (27 * HID + 4 * (K3 * HID + HID * HID) + 2 * HID) + 450 * POS
DQN_MACS = 3 * POS * DQN_H + DQN_H * DQN_H + DQN_H * POS


def _split(x):
    hi = x.astype(np.float16)
    lo = (x - hi.astype(np.float32)).astype(np.float16)
    return hi, lo


def _frag(wt, ks):
    """W^T [64][32*ks] -> MFMA A-fragment order [ks][n-tile 4][lane 64][8]
    (n = 16*n_tile + lane%16, k = 32*ks + 8*(lane//16) + j)."""
    return wt.reshape(4, 16, ks, 4, 8).transpose(2, 0, 3, 1, 4).reshape(-1)


def pack_planner_weights(gn_sd, dqn_sd):
    """GraphNet + OpponentDQN state dicts (reference names) -> float32 blob of GN_TOTAL floats."""
    g = {k: v.detach().cpu().float().numpy() for k, v in gn_sd.items()}
    d = {k: v.detach().cpu().float().numpy() for k, v in dqn_sd.items()}
    blob = np.zeros(GN_TOTAL, np.float32)
    we = g["embed.weight"].transpose(2, 3, 1, 0).reshape(27, HID)  # k = (kh*3+kw)*3 + cin
    blob[GE_W:GE_W + 27 * HID] = we.reshape(-1)
    blob[GE_B:GE_B + HID] = g["embed.bias"]
    wp = np.zeros((32, HID), np.float32)
    wp[:27] = we
    h, l = _split(wp.T.copy())
    blob[GH_E:GH_E + 4 * 64 * 8] = np.concatenate([_frag(h, 1), _frag(l, 1)]).view(np.float32)
    for i in range(8):
        w = g[f"layers.{i}.weight"]
        off = _layer_off(i)
        if i % 2 == 0:
            wk = w.transpose(2, 3, 1, 0).reshape(K3, HID)  # k = (kh*3+kw)*64 + cin
            ks = GH_KS3
        else:
            wk = w.reshape(HID, HID).T  # [cin][cout]
            ks = GH_KS1
        blob[off:off + wk.size] = wk.reshape(-1)
        blob[off + wk.size:off + wk.size + HID] = g[f"layers.{i}.bias"]
        h, l = _split(np.ascontiguousarray(wk.T))
        ho = _h_layer_off(i)
        n = ks * 4 * 64 * 8
        blob[ho:ho + n] = np.concatenate([_frag(h, ks), _frag(l, ks)]).view(np.float32)
    blob[GP_W:GP_W + 2 * HID] = g["policy_head.0.weight"].reshape(2, HID).reshape(-1)
    blob[GP_B:GP_B + 2] = g["policy_head.0.bias"]
    blob[GF_WT:GF_WT + 450 * POS] = g["policy_head.2.weight"].T.reshape(-1)
    blob[GF_B:GF_B + POS] = g["policy_head.2.bias"]
    blob[D0_WT:D0_WT + 3 * POS * DQN_H] = d["net.0.weight"].T.reshape(-1)
    blob[D0_B:D0_B + DQN_H] = d["net.0.bias"]
    blob[D1_WT:D1_WT + DQN_H * DQN_H] = d["net.2.weight"].T.reshape(-1)
    blob[D1_B:D1_B + DQN_H] = d["net.2.bias"]
    blob[D2_WT:D2_WT + DQN_H * POS] = d["net.4.weight"].T.reshape(-1)
    blob[D2_B:D2_B + POS] = d["net.4.bias"]
    w0 = d["net.0.weight"].T.astype(np.float64)  # [675][256]
    blob[D0_BASE:D0_BASE + DQN_H] = (d["net.0.bias"].astype(np.float64) + w0[2 * POS:].sum(0)).astype(np.float32)
    delta = np.concatenate([w0[:POS] - w0[2 * POS:], w0[POS:2 * POS] - w0[2 * POS:]])
    blob[D0_DELTA:D0_DELTA + 450 * DQN_H] = delta.astype(np.float32).reshape(-1)
    blob[GF_P:D0_P] = pack_mfma_b(g["policy_head.2.weight"].T, 29, 15)
    blob[D0_P:D1_P] = pack_mfma_b(delta.astype(np.float32), 29, 16)
    blob[D1_P:D2_P] = pack_mfma_b(d["net.2.weight"].T, 16, 16)
    blob[D2_P:GN_TOTAL] = pack_mfma_b(d["net.4.weight"].T, 16, 15)
    return blob


def reference_forward(gn_sd, dqn_sd, planes):
    """fp32 torch CPU: (softmax(GraphNet(x)), OpponentDQN(x)) as in BGPlannerAI.get_move (bg_planner.py:243-250)."""
    gn, dq = GraphNet(), OpponentDQN()
    gn.load_state_dict(gn_sd)
    dq.load_state_dict(dqn_sd)
    gn.eval()
    dq.eval()
    x = torch.as_tensor(planes, dtype=torch.float32)
    with torch.no_grad():
        logits = gn(x)
        p = torch.softmax(logits, dim=1)
        q = dq(x)
    return logits.numpy(), p.numpy(), q.numpy()
