"""Policy-value network definition, deterministic initialisation and packing
into the device weight blob (csrc/gz_pvnet.h).

``PolicyValueNet`` has exactly the parameter names of the reference's
``AlphaZeroGomokuNet`` (neural_network.py:94-159): ``conv``/``bn``,
``residual_tower.{0,1}.{conv1,bn1,conv2,bn2}``, ``policy_conv``, ``policy_fc``,
``value_conv``, ``value_fc1``, ``value_fc2`` -- so ``.pth`` checkpoints move
between the two unchanged.  It is the training-side module (``GomokuModel.model``);
inference during self-play runs the packed blob on the MFMA kernel.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

CH = 128
N = 15
POS = N * N
BN_EPS = 1e-5


class _Block(nn.Module):
    """conv3x3-BN-ReLU-conv3x3-BN, identity skip, ReLU (neural_network.py:74-91)."""

    def __init__(self, ch):
        super().__init__()
        # registration order of the reference (parameters() order feeds clip_grad_norm_'s sum)
        self.conv1 = nn.Conv2d(ch, ch, 3, padding=1)
        self.conv2 = nn.Conv2d(ch, ch, 3, padding=1)
        self.bn1 = nn.BatchNorm2d(ch)
        self.bn2 = nn.BatchNorm2d(ch)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + x)


class PolicyValueNet(nn.Module):
    def __init__(self, board_size=N, channels=3, num_residual=2):
        super().__init__()
        self.board_size = board_size
        self.channels = channels
        self.num_residual = num_residual
        cells = board_size * board_size
        self.conv = nn.Conv2d(channels, CH, 3, padding=1)
        self.bn = nn.BatchNorm2d(CH)
        self.residual_tower = nn.ModuleList([_Block(CH) for _ in range(num_residual)])
        self.policy_conv = nn.Conv2d(CH, 2, 1)
        self.policy_fc = nn.Linear(2 * cells, cells)
        self.value_conv = nn.Conv2d(CH, 1, 1)
        self.value_fc1 = nn.Linear(cells, 64)
        self.value_fc2 = nn.Linear(64, 1)

    def forward(self, x):
        h = F.relu(self.bn(self.conv(x)))
        for blk in self.residual_tower:
            h = blk(h)
        logits = self.policy_fc(torch.flatten(self.policy_conv(h), 1))
        v = F.relu(self.value_fc1(torch.flatten(self.value_conv(h), 1)))
        return logits, torch.tanh(self.value_fc2(v))


def _init_order(state):
    """Draw order of init_state_dict: residual blocks as conv1, bn1, conv2, bn2 (the
    order the fixtures were generated in), whatever the module registration order."""
    rank = {"conv1": 0, "bn1": 1, "conv2": 2, "bn2": 3}
    items = list(state.items())
    first = {}
    keys = []
    for i, (name, _) in enumerate(items):
        p = name.split(".")
        if p[0] == "residual_tower":
            keys.append((first.setdefault(p[1], i), rank[p[2]], i))
        else:
            keys.append((i, 0, i))
    return [items[k[2]] for k in sorted(keys)]


def init_state_dict(seed=0, bn_noise=True):
    """Deterministic weights from numpy's default_rng(seed), identical on every
    machine (torch's CPU RNG is not used).  Uniform(+-1/sqrt(fan_in)) like
    torch's default init; BatchNorm running stats are randomised too when
    ``bn_noise`` so that BN folding is exercised."""
    rng = np.random.default_rng(seed)
    net = PolicyValueNet()
    sd = {}
    for name, t in _init_order(net.state_dict()):
        shape = tuple(t.shape)
        if name.endswith("num_batches_tracked"):
            sd[name] = torch.zeros((), dtype=torch.long)
            continue
        if ".bn" in name or name.startswith("bn."):
            if name.endswith("running_var"):
                a = rng.uniform(0.5, 1.5, shape) if bn_noise else np.ones(shape)
            elif name.endswith("running_mean"):
                a = rng.uniform(-0.2, 0.2, shape) if bn_noise else np.zeros(shape)
            elif name.endswith("weight"):
                a = rng.uniform(0.8, 1.2, shape) if bn_noise else np.ones(shape)
            else:
                a = rng.uniform(-0.1, 0.1, shape) if bn_noise else np.zeros(shape)
        else:
            if name.endswith("weight"):
                fan_in = int(np.prod(shape[1:]))
            else:  # bias: fan_in of the owning layer
                w = net.state_dict()[name[: -len("bias")] + "weight"]
                fan_in = int(np.prod(w.shape[1:]))
            bound = 1.0 / np.sqrt(fan_in)
            a = rng.uniform(-bound, bound, shape)
        sd[name] = torch.from_numpy(np.asarray(a, dtype=np.float32))
    return sd


def _affine(sd, conv, bn):
    w = sd[conv + ".weight"].double()
    b = sd[conv + ".bias"].double()
    g = sd[bn + ".weight"].double()
    beta = sd[bn + ".bias"].double()
    mean = sd[bn + ".running_mean"].double()
    var = sd[bn + ".running_var"].double()
    s = g / torch.sqrt(var + BN_EPS)
    t = (b - mean) * s + beta
    return w, s.float(), t.float()


# float offsets, mirror of csrc/gz_pvnet.h
K0 = 28
K = 9 * CH
C0_W = 0
C0_S = C0_W + K0 * CH
C0_T = C0_S + CH
RES0 = C0_T + CH
RES_STRIDE = K * CH + 2 * CH
P_W = RES0 + 4 * RES_STRIDE
P_B = P_W + 2 * CH
PF_WT = P_B + 4
PF_B = PF_WT + 450 * 225
V_W = PF_B + 228
V_B = V_W + CH
V1_WT = V_B + 4
V1_B = V1_WT + 225 * 64
V2_W = V1_B + 64
V2_B = V2_W + 64
F16_RES0 = (V2_B + 4 + 3) & ~3  # 16-byte aligned (h8 loads)
F16_STRIDE = K * CH
F16_C0 = F16_RES0 + 4 * F16_STRIDE
PF_P = F16_C0 + 8 * 64 * 8
PF_KB, PF_NT = 29, 15
V1_P = PF_P + PF_KB * PF_NT * 256
V1_KB, V1_NT = 15, 4
TOTAL = V1_P + V1_KB * V1_NT * 256

PRECISIONS = {"fp32": 0, "f16x3": 1}  # GZ_PV_FP32, GZ_PV_F16X3

PV_MACS = 133_690_114  # conv0 777,600 + 4 x 33,177,600 + heads 202,114
PV_FLOPS = 2 * PV_MACS


def pack_mfma_b(wt, kb, nt):
    """W^T [K][N] (K-major) -> MFMA B-fragment order [kb][nt][lane 64][4] of the
    batched heads (csrc/gz_f16conv.h heads_gemm_block): element (kb, t, lane, j) =
    W^T[16 kb + 4 (lane // 16) + j][16 t + lane % 16], zero past K and N."""
    wt = np.asarray(wt, np.float32)
    pad = np.zeros((16 * kb, 16 * nt), np.float32)
    pad[:wt.shape[0], :wt.shape[1]] = wt
    # [kb][g 4][j 4][nt][li 16] -> [kb][nt][g][li][j]
    return pad.reshape(kb, 4, 4, nt, 16).transpose(0, 3, 1, 4, 2).reshape(-1)


def pack_pv_weights(sd):
    """state_dict (reference names) -> float32 blob of TOTAL floats."""
    sd = {k: v.detach().cpu() for k, v in sd.items()}
    blob = np.zeros(TOTAL, np.float32)
    w, s, t = _affine(sd, "conv", "bn")  # [128,3,3,3]
    w0 = w.permute(2, 3, 1, 0).reshape(27, CH)  # k = (kh*3+kw)*3 + cin
    blob[C0_W:C0_W + 27 * CH] = w0.float().numpy().reshape(-1)
    blob[C0_S:C0_S + CH] = s.numpy()
    blob[C0_T:C0_T + CH] = t.numpy()
    # fp16 conv0 A fragments: [n-tile][lane][8], n = 16*nt + lane%16, k = 8*(lane//16) + j
    w0p = np.zeros((32, CH), np.float32)
    w0p[:27] = w0.float().numpy()
    w0t = w0p.T  # [n][k]
    h0 = w0t.astype(np.float16)
    l0 = (w0t - h0.astype(np.float32)).astype(np.float16)

    def frag0(x):  # [n=(nt,li)][k=(q,j)] -> [nt][q][li][j]
        return x.reshape(8, 16, 4, 8).transpose(0, 2, 1, 3).reshape(-1)
    blob[F16_C0:F16_C0 + 8 * 64 * 8] = np.concatenate([frag0(h0), frag0(l0)]).view(np.float32)
    convs = []
    for i in range(2):
        convs.append((f"residual_tower.{i}.conv1", f"residual_tower.{i}.bn1"))
        convs.append((f"residual_tower.{i}.conv2", f"residual_tower.{i}.bn2"))
    for j, (cn, bn) in enumerate(convs):
        w, s, t = _affine(sd, cn, bn)  # [128(out),128(in),3,3]
        wk = w.permute(2, 3, 1, 0).reshape(K, CH)  # k = (kh*3+kw)*128 + cin
        base = RES0 + j * RES_STRIDE
        blob[base:base + K * CH] = wk.float().numpy().reshape(-1)
        # fp16x3 copy: W^T split into hi = fp16(w), lo = fp16(w - hi), each in
        # MFMA B-fragment order [ks 36][n-tile 8][lane 64][8 halves] with
        # n = 16*n_tile + lane%16, k = 32*ks + 8*(lane//16) + j (1 KiB per wave load)
        wt = wk.float().numpy().T.copy()  # [n][k]
        hi = wt.astype(np.float16)
        lo = (wt - hi.astype(np.float32)).astype(np.float16)

        def frag(x):  # [n=(nt,li)][k=(ks,q,j)] -> [ks][nt][q][li][j]
            return x.reshape(8, 16, 36, 4, 8).transpose(2, 0, 3, 1, 4).reshape(-1)
        halves = np.concatenate([frag(hi), frag(lo)])
        fb = F16_RES0 + j * F16_STRIDE
        blob[fb:fb + F16_STRIDE] = halves.view(np.float32)
        blob[base + K * CH:base + K * CH + CH] = s.numpy()
        blob[base + K * CH + CH:base + K * CH + 2 * CH] = t.numpy()
    blob[P_W:P_W + 2 * CH] = sd["policy_conv.weight"].reshape(2, CH).numpy().reshape(-1)
    blob[P_B:P_B + 2] = sd["policy_conv.bias"].numpy()
    blob[PF_WT:PF_WT + 450 * 225] = sd["policy_fc.weight"].t().contiguous().numpy().reshape(-1)
    blob[PF_B:PF_B + 225] = sd["policy_fc.bias"].numpy()
    blob[V_W:V_W + CH] = sd["value_conv.weight"].reshape(CH).numpy()
    blob[V_B] = float(sd["value_conv.bias"][0])
    blob[V1_WT:V1_WT + 225 * 64] = sd["value_fc1.weight"].t().contiguous().numpy().reshape(-1)
    blob[V1_B:V1_B + 64] = sd["value_fc1.bias"].numpy()
    blob[V2_W:V2_W + 64] = sd["value_fc2.weight"].reshape(64).numpy()
    blob[V2_B] = float(sd["value_fc2.bias"][0])
    blob[PF_P:V1_P] = pack_mfma_b(sd["policy_fc.weight"].t().numpy(), PF_KB, PF_NT)
    blob[V1_P:TOTAL] = pack_mfma_b(sd["value_fc1.weight"].t().numpy(), V1_KB, V1_NT)
    return blob


def pack_pv_weights_torch(sd, device="cuda"):
    """pack_pv_weights with torch ops on ``device``: the same blob, bit for bit (the BN
    fold in float64, fp16 rounding to nearest even on both sides), as a float32 tensor
    there.  The training loop repacks after every SGD phase; on the host that took
    ~0.4-0.8 s of numpy per iteration (tests/test_weights_pack.py checks the two agree)."""
    dev = torch.device(device)
    sd = {k: v.detach().to(dev) for k, v in sd.items()}
    blob = torch.zeros(TOTAL, dtype=torch.float32, device=dev)

    def split(x):  # fp32 -> (fp16 hi, fp16 lo)
        hi = x.half()
        return hi, (x - hi.float()).half()

    def as_f32(halves):
        return halves.contiguous().view(torch.float32)

    w, s, t = _affine(sd, "conv", "bn")
    w0 = w.permute(2, 3, 1, 0).reshape(27, CH).float()
    blob[C0_W:C0_W + 27 * CH] = w0.reshape(-1)
    blob[C0_S:C0_S + CH] = s
    blob[C0_T:C0_T + CH] = t
    w0p = torch.zeros(32, CH, dtype=torch.float32, device=dev)
    w0p[:27] = w0
    h0, l0 = split(w0p.t().contiguous())

    def frag0(x):
        return x.reshape(8, 16, 4, 8).permute(0, 2, 1, 3).reshape(-1)
    blob[F16_C0:F16_C0 + 8 * 64 * 8] = as_f32(torch.cat([frag0(h0), frag0(l0)]))

    def frag(x):
        return x.reshape(8, 16, 36, 4, 8).permute(2, 0, 3, 1, 4).reshape(-1)
    for j in range(4):
        i, c = divmod(j, 2)
        w, s, t = _affine(sd, f"residual_tower.{i}.conv{c + 1}", f"residual_tower.{i}.bn{c + 1}")
        wk = w.permute(2, 3, 1, 0).reshape(K, CH).float()
        base = RES0 + j * RES_STRIDE
        blob[base:base + K * CH] = wk.reshape(-1)
        hi, lo = split(wk.t().contiguous())
        fb = F16_RES0 + j * F16_STRIDE
        blob[fb:fb + F16_STRIDE] = as_f32(torch.cat([frag(hi), frag(lo)]))
        blob[base + K * CH:base + K * CH + CH] = s
        blob[base + K * CH + CH:base + K * CH + 2 * CH] = t

    def mfma_b(wt, kb, nt):
        pad = torch.zeros(16 * kb, 16 * nt, dtype=torch.float32, device=dev)
        pad[:wt.shape[0], :wt.shape[1]] = wt
        return pad.reshape(kb, 4, 4, nt, 16).permute(0, 3, 1, 4, 2).reshape(-1)
    pw, vw1 = sd["policy_fc.weight"].float(), sd["value_fc1.weight"].float()
    blob[P_W:P_W + 2 * CH] = sd["policy_conv.weight"].reshape(-1)
    blob[P_B:P_B + 2] = sd["policy_conv.bias"]
    blob[PF_WT:PF_WT + 450 * 225] = pw.t().reshape(-1)
    blob[PF_B:PF_B + 225] = sd["policy_fc.bias"]
    blob[V_W:V_W + CH] = sd["value_conv.weight"].reshape(-1)
    blob[V_B:V_B + 1] = sd["value_conv.bias"][:1]
    blob[V1_WT:V1_WT + 225 * 64] = vw1.t().reshape(-1)
    blob[V1_B:V1_B + 64] = sd["value_fc1.bias"]
    blob[V2_W:V2_W + 64] = sd["value_fc2.weight"].reshape(-1)
    blob[V2_B:V2_B + 1] = sd["value_fc2.bias"][:1]
    blob[PF_P:V1_P] = mfma_b(pw.t(), PF_KB, PF_NT)
    blob[V1_P:TOTAL] = mfma_b(vw1.t(), V1_KB, V1_NT)
    return blob


def reference_forward(sd, planes):
    """fp32 torch CPU forward of the same network (test oracle for the kernel)."""
    net = PolicyValueNet()
    net.load_state_dict(sd)
    net.eval()
    with torch.no_grad():
        lg, v = net(torch.as_tensor(planes, dtype=torch.float32))
    return lg.numpy(), v.numpy().reshape(-1)
