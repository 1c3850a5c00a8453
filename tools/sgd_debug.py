"""Diagnostics of the device training tower (csrc/gz_sgd.hip) on one batch: reads the
workspace after gz_sgd_forward (layout of ws_layout) and compares every stage with a
float64 torch computation from the same saved inputs -- weight fragments (hi + lo vs
w x 2^k), the conv outputs y1..y4, the activations, the BN coefficients.
usage: python tools/sgd_debug.py [boards]"""
import copy
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "alphazero-gomoku_amd"), REPO]
from gzero import sgd, weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
FRAG = 36 * 8 * 64 * 8
A = lambda x: (x + 255) // 256 * 256  # noqa: E731


def main():
    net = weights.PolicyValueNet()
    net.load_state_dict(weights.init_state_dict(20251131))
    rng = np.random.default_rng(20251231)
    cells = rng.choice(np.array([0, 0, 0, 1, 2], np.int8), size=(B, 225))
    x = torch.from_numpy(np.stack([cells == 1, cells == 2, cells == 0], 1).reshape(B, 3, 15, 15).astype(np.float32))
    dev = copy.deepcopy(net).cuda().train()
    keep = {}
    orig = sgd._Tower.forward

    def spy(ctx, y0, n, *params):
        out = orig(ctx, y0, n, *params)
        keep["ws"], keep["y0"] = ctx.ws, ctx.keep[0]
        return out
    sgd._Tower.forward = staticmethod(spy)
    with torch.no_grad():
        h = sgd.tower(dev, dev.conv(x.cuda()))
    torch.cuda.synchronize()
    ws = keep["ws"]
    R = B * 225 * 128 * 4
    off = 0

    def take(n):
        nonlocal off
        o = off
        off += A(n)
        return o
    o_frag = take(4 * 2 * 2 * FRAG * 2)
    o_y = [None] + [take(R) for _ in range(4)]
    o_act = [take(R) for _ in range(4)]
    [take(R) for _ in range(5)]
    take(R)
    o_coef = take(5 * 1152 * 4)
    o_wsc = take(32)
    o_xmax = take(4 * B * 4)

    def f32(o, n):
        return ws[o:o + 4 * n].view(torch.float32).double().cpu()
    frag = ws[o_frag:o_frag + 4 * 2 * 2 * FRAG * 2].view(torch.float16).double().cpu().view(4, 2, 2, FRAG)
    wsc = f32(o_wsc, 8)
    print("weight inverse scales", wsc[4:].tolist())
    convs = sgd._convs(dev)
    for L in range(4):
        W = convs[L].weight.detach().double().cpu()  # [n][c][3][3]
        i = torch.arange(FRAG)
        j, lane, nt, ks = i & 7, (i >> 3) & 63, (i >> 9) & 7, i >> 12
        n, k = 16 * nt + (lane & 15), 32 * ks + 8 * (lane >> 4) + j
        tap, c = k >> 7, k & 127
        want = W.reshape(128, 128, 9)[n, c, tap]
        got = (frag[L, 0, 0] + frag[L, 0, 1]) * wsc[4 + L]
        lo = frag[L, 0, 1]
        print(f"conv{L + 1}: fragments max|hi+lo - w| / max|w| = {float((got - want).abs().max() / want.abs().max()):.2e}, "
              f"lo subnormal share {float(((lo.abs() < 6.1e-5) & (lo != 0)).double().mean()):.3f}")
    # stage by stage in float64 from the saved inputs
    act = [f32(o, B * 225 * 128).view(B, 15, 15, 128).permute(0, 3, 1, 2) for o in o_act]
    ys = [None] + [f32(o, B * 225 * 128).view(B, 15, 15, 128).permute(0, 3, 1, 2) for o in o_y[1:]]
    for L in range(4):
        cv = convs[L]
        ref = F.conv2d(act[L], cv.weight.detach().double().cpu(), cv.bias.detach().double().cpu(), padding=1)
        err = (ys[L + 1] - ref).abs().max() / ref.abs().max()
        mio = F.conv2d(act[L].float().cuda(), cv.weight.detach().float(), cv.bias.detach().float(), padding=1).double().cpu()
        emio = (mio - ref).abs().max() / ref.abs().max()
        # per-channel error relative to the channel's batch std (what BatchNorm amplifies)
        sd = ref.std(dim=(0, 2, 3)).view(1, -1, 1, 1)
        rel = lambda t: float(((t - ref) / sd).pow(2).mean().sqrt())  # noqa: E731
        print(f"y{L + 1}: max err / max|y| native {float(err):.2e}, MIOpen {float(emio):.2e}; rms err / channel std "
              f"native {rel(ys[L + 1]):.2e}, MIOpen {rel(mio):.2e}; min channel std {float(sd.min()):.3g}")
    print("tower output max", float(h.abs().max()))
    # backward: the gradient torch's heads hand to the tower, native vs float64
    ref = copy.deepcopy(net).double().train()
    xd = x.double()
    hr = F.relu(ref.bn(ref.conv(xd)))
    hr = ref.residual_tower[0](hr)
    blk = ref.residual_tower[1]
    z3 = blk.bn1(blk.conv1(hr))
    z3.retain_grad()
    hr = F.relu(blk.bn2(blk.conv2(F.relu(z3))) + hr)
    hr.retain_grad()
    lg = ref.policy_fc(torch.flatten(ref.policy_conv(hr), 1))
    v = torch.tanh(ref.value_fc2(F.relu(ref.value_fc1(torch.flatten(ref.value_conv(hr), 1)))))
    yl = torch.from_numpy(rng.integers(0, 225, B))
    yv = torch.from_numpy(rng.uniform(-1, 1, (B, 1)))
    (torch.nn.CrossEntropyLoss()(lg, yl) + torch.nn.MSELoss()(v, yv)).backward()
    dev2 = copy.deepcopy(net).cuda().train()
    got = {}
    ob = sgd._Tower.backward

    def spyb(ctx, gout):
        got["gout"] = gout.detach().double().cpu()
        got["ws"] = ctx.ws
        r = ob(ctx, gout)
        torch.cuda.synchronize()
        return r
    sgd._Tower.backward = staticmethod(spyb)
    lg2, v2 = sgd.train_forward(dev2, x.cuda())
    (torch.nn.CrossEntropyLoss()(lg2, yl.cuda()) + torch.nn.MSELoss()(v2, yv.float().cuda())).backward()
    go = got["gout"]
    # g3 = dL/d(BN3 output) (workspace g[3]) against float64
    o_g = A(4 * 2 * 2 * FRAG * 2) + 8 * A(R)
    ws2 = got["ws"]
    g3 = ws2[o_g + 3 * A(R):o_g + 3 * A(R) + R].view(torch.float32).double().cpu().view(B, 15, 15, 128)
    r3 = z3.grad.permute(0, 2, 3, 1)
    d = g3 - r3
    print(f"g3: rms err / rms g {float(d.pow(2).mean().sqrt() / r3.pow(2).mean().sqrt()):.2e}; per channel "
          f"|sum err| / sum|g| max {float((d.sum((0, 1, 2)).abs() / r3.abs().sum((0, 1, 2))).max()):.2e}, "
          f"|sum g| / sum|g| min {float((r3.sum((0, 1, 2)).abs() / r3.abs().sum((0, 1, 2))).min()):.2e}; "
          f"mean signed err / mean|g| {float(d.mean() / r3.abs().mean()):.2e}")
    h2n = ws2[o_act[3]:o_act[3] + R].view(torch.float32).double().cpu().view(B, 15, 15, 128)
    zr = z3.detach().permute(0, 2, 3, 1)
    agree = (h2n > 0) == (zr > 0)
    dd = torch.where(agree, d, torch.zeros_like(d))
    print(f"mask flips {int((~agree).sum())} of {agree.numel()} (|z3| there max {float(zr[~agree].abs().max()) if (~agree).any() else 0:.2e}); "
          f"g3 rms err on agreeing elements / rms g {float(dd.pow(2).mean().sqrt() / r3.pow(2).mean().sqrt()):.2e}; "
          f"flip-element share of err^2 {float((d.pow(2).sum() - dd.pow(2).sum()) / d.pow(2).sum()):.3f}")
    print(f"dL/d(tower output): native-run heads vs float64: {float((go - hr.grad).norm() / hr.grad.norm()):.2e}")
    for (k, p1), (_, p2) in zip(ref.named_parameters(), dev2.named_parameters()):
        e = float((p2.grad.double().cpu() - p1.grad).norm() / max(p1.grad.norm(), 1e-30))
        print(f"  grad {k}: {e:.2e}")


if __name__ == "__main__":
    main()
