// gz_pvnet.h -- packed weight layout of AlphaZeroGomokuNet (neural_network.py:94-159)
// for the fp32 MFMA forward.  Produced by gzero/weights.py:pack_pv_weights().
//
// Conv weights are stored K-major as the GEMM B operand W[k][n]:
//   conv0:     k = tap*3 + cin   (27 rows + 1 zero row), n = out channel (128)
//   res convs: k = tap*128 + cin (1152 rows),           n = out channel (128)
// with tap = kh*3 + kw.  Bias and eval-mode BatchNorm are folded into a
// per-channel affine epilogue: y = acc*S[n] + T[n],
//   S = gamma / sqrt(running_var + eps), T = (bias - running_mean)*S + beta.
// Head weights: 1x1 convs as [out][128]; FCs stored transposed ([in][out]) so a
// thread per output reads coalesced rows.
#pragma once

namespace gzpv {
constexpr int CH = 128;
constexpr int POS = 225;
constexpr int K0 = 28;          // 27 padded to a multiple of the MFMA K-step (2)
constexpr int K = 9 * CH;       // 1152

constexpr int C0_W = 0;
constexpr int C0_S = C0_W + K0 * CH;
constexpr int C0_T = C0_S + CH;
constexpr int RES0 = C0_T + CH;
constexpr int RES_STRIDE = K * CH + 2 * CH;  // W, S, T
constexpr int RES_W = 0, RES_S = K * CH, RES_T = K * CH + CH;
constexpr int P_W = RES0 + 4 * RES_STRIDE;   // [2][128]
constexpr int P_B = P_W + 2 * CH;            // [2] (+2 pad)
constexpr int PF_WT = P_B + 4;               // [450][225]
constexpr int PF_B = PF_WT + 450 * 225;      // [225] (+3 pad)
constexpr int V_W = PF_B + 228;              // [128]
constexpr int V_B = V_W + CH;                // [1] (+3 pad)
constexpr int V1_WT = V_B + 4;               // [225][64]
constexpr int V1_B = V1_WT + 225 * 64;       // [64]
constexpr int V2_W = V1_B + 64;              // [64]
constexpr int V2_B = V2_W + 64;              // [1] (+3 pad)
// fp16x3 section: per residual conv, fp16 hi then fp16 lo (2 halves per float
// slot), each in v_mfma_f32_16x16x32_f16 B-fragment order
//   [ks 36][n-tile 8][lane 64][8]:  n = 16*n_tile + lane%16, k = 32*ks + 8*(lane/16) + j
// so one wave's fragment is one contiguous 1 KiB load; S/T are shared with the fp32 section
constexpr int F16_RES0 = (V2_B + 4 + 3) & ~3;  // 16-byte aligned for h8 loads
constexpr int F16_STRIDE = K * CH;           // floats: K*CH halves hi + K*CH halves lo
// conv0 in fp16 MFMA A-fragment order [n-tile 8][lane 64][8]: n = 16*n_tile + lane%16,
// k = 8*(lane/16) + j (k >= 27 zero); hi then lo
constexpr int F16_C0 = F16_RES0 + 4 * F16_STRIDE;
// FC heads in MFMA B-fragment order for the batched heads kernel (gz_f16conv.h
// heads_gemm_block): policy_fc [29 k-blocks][15 n-tiles][64][4], value_fc1 [15][4][64][4]
constexpr int PF_P = F16_C0 + 8 * 64 * 8;
constexpr int PF_KB = 29, PF_NT = 15;
constexpr int V1_P = PF_P + PF_KB * PF_NT * 256;
constexpr int V1_KB = 15, V1_NT = 4;
constexpr int TOTAL = V1_P + V1_KB * V1_NT * 256;

// incremental forward (gz_pvinc.hip): a root board's intermediate maps x0, y1, x1,
// y2 are stored in the LDS layout of the f16x3 kernel: hi plane [16 ch-groups]
// [256 rows][8] then the lo plane -- PV_MAP_HALVES halves per map
constexpr int PV_MAP_PLANE = CH * 256;
constexpr int PV_MAP_HALVES = 2 * PV_MAP_PLANE;
// delta tree forward (gz_pvinc.hip, pv_delta_kernel): a root board's pre-ReLU values
// of the 4 residual layers (y1, x1, y2, x2: z = BN(conv) [+ skip input]), fp32
// position-major [256 positions][128 channels] -- PV_PRE_FLOATS floats per layer
constexpr int PV_PRE_FLOATS = 256 * CH;
// a root child's recomputed squares / D squares (x0 r1, y1 r2, x1 r3, y2 r4: 164
// positions x 256 halves), the unit of the patch slots and of the tree scratch
constexpr int PV_PATCH_HALVES = 164 * 256;
// tree scratch per grid entry (one per CU): PV_SCRATCH_PATCHES patch-sized areas,
// shared by the workgroups of pv_sib_kernel / pv_dg_kernel on that entry (each kernel
// static_asserts its workgroups x nodes per chunk against it)
constexpr int PV_SCRATCH_PATCHES = 12;
// per-board record of the 1x1 head convs' outputs between the tower and the FC heads
// (gz_pvnet.hip / gz_pvinc.hip -> pv_heads_kernel): hp [0, 450) channel-major, zero to
// HP_K; hv [HV_OFF, HV_OFF + 225), zero to HSTRIDE
constexpr int HP_K = 464, HV_OFF = HP_K, HV_K = 240, HSTRIDE = HV_OFF + HV_K;

// algorithmic work of one forward (neural_network.py:132-159), MACs
constexpr long long MACS = 133690114LL;
}  // namespace gzpv
