// gz_gnet.h -- packed weight layout of the BG planner's GraphNet + OpponentDQN
// (bg_planner.py:22-78), produced by gzero/planner_nets.py:pack_planner_weights().
//
// fp32 section (K-major like gz_pvnet.h; the C oracle reads it too):
//   embed W [28][64] (k = tap*3 + cin, row 27 zero), b [64]
//   layers 0..7: W then b; even = 3x3 [576][64] (k = tap*64 + cin), odd = 1x1 [64][64]
//   policy conv W [2][64], b [2](+2); policy fc W^T [450][225], b [225](+3)
//   dqn fc0 W^T [675][256], b; fc1 W^T [256][256], b; fc2 W^T [256][225], b (+3)
// then the fc0 restatement below; fp16 section: embed A fragments hi/lo [4][64][8]; per layer hi then lo in
// v_mfma_f32_16x16x32_f16 A-fragment order [ks][n-tile 4][lane 64][8]
// (n = 16*n_tile + lane%16, k = 32*ks + 8*(lane/16) + j).
#pragma once

namespace gzgn {
constexpr int HID = 64;
constexpr int DQH = 256;
constexpr int POS = 225;
constexpr int K3 = 9 * HID;

constexpr int GE_W = 0;
constexpr int GE_B = GE_W + 28 * HID;
constexpr int GL0 = GE_B + HID;
constexpr int layer_off(int i) {
    int off = GL0;
    for (int j = 0; j < i; j++) off += ((j % 2 == 0) ? K3 * HID : HID * HID) + HID;
    return off;
}
constexpr int layer_bias(int i) { return layer_off(i) + ((i % 2 == 0) ? K3 * HID : HID * HID); }
constexpr int GP_W = layer_off(8);
constexpr int GP_B = GP_W + 2 * HID;
constexpr int GF_WT = GP_B + 4;
constexpr int GF_B = GF_WT + 450 * POS;
constexpr int D0_WT = GF_B + 228;
constexpr int D0_B = D0_WT + 3 * POS * DQH;
constexpr int D1_WT = D0_B + DQH;
constexpr int D1_B = D1_WT + DQH * DQH;
constexpr int D2_WT = D1_B + DQH;
constexpr int D2_B = D2_WT + DQH * POS;
constexpr int GH_E = (D2_B + 228 + 3) & ~3;
constexpr int GH_L0 = GH_E + 4 * 64 * 8;
constexpr int KS3 = 18, KS1 = 2;
constexpr int h_layer_off(int i) {
    int off = GH_L0;
    for (int j = 0; j < i; j++) off += ((j % 2 == 0) ? KS3 : KS1) * 4 * 64 * 8;
    return off;
}
// DQN fc0 for one-hot inputs: base [256] = bias + sum of the empty rows;
// delta [450][256] = (black - empty) rows, then (white - empty) rows
constexpr int D0_BASE = h_layer_off(8);
constexpr int D0_DELTA = D0_BASE + DQH;
// the batched heads' GEMMs in MFMA B-fragment order (gz_f16conv.h heads_gemm_block):
// [k-blocks of 16][n-tiles][64][4] of policy fc (450->225), the fc0 delta rows
// (450->256), fc1 (256->256), fc2 (256->225)
constexpr int GF_P = D0_DELTA + 450 * DQH;
constexpr int D0_P = GF_P + 29 * 15 * 256;
constexpr int D1_P = D0_P + 29 * 16 * 256;
constexpr int D2_P = D1_P + 16 * 16 * 256;
constexpr int TOTAL = D2_P + 16 * 15 * 256;

// per-board record between gn_kernel (GraphNet tower + policy conv 1x1) and
// gn_heads_kernel (policy FC + softmax, OpponentDQN): floats
//   [0, 450) policy conv output (channel-major flatten), zero to REC_X;
//   [REC_X, REC_X + 450) the one-hot stone inputs [black 225 | white 225], zero to REC
constexpr int REC_X = 464;
constexpr int REC = 928;

// Incremental GraphNet (gn_inc_kernel): a map slot holds one board's 4 conv inputs
// embed, L1, L3, L5 (each [plane hi/lo][cg 8][225][8] halves) and its policy-conv
// output (450 floats, channel-major, padded to 512)
constexpr int SLOT_MAP_HALVES = 2 * 8 * POS * 8;   // 28,800
constexpr int SLOT_POL = 4 * SLOT_MAP_HALVES / 2;  // floats from the slot start
constexpr size_t SLOT_BYTES = (size_t)4 * SLOT_MAP_HALVES * 2 + 512 * 4;

// one GN row's incremental tag (written by gz_plan.hip's collect kernel)
constexpr int TAG_STONES = 6;
struct GnTag {
    int32_t mode;  // 0: full forward, maps stored into slot `job`; 1: incremental
    int32_t base;  // slot of the maps the board adds stones to
    int32_t job;   // slot this row writes its maps (and policy-conv output) to
    int32_t cell;  // incremental: the new stone (r*15+c)
    int32_t nst;   // stones already added to `base` whose squares live in slot `job`
    uint8_t st[TAG_STONES];
    uint8_t pad[2];
    int32_t pad2;
};
static_assert(sizeof(GnTag) == 32, "tag size");
}  // namespace gzgn
