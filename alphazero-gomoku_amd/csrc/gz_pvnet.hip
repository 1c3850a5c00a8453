// gz_pvnet.hip -- AlphaZeroGomokuNet forward (neural_network.py:94-159) plus the
// softmax of GomokuModel.predict (neural_network.py:214-252) on gfx950.
//
// One 512-thread workgroup (8 waves) evaluates one board at a time and loops
// over boards.  The board's 128x225 activation map stays in LDS for the whole
// tower; every 3x3 conv is an implicit GEMM
//   C[pos][ch] = sum_k A[pos][k] * W[k][ch],  A[pos][tap*128+cin] = act[cin][pos+tap]
// with M = 225 positions (15 tiles of 16), N = 128 channels (8 tiles of 16).
// Off-board neighbours read a zero slot instead of predicating.  Two precisions:
//
//  * GZ_PV_FP32: v_mfma_f32_16x16x4_f32 -- exact f32 products, f32 accumulate.
//    Wave w owns N tile w for all 15 M tiles (each weight fragment read once per
//    board per workgroup).  Activations fp32, channel-major [ch][240].  The skip
//    input of a residual block is parked in a per-wave global slab.
//  * GZ_PV_F16X3: v_mfma_f32_16x16x32_f16 on a 3-term split, x = x_hi + x_lo
//    (x_hi = fp16(x), x_lo = fp16(x - x_hi)):  a*w ~ a_hi*w_hi + a_hi*w_lo +
//    a_lo*w_hi, every product exact in the f32 accumulator, ~22-bit operands.
//    16x the f32 MFMA rate per instruction, 5.3x per fp32-equivalent product.
//    Wave w owns 2 N tiles x 8 (or 7) M tiles, halving the LDS A-fragment reads
//    per MFMA; activations as hi/lo fp16 planes [16 ch-groups][240][8]
//    (conflict-free ds_read_b128); weights pre-arranged in B-fragment order.
//    The skip input of a residual block stays in registers.
#include <hip/hip_runtime.h>

#include <string>

#include "gz_f16conv.h"
#include "gz_pvnet.h"
#include "../../include/gzero.h"

using namespace gzpv;

namespace {

using namespace gzc;

constexpr int MT = 15;     // 16-position M tiles (240 >= 225)
constexpr int ROWS = 240;  // positions incl. 15 zero rows / slots
constexpr int ZERO = POS;  // index of a zero slot: the out-of-board neighbour
constexpr int SLAB_F = 4096;  // per-wave skip slab (floats): fp32 15*4*64, f16x3 2*8*4*64

// LDS layout (bytes): activation area first, then shared small buffers
constexpr int ACT_BYTES_F32 = CH * ROWS * 4;      // 122880
constexpr int ACT_BYTES_F16 = 2 * CH * 256 * 2;  // 131072: hi + lo planes of 256 rows
constexpr int ACT_BYTES = ACT_BYTES_F16 > ACT_BYTES_F32 ? ACT_BYTES_F16 : ACT_BYTES_F32;


// Phase stamps (tools/pv_stamps.py only): -DGZ_PV_STAMPS accumulates s_memtime
// deltas of workgroup 0 / wave 0 per phase; compiled out otherwise.
#ifdef GZ_PV_STAMPS
__device__ unsigned long long gz_pv_stamps[32];
#define PV_STAMP(i)                                                             \
    do {                                                                        \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                              \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
            gz_pv_stamps[i] += t_ - gz_pv_stamps[31];                           \
            gz_pv_stamps[31] = t_;                                              \
        }                                                                       \
    } while (0)
#define PV_WAVE_T0() unsigned long long wt0_ = __builtin_amdgcn_s_memtime()
#define PV_WAVE_STAMP(slot)                                                                          \
    do {                                                                                             \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) {                                            \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();                                    \
            atomicAdd(&gz_pv_stamps[(slot) + (threadIdx.x >> 6)], t_ - wt0_);                         \
            wt0_ = t_;                                                                               \
        }                                                                                            \
    } while (0)
#else
#define PV_WAVE_T0() \
    do {             \
    } while (0)
#define PV_WAVE_STAMP(slot) \
    do {                    \
    } while (0)
#define PV_STAMP(i) \
    do {            \
    } while (0)
#endif

// neighbour index of the lane's position in M tile m for tap (dr, dc); ZERO if off-board
__device__ inline int nbr(int m, int li, int dr, int dc) {
    int pos = m * 16 + li;
    int r = pos / 15 + dr, c = pos % 15 + dc;
    bool ok = pos < POS && r >= 0 && r < 15 && c >= 0 && c < 15;
    return ok ? r * 15 + c : ZERO;
}

// ============================================================ fp32 policy
struct ActF32 {
    float* a;  // [CH][ROWS]
    float* slab;
    __device__ float get(int ch, int pos) const { return a[ch * ROWS + pos]; }
    __device__ void put(int ch, int pos, float y) { a[ch * ROWS + pos] = y; }
    __device__ void get8(int c0, int pos, float* x) const {
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = a[(c0 + j) * ROWS + pos];
    }
    __device__ void zero_slots(int tid, int nth) {
        for (int i = tid; i < CH * (ROWS - POS); i += nth) a[(i / (ROWS - POS)) * ROWS + POS + i % (ROWS - POS)] = 0.f;
    }
    // k = tap*128 + cin, 4 input channels per k-step; B double-buffered 8 k-steps ahead
    __device__ __forceinline__ void conv(const float* __restrict__ Wk, int nt, int lane, f32x4 acc[MT]) const {
        const int li = lane & 15, g = lane >> 4;
        const float* wbase = Wk + (size_t)g * CH + nt * 16 + li;
        float bq[8], bn[8];
#pragma unroll
        for (int s = 0; s < 8; s++) bq[s] = wbase[(size_t)(4 * s) * CH];
        for (int blk = 0; blk < 36; blk++) {  // 9 taps x 4 blocks of 8 k-steps
            const int tap = blk >> 2, sb = blk & 3;
            const int dr = tap / 3 - 1, dc = tap % 3 - 1;
            int lv = li;
            asm volatile("" : "+v"(lv));  // keep the 9x15 neighbour indices from being hoisted (spills)
            int nb[MT];
#pragma unroll
            for (int m = 0; m < MT; m++) nb[m] = nbr(m, lv, dr, dc);
            if (blk + 1 < 36) {
                const int t2 = (blk + 1) >> 2, s2 = (blk + 1) & 3;
                const float* wp = wbase + (size_t)(t2 * CH + 32 * s2) * CH;
#pragma unroll
                for (int s = 0; s < 8; s++) bn[s] = wp[(size_t)(4 * s) * CH];
            }
            const float* ab = a + (32 * sb + g) * ROWS;
#pragma unroll
            for (int s = 0; s < 8; s++) {
                const float* ap = ab + 4 * s * ROWS;
                float av[MT];
#pragma unroll
                for (int m = 0; m < MT; m++) av[m] = ap[nb[m]];
#pragma unroll
                for (int m = 0; m < MT; m++)
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bq[s], acc[m], 0, 0, 0);
            }
#pragma unroll
            for (int s = 0; s < 8; s++) bq[s] = bn[s];
        }
    }
};

// ============================================================ fp16x3 policy (gz_f16conv.h)
template <int NM>
__device__ __forceinline__ void f16_load(const ActF16x3& act, f32x4 (&out)[2][NM], int np, int m0, int lane) {
    asm volatile("" : "+v"(lane));  // addresses are recomputed per layer, not hoisted (and spilled)
    lane &= 63;
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int m = 0; m < NM; m++) {
            const int pos = (m0 + m) * 16 + (lane & 15);
            if (pos < POS) f16_get4(act, ch0, pos, out[n][m]);
            else out[n][m] = zero4();
        }
    }
}

// f16_put4 that also stores the result to the global copy g of the map (the same
// [hi plane][lo plane] layout as LDS) when g != nullptr: a root board's
// intermediate maps for the incremental forward of its children (gz_pvinc.hip)
template <bool SKIP>
__device__ __forceinline__ void pv_put4(ActF16x3& act, const f32x4& acc, const f32x4& s, const f32x4& t,
                                        const f32x4& skip, int ch0, int pos, _Float16* __restrict__ g,
                                        float* __restrict__ pre) {
    h4 hi, lo;
    f32x4 z;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        float y = __builtin_fmaf(acc[r], s[r], t[r]);
        if (SKIP) y += skip[r];
        z[r] = y;
        y = y > 0.f ? y : 0.f;
        const _Float16 h = (_Float16)y;
        hi[r] = h;
        lo[r] = (_Float16)(y - (float)h);
    }
    const int o = ActF16x3::off(ch0, pos);
    *(h4*)(act.hi + o) = hi;
    *(h4*)(act.lo + o) = lo;
    if (g) {
        *(h4*)(g + o) = hi;
        *(h4*)(g + PV_MAP_PLANE + o) = lo;
    }
    if (pre) *(f32x4*)(pre + pos * CH + ch0) = z;
}

// pre (root boards of the delta tree forward, else nullptr): the layer's pre-ReLU
// values z = BN(acc) (+ the skip input), [pos][128] fp32

template <int NM, bool SKIP>
__device__ __forceinline__ void f16_store(ActF16x3& act, const f32x4 (&acc)[2][NM], const float* __restrict__ S,
                                          const float* __restrict__ T, const f32x4 (&skip)[2][NM], int np, int m0,
                                          int lane, _Float16* __restrict__ g, float* __restrict__ pre) {
    asm volatile("" : "+v"(lane));  // addresses are recomputed per layer, not hoisted (and spilled)
    lane &= 63;
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
        const f32x4 s = *(const f32x4*)(S + ch0), t = *(const f32x4*)(T + ch0);
#pragma unroll
        for (int m = 0; m < NM; m++) {
            const int pos = (m0 + m) * 16 + (lane & 15);
            if (pos < POS) pv_put4<SKIP>(act, acc[n][m], s, t, skip[n][m], ch0, pos, g, pre);
        }
    }
}

// last residual layer: y = relu(acc*S + T + skip) is only consumed by the 1x1
// heads (policy 128->2, value 128->1), so the epilogue reduces it straight into
// per-wave partial head sums hpart[np][3][256] (32 channels each) instead of
// storing the map (neural_network.py:132-142)
template <int NM>
__device__ __forceinline__ void f16_store_heads(const f32x4 (&acc)[2][NM], const float* __restrict__ W,
                                                const float* __restrict__ S, const float* __restrict__ T,
                                                const f32x4 (&skip)[2][NM], int np, int m0, int lane,
                                                float* __restrict__ hpart, float* __restrict__ pre) {
    asm volatile("" : "+v"(lane));
    lane &= 63;
    float s0[NM], s1[NM], sv[NM];
#pragma unroll
    for (int m = 0; m < NM; m++) s0[m] = s1[m] = sv[m] = 0.f;
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
        const f32x4 s = *(const f32x4*)(S + ch0), t = *(const f32x4*)(T + ch0);
        const f32x4 w0 = *(const f32x4*)(W + P_W + ch0), w1 = *(const f32x4*)(W + P_W + CH + ch0);
        const f32x4 wv = *(const f32x4*)(W + V_W + ch0);
#pragma unroll
        for (int m = 0; m < NM; m++) {
            const int pos = (m0 + m) * 16 + (lane & 15);
            if (pre && pos < POS) {
                f32x4 z;
#pragma unroll
                for (int r = 0; r < 4; r++) z[r] = __builtin_fmaf(acc[n][m][r], s[r], t[r]) + skip[n][m][r];
                *(f32x4*)(pre + pos * CH + ch0) = z;
            }
        }
#pragma unroll
        for (int m = 0; m < NM; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float y = __builtin_fmaf(acc[n][m][r], s[r], t[r]) + skip[n][m][r];
                y = y > 0.f ? y : 0.f;
                s0[m] = __builtin_fmaf(w0[r], y, s0[m]);
                s1[m] = __builtin_fmaf(w1[r], y, s1[m]);
                sv[m] = __builtin_fmaf(wv[r], y, sv[m]);
            }
    }
#pragma unroll
    for (int m = 0; m < NM; m++) {
        float a = s0[m], c = s1[m], v = sv[m];
        a += __shfl_xor(a, 16);
        c += __shfl_xor(c, 16);
        v += __shfl_xor(v, 16);
        a += __shfl_xor(a, 32);
        c += __shfl_xor(c, 32);
        v += __shfl_xor(v, 32);
        const int pos = (m0 + m) * 16 + (lane & 15);
        if (lane < 16 && pos < POS) {
            hpart[(np * 3 + 0) * 256 + pos] = a;
            hpart[(np * 3 + 1) * 256 + pos] = c;
            hpart[(np * 3 + 2) * 256 + pos] = v;
        }
    }
}

// gmaps: nullptr, or the root's 4 map copies (x0, y1, x1, y2); y1, x1, y2 are stored here.
// gpre: nullptr, or the root's 4 pre-ReLU maps (PV_PRE_FLOATS each)
template <int NM, int m0>
__device__ __forceinline__ void f16_tower(ActF16x3& act, const float* __restrict__ W, int wave, int lane,
                                          float* __restrict__ hpart, _Float16* __restrict__ gmaps,
                                          float* __restrict__ gpre) {
    const int np = wave & 3;
    for (int blk = 0; blk < 2; blk++) {
        f32x4 skip[2][NM];
        for (int half = 0; half < 2; half++) {
            const int layer = 2 * blk + half;
            const float* R = W + RES0 + layer * RES_STRIDE;
            f32x4 acc[2][NM];
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int m = 0; m < NM; m++) acc[n][m] = zero4();
            PV_WAVE_T0();
            f16_conv<NM, 4, 8, 9>(act, (const _Float16*)(W + F16_RES0 + layer * F16_STRIDE), np, m0, lane, acc);
            PV_STAMP(2);
            PV_WAVE_STAMP(8);
            if (half == 0) f16_load<NM>(act, skip, np, m0, lane);  // block input, for the skip connection
            __syncthreads();
            PV_WAVE_STAMP(16);
            PV_STAMP(3);
            float* pre = gpre ? gpre + (size_t)layer * PV_PRE_FLOATS : nullptr;
            if (half == 0)
                f16_store<NM, false>(act, acc, R + RES_S, R + RES_T, skip, np, m0, lane,
                                     gmaps ? gmaps + (size_t)(1 + layer) * PV_MAP_HALVES : nullptr, pre);
            else if (blk == 0)
                f16_store<NM, true>(act, acc, R + RES_S, R + RES_T, skip, np, m0, lane,
                                    gmaps ? gmaps + (size_t)2 * PV_MAP_HALVES : nullptr, pre);
            else
                f16_store_heads<NM>(acc, W, R + RES_S, R + RES_T, skip, np, m0, lane, hpart, pre);
            __syncthreads();
            PV_STAMP(4);
        }
    }
}

// conv0 3->128 + BN + ReLU in f16 (C^T form): the input planes are 0/1, exact in
// fp16, so a*w = a*w_hi + a*w_lo (2 MFMAs, no a_lo term); K = 27 (k = tap*3 + cin)
// padded to one 32-deep k-step.  Wave w: N tile w, all 15 M tiles.
// im2col of conv0 for the board in `planes`: col[row][k] (fp16, 0/1 exactly),
// k = tap*3 + cin (27 -> 32 zero-padded), row = position (rows >= 225 zero).
// One thread per (row, k-half); built once per board for all 8 waves.
template <int NTH>
__device__ __forceinline__ void build_im2col(_Float16* __restrict__ col, const float* __restrict__ planes, int tid) {
    for (int t = tid; t < 256 * 2; t += NTH) {
        const int row = t >> 1, k0 = (t & 1) * 16;
        const int r = row / 15, c = row % 15;
        h8 v[2];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int k = k0 + j;
            const int tap = k / 3, cin = k % 3;
            const int rr = r + tap / 3 - 1, cc = c + tap % 3 - 1;
            const bool ok = k < 27 && row < POS && rr >= 0 && rr < 15 && cc >= 0 && cc < 15;
            v[j >> 3][j & 7] = ok ? (_Float16)planes[cin * ROWS + rr * 15 + cc] : (_Float16)0.f;
        }
        *(h8*)(col + row * 32 + k0) = v[0];
        *(h8*)(col + row * 32 + k0 + 8) = v[1];
    }
}

// conv0 3->128 + BN + ReLU in f16 (C^T form): the input planes are 0/1, exact in
// fp16, so a*w = a*w_hi + a*w_lo (2 MFMAs, no a_lo term); K = 27 (k = tap*3 + cin)
// padded to one 32-deep k-step.  Wave w: N tile w, all 15 M tiles.
__device__ __forceinline__ void conv0_f16(ActF16x3& act, const float* __restrict__ W, const _Float16* col, int nt,
                                          int lane, _Float16* __restrict__ g) {
    const int li = lane & 15, q = lane >> 4;
    const _Float16* wf = (const _Float16*)(W + F16_C0) + ((size_t)nt * 64 + lane) * 8;
    const h8 bh = *(const h8*)wf, bl = *(const h8*)(wf + 8 * 64 * 8);
    const int ch0 = nt * 16 + 4 * q;
    const f32x4 s = *(const f32x4*)(W + C0_S + ch0), t = *(const f32x4*)(W + C0_T + ch0);
    const f32x4 none = zero4();
    h8 a[MT];
#pragma unroll
    for (int m = 0; m < MT; m++) a[m] = *(const h8*)(col + (m * 16 + li) * 32 + 8 * q);
#pragma unroll
    for (int m = 0; m < MT; m++) {
        f32x4 acc = zero4();
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, a[m], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl, a[m], acc, 0, 0, 0);
        const int pos = m * 16 + li;
        if (pos < POS) pv_put4<false>(act, acc, s, t, none, ch0, pos, g, nullptr);
    }
}

// epilogue: y = acc*S + T (+ skip), ReLU, back into the map.
// C layout of the 16x16 MFMAs: column (channel) = lane&15, row (position) = 4*(lane>>4) + r.
template <class Act>
__device__ __forceinline__ void store_tiles(Act& act, const f32x4 acc[MT], const float* __restrict__ S,
                                           const float* __restrict__ T, const f32x4* skip, int nt, int lane) {
    const int ch = nt * 16 + (lane & 15), g = lane >> 4;
    const float s = S[ch], t = T[ch];
#pragma unroll
    for (int m = 0; m < MT; m++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int pos = m * 16 + 4 * g + r;
            if (pos < POS) {
                float y = __builtin_fmaf(acc[m][r], s, t);
                if (skip) y += skip[m][r];
                act.put(ch, pos, y > 0.f ? y : 0.f);
            }
        }
    }
}

// fp32 path: the block input goes to a lane-contiguous global slab (one 256-B
// access per value per wave) because 60 more VGPRs do not fit beside the B ring
__device__ __forceinline__ void slab_save(const ActF32& act, float* __restrict__ slab, int nt, int lane) {
    const int ch = nt * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int pos = m * 16 + 4 * g + r;
            slab[(m * 4 + r) * 64 + lane] = pos < POS ? act.get(ch, pos) : 0.f;
        }
}

__device__ __forceinline__ void slab_load(const float* __restrict__ slab, f32x4 out[MT], int lane) {
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) out[m][r] = slab[(m * 4 + r) * 64 + lane];
}

// ---- shared pieces of both kernels; NTH = threads per workgroup

struct Smem {
    float* planes;  // [3][ROWS] fp32 input planes
    float* hp;      // [2*POS] policy 1x1 conv output (channel-major flatten)
    float* hv;      // [POS] value 1x1 conv output
    float* red;     // [32] softmax reductions
    float* lg;      // [256] logits, then exp(logit - max)
    float* part;    // [2][256] policy_fc partial sums
    float* vq;      // [3][64] value_fc1 partial sums
    float* hpart;   // [4][3][256] fused 1x1 head partial sums (f16x3 kernel)
};
// the f16x3 kernel's conv0 im2col (256 x 32 halves) reuses hp..hpart
static_assert((2 * POS + POS + 32 + 256 + 512 + 192 + 4 * 3 * 256) * 4 >= 256 * 32 * 2, "im2col space");
constexpr int SMALL_F = 3 * ROWS + 2 * POS + POS + 32 + 256 + 512 + 192 + 4 * 3 * 256;
constexpr int LDS_BYTES = ACT_BYTES + SMALL_F * 4;

__device__ inline Smem smem_layout(char* lds) {
    Smem m;
    m.planes = (float*)(lds + ACT_BYTES);
    m.hp = m.planes + 3 * ROWS;
    m.hv = m.hp + 2 * POS;
    m.red = m.hv + POS;
    m.lg = m.red + 32;
    m.part = m.lg + 256;
    m.vq = m.part + 512;
    m.hpart = m.vq + 192;
    return m;
}

// input planes [black, white, empty] (gomoku_board.py:239-260, absolute colours)
template <int NTH>
__device__ __forceinline__ void load_planes(float* planes, const uint32_t* __restrict__ bd, int tid) {
    for (int p = tid; p < POS; p += NTH) {
        int bit = (p / 15) * 16 + (p % 15);
        uint32_t bl = (bd[bit >> 5] >> (bit & 31)) & 1u;
        uint32_t wh = (bd[8 + (bit >> 5)] >> (bit & 31)) & 1u;
        planes[p] = (float)bl;
        planes[ROWS + p] = (float)wh;
        planes[2 * ROWS + p] = (float)(1u - (bl | wh));
    }
}

// conv0 3->128 + BN + ReLU for N tile nt (exact f32 MFMA in both modes): K = 27 (k = tap*3+cin) -> 28
template <class Act>
__device__ __forceinline__ void conv0_tile(Act& act, const float* __restrict__ W, const float* planes, int nt,
                                           int lane) {
    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; m++) acc[m] = zero4();
    int li = lane & 15;
    asm volatile("" : "+v"(li));
    const int g = lane >> 4;
#pragma unroll
    for (int s = 0; s < K0 / 4; s++) {
        const int k = 4 * s + g;
        const int tap = k / 3, cin = k % 3;
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        const float bw = W[C0_W + k * CH + nt * 16 + li];  // row 27 is zero
#pragma unroll
        for (int m = 0; m < MT; m++) {
            int idx = k < 27 ? nbr(m, li, dr, dc) : ZERO;
            float a = planes[(k < 27 ? cin : 0) * ROWS + idx];
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw, acc[m], 0, 0, 0);
        }
    }
    store_tiles(act, acc, W + C0_S, W + C0_T, (const f32x4*)nullptr, nt, lane);
}

// heads (neural_network.py:132-159) + softmax (neural_network.py:240-247) for board b;
// the tower's output map is in act.  Ends with a barrier.
template <int NTH, class Act>
__device__ __forceinline__ void heads(const Act& act, const Smem& sm, const float* __restrict__ W, int b, int tid,
                                      float* __restrict__ logits, float* __restrict__ value,
                                      float* __restrict__ probs) {
    const int lane = tid & 63, wave = tid >> 6;
    // 1x1 convs (policy 128->2, value 128->1), one thread per position
    if (tid < POS) {
        const int pos = tid;
        float p0 = W[P_B], p1 = W[P_B + 1], v = W[V_B];
        for (int c0 = 0; c0 < CH; c0 += 8) {
            float a[8];
            act.get8(c0, pos, a);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                p0 += W[P_W + c0 + j] * a[j];
                p1 += W[P_W + CH + c0 + j] * a[j];
                v += W[V_W + c0 + j] * a[j];
            }
        }
        sm.hp[pos] = p0;  // flatten order: channel-major (policy.view(B, -1))
        sm.hp[POS + pos] = p1;
        sm.hv[pos] = v;
    }
    __syncthreads();
    PV_STAMP(5);
    // policy_fc 450->225: thread (h, o) sums input part h of NTH/256 for output o
    constexpr int NH = NTH / 256, HI = 2 * POS / NH;
    {
        const int o = tid & 255, h = tid >> 8;
        if (o < POS) sm.part[h * 256 + o] = dot_col<HI, 45>(W + PF_WT + (size_t)h * HI * POS + o, POS, sm.hp + h * HI);
    }
    __syncthreads();
    // logits = bias + parts; value_fc1 225->64 in input thirds (192 threads: waves 4-6, or 0-2 at 256 threads)
    if (tid < POS) {
        float l = W[PF_B + tid];
#pragma unroll
        for (int h = 0; h < NH; h++) l += sm.part[h * 256 + tid];
        sm.lg[tid] = l;
    }
    {
        const int t = NTH == 512 ? tid - 256 : tid;
        if (t >= 0 && t < 192) {
            const int j = t & 63, t3 = t >> 6;
            sm.vq[t3 * 64 + j] = dot_col<75, 25>(W + V1_WT + t3 * 75 * 64 + j, 64, sm.hv + t3 * 75);
        }
    }
    __syncthreads();
    PV_STAMP(6);
    // value_fc1 bias + ReLU, value_fc2 + tanh (wave 0); softmax max/sum over 225 logits (waves 0..3)
    if (wave == 0) {
        float h1 = W[V1_B + lane] + (sm.vq[lane] + sm.vq[64 + lane] + sm.vq[128 + lane]);
        h1 = h1 > 0.f ? h1 : 0.f;
        float part2 = W[V2_W + lane] * h1;
        float tot = wave_sum(part2) + W[V2_B];
        if (lane == 0) value[b] = tanhf(tot);
    }
    if (wave < 4) {
        float x = tid < POS ? sm.lg[tid] : -3.0e38f;
        float mx = wave_max(x);
        if (lane == 0) sm.red[wave] = mx;
    }
    __syncthreads();
    if (wave < 4) {
        const float mx = fmaxf(fmaxf(sm.red[0], sm.red[1]), fmaxf(sm.red[2], sm.red[3]));
        float e = tid < POS ? __expf(sm.lg[tid] - mx) : 0.f;
        float s = wave_sum(e);
        if (lane == 0) sm.red[8 + wave] = s;
        if (tid < POS) {
            logits[(size_t)b * POS + tid] = sm.lg[tid];
            sm.lg[tid] = e;
        }
    }
    __syncthreads();
    if (wave < 4 && probs) {
        const float s = (sm.red[8] + sm.red[9]) + (sm.red[10] + sm.red[11]);
        if (tid < POS) probs[(size_t)b * POS + tid] = sm.lg[tid] / s;
    }
    __syncthreads();
    PV_STAMP(7);
}

__device__ inline int board_count(int n, const int32_t* d_count) {
    if (!d_count) return n;
    int c = *d_count;
    return c < n ? c : n;
}

// ============================================================ fp32 kernel: 8 waves, wave w = N tile w
constexpr int NT32 = 512;
__global__ __launch_bounds__(NT32, 1) void pv_kernel_f32(const float* __restrict__ W,
                                                       const uint32_t* __restrict__ boards, int n,
                                                       const int32_t* d_count, float* __restrict__ logits,
                                                       float* __restrict__ value, float* __restrict__ probs,
                                                       float* __restrict__ scratch) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    const Smem sm = smem_layout(lds);
    ActF32 act;
    act.a = (float*)lds;
    const int count = board_count(n, d_count);
    float* slab = scratch + ((size_t)blockIdx.x * (NT32 / 64) + (threadIdx.x >> 6)) * SLAB_F;
    act.zero_slots(threadIdx.x, NT32);
    for (int i = threadIdx.x; i < 3 * (ROWS - POS); i += NT32)
        sm.planes[(i / (ROWS - POS)) * ROWS + POS + i % (ROWS - POS)] = 0.f;

    for (int b = blockIdx.x; b < count; b += gridDim.x) {
        // re-derive the lane ids per board: nothing lane-dependent is hoisted out
        // of this loop and kept live (spilled) across the whole tower
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, nt = __builtin_amdgcn_readfirstlane(tid >> 6);
        load_planes<NT32>(sm.planes, boards + (size_t)b * 16, tid);
        __syncthreads();
        conv0_tile(act, W, sm.planes, nt, lane);
        __syncthreads();
        // residual tower (ResidualBlock, neural_network.py:74-91)
        for (int blk = 0; blk < 2; blk++) {
            for (int half = 0; half < 2; half++) {
                const int layer = 2 * blk + half;
                const float* R = W + RES0 + layer * RES_STRIDE;
                f32x4 acc[MT];
#pragma unroll
                for (int m = 0; m < MT; m++) acc[m] = zero4();
                act.conv(R + RES_W, nt, lane, acc);
                if (half == 0) slab_save(act, slab, nt, lane);  // keep the block input for the skip connection
                __syncthreads();
                if (half == 0) {
                    store_tiles(act, acc, R + RES_S, R + RES_T, (const f32x4*)nullptr, nt, lane);
                } else {
                    f32x4 skip[MT];
                    slab_load(slab, skip, lane);
                    store_tiles(act, acc, R + RES_S, R + RES_T, skip, nt, lane);
                }
                __syncthreads();
            }
        }
        heads<NT32, ActF32>(act, sm, W, b, tid, logits, value, probs);
    }
}

// ============================================================ f16x3 kernel: 8 waves (two per SIMD)
// (one wave per SIMD with 512 registers and all 15 M tiles per wave measured 37%
// slower: the compiler serialises the A-fragment reads of a single stream)
constexpr int NT16 = 512;
constexpr int PV_SPLIT = 8;  // M tiles of the older wave of each SIMD pair (it wins MFMA arbitration)
constexpr int PV_YOUNG_TILES = 15 - PV_SPLIT;
// list (optional): the boards to run, list[0 .. *list_count); ord / maps: the
// root ordinal of every board (-1: none) and the root map area -- a board with
// 0 <= ord < root_cap also stores its x0, y1, x1, y2 maps (gz_pvinc.hip)
template <bool LIST, bool DUMP>
__global__ __launch_bounds__(NT16, 1) void pv_kernel_f16x3(const float* __restrict__ W,
                                                         const uint32_t* __restrict__ boards, int n,
                                                         const int32_t* d_count, float* __restrict__ hbuf,
                                                         const int32_t* __restrict__ list,
                                                         const int32_t* __restrict__ list_count,
                                                         const int32_t* __restrict__ ord,
                                                         _Float16* __restrict__ maps, int root_cap,
                                                         float* __restrict__ pres = nullptr) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    const Smem sm = smem_layout(lds);
    ActF16x3 act;
    act.hi = (_Float16*)lds;
    act.lo = act.hi + CH * ROWS16;
    const int count = LIST ? *list_count : board_count(n, d_count);
    act.zero_slots(threadIdx.x, NT16, CH);
    for (int i = threadIdx.x; i < 3 * (ROWS - POS); i += NT16)
        sm.planes[(i / (ROWS - POS)) * ROWS + POS + i % (ROWS - POS)] = 0.f;

    PV_STAMP(30);  // start of the clock (slot 30 is not a phase)
    for (int li_ = blockIdx.x; li_ < count; li_ += gridDim.x) {
        const int b = LIST ? list[li_] : li_;
        _Float16* gm = nullptr;
        float* gp = nullptr;
        if (DUMP) {
            const int o = ord[b];
            if (o >= 0 && o < root_cap) {
                gm = maps + (size_t)o * 4 * PV_MAP_HALVES;
                if (pres) gp = pres + (size_t)o * 4 * PV_PRE_FLOATS;
            }
        }
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        load_planes<NT16>(sm.planes, boards + (size_t)b * 16, tid);
        __syncthreads();
        PV_STAMP(0);
        // im2col in the heads' scratch area (dead until this board's heads)
        _Float16* col = (_Float16*)sm.hp;
        build_im2col<NT16>(col, sm.planes, tid);
        __syncthreads();
        conv0_f16(act, W, col, wave, lane, gm);
        __syncthreads();
        PV_STAMP(1);
        if (wave >> 2)
            f16_tower<PV_YOUNG_TILES, PV_SPLIT>(act, W, wave, lane, sm.hpart, gm, gp);
        else
            f16_tower<PV_SPLIT, 0>(act, W, wave, lane, sm.hpart, gm, gp);
        int tid_h = threadIdx.x;  // re-read: a pinned tid kept live across the tower is spilled
        asm volatile("" : "+v"(tid_h));
        // the 1x1 head convs' outputs go to HBM; the FC heads run batched over boards
        // in pv_heads_kernel.  hpart is next written in the next board's last epilogue,
        // many barriers later, so no barrier is needed here.
        if (tid_h < POS) {
            float p0 = W[P_B], p1 = W[P_B + 1], v = W[V_B];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                p0 += sm.hpart[(q * 3 + 0) * 256 + tid_h];
                p1 += sm.hpart[(q * 3 + 1) * 256 + tid_h];
                v += sm.hpart[(q * 3 + 2) * 256 + tid_h];
            }
            float* h = hbuf + (size_t)b * HSTRIDE;
            h[tid_h] = p0;  // flatten order: channel-major (policy.view(B, -1))
            h[POS + tid_h] = p1;
            h[HV_OFF + tid_h] = v;
        } else if (tid_h < POS + (HV_OFF - 2 * POS)) {
            hbuf[(size_t)b * HSTRIDE + 2 * POS + (tid_h - POS)] = 0.f;  // hp k-padding
        } else if (tid_h < POS + (HV_OFF - 2 * POS) + (HSTRIDE - HV_OFF - POS)) {
            hbuf[(size_t)b * HSTRIDE + HV_OFF + POS + (tid_h - POS - (HV_OFF - 2 * POS))] = 0.f;  // hv padding
        }
    }
}

// ============================================================ batched FC heads (f16x3 path)
// policy_fc 450->225 and value_fc1 225->64 for HB = 64 boards per workgroup as fp32
// MFMA GEMMs (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation) over
// the 1x1-conv outputs the tower kernel left in hbuf, then value_fc2 + tanh and the
// softmax (neural_network.py:146-159, 240-247).  K is taken in blocks of 16: in the
// t-th k-step of block j, lane group g multiplies k = 16j + 4g + t, so a lane's A
// operand for 4 k-steps is one 16-byte load.  Wave w: policy n-tiles {w, w+4, w+8,
// w+12} (< 15) and value n-tile w, all 4 board tiles.
constexpr int HB = 64;
constexpr int NTH_H = 256;
constexpr int LG_STRIDE = 228;
static_assert(HP_K == 16 * PF_KB && HV_K == 16 * V1_KB && HP_K % 16 == 0 && HV_K % 16 == 0 && HV_OFF % 4 == 0 && HSTRIDE % 4 == 0, "16-B A loads");

// The f16x3 tower's heads run the same two GEMMs on v_mfma_f32_16x16x32_f16 with the
// 3-product split (a_hi w_hi + a_hi w_lo + a_lo w_hi): 32-deep k-blocks, lane group g
// multiplying k = 32 kb + 8 g + j (j < 8) of its board row (A) and its output column (B).
// The B fragments -- policy_fc / value_fc1 x 2^8 (exact; it keeps the small weights' lo
// halves out of fp16's subnormals), split into fp16 hi / lo -- are cut from the fp32
// fragments once per forward (pv_heads_pack_kernel) into the workspace: [kb][n-tile][lane]
// [8] hi plane, then the lo plane.  The exact-fp32 path keeps the fp32-MFMA heads.
constexpr int HF_PKB = 15, HF_VKB = 8;  // k-blocks: policy 480 >= 450 inputs, value 256 >= 225
constexpr int HF_VAL = HF_PKB * PF_NT * 64 * 8;           // halves: value_fc1's fragments
constexpr int HF_PLANE = HF_VAL + HF_VKB * V1_NT * 64 * 8;  // halves per plane (hi, lo)
constexpr size_t HF_BYTES = 2 * (size_t)HF_PLANE * sizeof(_Float16);
constexpr float HF_SCALE = 256.f, HF_UNSCALE = 1.f / 256.f;
static_assert(HF_PKB * 32 >= HP_K - 8 && HF_VKB * 32 >= HV_K, "k-blocks");

__global__ __launch_bounds__(256) void pv_heads_pack_kernel(const float* __restrict__ W, _Float16* __restrict__ hf) {
    constexpr int NPF = HF_PKB * PF_NT * 64, NV = HF_VKB * V1_NT * 64;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= NPF + NV) return;
    const bool pol = i < NPF;
    const int f = pol ? i : i - NPF, nts = pol ? PF_NT : V1_NT, kb16max = pol ? PF_KB : V1_KB;
    const float* Wp = W + (pol ? PF_P : V1_P);
    const int lane = f & 63, nt = (f >> 6) % nts, kb = (f >> 6) / nts, li = lane & 15, g = lane >> 4;
    h8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int k = 32 * kb + 8 * g + j, kb16 = k >> 4, r = k & 15;
        float v = kb16 < kb16max ? Wp[(((size_t)kb16 * nts + nt) * 64 + li + 16 * (r >> 2)) * 4 + (r & 3)] : 0.f;
        v *= HF_SCALE;
        hi[j] = (_Float16)v;
        lo[j] = (_Float16)(v - (float)hi[j]);
    }
    _Float16* o = hf + (pol ? 0 : HF_VAL) + (size_t)f * 8;
    *(h8*)o = hi;
    *(h8*)(o + HF_PLANE) = lo;
}

// KB 32-deep k-blocks of the f16x3 heads GEMM over the workgroup's 4 board tiles and the
// wave's n-tiles nt[0..ntn).  The A operand is split once per workgroup: thread t takes 8
// k of board t / 4 (its row srow, k >= klim read as 0) into hi / lo fragments in LDS
// (stage: 2 buffers x [hi, lo] x 256 fragments, 16 KB), so the 4 waves do not each split
// the same rows; the next k-block is split while this one's MFMAs run (one barrier per block)
template <int KB>
__device__ __forceinline__ void heads_gemm_f16x3(const _Float16* __restrict__ hf, int ntiles, int klim,
                                                 const float* __restrict__ srow, h8* stage, int tid, int lane,
                                                 const int (&nt)[4], int ntn, f32x4 (&acc)[4][4]) {
    const int li = lane & 15, g = lane >> 4, kq = tid & 3;
    auto split = [&](int kb, int buf) {
        const int k0 = 32 * kb + 8 * kq;
        f32x4 x0 = zero4(), x1 = zero4();
        if (k0 < klim) {
            x0 = *(const f32x4*)(srow + k0);
            x1 = *(const f32x4*)(srow + k0 + 4);
        }
        h8 vh, vl;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            vh[j] = (_Float16)x0[j];
            vl[j] = (_Float16)(x0[j] - (float)vh[j]);
            vh[4 + j] = (_Float16)x1[j];
            vl[4 + j] = (_Float16)(x1[j] - (float)vh[4 + j]);
        }
        stage[buf * 512 + tid] = vh;  // fragment (board, kq) = tid: board 16 m + li, kq = g
        stage[buf * 512 + 256 + tid] = vl;
    };
    split(0, 0);
    __syncthreads();
#pragma unroll 1
    for (int kb = 0; kb < KB; kb++) {
        const int buf = kb & 1;
        if (kb + 1 < KB) split(kb + 1, buf ^ 1);
        h8 bh[4], bl[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (q >= ntn) continue;
            const _Float16* b = hf + (((size_t)kb * ntiles + nt[q]) * 64 + lane) * 8;
            bh[q] = *(const h8*)b;
            bl[q] = *(const h8*)(b + HF_PLANE);
        }
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const h8 ah = stage[buf * 512 + (16 * m + li) * 4 + g], al = stage[buf * 512 + 256 + (16 * m + li) * 4 + g];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (q >= ntn) continue;
                acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[q], acc[m][q], 0, 0, 0);
                acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[q], acc[m][q], 0, 0, 0);
                acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[q], acc[m][q], 0, 0, 0);
            }
        }
        __syncthreads();  // every wave is done with buffer buf before it is split into again
    }
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (q < ntn) acc[m][q] = acc[m][q] * HF_UNSCALE;
}

// hf == nullptr: the fp32-MFMA GEMMs (exact f32 products); else the f16x3 ones
__global__ __launch_bounds__(NTH_H, 2) void pv_heads_kernel(const float* __restrict__ W, const float* __restrict__ hbuf,
                                                           int n, const int32_t* d_count, float* __restrict__ logits,
                                                           float* __restrict__ value, float* __restrict__ probs,
                                                           const _Float16* __restrict__ hf) {
    __shared__ __attribute__((aligned(16))) float lg[HB * LG_STRIDE];  // (the policy GEMM's A stage before)
    __shared__ __attribute__((aligned(16))) float h1[HB * 64];         // (the value GEMM's A stage before)
    static_assert(HB == 64 && HB * LG_STRIDE * 4 >= 16384 && HB * 64 * 4 >= 16384, "A stages");
    const int count = board_count(n, d_count);
    const int b0 = blockIdx.x * HB;
    if (b0 >= count) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, g = lane >> 4;
    // board rows of the lane (row li of each of the 4 board tiles); rows past count
    // re-read the last board and their outputs are dropped
    const float* arow[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int b = b0 + 16 * m + li;
        arow[m] = hbuf + (size_t)(b < count ? b : count - 1) * HSTRIDE;
    }
    {  // policy_fc
        int nt[4];
        int ntn = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            nt[q] = wave + 4 * q;
            ntn += nt[q] < 15;
        }
        f32x4 acc[4][4];
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
            for (int q = 0; q < 4; q++) acc[m][q] = zero4();
        if (hf) {
            const int sb = b0 + (tid >> 2);
            heads_gemm_f16x3<HF_PKB>(hf, PF_NT, HP_K, hbuf + (size_t)(sb < count ? sb : count - 1) * HSTRIDE,
                                     (h8*)lg, tid, lane, nt, ntn, acc);
        } else
            for (int kb = 0; kb < HP_K / 16; kb++)
                heads_gemm_block(W + PF_P, PF_NT, kb, lane, nt, ntn, acc, arow);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (q >= ntn) continue;
            const int o = 16 * nt[q] + li;
            if (o >= POS) continue;
            const float bias = W[PF_B + o];
#pragma unroll
            for (int m = 0; m < 4; m++)
#pragma unroll
                for (int r = 0; r < 4; r++) lg[(16 * m + 4 * g + r) * LG_STRIDE + o] = acc[m][q][r] + bias;
        }
    }
    {  // value_fc1 (+ bias, ReLU)
        const float* arv[4];
#pragma unroll
        for (int m = 0; m < 4; m++) arv[m] = arow[m] + HV_OFF;
        int nt[4] = {wave, 0, 0, 0};
        f32x4 acc[4][4];
#pragma unroll
        for (int m = 0; m < 4; m++) acc[m][0] = zero4();
        if (hf) {
            const int sb = b0 + (tid >> 2);
            heads_gemm_f16x3<HF_VKB>(hf + HF_VAL, V1_NT, HV_K,
                                     hbuf + (size_t)(sb < count ? sb : count - 1) * HSTRIDE + HV_OFF, (h8*)h1, tid,
                                     lane, nt, 1, acc);
        } else
            for (int kb = 0; kb < HV_K / 16; kb++)
                heads_gemm_block(W + V1_P, V1_NT, kb, lane, nt, 1, acc, arv);
        const int j = 16 * wave + li;
        const float bias = W[V1_B + j];
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float y = acc[m][0][r] + bias;
                h1[(16 * m + 4 * g + r) * 64 + j] = y > 0.f ? y : 0.f;
            }
    }
    __syncthreads();
    // value_fc2 + tanh: one thread per board
    if (tid < HB && b0 + tid < count) {
        float tot = 0.f;
        for (int j = 0; j < 64; j++) tot = __builtin_fmaf(W[V2_W + j], h1[tid * 64 + j], tot);
        value[b0 + tid] = tanhf(tot + W[V2_B]);
    }
    // softmax: wave w handles boards w, w+4, ...; lane covers outputs lane + 64u
    for (int bb = wave; bb < HB && b0 + bb < count; bb += 4) {
        const float* l = lg + bb * LG_STRIDE;
        float x[4];
        float mx = -3.0e38f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int o = lane + 64 * u;
            x[u] = o < POS ? l[o] : -3.0e38f;
            mx = fmaxf(mx, x[u]);
        }
        mx = wave_max(mx);
        float e[4], sum = 0.f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int o = lane + 64 * u;
            e[u] = o < POS ? __expf(x[u] - mx) : 0.f;
            sum += e[u];
        }
        sum = wave_sum(sum);
        const size_t base = (size_t)(b0 + bb) * POS;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int o = lane + 64 * u;
            if (o < POS) {
                logits[base + o] = x[u];
                if (probs) probs[base + o] = e[u] / sum;
            }
        }
    }
}

// ============================================================ masked prior (ai_agent.py:564-582)
// MCTSNode._get_prior_probability: the float32 softmax at the node's unexplored
// moves (the empty cells in row-major order, gomoku_board.py:201-213) as float64,
// divided by their float64 np.sum when it is > 0.  np.sum of a contiguous float64
// vector is numpy's pairwise summation (blocks of <= 128 terms: < 8 terms left to
// right from 0.0, else 8 interleaved accumulators combined ((0+1)+(2+3))+((4+5)+(6+7))
// plus the remainder left to right; longer vectors split at n/2 rounded down to a
// multiple of 8), restated here term for term so the sum rounds exactly like the
// reference's (oracle.np_pairwise_sum).  Output: dense [n][225] float64, the prior at
// empty cells and 0 at stones (the reference's compact vector = dense[empty cells]).
// One workgroup per 64 boards, a wave per board (16 in turn): the empty cells'
// terms compacted in row-major order by ballot prefix counts, then the pairwise sum
// with numpy's association -- lane j < 8 of block k runs the j-th of its 8 interleaved
// accumulators (<= 16 terms in order), one lane combines them and adds the remainder.
constexpr int PR_B = 64;
constexpr int PR_PER_WAVE = PR_B / 4;

// one block of np_pairwise_block (n terms at a[0..n)) with lanes l0 .. l0 + 7 of the
// wave; every lane returns the block's sum
__device__ __forceinline__ double np_pairwise_block_wave(const float* a, int n, int l0, int lane) {
    const int j = lane - l0;
    const int nfull = n - n % 8;
    double r = 0.0;
    if (n >= 8 && j >= 0 && j < 8) {
        r = (double)a[j];
        for (int i = 8 + j; i < nfull; i += 8) r += (double)a[i];
    }
    double rr[8];
#pragma unroll
    for (int t = 0; t < 8; t++) rr[t] = __shfl(r, l0 + t);
    double res;
    if (n < 8) {
        res = 0.0;
        for (int i = 0; i < n; i++) res += (double)a[i];
    } else {
        res = ((rr[0] + rr[1]) + (rr[2] + rr[3])) + ((rr[4] + rr[5]) + (rr[6] + rr[7]));
        for (int i = nfull; i < n; i++) res += (double)a[i];
    }
    return res;
}

__global__ __launch_bounds__(256) void pv_prior_kernel(const uint32_t* __restrict__ boards, int n, const int32_t* d_count,
                                                       const float* __restrict__ probs, double* __restrict__ prior) {
    __shared__ float terms[4][256];  // a wave's board: the empty cells' terms, compacted
    const int count = board_count(n, d_count);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float* a = terms[wave];
    for (int i = 0; i < PR_PER_WAVE; i++) {
        const int b = blockIdx.x * PR_B + wave * PR_PER_WAVE + i;
        if (b >= count) break;
        const uint32_t* bd = boards + (size_t)b * 16;
        float pv[4];
        bool empty[4];
        int m = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int cell = 64 * u + lane;
            const int bit = (cell / 15) * 16 + cell % 15;
            const int w = cell < POS ? bit >> 5 : 0;
            const bool occ = ((bd[w] | bd[8 + w]) >> (bit & 31)) & 1u;
            empty[u] = cell < POS && !occ;
            pv[u] = cell < POS ? probs[(size_t)b * POS + cell] : 0.f;
            const uint64_t mk = __ballot(empty[u]);
            if (empty[u]) a[m + __popcll(mk & ((1ull << lane) - 1ull))] = pv[u];
            m += __popcll(mk);
        }
        asm volatile("" ::: "memory");  // (a wave's LDS accesses execute in order)
        double s;
        if (m <= 128) {
            s = np_pairwise_block_wave(a, m, 0, lane);
        } else {
            int k2 = m / 2;
            k2 -= k2 % 8;
            const double s0 = np_pairwise_block_wave(a, k2, 0, lane);
            const double s1 = np_pairwise_block_wave(a + k2, m - k2, 8, lane);
            s = s0 + s1;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int cell = 64 * u + lane;
            if (cell >= POS) continue;
            double v = 0.0;
            if (empty[u]) {
                const double x = (double)pv[u];
                v = s > 0.0 ? x / s : x;
            }
            prior[(size_t)b * POS + cell] = v;
        }
        asm volatile("" ::: "memory");  // the terms are read before the next board's compaction
    }
}

}  // namespace

#ifdef GZ_PV_STAMPS
extern "C" int gz_pv_stamps_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gz_pv_stamps), 32 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gz_pv_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

extern "C" void gz_internal_set_error(const char* msg);

extern "C" size_t gz_pv_weight_floats(void) { return (size_t)TOTAL; }

static int pv_grid(int n) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return n < cus ? n : cus;
}

// f16x3: the tower -> heads records, then the heads' fp16 fragments (HF_BYTES)
static size_t pv_hf_offset(int32_t n) { return ((size_t)(n < 1 ? 1 : n) * HSTRIDE * sizeof(float) + 255) & ~(size_t)255; }

extern "C" size_t gz_pv_workspace_bytes(int32_t n) {
    const int grid = pv_grid(n < 1 ? 1 : n);
    const size_t slab = (size_t)grid * (NT32 / 64) * SLAB_F * sizeof(float);  // fp32 kernel
    const size_t heads = pv_hf_offset(n) + HF_BYTES;
    return slab > heads ? slab : heads;
}

static void pv_heads_launch(const float* d_weights, const float* hbuf, int32_t n, const int32_t* d_count,
                            float* d_logits, float* d_value, float* d_probs, _Float16* hf, hipStream_t s) {
    if (hf) {
        constexpr int NF = HF_PKB * PF_NT * 64 + HF_VKB * V1_NT * 64;
        pv_heads_pack_kernel<<<(NF + 255) / 256, 256, 0, s>>>(d_weights, hf);
    }
    pv_heads_kernel<<<(n + HB - 1) / HB, NTH_H, 0, s>>>(d_weights, hbuf, n, d_count, d_logits, d_value, d_probs, hf);
}

extern "C" int gz_pv_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                             float* d_logits, float* d_value, float* d_probs, double* d_prior, void* d_workspace,
                             int32_t precision, void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_logits || !d_value))) {
        gz_internal_set_error("gz_pv_forward: bad arguments");
        return GZ_ERR_ARG;
    }
    if (precision != GZ_PV_FP32 && precision != GZ_PV_F16X3) {
        gz_internal_set_error("gz_pv_forward: unknown precision");
        return GZ_ERR_ARG;
    }
    if (!d_workspace) {
        gz_internal_set_error("gz_pv_forward: d_workspace is required");
        return GZ_ERR_ARG;
    }
    if (d_prior && !d_probs) {
        gz_internal_set_error("gz_pv_forward: d_prior needs d_probs (the prior is renormalised from the softmax)");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    int grid = pv_grid(n);
    hipStream_t s = (hipStream_t)stream;
    if (precision == GZ_PV_FP32)
        pv_kernel_f32<<<grid, NT32, 0, s>>>(d_weights, d_boards, n, d_count, d_logits, d_value, d_probs,
                                            (float*)d_workspace);
    else
    {
        pv_kernel_f16x3<false, false><<<grid, NT16, 0, s>>>(d_weights, d_boards, n, d_count, (float*)d_workspace, nullptr,
                                                     nullptr, nullptr, nullptr, 0);
        pv_heads_launch(d_weights, (const float*)d_workspace, n, d_count, d_logits, d_value, d_probs,
                        (_Float16*)((char*)d_workspace + pv_hf_offset(n)), s);
    }
    if (d_prior) pv_prior_kernel<<<(n + PR_B - 1) / PR_B, 256, 0, s>>>(d_boards, n, d_count, d_probs, d_prior);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("pv_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}

// ============================================================ incremental forward (gz_pvinc.hip)
extern "C" int gz_internal_tree_classify(const int32_t* d_meta, int32_t n, const int32_t* d_count, int32_t root_cap,
                                         int32_t patch_cap, int32_t* d_ord, int32_t* d_pslot, int32_t* d_ctr,
                                         int32_t* d_roots, int32_t* d_full, int32_t* d_grand, int32_t* d_ghead,
                                         int32_t* d_gnext, const uint32_t* d_boards, int32_t* d_cinfo,
                                         int32_t* d_children, void* stream);
extern "C" int gz_internal_tree_children(const float* d_weights, const uint32_t* d_boards, const int32_t* d_meta,
                                         const int32_t* d_ord, const int32_t* d_pslot, int32_t n,
                                         const int32_t* d_count, const _Float16* d_maps, _Float16* d_patches,
                                         float* d_hbuf, const int32_t* d_grand, const int32_t* d_ngrand,
                                         const int32_t* d_cinfo, _Float16* d_scratch, int32_t* d_tiles,
                                         const int32_t* d_children, const int32_t* d_nchildren, int grid,
                                         const float* d_pres, int32_t* d_queue, void* stream);

namespace {
constexpr size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
// per grid entry (gz_pvnet.h): pv_sib_kernel's workgroup x 6 nodes, pv_dg_kernel's 2 x 6
constexpr size_t SIB_SCRATCH_HALVES = PV_SCRATCH_PATCHES * (size_t)PV_PATCH_HALVES;
inline int32_t patch_cap_of(int32_t root_cap) { return 16 * (root_cap < 0 ? 0 : root_cap); }
struct TreeWs {
    float* hbuf;
    int32_t *ord, *pslot, *roots, *full, *grand, *gnext, *cinfo, *children, *ghead, *ctr;
    _Float16* maps;
    float* pres;        // the roots' pre-BN accumulators (pv_dg_kernel)
    _Float16* patches;
    _Float16* scratch;  // pv_sib_kernel / pv_dg_kernel: 12 patch-sized areas per workgroup
    _Float16* hf;       // the heads' fp16 fragments (HF_BYTES)
};
TreeWs tree_carve(void* ws, int32_t n, int32_t root_cap) {
    const size_t m = (size_t)(n < 1 ? 1 : n);
    char* p = (char*)ws;
    TreeWs t;
    t.hbuf = (float*)p;
    p += al256(m * HSTRIDE * sizeof(float));
    int32_t** arrays[7] = {&t.ord, &t.pslot, &t.roots, &t.full, &t.grand, &t.gnext, &t.cinfo};
    for (auto a : arrays) {
        *a = (int32_t*)p;
        p += al256(m * 4);
    }
    t.children = (int32_t*)p;  // n entries + the per-wave counts of tree_children_kernel
    p += al256((m + m / 64 + 1) * 4);
    t.ctr = (int32_t*)p;
    p += 256;
    t.ghead = (int32_t*)p;
    p += al256((size_t)patch_cap_of(root_cap) * 4);
    t.maps = (_Float16*)p;
    p += (size_t)(root_cap < 0 ? 0 : root_cap) * 4 * PV_MAP_HALVES * sizeof(_Float16);
    t.pres = (float*)p;
    p += (size_t)(root_cap < 0 ? 0 : root_cap) * 4 * PV_PRE_FLOATS * sizeof(float);
    t.patches = (_Float16*)p;
    p += (size_t)patch_cap_of(root_cap) * PV_PATCH_HALVES * sizeof(_Float16);
    t.scratch = (_Float16*)p;
    p += (size_t)pv_grid(1 << 30) * SIB_SCRATCH_HALVES * sizeof(_Float16);
    t.hf = (_Float16*)p;
    return t;
}
}  // namespace

extern "C" size_t gz_pv_tree_workspace_bytes(int32_t n, int32_t root_cap) {
    const size_t m = (size_t)(n < 1 ? 1 : n);
    return al256(m * HSTRIDE * sizeof(float)) + 7 * al256(m * 4) + al256((m + m / 64 + 1) * 4) + 256 +
           al256((size_t)patch_cap_of(root_cap) * 4) +
           (size_t)(root_cap < 0 ? 0 : root_cap) * 4 * PV_MAP_HALVES * sizeof(_Float16) +
           (size_t)(root_cap < 0 ? 0 : root_cap) * 4 * PV_PRE_FLOATS * sizeof(float) +
           (size_t)patch_cap_of(root_cap) * PV_PATCH_HALVES * sizeof(_Float16) +
           (size_t)pv_grid(1 << 30) * SIB_SCRATCH_HALVES * sizeof(_Float16) + HF_BYTES;
}

extern "C" int gz_pv_forward_tree(const float* d_weights, const uint32_t* d_boards, const int32_t* d_meta, int32_t n,
                                  const int32_t* d_count, int32_t root_cap, float* d_logits, float* d_value,
                                  float* d_probs, double* d_prior, void* d_workspace, void* stream) {
    if (n < 0 || root_cap < 0 || (n > 0 && (!d_weights || !d_boards || !d_meta || !d_logits || !d_value || !d_workspace))) {
        gz_internal_set_error("gz_pv_forward_tree: bad arguments");
        return GZ_ERR_ARG;
    }
    if (d_prior && !d_probs) {
        gz_internal_set_error("gz_pv_forward_tree: d_prior needs d_probs");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    hipStream_t s = (hipStream_t)stream;
    TreeWs t = tree_carve(d_workspace, n, root_cap);
    int rc = gz_internal_tree_classify(d_meta, n, d_count, root_cap, patch_cap_of(root_cap), t.ord, t.pslot, t.ctr,
                                       t.roots, t.full, t.grand, t.ghead, t.gnext, d_boards, t.cinfo, t.children,
                                       stream);
    if (rc) return rc;
    const int grid = pv_grid(n);
    // roots (full forward, maps stored), then every board without a stored root or
    // patch (full forward), then the roots' children and their children (incremental);
    // ctr = [roots seen, #roots, #children, #full, #grandchildren, patch slots claimed, .., .,
    //        executed tile-taps (children, grandchildren) at 8, 9, pv_dg_kernel's / pv_sib_kernel's XCD queue heads at 16..23 / 24..31]
    pv_kernel_f16x3<true, true><<<grid, NT16, 0, s>>>(d_weights, d_boards, n, d_count, t.hbuf, t.roots, t.ctr + 1,
                                                     t.ord, t.maps, root_cap, t.pres);
    pv_kernel_f16x3<true, false><<<grid, NT16, 0, s>>>(d_weights, d_boards, n, d_count, t.hbuf, t.full, t.ctr + 3,
                                                      nullptr, nullptr, 0);
    rc = gz_internal_tree_children(d_weights, d_boards, d_meta, t.ord, t.pslot, n, d_count, t.maps, t.patches, t.hbuf,
                                   t.grand, t.ctr + 4, t.cinfo, t.scratch, t.ctr + 8, t.children, t.ctr + 2, grid,
                                   t.pres, t.ctr + 16, stream);
    if (rc) return rc;
    pv_heads_launch(d_weights, t.hbuf, n, d_count, d_logits, d_value, d_probs, t.hf, s);
    if (d_prior) pv_prior_kernel<<<(n + PR_B - 1) / PR_B, 256, 0, s>>>(d_boards, n, d_count, d_probs, d_prior);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("gz_pv_forward_tree: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}


// the 16-row MFMA tiles of the residual convs the last tree forward's incremental
// kernels executed: [root children, grandchildren]
extern "C" int gz_pv_tree_exec_tiles(const void* d_workspace, int32_t n, int32_t* d_out2, void* stream) {
    TreeWs t = tree_carve((void*)d_workspace, n, 0);
    if (hipMemcpyAsync(d_out2, t.ctr + 8, 2 * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess) {
        gz_internal_set_error("gz_pv_tree_exec_tiles: copy");
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}

// counts of the last tree forward's lists: [roots seen, roots with maps, children, full,
// grandchildren, patch slots claimed]
extern "C" int gz_pv_tree_stats(const void* d_workspace, int32_t n, int32_t* d_out6, void* stream) {
    TreeWs t = tree_carve((void*)d_workspace, n, 0);
    if (hipMemcpyAsync(d_out6, t.ctr, 6 * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess) {
        gz_internal_set_error("gz_pv_tree_stats: copy");
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
