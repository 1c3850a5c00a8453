// gz_gnet.hip -- the BG planner's nets for a batch of boards on gfx950:
//   p = softmax(GraphNet(planes)), q = OpponentDQN(planes)   (bg_planner.py:22-78,243-250)
//
// One 512-thread workgroup (8 waves) evaluates one board at a time and loops over
// boards; two workgroups share a CU (LDS 76 KB each).  GraphNet's 64x225 map
// stays in LDS as f16x3 hi/lo planes (gz_f16conv.h); every conv is an implicit
// GEMM on v_mfma_f32_16x16x32_f16 in C^T form.  Wave w owns n-tiles
// {2(w&1), 2(w&1)+1} x M tiles [4(w>>1), 4(w>>1)+4), waves 6-7 three tiles (tile 15
// would be zero rows only).
// The embed conv reads 0/1 planes, exact in fp16, so it takes 2 MFMAs (w_hi, w_lo).
// The policy conv 1x1 (64->2) runs on VALU at the end of the tower and goes to a
// per-board record in the workspace with the stone inputs; gn_heads_kernel then runs
// the policy FC 450->225 + softmax and the OpponentDQN MLP for 64 boards per
// workgroup as fp32-MFMA GEMMs (weights read once per 64 boards, not per board).
#include <hip/hip_runtime.h>

#include <string>
#include <type_traits>

#include "gz_f16conv.h"
#include "gz_gnet.h"
#include "../../include/gzero.h"

using namespace gzc;
using namespace gzgn;

namespace {

// Phase stamps (tools/gn_stamps.py only): -DGZ_GN_STAMPS accumulates s_memtime
// deltas of workgroup 0 / wave 0 per phase; compiled out otherwise.
#ifdef GZ_GN_STAMPS
__device__ unsigned long long gz_gn_stamps[32];
#define GN_STAMP(i)                                                \
    do {                                                           \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                 \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
            gz_gn_stamps[i] += t_ - gz_gn_stamps[31];              \
            gz_gn_stamps[31] = t_;                                 \
        }                                                          \
    } while (0)
#else
#define GN_STAMP(i) \
    do {            \
    } while (0)
#endif

constexpr int NT = 512;
constexpr int NM = 4;        // M tiles per wave
constexpr int PROWS = 240;   // fp32 planes [3][240]
constexpr int ACT_BYTES = 2 * HID * ROWS16 * 2;  // 65536
constexpr int SMALL_F = 3 * PROWS;
constexpr int LDS_BYTES = ACT_BYTES + SMALL_F * 4;

// neighbour of the lane's position in M tile m for tap (dr, dc); POS (a zero plane slot) if off-board
__device__ inline int pnbr(int m, int li, int dr, int dc) {
    int pos = m * 16 + li;
    int r = pos / 15 + dr, c = pos % 15 + dc;
    bool ok = pos < POS && r >= 0 && r < 15 && c >= 0 && c < 15;
    return ok ? r * 15 + c : POS;
}

// epilogue: y = relu(acc + bias) for the wave's 2 n-tiles x NMW M tiles
template <int NMW>
__device__ __forceinline__ void gn_store(ActF16x3& act, const f32x4 (&acc)[2][NMW], const float* __restrict__ bias,
                                         int np, int m0, int lane) {
    asm volatile("" : "+v"(lane));
    lane &= 63;
    const f32x4 one = {1.f, 1.f, 1.f, 1.f};
    const f32x4 none = zero4();
#pragma unroll
    for (int n = 0; n < 2; n++) {
        const int ch0 = (2 * np + n) * 16 + 4 * (lane >> 4);
        const f32x4 t = *(const f32x4*)(bias + ch0);
#pragma unroll
        for (int m = 0; m < NMW; m++) {
            const int pos = (m0 + m) * 16 + (lane & 15);
            if (pos < POS) f16_put4<false>(act, acc[n][m], one, t, none, ch0, pos);
        }
    }
}

// embed conv MFMAs (fragments from the im2col in act.hi) and the 8 tower layers
// for a wave owning NMW M tiles from m0; every barrier of the board's tower is here
// the map in LDS (all 225 positions) -> map slot map `m` ([plane][cg][225][8] halves)
__device__ __forceinline__ void gn_store_map(const ActF16x3& act, _Float16* __restrict__ slot, int m) {
    _Float16* dst = slot + (size_t)m * SLOT_MAP_HALVES;
    for (int i = threadIdx.x; i < 2 * 8 * POS; i += NT) {
        const int pcg = i / POS, pos = i - pcg * POS;
        const _Float16* src = (pcg < 8 ? act.hi : act.lo) + ((pcg & 7) * ROWS16 + pos) * 8;
        *(uint4*)(dst + (size_t)i * 8) = *(const uint4*)src;
    }
}

template <int NMW>
__device__ __forceinline__ void gn_tower(ActF16x3& act, const float* __restrict__ W, int np, int m0, int lane,
                                         _Float16* __restrict__ slot) {
    {
        const _Float16* col = act.hi;
        const int li = lane & 15, q = lane >> 4;
        h8 a[NMW];
#pragma unroll
        for (int m = 0; m < NMW; m++) a[m] = *(const h8*)(col + (q * ROWS16 + (m0 + m) * 16 + li) * 8);
        h8 wa[2][2];
#pragma unroll
        for (int nn = 0; nn < 2; nn++) {
            const _Float16* wf = (const _Float16*)(W + GH_E) + ((size_t)(2 * np + nn) * 64 + lane) * 8;
            wa[nn][0] = *(const h8*)wf;
            wa[nn][1] = *(const h8*)(wf + 4 * 64 * 8);
        }
        f32x4 acc[2][NMW];
#pragma unroll
        for (int m = 0; m < NMW; m++)
#pragma unroll
            for (int nn = 0; nn < 2; nn++) {
                acc[nn][m] = zero4();
                acc[nn][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nn][0], a[m], acc[nn][m], 0, 0, 0);
                acc[nn][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[nn][1], a[m], acc[nn][m], 0, 0, 0);
            }
        __syncthreads();  // every wave has its im2col fragments
        gn_store<NMW>(act, acc, W + GE_B, np, m0, lane);
    }
    __syncthreads();
    if (slot) gn_store_map(act, slot, 0);  // (read only: the next write to act follows a barrier)
    GN_STAMP(2);

    // ---- 4 x [conv3x3 + ReLU, conv1x1 + ReLU] (bg_planner.py:50-54)
    for (int i = 0; i < 8; i++) {
        f32x4 acc[2][NMW];
#pragma unroll
        for (int nn = 0; nn < 2; nn++)
#pragma unroll
            for (int m = 0; m < NMW; m++) acc[nn][m] = zero4();
        const _Float16* wf = (const _Float16*)(W + h_layer_off(i));
        if (i % 2 == 0)
            f16_conv<NMW, 2, 4, 9>(act, wf, np, m0, lane, acc);
        else
            f16_conv<NMW, 2, 4, 1>(act, wf, np, m0, lane, acc);
        __syncthreads();  // every wave has read the layer input
        if (i % 2 == 0) GN_STAMP(3);
        else GN_STAMP(5);
        gn_store<NMW>(act, acc, W + layer_bias(i), np, m0, lane);
        __syncthreads();
        if (slot && (i & 1) && i < 7) gn_store_map(act, slot, (i + 1) / 2);  // L1, L3, L5: the 3x3 inputs
        if (i % 2 == 0) GN_STAMP(4);
        else GN_STAMP(6);
    }
}

// the policy conv 1x1 64->2 at one position (bg_planner.py:45): hp / lp = the
// position's channel group 0 in the hi / lo plane, cgs = the channel-group stride
__device__ __forceinline__ void gn_pconv(const float* __restrict__ W, const _Float16* hp, const _Float16* lp, int cgs,
                                         float& o0, float& o1) {
    float p0 = W[GP_B], p1 = W[GP_B + 1];
    for (int c0 = 0; c0 < HID; c0 += 8) {
        const h8 xh = *(const h8*)(hp + (c0 >> 3) * cgs);
        const h8 xl = *(const h8*)(lp + (c0 >> 3) * cgs);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float a = (float)xh[j] + (float)xl[j];
            p0 = __builtin_fmaf(W[GP_W + c0 + j], a, p0);
            p1 = __builtin_fmaf(W[GP_W + HID + c0 + j], a, p1);
        }
    }
    o0 = p0;
    o1 = p1;
}

// boards b = list[i] (list: NULL = 0..count-1).  slots (optional): every board's
// maps and policy-conv output also go to a map slot -- tags[b].job, or slot b
// when tags is NULL (the search roots)
__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4))) void gn_kernel(
    const float* __restrict__ W, const uint32_t* __restrict__ boards, int n, const int32_t* d_count,
    float* __restrict__ rec, const int32_t* __restrict__ list, char* __restrict__ slots,
    const GnTag* __restrict__ tags) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    ActF16x3 act;
    act.hi = (_Float16*)lds;
    act.lo = act.hi + HID * ROWS16;
    float* planes = (float*)(lds + ACT_BYTES);  // [3][240]

    int count = n;
    if (d_count) {
        int c = *d_count;
        count = c < n ? c : n;
    }
    act.zero_slots(threadIdx.x, NT, HID);
    for (int i = threadIdx.x; i < 3 * (PROWS - POS); i += NT)
        planes[(i / (PROWS - POS)) * PROWS + POS + i % (PROWS - POS)] = 0.f;

    GN_STAMP(30);
    for (int i = blockIdx.x; i < count; i += gridDim.x) {
        const int b = list ? list[i] : i;
        _Float16* slot = nullptr;
        if (slots) slot = (_Float16*)(slots + (size_t)(tags ? tags[b].job : b) * SLOT_BYTES);
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int np = wave & 1, m0 = (wave >> 1) * NM;
        float* rb = rec + (size_t)b * REC;
        // ---- input planes [black, white, empty] (bg_planner.py:225-230); the stone
        // planes also go to the record (the DQN's one-hot inputs, gn_heads_kernel)
        const uint32_t* bd = boards + (size_t)b * 16;
        for (int p = tid; p < POS; p += NT) {
            int bit = (p / 15) * 16 + (p % 15);
            uint32_t bl = (bd[bit >> 5] >> (bit & 31)) & 1u;
            uint32_t wh = (bd[8 + (bit >> 5)] >> (bit & 31)) & 1u;
            planes[p] = (float)bl;
            planes[PROWS + p] = (float)wh;
            planes[2 * PROWS + p] = (float)(1u - (bl | wh));
            rb[REC_X + p] = (float)bl;
            rb[REC_X + POS + p] = (float)wh;
        }
        if (tid < (REC_X - 2 * POS) + (REC - REC_X - 2 * POS)) {  // record padding (A rows past K are zero)
            const int z = tid < REC_X - 2 * POS ? 2 * POS + tid : REC_X + 2 * POS + (tid - (REC_X - 2 * POS));
            rb[z] = 0.f;
        }
        __syncthreads();
        GN_STAMP(0);

        // ---- embed conv 3->64 (K = 27 -> 32): planes are 0/1, so a*w = a*w_hi + a*w_lo.
        // im2col (256 rows x 32 halves, built once per board) lives in the activation
        // area, k-chunk q of row r at channel-group slot (q, r) so the zero rows
        // POS..255 stay zero, until every wave holds its fragments in registers.
        {
            _Float16* col = act.hi;
            for (int t = tid; t < 256 * 2; t += NT) {
                const int row = t >> 1, k0 = (t & 1) * 16;
                const int r = row / 15, c = row % 15;
                h8 v[2];
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const int k = k0 + j;
                    const int tap = k / 3, cin = k % 3;
                    const int rr = r + tap / 3 - 1, cc = c + tap % 3 - 1;
                    const bool ok = k < 27 && row < POS && rr >= 0 && rr < 15 && cc >= 0 && cc < 15;
                    v[j >> 3][j & 7] = ok ? (_Float16)planes[cin * PROWS + rr * 15 + cc] : (_Float16)0.f;
                }
                *(h8*)(col + ((k0 >> 3) * ROWS16 + row) * 8) = v[0];
                *(h8*)(col + ((k0 >> 3) * ROWS16 + ROWS16 + row) * 8) = v[1];
            }
            __syncthreads();
        }
        // waves 6-7 own M tiles 12-14 only (tile 15 is all zero rows): 15 tiles, not 16
        if ((wave >> 1) == 3)
            gn_tower<NM - 1>(act, W, np, m0, lane, slot);
        else
            gn_tower<NM>(act, W, np, m0, lane, slot);

        // ---- policy head conv1x1 64->2 (one thread per position), flattened
        // channel-major into the record.  The next board's first LDS write that
        // could clobber the map (its im2col) comes after a barrier, so none here.
        int tid_h = threadIdx.x;  // re-read (not kept live across the tower)
        asm volatile("" : "+v"(tid_h));
        if (tid_h < POS) {
            float p0, p1;
            gn_pconv(W, act.hi + tid_h * 8, act.lo + tid_h * 8, ROWS16 * 8, p0, p1);
            rb[tid_h] = p0;
            rb[POS + tid_h] = p1;
            if (slot) {
                float* pol = (float*)slot + SLOT_POL;
                pol[tid_h] = p0;
                pol[POS + tid_h] = p1;
            }
        }
        GN_STAMP(7);
    }
}

// ============================================================ batched heads
// policy FC 450->225 + softmax (bg_planner.py:55-56, 243-246) and OpponentDQN
// (bg_planner.py:68-78) for HB (32) boards per workgroup as fp32-MFMA GEMMs over
// the records gn_kernel left (heads_gemm_block, gz_f16conv.h).  DQN fc0 on the one-hot
// planes = base + the (colour - empty) delta rows of the stones (gz_gnet.h): a GEMM
// with K = 450 over the record's stone inputs (only the k-blocks holding a stone on
// one of the workgroup's boards).  Wave w: n-tiles {w, w+4, w+8, w+12}.
constexpr int HB = 32;  // boards per workgroup: 66 KB of LDS, two workgroups per CU
constexpr int HMT = HB / 16;  // M tiles (16 boards each)
constexpr int NTH_H = 256;
constexpr int LG_STRIDE = 228;   // logits rows
constexpr int H_STRIDE = 260;    // DQN hidden rows (16 B apart in bank space per row)
static_assert(REC_X == 29 * 16 && REC - REC_X == 29 * 16 && REC % 4 == 0 && REC_X % 16 == 0 && H_STRIDE % 4 == 0, "16-B A loads");

// heads_gemm_block's products in its order, with the next k-block's A and B fragments
// loaded while the current one's MFMAs run (4 waves per workgroup leave little else
// to hide the loads behind)
template <int KB, int NTILES>
__device__ __forceinline__ void heads_gemm(const float* __restrict__ Wp, int lane, const int (&nt)[4], int ntn,
                                           f32x4 (&acc)[HMT][4], const float* __restrict__ arow[HMT]) {
#pragma unroll
    for (int m = 0; m < HMT; m++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc[m][q] = zero4();
    const int g = lane >> 4;
    auto load = [&](int kb, f32x4 (&a)[HMT], f32x4 (&b)[4]) {
#pragma unroll
        for (int m = 0; m < HMT; m++) a[m] = *(const f32x4*)(arow[m] + 16 * kb + 4 * g);
#pragma unroll
        for (int q = 0; q < 4; q++)
            b[q] = q < ntn ? *(const f32x4*)(Wp + (((size_t)kb * NTILES + nt[q]) * 64 + lane) * 4) : zero4();
    };
    f32x4 a[2][HMT], b[2][4];
    load(0, a[0], b[0]);
#pragma unroll 2
    for (int kb = 0; kb < KB; kb++) {
        const int cur = kb & 1;
        if (kb + 1 < KB) load(kb + 1, a[cur ^ 1], b[cur ^ 1]);
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int m = 0; m < HMT; m++)
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (q < ntn) acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][m][t], b[cur][q][t], acc[m][q], 0, 0, 0);
    }
}

// DQN fc0 over the k-blocks of the one-hot stone inputs that hold a stone
// on at least one of the workgroup's boards (mask: bit kb).  A skipped block's
// products are all zero, and adding them leaves every accumulator bit unchanged (the
// accumulators start at +0 and never become -0), so the outputs are bitwise those of
// the dense GEMM
template <int NTILES>
__device__ __forceinline__ void heads_gemm_mask(const float* __restrict__ Wp, int lane, const int (&nt)[4], int ntn,
                                                f32x4 (&acc)[HMT][4], const float* __restrict__ arow[HMT], uint32_t mask) {
#pragma unroll
    for (int m = 0; m < HMT; m++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc[m][q] = zero4();
    const int g = lane >> 4;
    auto load = [&](int kb, f32x4 (&a)[HMT], f32x4 (&b)[4]) {
#pragma unroll
        for (int m = 0; m < HMT; m++) a[m] = *(const f32x4*)(arow[m] + 16 * kb + 4 * g);
#pragma unroll
        for (int q = 0; q < 4; q++)
            b[q] = q < ntn ? *(const f32x4*)(Wp + (((size_t)kb * NTILES + nt[q]) * 64 + lane) * 4) : zero4();
    };
    mask = __builtin_amdgcn_readfirstlane(mask);
    if (!mask) return;
    f32x4 a0[HMT], b0[4];
    load(__builtin_ctz(mask), a0, b0);
    mask &= mask - 1;
    for (;;) {
        f32x4 a1[HMT], b1[4];
        const bool more = mask != 0;
        if (more) load(__builtin_ctz(mask), a1, b1);  // the next live block while this one's MFMAs run
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int m = 0; m < HMT; m++)
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (q < ntn) acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[m][t], b0[q][t], acc[m][q], 0, 0, 0);
        if (!more) break;
        mask &= mask - 1;
#pragma unroll
        for (int m = 0; m < HMT; m++) a0[m] = a1[m];
#pragma unroll
        for (int q = 0; q < 4; q++) b0[q] = b1[q];
    }
}

// acc + bias (ReLU if RELU) into LDS rows dst[board][n] for the wave's n-tiles
template <bool RELU>
__device__ __forceinline__ void heads_put(const f32x4 (&acc)[HMT][4], const float* __restrict__ bias, int nmax,
                                          const int (&nt)[4], int ntn, int lane, float* dst, int stride) {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q >= ntn) continue;
        const int o = 16 * nt[q] + li;
        if (o >= nmax) continue;
        const float bv = bias[o];
#pragma unroll
        for (int m = 0; m < HMT; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float y = acc[m][q][r] + bv;
                if (RELU) y = y > 0.f ? y : 0.f;
                dst[(16 * m + 4 * g + r) * stride + o] = y;
            }
    }
}

__global__ __launch_bounds__(NTH_H, 64 / HB) void gn_heads_kernel(const float* __restrict__ W, const float* __restrict__ rec,
                                                           int n, const int32_t* d_count, float* __restrict__ p_out,
                                                           float* __restrict__ q_out, float* __restrict__ logits_out) {
    __shared__ __attribute__((aligned(16))) float ra[HB * H_STRIDE];  // logits, then DQN hidden 2
    __shared__ __attribute__((aligned(16))) float rb[HB * H_STRIDE];  // DQN hidden 1
    int count = n;
    if (d_count) {
        int c = *d_count;
        count = c < n ? c : n;
    }
    const int b0 = blockIdx.x * HB;
    if (b0 >= count) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, g = lane >> 4;
    // board rows of the lane (row li of each of the 4 board tiles); rows past count
    // re-read the last board and their outputs are dropped
    const float* arow[HMT];
#pragma unroll
    for (int m = 0; m < HMT; m++) {
        const int b = b0 + 16 * m + li;
        arow[m] = rec + (size_t)(b < count ? b : count - 1) * REC;
    }
    int nt[4];
    int ntn_p = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        nt[q] = wave + 4 * q;
        ntn_p += nt[q] < 15;
    }
    f32x4 acc[HMT][4];
    // the fc0 k-blocks with a stone on any of this workgroup's boards (visible after the
    // barrier that follows the policy FC)
    __shared__ uint32_t kmask;
    if (tid == 0) kmask = 0;
    __syncthreads();
    {
        constexpr int KBX = (REC - REC_X) / 16;
        uint32_t mk = 0;
        for (int e = tid; e < HB * KBX; e += NTH_H) {
            const int bb = e / KBX, kb = e - bb * KBX;
            const int b = b0 + bb < count ? b0 + bb : count - 1;
            const f32x4* x = (const f32x4*)(rec + (size_t)b * REC + REC_X + 16 * kb);
            bool nz = false;
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const f32x4 y = x[v];
                nz |= y[0] != 0.f || y[1] != 0.f || y[2] != 0.f || y[3] != 0.f;
            }
            if (nz) mk |= 1u << kb;
        }
        if (mk) atomicOr(&kmask, mk);
    }
    // ---- policy FC 450 -> 225 (+ bias) into ra, then softmax per board
    heads_gemm<REC_X / 16, 15>(W + GF_P, lane, nt, ntn_p, acc, arow);
    heads_put<false>(acc, W + GF_B, POS, nt, ntn_p, lane, ra, LG_STRIDE);
    __syncthreads();
    for (int bb = wave; bb < HB && b0 + bb < count; bb += 4) {  // wave w: boards w, w+4, ...
        const float* l = ra + bb * LG_STRIDE;
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
                p_out[base + o] = e[u] / sum;
                if (logits_out) logits_out[base + o] = x[u];
            }
        }
    }
    // ---- DQN fc0 (one-hot planes -> 256) + ReLU into rb
    {
        const float* ax[HMT];
#pragma unroll
        for (int m = 0; m < HMT; m++) ax[m] = arow[m] + REC_X;
        heads_gemm_mask<16>(W + D0_P, lane, nt, 4, acc, ax, kmask);
        heads_put<true>(acc, W + D0_BASE, DQH, nt, 4, lane, rb, H_STRIDE);
    }
    __syncthreads();  // rb complete; ra (logits) no longer read
    const float* ah[HMT];
    // ---- fc1 256 -> 256 + ReLU into ra
#pragma unroll
    for (int m = 0; m < HMT; m++) ah[m] = rb + (16 * m + li) * H_STRIDE;
    heads_gemm<DQH / 16, 16>(W + D1_P, lane, nt, 4, acc, ah);
    heads_put<true>(acc, W + D1_B, DQH, nt, 4, lane, ra, H_STRIDE);
    __syncthreads();
    // ---- fc2 256 -> 225: q
#pragma unroll
    for (int m = 0; m < HMT; m++) ah[m] = ra + (16 * m + li) * H_STRIDE;
    heads_gemm<DQH / 16, 15>(W + D2_P, lane, nt, ntn_p, acc, ah);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q >= ntn_p) continue;
        const int o = 16 * nt[q] + li;
        if (o >= POS) continue;
        const float bv = W[D2_B + o];
#pragma unroll
        for (int m = 0; m < HMT; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int b = b0 + 16 * m + 4 * g + r;
                if (b < count) q_out[(size_t)b * POS + o] = acc[m][q][r] + bv;
            }
    }
}


// Small launches (the planner's sequential rounds: one row per game, 512 rows in config
// 5): gn_heads_kernel's 32 boards and 4 waves per workgroup give such a launch 16
// workgroups whose fp32-MFMA chains (90 k-blocks x 32 MFMAs per wave) set its time.
constexpr int HBS = 16, PFS = 6;  // boards per workgroup; k-blocks of fragments in flight

// The heads split over output tiles for them: three launches
// (policy FC + DQN fc0; fc1; fc2 + the softmax), each workgroup 16 boards x 4 output
// tiles (a wave per tile, the fragments 5 k-blocks ahead), the layers' outputs through
// a scratch in global memory.  A launch of 512 rows then has 256 / 128 / 160
// workgroups instead of 32, each with a quarter of a wave's MFMA chain per tile.
// Products, their order and the epilogues are gn_heads_kernel's, so p and q are the
// same bits.
constexpr int HN_LD = 256;  // scratch row stride (logits 225, hidden 256)
constexpr int HN_ROW = 3 * HN_LD;  // scratch floats per row: logits, h0, h1 (in the caller's workspace)

__device__ __forceinline__ void hn_tile(const float* __restrict__ Wp, int KB, int NTILES, int nt, int lane,
                                        const float* __restrict__ arow, f32x4& acc) {
    acc = zero4();
    const int g = lane >> 4;
    f32x4 a[PFS], b[PFS];
    const float* bp = Wp + ((size_t)nt * 64 + lane) * 4;
    const size_t bstep = (size_t)NTILES * 64 * 4;
#pragma unroll
    for (int k = 0; k < PFS - 1; k++)
        if (k < KB) {
            a[k] = *(const f32x4*)(arow + 16 * k + 4 * g);
            b[k] = *(const f32x4*)(bp + k * bstep);
        }
    __builtin_amdgcn_sched_barrier(0);
    for (int k0 = 0; k0 < KB; k0 += PFS) {
#pragma unroll
        for (int j = 0; j < PFS; j++) {
            const int kb = k0 + j;
            if (kb >= KB) break;
            const int kn = kb + PFS - 1, sn = (j + PFS - 1) % PFS;
            if (kn < KB) {
                a[sn] = *(const f32x4*)(arow + 16 * kn + 4 * g);
                b[sn] = *(const f32x4*)(bp + kn * bstep);
            }
            // (keeps the loads PFS - 1 blocks ahead: the scheduler would otherwise sink
            // them next to their MFMAs, 1-2 blocks ahead)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 4; t++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][t], b[j][t], acc, 0, 0, 0);
        }
    }
}

// acc + bias (ReLU) -> out[b][o] for the tile's live rows and columns
template <bool RELU>
__device__ __forceinline__ void hn_put(const f32x4& acc, const float* __restrict__ bias, int nmax, int nt, int lane,
                                       int b0, int count, float* __restrict__ out, int ld) {
    const int li = lane & 15, g = lane >> 4, o = 16 * nt + li;
    if (o >= nmax) return;
    const float bv = bias[o];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int b = b0 + 4 * g + r;
        float y = acc[r] + bv;
        if (RELU) y = y > 0.f ? y : 0.f;
        if (b < count) out[(size_t)b * ld + o] = y;
    }
}

__device__ __forceinline__ int hn_count(int n, const int32_t* d_count) {
    if (!d_count) return n;
    const int c = *d_count;
    return c < n ? c : n;
}

// stage 0: policy FC (y 0..3: tiles 4y + wave < 15) -> logits, DQN fc0 (y 4..7) -> h0
__global__ __launch_bounds__(256) void gn_hn0_kernel(const float* __restrict__ W, const float* __restrict__ rec, int n,
                                                     const int32_t* d_count, float* __restrict__ lg,
                                                     float* __restrict__ h0) {
    const int count = hn_count(n, d_count), b0 = blockIdx.x * HBS;
    if (b0 >= count) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, y = blockIdx.y;
    const float* arow = rec + (size_t)(b0 + li < count ? b0 + li : count - 1) * REC;
    f32x4 acc;
    if (y < 4) {
        const int nt = 4 * y + wave;
        if (nt >= 15) return;
        hn_tile(W + GF_P, REC_X / 16, 15, nt, lane, arow, acc);
        hn_put<false>(acc, W + GF_B, POS, nt, lane, b0, count, lg, HN_LD);
    } else {
        const int nt = 4 * (y - 4) + wave;
        hn_tile(W + D0_P, (REC - REC_X) / 16, 16, nt, lane, arow + REC_X, acc);
        hn_put<true>(acc, W + D0_BASE, DQH, nt, lane, b0, count, h0, HN_LD);
    }
}

// stage 1: fc1 (y 0..3) h0 -> h1
__global__ __launch_bounds__(256) void gn_hn1_kernel(const float* __restrict__ W, int n, const int32_t* d_count,
                                                     const float* __restrict__ h0, float* __restrict__ h1) {
    const int count = hn_count(n, d_count), b0 = blockIdx.x * HBS;
    if (b0 >= count) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, nt = 4 * blockIdx.y + wave;
    const float* arow = h0 + (size_t)(b0 + li < count ? b0 + li : count - 1) * HN_LD;
    f32x4 acc;
    hn_tile(W + D1_P, DQH / 16, 16, nt, lane, arow, acc);
    hn_put<true>(acc, W + D1_B, DQH, nt, lane, b0, count, h1, HN_LD);
}

// stage 2: fc2 (y 0..3) h1 -> q; y 4: the softmax of the 16 boards' logits -> p
__global__ __launch_bounds__(256) void gn_hn2_kernel(const float* __restrict__ W, int n, const int32_t* d_count,
                                                     const float* __restrict__ lg, const float* __restrict__ h1,
                                                     float* __restrict__ p_out, float* __restrict__ q_out) {
    const int count = hn_count(n, d_count), b0 = blockIdx.x * HBS;
    if (b0 >= count) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15;
    if (blockIdx.y < 4) {
        const int nt = 4 * blockIdx.y + wave;
        if (nt >= 15) return;
        const float* arow = h1 + (size_t)(b0 + li < count ? b0 + li : count - 1) * HN_LD;
        f32x4 acc;
        hn_tile(W + D2_P, DQH / 16, 15, nt, lane, arow, acc);
        const int g = lane >> 4, o = 16 * nt + li;
        if (o >= POS) return;
        const float bv = W[D2_B + o];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int b = b0 + 4 * g + r;
            if (b < count) q_out[(size_t)b * POS + o] = acc[r] + bv;
        }
        return;
    }
    for (int bb = wave; bb < HBS && b0 + bb < count; bb += 4) {  // gn_heads_kernel's softmax
        const float* l = lg + (size_t)(b0 + bb) * HN_LD;
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
            if (o < POS) p_out[base + o] = e[u] / sum;
        }
    }
}

// the heads over max_rows rows (d_count of them live): split over output tiles when
// gn_heads_kernel would not give every CU 2 workgroups of 32 boards, no logits are asked
// for and the caller's workspace holds the scratch (sc: max_rows x HN_ROW floats)
static void gn_heads_launch(const float* W, const float* rec, int max_rows, const int32_t* d_count, float* d_p,
                            float* d_q, float* d_logits, int cus, hipStream_t s, float* sc) {
    static const int small_cap = [] {  // GZ_GN_SMALL_HEADS: rows below which the small kernel runs (A/B)
        const char* e = getenv("GZ_GN_SMALL_HEADS");
        return e ? atoi(e) : -1;
    }();
    const int cap = small_cap >= 0 ? small_cap : 2 * HB * cus;
    if (sc && !d_logits && max_rows < cap) {
        const unsigned gx = (unsigned)((max_rows + HBS - 1) / HBS);
        float *lg = sc, *h0 = sc + (size_t)max_rows * HN_LD, *h1 = sc + 2 * (size_t)max_rows * HN_LD;
        gn_hn0_kernel<<<dim3(gx, 8), 256, 0, s>>>(W, rec, max_rows, d_count, lg, h0);
        gn_hn1_kernel<<<dim3(gx, 4), 256, 0, s>>>(W, max_rows, d_count, h0, h1);
        gn_hn2_kernel<<<dim3(gx, 5), 256, 0, s>>>(W, max_rows, d_count, lg, h1, d_p, d_q);
    } else
        gn_heads_kernel<<<(max_rows + HB - 1) / HB, NTH_H, 0, s>>>(W, rec, max_rows, d_count, d_p, d_q, d_logits);
}

// ============================================================ incremental GraphNet
// A planner ply's board is its predecessor plus one stone (bg_planner.py:243-250 on
// the board _simulate's previous ply left, ai_agent.py:265-271), and a rollout's
// first board is usually the search root plus the expanded child's stone.  GraphNet
// (embed 3x3, then 4 x [3x3, 1x1]) has receptive radius 5, so a board that adds
// stone c to a board whose maps are kept only changes, at each layer's output,
// the square of radius 1 (embed), 2 (L0, L1), 3 (L2, L3), 4 (L4, L5), 5 (L6, L7)
// around c.  gn_inc_kernel recomputes just those squares, IG boards per chunk,
// layer-major: each 3x3 layer reads the windows (square radius + 1) of its input
// map, assembled in LDS from the layer's own new square and, elsewhere, the stored
// maps (LDS-DMA); the 1x1 layers read the new square only.  The policy conv then
// runs on the radius-5 square; the rest of the 450 policy-conv outputs are the
// predecessor's.  The stored maps are the 3x3 inputs (embed, L1, L3, L5, map
// slots in gz_gnet.h): a chain of boards keeps its base's maps (the search root's,
// or a full forward's) plus, in its own slot, the squares of the stones added since
// (a window position inside one of those squares reads the slot, else the base).
// Every output element takes gn_kernel's products in gn_kernel's order (the same
// k-steps, MFMA operand splits and epilogues), so the records -- and p, q from
// gn_heads_kernel -- are bitwise those of the full forward.
constexpr int IG = 3;  // boards per chunk
constexpr int IMH = IG == 1 ? 1 : 2;      // M parts: waves = 4 n-tiles x IMH
constexpr int NTI = 256 * IMH;            // wave: n-tile wave & 3, M part wave >> 2
constexpr int IWG = IG == 1 ? 2 : 1;      // workgroups per CU
// a window of radius R: (2R+1)^2 positions, each channel-group plane padded to a multiple
// of 16 positions, so that the plane stride is a whole number of 256-B bank rows (the
// ds_read_b128 of a tile row then lands on the same bank slot in every plane)
__host__ __device__ constexpr int ig_pw(int R) { return ((2 * R + 1) * (2 * R + 1) + 15) / 16 * 16; }
constexpr int IWIN_MAX = ig_pw(6) * 256;  // bytes of a radius-6 window (2 planes x 8 cg x 176 x 16 B)
// LDS: the windows at 0 (up to IG x 43 KB), each 3x3 layer's output rows at the top of
// [0, IA) (B(ro): [plane][8 cg][ig_brows(ro)][8] halves at IA - 256 ig_brows(ro)), so
// that the next window's fill can start as soon as the 3x3 k-loop has read its window
constexpr int IA = IG == 1 ? 65536 : 153344;
__host__ __device__ constexpr int ig_brows(int ro) { return (IG * (2 * ro + 1) * (2 * ro + 1) + 15) / 16 * 16; }
__host__ __device__ constexpr int ig_boff(int ro) { return IA - 256 * ig_brows(ro); }
constexpr int ICOL = IA;                  // embed im2col [IG][4][16][8] halves
constexpr int IPC = ICOL + IG * 1024;     // policy-conv outputs [IG][2][128] floats
constexpr int IU = IPC + IG * 2 * 128 * 4;
constexpr int ITAB = IU + IG * 128;         // row tables of the radius 1..5 passes, then their totals
// (radius 1 has no table: the embed works on its squares directly)
__host__ __device__ constexpr int itab_off(int ro) { return ro <= 2 ? 0 : itab_off(ro - 1) + ig_brows(ro - 1); }
constexpr int ITOT = itab_off(6);            // 864 entries (radius 2..5 rows, padded to whole tiles)
constexpr int ILDS = ITAB + (ITOT + 8 + 5 * IG * 8) * 4;
static_assert(ILDS * IWG <= 160 * 1024 && IG * IWIN_MAX <= IA && ig_boff(5) >= 0, "LDS");
// the next window vs the rows the 1x1 layer before it reads: map 1, 2 windows clear
// of B(2), B(3); the map-3 window overlaps B(4) above ig_boff(4) (filled in two parts)
static_assert(IG * ig_pw(4) * 256 <= ig_boff(2) && IG * ig_pw(5) * 256 <= ig_boff(3), "window / rows overlap");

struct GnUnit {
    const _Float16* base;  // maps the chain adds stones to
    _Float16* job;         // this row's slot (its new squares; earlier stones' squares)
    const float* pol_src;  // policy-conv outputs of the predecessor
    float* pol_job;
    float* rec;            // the row's record (gn_heads_kernel input)
    int32_t cell, nst;
    uint8_t st[8];
    uint32_t board[16];
    int32_t pad[2];
};
static_assert(sizeof(GnUnit) == 128, "unit");

typedef __attribute__((address_space(3))) void ig_lds_t;
typedef __attribute__((address_space(1))) void ig_glb_t;
__device__ uint4 gz_gn_zero16[1];  // zero-initialised (off-board window positions)

__device__ __forceinline__ int iabs_(int x) { return x < 0 ? -x : x; }

struct Sq {  // clipped square around a cell: rows r0.., cols c0.., h x w
    int r0, c0, h, w;
};
__device__ __forceinline__ Sq square(int cell, int rad) {
    const int cr = cell / 15, cc = cell - (cell / 15) * 15;
    Sq q;
    q.r0 = cr - rad > 0 ? cr - rad : 0;
    q.c0 = cc - rad > 0 ? cc - rad : 0;
    q.h = (cr + rad < 14 ? cr + rad : 14) - q.r0 + 1;
    q.w = (cc + rad < 14 ? cc + rad : 14) - q.c0 + 1;
    return q;
}

__device__ __forceinline__ const _Float16* ig_rfl(const _Float16* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const _Float16*)(((uint64_t)hi << 32) | lo);
}

// window of map MAP (radius R = MAP + 3, [plane][8 cg][P][8] halves) for every unit,
// unit g at halves g * P * 128: LDS-DMA of every on-board position outside the
// unit's new square (radius MAP + 1, written by the producing epilogue), zeros off
// the board; drained by the caller's barrier
template <int MAP>
__device__ __forceinline__ void ig_fill(char* lds, const GnUnit* U, int ng, int tid, int lo = 0, int hi = 1 << 30) {
    constexpr int R = MAP + 3, Wd = 2 * R + 1, PW = Wd * Wd, P = ig_pw(R), NB = (PW + 63) / 64, rc = MAP + 1;
    // work blocks (unit g, 64 window positions): the lane's position and its source
    // are worked out once, then its 16 channel-group planes go by LDS-DMA (for a given
    // plane a wave's 64 positions are contiguous in LDS)
    const int lane = tid & 63, wave = tid >> 6;
    for (int blk = wave; blk < ng * NB; blk += NTI / 64) {
        const int g = blk / NB, b0 = (blk - g * NB) * 64, loc = b0 + lane;
        const _Float16* base = ig_rfl(U[g].base) + MAP * SLOT_MAP_HALVES;
        const _Float16* job = ig_rfl(U[g].job) + MAP * SLOT_MAP_HALVES;
        const int cell = __builtin_amdgcn_readfirstlane(U[g].cell), nst = __builtin_amdgcn_readfirstlane(U[g].nst);
        const int cr = cell / 15, cc = cell - cr * 15;
        const int dr = loc / Wd - R, dc = loc % Wd - R;
        const int pr = cr + dr, pc = cc + dc;
        const bool on = pr >= 0 && pr < 15 && pc >= 0 && pc < 15;
        // positions past the window, and the new square (its epilogue writes it): no load
        const bool skip = loc >= PW || (on && iabs_(dr) <= rc && iabs_(dc) <= rc);
        const char* src = (const char*)gz_gn_zero16;
        int step = 0;  // bytes between planes at the source
        if (on) {
            bool mine = false;
            for (int s = 0; s < nst; s++) {
                const int sc = U[g].st[s], sr = sc / 15, scc = sc - sr * 15;
                mine |= iabs_(pr - sr) <= rc && iabs_(pc - scc) <= rc;
            }
            src = (const char*)((mine ? job : base) + (pr * 15 + pc) * 8);
            step = POS * 16;
        }
        char* dst = lds + (size_t)g * P * 256 + (size_t)b0 * 16;  // + lane * 16 by the DMA
        const int byte0 = g * P * 256 + loc * 16;
#pragma unroll
        for (int pcg = 0; pcg < 16; pcg++) {
            const int byte = byte0 + pcg * P * 16;
            if (!skip && byte >= lo && byte < hi)
                __builtin_amdgcn_global_load_lds((ig_glb_t*)(src + pcg * step), (ig_lds_t*)(dst + pcg * P * 16), 16, 0, 0);
        }
    }
}

// a workgroup barrier that waits for this wave's LDS accesses only, not for its
// outstanding global loads -- a window fill (LDS-DMA) issued before it stays in flight
__device__ __forceinline__ void ig_bar() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt, expcnt unconstrained
    __builtin_amdgcn_s_barrier();
}

// the rows of a pass: every unit's square of radius ro (clipped, row-major), packed;
// row i -> unit g, position (pr, pc), index j in its square
struct IgRow {
    int g, pr, pc, j;
};
constexpr int IG_PAD = 1 << 30;  // a table entry that pads a tile (a real row's geometry, no output)
__device__ __forceinline__ IgRow ig_row(const char* lds, int ro, int i) {
    const int v = ((const int*)(lds + ITAB))[itab_off(ro) + i];
    IgRow r;
    r.g = v & 3;
    r.pr = (v >> 2) & 15;
    r.pc = (v >> 6) & 15;
    r.j = (v >> 10) & 1023;
    return r;
}
__device__ __forceinline__ bool ig_valid(const char* lds, int ro, int i) {
    return !(((const int*)(lds + ITAB))[itab_off(ro) + i] & IG_PAD);
}
__device__ __forceinline__ int ig_total(const char* lds, int ro) { return ((const int*)(lds + ITAB))[ITOT + ro]; }

// The row tables of a chunk (radius 2..5), built once by the whole workgroup: entry i
// of radius ro = unit | pr << 2 | pc << 6 | (index in its square) << 10, N rows in
// T = ceil(N / 16) tiles.  A 3x3 layer's tile reads, per lane, 16 B of a window plane at
// its row's window position p, so a tile whose 16 rows share p mod 16 serialises its
// ds_read_b128 (one bank slot per 16-B position).  The rows of radius >= 2 are therefore
// ordered by that slot (a counting sort, p in the window of radius ro + 1 the layer
// reads) and dealt to the tiles round-robin -- sorted row k -> tile k mod T, lane k / T
// -- so each tile takes an even share of every slot.  The lanes past N in the deal are
// padding entries (IG_PAD) that hold row 0's geometry.  Which lane computes a row does
// not change its result (an MFMA output element depends on its own row only).
__device__ __forceinline__ void ig_build_rows(char* lds, const GnUnit* U, int ng, int tid) {
    int* tab = (int*)(lds + ITAB);
    int* sqt = tab + ITOT + 8;  // [radius - 1][unit]: r0, c0, h, w, first natural row
    int* rk = (int*)lds;        // scratch in the (not yet filled) window area: rank in its slot
    int* hist = rk + 5 * IG * 121;  // [radius - 1][16] slot counts, then [radius - 1][16] starts
    if (tid < 5) {
        const int ro = tid + 1;
        int start = 0;
        for (int g = 0; g < ng; g++) {
            const Sq q = square(U[g].cell, ro);
            int* e = sqt + ((ro - 1) * IG + g) * 8;
            e[0] = q.r0, e[1] = q.c0, e[2] = q.h, e[3] = q.w, e[4] = start;
            start += q.h * q.w;
        }
        tab[ITOT + ro] = start;
    }
    if (tid < 5 * 16) hist[tid] = 0;
    __syncthreads();
    // every entry of the padded tables: padding with row 0's geometry
#pragma unroll
    for (int ro = 2; ro <= 5; ro++) {
        const int* q = sqt + (ro - 1) * IG * 8;
        for (int e = tid; e < ig_brows(ro); e += NTI) tab[itab_off(ro) + e] = IG_PAD | q[0] << 2 | q[1] << 6;
    }
    auto row_of = [&](int e, int& ro, int& nat, int& v, int& slot) -> bool {
        ro = 1 + e / (IG * 121);
        const int r = e - (ro - 1) * IG * 121, g = r / 121, j = r - g * 121;
        if (g >= ng) return false;
        const int* q = sqt + ((ro - 1) * IG + g) * 8;
        const int w = q[3];
        if (j >= q[2] * w) return false;
        const int rr = (int)(((float)j + 0.5f) / (float)w);  // exact: j < 121, w <= 11
        const int pr = q[0] + rr, pc = q[1] + j - rr * w;
        nat = q[4] + j;
        v = g | pr << 2 | pc << 6 | j << 10;
        const int cell = U[g].cell, cr = cell / 15, cc = cell - cr * 15, R = ro + 1, Wd = 2 * R + 1;
        slot = ((pr - cr + R) * Wd + (pc - cc + R)) & 15;
        return true;
    };
    for (int e = tid; e < 5 * IG * 121; e += NTI) {
        int ro, nat, v, slot;
        if (!row_of(e, ro, nat, v, slot) || ro == 1) continue;
        rk[(ro - 1) * IG * 121 + nat] = atomicAdd(&hist[(ro - 1) * 16 + slot], 1);
    }
    __syncthreads();
    if (tid < 5) {
        int a = 0;
        for (int sl = 0; sl < 16; sl++) {
            const int c = hist[tid * 16 + sl];
            hist[80 + tid * 16 + sl] = a;
            a += c;
        }
    }
    __syncthreads();
    for (int e = tid; e < 5 * IG * 121; e += NTI) {
        int ro, nat, v, slot;
        if (!row_of(e, ro, nat, v, slot) || ro == 1) continue;
        const int k = hist[80 + (ro - 1) * 16 + slot] + rk[(ro - 1) * IG * 121 + nat];
        const int T = (tab[ITOT + ro] + 15) >> 4;
        tab[itab_off(ro) + (k % T) * 16 + k / T] = v;
    }
    __syncthreads();  // the scratch (window area) is free for the first fill
}

// tiles per group of the 3x3 k-loop: a group's 3 products interleave over its tiles, so
// an MFMA's accumulator was last written GT - 1 MFMAs earlier
constexpr int IG_GT = 3;

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1
template <class F, int... I>
__device__ __forceinline__ void ig_sfor(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// 3x3 k-loop for the wave's n-tile over NT M tiles, with gn_kernel's k-steps (tap-major,
// cq inner) and per-element product order (w_hi*a_hi, w_lo*a_hi, w_hi*a_lo).  act = the
// windows (radius R, [plane][8 cg][P][8] halves per unit); ctr[m] = the lane's row's
// window position (unit offset included, in units of 8 halves within a cg plane).
// Tiles go in groups of 3 (the 3 products interleaved over the group, so no MFMA waits
// on its predecessor's result); each group's fragments are read while the previous
// group's MFMAs run (two fragment buffers); weight fragments 3 k-steps ahead.
template <int NT, int NMAX, int R>
__device__ __forceinline__ void ig_conv3_nt(const _Float16* act, const int (&ctr)[NMAX], const _Float16* __restrict__ Wf,
                                            int nt, int lane, f32x4 (&acc)[NMAX]) {
    constexpr int Wd = 2 * R + 1, P = ig_pw(R), KS = 18, LO = 64 * P, GT = IG_GT < NT ? IG_GT : NT, NG = (NT + GT - 1) / GT;
    const int q = lane >> 4;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)Wf, 0, 0x7fffffff, 0x00020000);
    const int wo = (nt * 64 + lane) * 16;
    auto wload = [&](int ks, int lo) -> h8 {
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wo, ks * 4096 + lo * KS * 4096, 0));
    };
    h8 b[4][2];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        b[c][0] = wload(c, 0);
        b[c][1] = wload(c, 1);
    }
    f32x4 c[NT];
#pragma unroll
    for (int m = 0; m < NT; m++) c[m] = acc[m];
    int c8[NT];  // the lane's fragment offset (halves) of tile m at tap (0, 0), cq 0
#pragma unroll
    for (int m = 0; m < NT; m++) c8[m] = (ctr[m] + q * P) * 8;
    h8 fa[2][GT][2];
    auto toff = [&](int t) {
        t = t < 9 ? t : t - 9;
        return ((t / 3 - 1) * Wd + (t % 3 - 1)) * 8;
    };
    // fragments of tile group G for (tap, CQ) into buffer PB
    auto load = [&](auto pb_, auto g_, auto cq_, int tap) {
        constexpr int PB = decltype(pb_)::value, G = decltype(g_)::value, CQ = decltype(cq_)::value;
#pragma unroll
        for (int j = 0; j < GT; j++) {
            const int m = G * GT + j;
            if (m < NT) {
                const int o = c8[m] + toff(tap) + CQ * 4 * P * 8;
                fa[PB][j][0] = *(const h8*)(act + o);
                fa[PB][j][1] = *(const h8*)(act + LO + o);
            }
        }
    };
    auto mfmas = [&](auto pb_, auto g_, auto sl_) {
        constexpr int PB = decltype(pb_)::value, G = decltype(g_)::value, SL = decltype(sl_)::value;
#pragma unroll
        for (int j = 0; j < GT; j++)
            if (G * GT + j < NT) c[G * GT + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[SL][0], fa[PB][j][0], c[G * GT + j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < GT; j++)
            if (G * GT + j < NT) c[G * GT + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[SL][1], fa[PB][j][0], c[G * GT + j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < GT; j++)
            if (G * GT + j < NT) c[G * GT + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[SL][0], fa[PB][j][1], c[G * GT + j], 0, 0, 0);
    };
    auto tiles_of = [](int g) { return NT - g * GT < GT ? NT - g * GT : GT; };
    using I0 = std::integral_constant<int, 0>;
    load(I0{}, I0{}, I0{}, 0);
    // NK k-steps from slot 0 (ks0 = 4 tp or 16), tap0 = their first tap; items k = (k-step i, group g)
    auto ksteps = [&](auto nk_, int ks0, int tap0) {
        constexpr int NK = decltype(nk_)::value;
        ig_sfor([&](auto k_) {
            constexpr int k = decltype(k_)::value, i = k / NG, g = k % NG, pb = k & 1;
            constexpr int kn = k + 1, in = kn / NG, gn = kn % NG;
            if (g == 0) {  // weights of k-step ks0 + i + 3 into the slot k-step ks0 + i - 1 released
                const int ksr = ks0 + i + 3, kn2 = ksr < KS ? ksr : ksr - KS;
                b[(i + 3) & 3][0] = wload(kn2, 0);
                b[(i + 3) & 3][1] = wload(kn2, 1);
            }
            // the next item's fragments (past the last k-step here: the next tap's cq 0)
            if (kn < NK * NG)
                load(std::integral_constant<int, 1 - pb>{}, std::integral_constant<int, gn>{},
                     std::integral_constant<int, in & 1>{}, tap0 + (in >> 1));
            else
                load(std::integral_constant<int, 1 - pb>{}, I0{}, I0{}, tap0 + (NK >> 1));
            mfmas(std::integral_constant<int, pb>{}, std::integral_constant<int, g>{}, std::integral_constant<int, i>{});
            if (g == 0) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // VMEM read
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * (kn < NK * NG ? tiles_of(gn) : tiles_of(0)), 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 3 * tiles_of(g), 0);  // MFMA
        }, std::make_integer_sequence<int, NK * NG>{});
    };
#pragma unroll 1
    for (int tp = 0; tp < 4; tp++) ksteps(std::integral_constant<int, 4>{}, 4 * tp, 2 * tp);  // taps 2tp, 2tp+1
    ksteps(std::integral_constant<int, 2>{}, 16, 8);                                          // tap 8
#pragma unroll
    for (int m = 0; m < NT; m++) acc[m] = c[m];
}

template <int NMAX, int R>
__device__ __forceinline__ void ig_conv3(const _Float16* act, const int (&ctr)[NMAX], int nt_tiles,
                                         const _Float16* __restrict__ Wf, int nt, int lane, f32x4 (&acc)[NMAX]) {
    static_assert(NMAX >= 1 && NMAX <= 12, "tile counts");
    switch (nt_tiles) {
        case 1: ig_conv3_nt<1, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 2: if constexpr (NMAX >= 2) ig_conv3_nt<2, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 3: if constexpr (NMAX >= 3) ig_conv3_nt<3, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 4: if constexpr (NMAX >= 4) ig_conv3_nt<4, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 5: if constexpr (NMAX >= 5) ig_conv3_nt<5, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 6: if constexpr (NMAX >= 6) ig_conv3_nt<6, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 7: if constexpr (NMAX >= 7) ig_conv3_nt<7, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 8: if constexpr (NMAX >= 8) ig_conv3_nt<8, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 9: if constexpr (NMAX >= 9) ig_conv3_nt<9, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 10: if constexpr (NMAX >= 10) ig_conv3_nt<10, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 11: if constexpr (NMAX >= 11) ig_conv3_nt<11, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        case 12: if constexpr (NMAX >= 12) ig_conv3_nt<12, NMAX, R>(act, ctr, Wf, nt, lane, acc); break;
        default: break;
    }
}

// The wave's rows of a pass over radius-ro squares: its M half of the tiles
// (the lane's packed row index of tile m is i0 + 16 m; rows >= total are padding)
struct IgTiles {
    int i0, total, nt;
};
__device__ __forceinline__ IgTiles ig_tiles(const char* lds, int ro, int mh, int lane) {
    IgTiles t;
    t.total = ig_total(lds, ro);
    const int T = (t.total + 15) >> 4, T0 = (T + IMH - 1) / IMH, t0 = mh * T0;
    t.nt = T - t0 < T0 ? (T - t0 > 0 ? T - t0 : 0) : T0;
    t.i0 = t0 * 16 + (lane & 15);
    return t;
}

constexpr int ig_nmax(int ro) { return ((IG * (2 * ro + 1) * (2 * ro + 1) + 15) / 16 + IMH - 1) / IMH; }

// 3x3 layer (L0, L2, L4, L6: input map MAP window, output square radius MAP + 2) ->
// relu(acc + bias) as hi / lo into the square rows B(ro); pre() (the next window's
// fill) runs right after the k-loop's barrier
struct Ig1x1W {  // a 1x1 layer's weight fragments and bias for the wave (loaded ahead)
    h8 w0h, w1h, w0l, w1l;
    f32x4 bias;
};
__device__ __forceinline__ Ig1x1W ig_w1x1(const float* __restrict__ W, int layer, int nt, int lane) {
    const _Float16* wf = (const _Float16*)(W + h_layer_off(layer)) + ((size_t)nt * 64 + lane) * 8;
    Ig1x1W w;
    w.w0h = *(const h8*)wf;
    w.w1h = *(const h8*)(wf + 4 * 64 * 8);
    w.w0l = *(const h8*)(wf + 2 * 4 * 64 * 8);
    w.w1l = *(const h8*)(wf + 3 * 4 * 64 * 8);
    w.bias = *(const f32x4*)(W + layer_bias(layer) + nt * 16 + 4 * (lane >> 4));
    return w;
}

template <int MAP, int NMAX, class Pre>
__device__ __forceinline__ void ig_layer3(char* lds, const GnUnit* U, int ng, const float* __restrict__ W, int layer,
                                          int nt, int mh, int lane, Ig1x1W& next, Pre&& pre) {
    constexpr int R = MAP + 3, Wd = 2 * R + 1, P = ig_pw(R), ro = MAP + 2;
    static_assert(NMAX >= ig_nmax(ro), "tiles per M half");
    const IgTiles t = ig_tiles(lds, ro, mh, lane);
    int ctr[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const int i = t.i0 + 16 * m;
        const IgRow r = ig_row(lds, ro, i < 16 * ((t.total + 15) >> 4) ? i : 0);  // (padding: row 0's geometry)
        const int cell = U[r.g].cell, cr = cell / 15, cc = cell - (cell / 15) * 15;
        ctr[m] = r.g * 16 * P + (r.pr - cr + R) * Wd + (r.pc - cc + R);
    }
    f32x4 acc[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) acc[m] = zero4();
    const _Float16* wf = (const _Float16*)(W + h_layer_off(layer));
    if constexpr (NMAX <= 6) {
        if (t.nt > 0) ig_conv3<NMAX, R>((const _Float16*)lds, ctr, t.nt, wf, nt, lane, acc);
    } else {
        // more than 6 tiles: two k-loops over tiles [0, 6) and [6, nt) (the second
        // streams the weights again), so that one k-loop's registers stay small
        constexpr int NB = NMAX - 6;
        int c0[6], c1[NB];
        f32x4 a0[6], a1[NB];
#pragma unroll
        for (int m = 0; m < 6; m++) {
            c0[m] = ctr[m];
            a0[m] = zero4();
        }
#pragma unroll
        for (int m = 0; m < NB; m++) {
            c1[m] = ctr[6 + m];
            a1[m] = zero4();
        }
        if (t.nt > 0) ig_conv3<6, R>((const _Float16*)lds, c0, t.nt < 6 ? t.nt : 6, wf, nt, lane, a0);
        if (t.nt > 6) ig_conv3<NB, R>((const _Float16*)lds, c1, t.nt - 6, wf, nt, lane, a1);
#pragma unroll
        for (int m = 0; m < 6; m++) acc[m] = a0[m];
#pragma unroll
        for (int m = 0; m < NB; m++) acc[6 + m] = a1[m];
    }
    const int ch0 = nt * 16 + 4 * (lane >> 4);
    const f32x4 bias = *(const f32x4*)(W + layer_bias(layer) + ch0);
    next = ig_w1x1(W, layer + 1, nt, lane);
    __syncthreads();  // every wave is past the k-loop: the windows are dead
    // every global load so far has landed (the bias, the next 1x1 layer's weights): the
    // fill issued next is the only VMEM traffic in flight until the 1x1 layer's end
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    pre();
    constexpr int BR = ig_brows(ro);
    _Float16* sq = (_Float16*)(lds + ig_boff(ro));
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const int i = t.i0 + 16 * m;
        if (m >= t.nt || !ig_valid(lds, ro, i)) continue;
        h4 hi, lo;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float y = acc[m][r] + bias[r];
            y = y > 0.f ? y : 0.f;
            const _Float16 h = (_Float16)y;
            hi[r] = h;
            lo[r] = (_Float16)(y - (float)h);
        }
        const int o = ((ch0 >> 3) * BR + i) * 8 + (ch0 & 7);
        *(h4*)(sq + o) = hi;
        *(h4*)(sq + 8 * BR * 8 + o) = lo;
    }
    ig_bar();  // the rows are complete; the fill stays in flight through the 1x1 layer
}

// 1x1 layer (L1, L3, L5, L7) over the square rows B(ro): acc only
template <int NMAX, int BR>
__device__ __forceinline__ void ig_conv1(const _Float16* sq, const IgTiles& t, const Ig1x1W& w, int lane,
                                         f32x4 (&acc)[NMAX]) {
    const h8 w0h = w.w0h, w1h = w.w1h, w0l = w.w0l, w1l = w.w1l;
    const int q = lane >> 4;
#pragma unroll
    for (int m = 0; m < NMAX; m++) acc[m] = zero4();
    // groups of 3 tiles; per element gn_kernel's order: k-step 0 (hi*hi, w_lo*hi, hi*a_lo), k-step 1
#pragma unroll
    for (int g0 = 0; g0 < NMAX; g0 += 3) {
        if (g0 >= t.nt) break;
        h8 a[3][4];
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int o = (q * BR + t.i0 + 16 * (g0 + j < NMAX ? g0 + j : g0)) * 8;
            a[j][0] = *(const h8*)(sq + o);
            a[j][1] = *(const h8*)(sq + 8 * BR * 8 + o);
            a[j][2] = *(const h8*)(sq + 4 * BR * 8 + o);
            a[j][3] = *(const h8*)(sq + 8 * BR * 8 + 4 * BR * 8 + o);
        }
#define IG_P(W_, A_)                                                                                \
    _Pragma("unroll") for (int j = 0; j < 3; j++) if (g0 + j < NMAX)                                \
        acc[g0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(W_, a[j][A_], acc[g0 + j], 0, 0, 0);
        IG_P(w0h, 0)
        IG_P(w0l, 0)
        IG_P(w0h, 1)
        IG_P(w1h, 2)
        IG_P(w1l, 2)
        IG_P(w1h, 3)
#undef IG_P
    }
}

// relu(acc + bias) split hi / lo
__device__ __forceinline__ void ig_split(const f32x4& acc, const f32x4& bias, h4& hi, h4& lo) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        float y = acc[r] + bias[r];
        y = y > 0.f ? y : 0.f;
        const _Float16 h = (_Float16)y;
        hi[r] = h;
        lo[r] = (_Float16)(y - (float)h);
    }
}

// 1x1 layer producing stored map MAP (L1 -> 1, L3 -> 2, L5 -> 3; square radius
// MAP + 1): k-loop over the square rows B(ro), barrier, rest() (what remains of the
// next window's fill), then the outputs into that window's new square and the row's
// map slot
template <int MAP, int NMAX, class Rest>
__device__ __forceinline__ void ig_layer1_map(char* lds, const GnUnit* U, int ng, const Ig1x1W& w, int nt, int mh,
                                              int lane, Rest&& rest) {
    constexpr int R = MAP + 3, Wd = 2 * R + 1, P = ig_pw(R), ro = MAP + 1;
    static_assert(NMAX >= ig_nmax(ro), "tiles per M half");
    const IgTiles t = ig_tiles(lds, ro, mh, lane);
    f32x4 acc[NMAX];
    ig_conv1<NMAX, ig_brows(ro)>((const _Float16*)(lds + ig_boff(ro)), t, w, lane, acc);
    const int ch0 = nt * 16 + 4 * (lane >> 4);
    const f32x4 bias = w.bias;
    ig_bar();  // the square rows are dead
    rest();
    _Float16* win = (_Float16*)lds;
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const int i = t.i0 + 16 * m;
        if (m >= t.nt || !ig_valid(lds, ro, i)) continue;
        h4 hi, lo;
        ig_split(acc[m], bias, hi, lo);
        const IgRow r = ig_row(lds, ro, i);
        const int cell = U[r.g].cell, cr = cell / 15, cc = cell - (cell / 15) * 15;
        const int w = (r.pr - cr + R) * Wd + (r.pc - cc + R);
        const int o = r.g * 16 * P * 8 + ((ch0 >> 3) * P + w) * 8 + (ch0 & 7);
        *(h4*)(win + o) = hi;
        *(h4*)(win + 8 * P * 8 + o) = lo;
        _Float16* g = U[r.g].job + MAP * SLOT_MAP_HALVES + ((ch0 >> 3) * POS + r.pr * 15 + r.pc) * 8 + (ch0 & 7);
        *(h4*)g = hi;
        *(h4*)(g + 8 * POS * 8) = lo;
    }
    __syncthreads();  // the window is complete (the barrier drains the fill)
}

__global__ __launch_bounds__(NTI, IWG) void gn_inc_kernel(const float* __restrict__ W, const uint32_t* __restrict__ boards,
                                                        const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ list_count,
                                                        const GnTag* __restrict__ tags, char* __restrict__ slots,
                                                        float* __restrict__ rec, int per, int* __restrict__ queue) {
    __shared__ __attribute__((aligned(16))) char lds[ILDS];
    GnUnit* U = (GnUnit*)(lds + IU);
    _Float16* col = (_Float16*)(lds + ICOL);
    float* pcv = (float*)(lds + IPC);
    const int count = *list_count;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), nt = wave & 3, mh = wave >> 2;
    // chunks of `per` (<= IG) boards: fewer than IG when the launch has too few rows to
    // give every CU a chunk of IG (a workgroup's time is a chain of short phases whose
    // k-loops scale with its tiles)
    // chunks claimed from the queue head in turn (a workgroup whose chunks were cheap takes
    // more: no static share, no tail); thread 0 claims one chunk ahead and hands the
    // claim over through pcv[0] (the policy-conv outputs are written at the chunk's end)
    int claim = 0;
    if (tid == 0) claim = atomicAdd(queue, per);
    for (;;) {
        __syncthreads();  // the previous chunk is done with U and pcv
        if (tid == 0) {
            *(int*)pcv = claim;
            if (claim < count) claim = atomicAdd(queue, per);
        }
        __syncthreads();
        const int pos0 = *(const int*)pcv;
        if (pos0 >= count) break;
        const int ng = count - pos0 < per ? count - pos0 : per;
        if (tid < ng) {
            const int b = list[pos0 + tid];
            const GnTag tg = tags[b];
            GnUnit u;
            char* bs = slots + (size_t)tg.base * SLOT_BYTES;
            char* js = slots + (size_t)tg.job * SLOT_BYTES;
            u.base = (const _Float16*)bs;
            u.job = (_Float16*)js;
            u.pol_src = (const float*)(tg.nst > 0 || tg.base == tg.job ? js : bs) + SLOT_POL;
            u.pol_job = (float*)js + SLOT_POL;
            u.rec = rec + (size_t)b * REC;
            u.cell = tg.cell;
            u.nst = tg.nst;
#pragma unroll
            for (int s = 0; s < 8; s++) u.st[s] = s < TAG_STONES ? tg.st[s] : 0;
#pragma unroll
            for (int w = 0; w < 16; w++) u.board[w] = boards[(size_t)b * 16 + w];
            u.pad[0] = u.pad[1] = 0;
            U[tid] = u;
        }
        __syncthreads();
        GN_STAMP(8);
        ig_build_rows(lds, U, ng, tid);  // (read after the embed's barriers)
        // (the asm barriers keep the compiler from hoisting every section's per-lane
        // addresses out of the chunk loop, where they would all stay live, and spill)
        auto fresh = [&](const float*& Wp, int& t) {
            Wp = W;
            t = tid;
            asm volatile("" : "+s"(Wp), "+v"(t));
        };
        const float* Wp;
        int t_;
        fresh(Wp, t_);
        // ---- embed: window of map 0 (fill) + im2col of the radius-1 squares
        ig_fill<0>(lds, U, ng, t_);
        for (int e = tid; e < IG * 512; e += NTI) {
            const int g = e >> 9, row = (e >> 5) & 15, k = e & 31;
            _Float16 v = (_Float16)0.f;
            if (g < ng) {
                const Sq q = square(U[g].cell, 1);
                if (row < q.h * q.w && k < 27) {
                    const int pr = q.r0 + row / q.w, pc = q.c0 + row % q.w;
                    const int tap = k / 3, cin = k % 3;
                    const int rr = pr + tap / 3 - 1, cc = pc + tap % 3 - 1;
                    if (rr >= 0 && rr < 15 && cc >= 0 && cc < 15) {
                        const int bit = rr * 16 + cc;
                        const uint32_t bl = (U[g].board[bit >> 5] >> (bit & 31)) & 1u;
                        const uint32_t wh = (U[g].board[8 + (bit >> 5)] >> (bit & 31)) & 1u;
                        v = (_Float16)(float)(cin == 0 ? bl : (cin == 1 ? wh : 1u - (bl | wh)));
                    }
                }
            }
            col[((g * 4 + (k >> 3)) * 16 + row) * 8 + (k & 7)] = v;
        }
        __syncthreads();  // the fill has landed; the im2col is complete
        GN_STAMP(9);
        fresh(Wp, t_);
        {
            const int ln = t_ & 63, li = ln & 15, q = ln >> 4, ch0 = nt * 16 + 4 * q;
            const _Float16* wf = (const _Float16*)(Wp + GH_E) + ((size_t)nt * 64 + ln) * 8;
            const h8 wh = *(const h8*)wf, wl = *(const h8*)(wf + 4 * 64 * 8);
            const f32x4 bias = *(const f32x4*)(Wp + GE_B + ch0);
            constexpr int P0 = ig_pw(3);
            for (int g = mh; g < ng; g += IMH) {
                const h8 a = *(const h8*)(col + ((g * 4 + q) * 16 + li) * 8);
                f32x4 acc = zero4();
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, a, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, a, acc, 0, 0, 0);
                const Sq sq = square(U[g].cell, 1);
                if (li < sq.h * sq.w) {
                    h4 hi, lo;
                    ig_split(acc, bias, hi, lo);
                    const int pr = sq.r0 + li / sq.w, pc = sq.c0 + li % sq.w;
                    const int cell = U[g].cell, cr = cell / 15, cc = cell - cr * 15;
                    const int w = (pr - cr + 3) * 7 + (pc - cc + 3);
                    _Float16* win = (_Float16*)lds + g * 16 * P0 * 8 + ((ch0 >> 3) * P0 + w) * 8 + (ch0 & 7);
                    *(h4*)win = hi;
                    *(h4*)(win + 8 * P0 * 8) = lo;
                    _Float16* gp = U[g].job + ((ch0 >> 3) * POS + pr * 15 + pc) * 8 + (ch0 & 7);
                    *(h4*)gp = hi;
                    *(h4*)(gp + 8 * POS * 8) = lo;
                }
            }
        }
        __syncthreads();
        // ---- the tower: 3x3 over a window -> square rows; 1x1 -> the next map
        fresh(Wp, t_);
        // NMAX = the tiles of a wave's M half: ceil(ceil(IG (2 ro + 1)^2 / 16) / 2)
        GN_STAMP(10);
        // the window fills: maps 1 and 2 right after the 3x3 k-loop before them, map 3
        // below B(4) then, the rest after L5's k-loop
        auto none = [] {};
        Ig1x1W w1;
        ig_layer3<0, ig_nmax(2)>(lds, U, ng, Wp, 0, nt, mh, t_ & 63, w1, [&] { ig_fill<1>(lds, U, ng, t_); });  // L0
        GN_STAMP(11);
        fresh(Wp, t_);
        ig_layer1_map<1, ig_nmax(2)>(lds, U, ng, w1, nt, mh, t_ & 63, none);
        GN_STAMP(12);
        fresh(Wp, t_);
        ig_layer3<1, ig_nmax(3)>(lds, U, ng, Wp, 2, nt, mh, t_ & 63, w1, [&] { ig_fill<2>(lds, U, ng, t_); });  // L2
        GN_STAMP(13);
        fresh(Wp, t_);
        ig_layer1_map<2, ig_nmax(3)>(lds, U, ng, w1, nt, mh, t_ & 63, none);
        GN_STAMP(14);
        fresh(Wp, t_);
        ig_layer3<2, ig_nmax(4)>(lds, U, ng, Wp, 4, nt, mh, t_ & 63, w1,
                        [&] { ig_fill<3>(lds, U, ng, t_, 0, ig_boff(4)); });  // L4: <= 243 rows
        GN_STAMP(15);
        fresh(Wp, t_);
        ig_layer1_map<3, ig_nmax(4)>(lds, U, ng, w1, nt, mh, t_ & 63, [&] { ig_fill<3>(lds, U, ng, t_, ig_boff(4)); });
        GN_STAMP(16);
        fresh(Wp, t_);
        ig_layer3<3, ig_nmax(5)>(lds, U, ng, Wp, 6, nt, mh, t_ & 63, w1, none);  // L6
        GN_STAMP(17);
        fresh(Wp, t_);
        {   // L7 (1x1) in place over the square rows, then the policy conv per row
            const int ln = t_ & 63;
            constexpr int N5 = ig_nmax(5);
            const IgTiles t = ig_tiles(lds, 5, mh, ln);
            f32x4 acc[N5];
            ig_conv1<N5, ig_brows(5)>((const _Float16*)(lds + ig_boff(5)), t, w1, ln, acc);
            const int ch0 = nt * 16 + 4 * (ln >> 4);
            const f32x4 bias = w1.bias;
            __syncthreads();
            constexpr int BR = ig_brows(5);
            _Float16* sq = (_Float16*)(lds + ig_boff(5));
#pragma unroll
            for (int m = 0; m < N5; m++) {
                const int i = t.i0 + 16 * m;
                if (m >= t.nt || !ig_valid(lds, 5, i)) continue;
                h4 hi, lo;
                ig_split(acc[m], bias, hi, lo);
                const int o = ((ch0 >> 3) * BR + i) * 8 + (ch0 & 7);
                *(h4*)(sq + o) = hi;
                *(h4*)(sq + 8 * BR * 8 + o) = lo;
            }
            __syncthreads();
            GN_STAMP(18);
            fresh(Wp, t_);
            const int total = ig_total(lds, 5);
            if (t_ < 16 * ((total + 15) >> 4) && ig_valid(lds, 5, t_)) {
                const IgRow r = ig_row(lds, 5, t_);
                float p0, p1;
                gn_pconv(Wp, sq + t_ * 8, sq + 8 * BR * 8 + t_ * 8, BR * 8, p0, p1);
                pcv[(r.g * 2 + 0) * 128 + r.j] = p0;
                pcv[(r.g * 2 + 1) * 128 + r.j] = p1;
            }
            __syncthreads();
            GN_STAMP(19);
        }
        // ---- records: policy-conv outputs (new square, else the predecessor's), stones
        for (int e = tid; e < ng * REC; e += NTI) {
            const int g = e / REC, i = e - g * REC;
            const GnUnit& u = U[g];
            float v = 0.f;
            if (i < 2 * POS) {
                const int ch = i >= POS ? 1 : 0, p = i - ch * POS, pr = p / 15, pc = p - (p / 15) * 15;
                const int* q = (const int*)(lds + ITAB) + ITOT + 8 + (4 * IG + g) * 8;  // radius 5
                if (pr >= q[0] && pr < q[0] + q[2] && pc >= q[1] && pc < q[1] + q[3])
                    v = pcv[(g * 2 + ch) * 128 + (pr - q[0]) * q[3] + (pc - q[1])];
                else
                    v = u.pol_src[i];
                u.pol_job[i] = v;
            } else if (i >= REC_X && i < REC_X + 2 * POS) {
                const int ch = i >= REC_X + POS ? 1 : 0, p = i - REC_X - ch * POS;
                const int bit = (p / 15) * 16 + (p % 15);
                v = (float)((u.board[ch * 8 + (bit >> 5)] >> (bit & 31)) & 1u);
            }
            u.rec[i] = v;
        }
        GN_STAMP(20);
    }
}
}  // namespace

#ifdef GZ_GN_STAMPS
extern "C" int gz_gn_stamps_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gz_gn_stamps), 32 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gz_gn_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

extern "C" void gz_internal_set_error(const char* msg);

extern "C" size_t gz_gn_weight_floats(void) { return (size_t)TOTAL; }

// n records, then the split heads' scratch for n rows
extern "C" size_t gz_gn_workspace_bytes(int32_t n) { return (size_t)(n < 1 ? 1 : n) * (REC + HN_ROW) * sizeof(float); }

static int gn_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return cus;
}

static int gn_launch_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string(what) + ": " + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}

// the search roots' full forward: maps and policy-conv outputs into slots 0..n-1
// (gz_plan.hip; d_rec: n record rows of scratch)
extern "C" int gz_internal_gn_roots(const float* d_weights, const uint32_t* d_rows, int32_t n, void* d_slots,
                                    float* d_rec, void* stream) {
    if (n <= 0) return GZ_OK;
    const int cus = gn_cus();
    gn_kernel<<<n < 2 * cus ? n : 2 * cus, NT, 0, (hipStream_t)stream>>>(d_weights, d_rows, n, nullptr, d_rec, nullptr,
                                                                       (char*)d_slots, nullptr);
    return gn_launch_check("gn_kernel (roots)");
}

// the planner nets over tagged rows (gz_plan.hip's collect kernel): full-forward
// rows (keeping their maps in their slots) and incremental rows, then the batched
// heads over all rows
extern "C" int gz_internal_gn_forward_tagged(const float* d_weights, const uint32_t* d_rows, int32_t max_rows,
                                             const int32_t* d_count, const int32_t* d_full_list,
                                             const int32_t* d_full_count, const int32_t* d_inc_list,
                                             const int32_t* d_inc_count, const void* d_tags, void* d_slots,
                                             float* d_p, float* d_q, float* d_rec, float* d_hscratch,
                                             int32_t* d_queue, void* stream) {
    if (max_rows <= 0) return GZ_OK;
    const int cus = gn_cus();
    hipStream_t s = (hipStream_t)stream;
    gn_kernel<<<max_rows < 2 * cus ? max_rows : 2 * cus, NT, 0, s>>>(d_weights, d_rows, max_rows, d_full_count, d_rec,
                                                                     d_full_list, (char*)d_slots, (const GnTag*)d_tags);
    int per = (max_rows + IWG * cus - 1) / (IWG * cus);
    per = per < 1 ? 1 : (per > IG ? IG : per);
    static const int per_env = [] {  // GZ_GN_INC_PER: a fixed chunk size (A/B)
        const char* e = getenv("GZ_GN_INC_PER");
        return e ? atoi(e) : 0;
    }();
    if (per_env >= 1 && per_env <= IG) per = per_env;
    const int chunks = (max_rows + per - 1) / per;
    gn_inc_kernel<<<chunks < IWG * cus ? chunks : IWG * cus, NTI, 0, s>>>(d_weights, d_rows, d_inc_list, d_inc_count,
                                                              (const GnTag*)d_tags, (char*)d_slots, d_rec, per,
                                                              d_queue);
    gn_heads_launch(d_weights, d_rec, max_rows, d_count, d_p, d_q, nullptr, cus, s, d_hscratch);
    return gn_launch_check("gn_inc_kernel");
}

// rows by kind for gz_gn_forward_chain
__global__ void gn_split_kernel(const GnTag* __restrict__ tags, int n, int32_t* __restrict__ lists,
                                int32_t* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int k = tags[i].mode == 1 ? 1 : 0;
    lists[(size_t)k * n + atomicAdd(&counts[k], 1)] = i;
}

extern "C" size_t gz_gn_slot_bytes(void) { return SLOT_BYTES; }

extern "C" size_t gz_gn_chain_workspace_bytes(int32_t n) {
    const size_t m = (size_t)(n < 1 ? 1 : n);
    return m * (REC + HN_ROW) * 4 + 2 * m * 4 + 256;
}

extern "C" int gz_gn_forward_chain(const float* d_weights, const uint32_t* d_boards, int32_t n, const void* d_tags,
                                   void* d_slots, float* d_p, float* d_q, void* d_workspace, void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_tags || !d_slots || !d_p || !d_q || !d_workspace))) {
        gz_internal_set_error("gz_gn_forward_chain: bad arguments");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    hipStream_t s = (hipStream_t)stream;
    float* rec = (float*)d_workspace;
    float* hsc = rec + (size_t)n * REC;
    int32_t* lists = (int32_t*)(hsc + (size_t)n * HN_ROW);
    int32_t* counts = lists + 2 * (size_t)n;
    if (hipMemsetAsync(counts, 0, 12, s) != hipSuccess) {  // the two list counts, gn_inc_kernel's queue head
        gz_internal_set_error("gz_gn_forward_chain: memset");
        return GZ_ERR_HIP;
    }
    gn_split_kernel<<<(n + 255) / 256, 256, 0, s>>>((const GnTag*)d_tags, n, lists, counts);
    int rc = gn_launch_check("gn_split_kernel");
    if (rc) return rc;
    return gz_internal_gn_forward_tagged(d_weights, d_boards, n, nullptr, lists, counts, lists + n, counts + 1,
                                         d_tags, d_slots, d_p, d_q, rec, hsc, counts + 2, stream);
}

extern "C" int gz_gn_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                             float* d_p, float* d_q, float* d_logits, void* d_workspace, void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_p || !d_q || !d_workspace))) {
        gz_internal_set_error("gz_gn_forward: bad arguments (d_workspace: gz_gn_workspace_bytes(n))");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    int grid = n < 2 * cus ? n : 2 * cus;
    hipStream_t s = (hipStream_t)stream;
    gn_kernel<<<grid, NT, 0, s>>>(d_weights, d_boards, n, d_count, (float*)d_workspace, nullptr, nullptr, nullptr);
    gn_heads_launch(d_weights, (const float*)d_workspace, n, d_count, d_p, d_q, d_logits, cus, s,
                    (float*)d_workspace + (size_t)n * REC);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("gn_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
