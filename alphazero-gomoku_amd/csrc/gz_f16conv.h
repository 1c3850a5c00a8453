// gz_f16conv.h -- shared pieces of the f16x3 MFMA convolutions (gz_pvnet.hip,
// gz_gnet.hip): the activation-plane layout, the pipelined implicit-GEMM 3x3 /
// 1x1 conv and the VALU helpers of the heads.
//
// f16x3: x = x_hi + x_lo (x_hi = fp16(x), x_lo = fp16(x - x_hi)); a*w ~ a_hi*w_hi +
// a_hi*w_lo + a_lo*w_hi on v_mfma_f32_16x16x32_f16, every product exact in the f32
// accumulator (~22-bit operands).  The MFMAs compute C^T[ch][pos] (A = weight
// fragment, B = activation fragment).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gzc {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int BN = 15;     // board side
constexpr int BPOS = 225;  // positions

__device__ inline f32x4 zero4() {
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    return z;
}

// Activations as hi/lo fp16 planes [channel group][ROWS16][8]: group cg = ch/8 holds
// 16 B per position, so the 16 lanes of a ds_read_b128 bank group read 16
// consecutive positions = 16 distinct 16-B bank slots.  Rows 225..255 are zero;
// an off-board neighbour with virtual index v reads zero row 225 + ((v-225) mod 16),
// which keeps its bank slot = v mod 16, so no tap or board edge conflicts.
constexpr int ROWS16 = 256;
__device__ inline int nbr16(int m, int li, int dr, int dc) {
    int pos = m * 16 + li;
    int r = pos / BN + dr, c = pos % BN + dc;
    bool ok = pos < BPOS && r >= 0 && r < BN && c >= 0 && c < BN;
    return ok ? r * BN + c : BPOS + ((pos + dr * BN + dc - BPOS) & 15);
}

struct ActF16x3 {
    _Float16* hi;
    _Float16* lo;
    __device__ static int off(int ch, int pos) { return ((ch >> 3) * ROWS16 + pos) * 8 + (ch & 7); }
    __device__ void get8(int c0, int pos, float* x) const {  // channels c0..c0+7, c0 % 8 == 0
        const h8 xh = *(const h8*)(hi + ((c0 >> 3) * ROWS16 + pos) * 8);
        const h8 xl = *(const h8*)(lo + ((c0 >> 3) * ROWS16 + pos) * 8);
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = (float)xh[j] + (float)xl[j];
    }
    __device__ void zero_slots(int tid, int nth, int channels) {
        constexpr int PAD = (ROWS16 - BPOS) * 8;
        for (int i = tid; i < (channels / 8) * PAD; i += nth) {
            int o = (i / PAD) * ROWS16 * 8 + BPOS * 8 + i % PAD;
            hi[o] = (_Float16)0.f;
            lo[o] = (_Float16)0.f;
        }
    }
};

// lane (li, g) of a C^T tile holds channels 4g..4g+3 of its N tile for position
// 16*tile + li: 4 consecutive channels = 8 bytes of the hi plane and 8 of the lo.
__device__ __forceinline__ void f16_get4(const ActF16x3& act, int ch0, int pos, f32x4& out) {
    const int o = ActF16x3::off(ch0, pos);
    const h4 xh = *(const h4*)(act.hi + o);
    const h4 xl = *(const h4*)(act.lo + o);
#pragma unroll
    for (int r = 0; r < 4; r++) out[r] = (float)xh[r] + (float)xl[r];
}

// y = acc*S + T (+ skip), ReLU, split into hi/lo and stored as two 8-byte writes
template <bool SKIP>
__device__ __forceinline__ void f16_put4(ActF16x3& act, const f32x4& acc, const f32x4& s, const f32x4& t,
                                         const f32x4& skip, int ch0, int pos) {
    h4 hi, lo;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        float y = acc[r] * s[r] + t[r];
        if (SKIP) y += skip[r];
        y = y > 0.f ? y : 0.f;
        const _Float16 h = (_Float16)y;
        hi[r] = h;
        lo[r] = (_Float16)(y - (float)h);  // y - h is exact in f32
    }
    const int o = ActF16x3::off(ch0, pos);
    *(h4*)(act.hi + o) = hi;
    *(h4*)(act.lo + o) = lo;
}

// Implicit-GEMM conv (3x3 with TAPS = 9, 1x1 with TAPS = 1) over CQ 32-channel
// input groups, for the wave's n-tiles {2np, 2np+1} of NTT and M tiles
// [m0, m0 + NM).  Weights: f16 hi then lo, each in A-fragment order
// [ks = tap*CQ + cq][n-tile NTT][lane 64][8] (gzero/weights.py, planner_nets.py).
//
// Software pipeline over half k-steps: the activation fragments of M tiles
// [HA, NM) are read while the MFMAs of tiles [0, HA) run, and those of [0, HA)
// for the next k-step while the MFMAs of [HA, NM) run; the weight fragments of
// the next k-step are prefetched.  The order is pinned with sched_group_barrier
// (the default scheduler sinks every read to its use).  Branch-free: the last
// k-step prefetches k-step 0 / the tap after the last (valid addresses, unused),
// so each tap is one basic block.
template <int NM, int CQ, int NTT, int TAPS>
__device__ __forceinline__ void f16_conv(const ActF16x3& act, const _Float16* __restrict__ Wf, int np, int m0,
                                         int lane, f32x4 (&acc)[2][NM]) {
    constexpr int HA = (NM + 1) / 2, HB = NM - HA;
    constexpr int KS = TAPS * CQ;
    constexpr int KS_HALVES = NTT * 64 * 8;  // fragments of one k-step, all n-tiles
    constexpr int KS_BYTES = KS_HALVES * 2, LO_BYTES = KS * KS_BYTES;
    const int li = lane & 15, q = lane >> 4;
    // weight fragments through a buffer resource: one 32-bit lane offset instead of
    // two 64-bit pointers (the k-step / hi-lo / n-tile parts are wave-uniform)
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)Wf, 0, 0x7fffffff, 0x00020000);
    const int wo = ((2 * np) * 64 + lane) * 16;
    auto wload = [&](int ks, int n, int lo) -> h8 {
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wo, ks * KS_BYTES + n * 1024 + lo * LO_BYTES, 0));
    };
    h8 b[2][2];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        b[n][0] = wload(0, n, 0);
        b[n][1] = wload(0, n, 1);
    }

    h8 ah[NM], al[NM];
    int nb[NM];
    int lv = li;
    asm volatile("" : "+v"(lv));
#pragma unroll
    for (int m = 0; m < NM; m++)
        nb[m] = (nbr16(m0 + m, lv, TAPS == 9 ? -1 : 0, TAPS == 9 ? -1 : 0) + q * ROWS16) * 8;
#pragma unroll
    for (int m = 0; m < HA; m++) {
        ah[m] = *(const h8*)(act.hi + nb[m]);
        al[m] = *(const h8*)(act.lo + nb[m]);
    }
    for (int tap = 0; tap < TAPS; tap++) {
#pragma unroll
        for (int cq = 0; cq < CQ; cq++) {
            const int ks = tap * CQ + cq;
            const int ao = cq * 4 * ROWS16 * 8;
#pragma unroll
            for (int m = HA; m < NM; m++) {
                ah[m] = *(const h8*)(act.hi + ao + nb[m]);
                al[m] = *(const h8*)(act.lo + ao + nb[m]);
            }
            h8 bn[2][2];
            {
                const int ks1 = ks + 1 < KS ? ks + 1 : 0;
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    bn[n][0] = wload(ks1, n, 0);
                    bn[n][1] = wload(ks1, n, 1);
                }
            }
#pragma unroll
            for (int m = 0; m < HA; m++) {
#pragma unroll
                for (int n = 0; n < 2; n++) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[n][0], ah[m], acc[n][m], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 2; n++) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[n][1], ah[m], acc[n][m], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 2; n++) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[n][0], al[m], acc[n][m], 0, 0, 0);
            }
            if (TAPS == 9 && cq == CQ - 1) {  // next tap: new neighbour offsets (tap 9 after the last: unused)
                const int t2 = tap + 1, dr = t2 / 3 - 1, dc = t2 % 3 - 1;
                int lw = li;
                asm volatile("" : "+v"(lw));
#pragma unroll
                for (int m = 0; m < NM; m++) nb[m] = (nbr16(m0 + m, lw, dr, dc) + q * ROWS16) * 8;
            }
            {
                const int ao2 = ((cq + 1) % CQ) * 4 * ROWS16 * 8;
#pragma unroll
                for (int m = 0; m < HA; m++) {
                    ah[m] = *(const h8*)(act.hi + ao2 + nb[m]);
                    al[m] = *(const h8*)(act.lo + ao2 + nb[m]);
                }
            }
#pragma unroll
            for (int m = HA; m < NM; m++) {
#pragma unroll
                for (int n = 0; n < 2; n++) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[n][0], ah[m], acc[n][m], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 2; n++) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[n][1], ah[m], acc[n][m], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < 2; n++) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[n][0], al[m], acc[n][m], 0, 0, 0);
            }
#pragma unroll
            for (int n = 0; n < 2; n++) {
                b[n][0] = bn[n][0];
                b[n][1] = bn[n][1];
            }
            // pin the interleave: weight prefetch first, then 2 activation reads per 6 MFMAs
            __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);  // VMEM read
#pragma unroll
            for (int m = 0; m < HA; m++) {
                if (m < HB) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);              // MFMA
            }
#pragma unroll
            for (int m = 0; m + 1 < HB; m++) {
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 2 + 2 * (HA - HB), 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
        }
    }
}

// wave-wide reductions (wave64)
__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ inline float wave_max(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// sum_i w[i*stride] * x[i] for one output column; BATCH independent loads in flight
template <int NI, int BATCH>
__device__ __forceinline__ float dot_col(const float* __restrict__ wp, int stride, const float* __restrict__ xp) {
    static_assert(NI % BATCH == 0, "batch must divide the input count");
    float acc = 0.f;
#pragma unroll 1
    for (int i0 = 0; i0 < NI; i0 += BATCH) {
        float w[BATCH];
#pragma unroll
        for (int j = 0; j < BATCH; j++) w[j] = wp[(size_t)(i0 + j) * stride];
#pragma unroll
        for (int j = 0; j < BATCH; j++) acc += w[j] * xp[i0 + j];
    }
    return acc;
}

// One 16-deep K block of a batched fp32-MFMA GEMM over 4 tiles of 16 rows
// (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation): in the t-th k-step
// of block kb, lane group g multiplies k = 16kb + 4g + t, so a lane's A operand for
// the 4 k-steps is one 16-byte load from its row arow[m] (rows zero past K), and its
// B operand is one 16-byte load from the packed weights
//   Wp[kb][n-tile][lane 64][t 4] = W^T[16kb + 4(lane/16) + t][16 n-tile + lane%16]
// (zero past K and N; gzero/weights.py pack_mfma_b).  n-tiles nt[0..ntn) of the wave.
// Used by the batched FC heads of the PV and planner nets.
__device__ __forceinline__ void heads_gemm_block(const float* __restrict__ Wp, int ntiles, int kb, int lane,
                                                 const int (&nt)[4], int ntn, f32x4 (&acc)[4][4],
                                                 const float* __restrict__ arow[4]) {
    const int g = lane >> 4;
    f32x4 a[4], b[4];
#pragma unroll
    for (int m = 0; m < 4; m++) a[m] = *(const f32x4*)(arow[m] + 16 * kb + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; q++)
        b[q] = q < ntn ? *(const f32x4*)(Wp + (((size_t)kb * ntiles + nt[q]) * 64 + lane) * 4) : zero4();
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (q < ntn) acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][t], b[q][t], acc[m][q], 0, 0, 0);
}

}  // namespace gzc
