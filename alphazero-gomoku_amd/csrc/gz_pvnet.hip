// gz_pvnet.hip -- AlphaZeroGomokuNet forward (neural_network.py:94-159) plus the
// softmax of GomokuModel.predict (neural_network.py:214-252) on gfx950.
//
// One 512-thread workgroup (8 waves) evaluates one board at a time and loops
// over boards.  The board's 128x225 activation map stays in LDS for the whole
// tower; every 3x3 conv is an implicit GEMM
//   C[pos][ch] = sum_k A[pos][k] * W[k][ch],  A[pos][tap*128+cin] = act[cin][pos+tap]
// with M = 225 positions (15 tiles of 16), N = 128 channels (8 tiles of 16):
// wave w owns N tile w for all 15 M tiles, so each weight fragment is read
// once per board per workgroup and reused 15 times.  Off-board neighbours read
// a zero slot instead of predicating.  Two precisions (same layout of work):
//
//  * GZ_PV_FP32: v_mfma_f32_16x16x4_f32 -- exact f32 products, f32 accumulate.
//    Activations fp32, channel-major [ch][240].  The skip input of a residual
//    block is parked in a per-wave global slab (registers are full).
//  * GZ_PV_F16X3: v_mfma_f32_16x16x32_f16 on a 3-term split, x = x_hi + x_lo
//    (x_hi = fp16(x), x_lo = fp16(x - x_hi)):  a*w ~ a_hi*w_hi + a_hi*w_lo +
//    a_lo*w_hi, every product exact in the f32 accumulator, ~22-bit operands.
//    16x the f32 MFMA rate per instruction, 5.3x per fp32-equivalent product.
//    Activations as hi/lo fp16 planes, position-major [240][136] (272-byte
//    rows: 16-byte A fragments by ds_read_b128 with few bank conflicts).  The
//    skip input stays in registers.
#include <hip/hip_runtime.h>

#include <string>

#include "gz_pvnet.h"
#include "../../include/gzero.h"

using namespace gzpv;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int NT = 512;    // 8 waves: wave w owns output channels [16w, 16w+16)
constexpr int MT = 15;     // 16-position M tiles (240 >= 225)
constexpr int ROWS = 240;  // positions incl. 15 zero rows / slots
constexpr int ZERO = POS;  // index of a zero slot: the out-of-board neighbour
constexpr int RS = 136;    // fp16 row: 128 channels + 8 pad (272 B)

// LDS layout (bytes): activation area first, then shared small buffers
constexpr int ACT_BYTES_F32 = CH * ROWS * 4;      // 122880
constexpr int ACT_BYTES_F16 = 2 * ROWS * RS * 2;  // 130560
constexpr int ACT_BYTES = ACT_BYTES_F16 > ACT_BYTES_F32 ? ACT_BYTES_F16 : ACT_BYTES_F32;
constexpr int PLANES_F = 3 * ROWS;
constexpr int SMALL_F = PLANES_F + 2 * POS + POS + 64 + 32 + 256;
constexpr int LDS_BYTES = ACT_BYTES + SMALL_F * 4;

__device__ inline f32x4 zero4() {
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    return z;
}

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
    __device__ void zero_slots(int tid) {
        for (int i = tid; i < CH * (ROWS - POS); i += NT) a[(i / (ROWS - POS)) * ROWS + POS + i % (ROWS - POS)] = 0.f;
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

// ============================================================ fp16x3 policy
struct ActF16x3 {
    _Float16* hi;  // [ROWS][RS]
    _Float16* lo;
    __device__ float get(int ch, int pos) const {
        int o = pos * RS + ch;
        return (float)hi[o] + (float)lo[o];
    }
    __device__ void put(int ch, int pos, float y) {
        _Float16 h = (_Float16)y;
        _Float16 l = (_Float16)(y - (float)h);  // y - h is exact in f32
        int o = pos * RS + ch;
        hi[o] = h;
        lo[o] = l;
    }
    __device__ void zero_slots(int tid) {
        for (int i = tid; i < (ROWS - POS) * RS; i += NT) {
            hi[POS * RS + i] = (_Float16)0.f;
            lo[POS * RS + i] = (_Float16)0.f;
        }
    }
    // k = tap*128 + cin, 32 input channels per k-step (lane group q = lane>>4 holds 8)
    __device__ __forceinline__ void conv(const _Float16* __restrict__ Whi, const _Float16* __restrict__ Wlo, int nt,
                                         int lane, f32x4 acc[MT]) const {
        const int li = lane & 15, q = lane >> 4;
        const _Float16* wh = Whi + (size_t)(nt * 16 + li) * K + 8 * q;  // W^T [n][k]
        const _Float16* wl = Wlo + (size_t)(nt * 16 + li) * K + 8 * q;
        h8 bh = *(const h8*)wh, bl = *(const h8*)wl;
        for (int tap = 0; tap < 9; tap++) {
            const int dr = tap / 3 - 1, dc = tap % 3 - 1;
            int lv = li;
            asm volatile("" : "+v"(lv));
            int nb[MT];
#pragma unroll
            for (int m = 0; m < MT; m++) nb[m] = nbr(m, lv, dr, dc) * RS + 8 * q;
#pragma unroll
            for (int cq = 0; cq < 4; cq++) {
                const int ks = tap * 4 + cq;
                h8 bhn = bh, bln = bl;
                if (ks + 1 < 36) {
                    bhn = *(const h8*)(wh + (ks + 1) * 32);
                    bln = *(const h8*)(wl + (ks + 1) * 32);
                }
                const _Float16* ahp = hi + cq * 32;
                const _Float16* alp = lo + cq * 32;
#pragma unroll
                for (int m = 0; m < MT; m++) {
                    const h8 ah = *(const h8*)(ahp + nb[m]);
                    const h8 al = *(const h8*)(alp + nb[m]);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[m], 0, 0, 0);
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[m], 0, 0, 0);
                }
                bh = bhn;
                bl = bln;
            }
        }
    }
};

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
                float y = acc[m][r] * s + t;
                if (skip) y += skip[m][r];
                act.put(ch, pos, y > 0.f ? y : 0.f);
            }
        }
    }
}

template <class Act>
__device__ __forceinline__ void load_tiles(const Act& act, f32x4 out[MT], int nt, int lane) {
    const int ch = nt * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
    for (int m = 0; m < MT; m++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int pos = m * 16 + 4 * g + r;
            out[m][r] = pos < POS ? act.get(ch, pos) : 0.f;
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

template <int PREC>
__global__ __launch_bounds__(NT, 1) void pv_kernel(const float* __restrict__ W, const uint32_t* __restrict__ boards, int n,
                                                   const int32_t* d_count, float* __restrict__ logits,
                                                   float* __restrict__ value, float* __restrict__ probs,
                                                   float* __restrict__ scratch) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    float* small = (float*)(lds + ACT_BYTES);
    float* planes = small;  // [3][ROWS] fp32
    float* hp = planes + PLANES_F;
    float* hv = hp + 2 * POS;
    float* hh = hv + POS;
    float* red = hh + 64;
    float* lg = red + 32;
    using Act = typename std::conditional<PREC == GZ_PV_FP32, ActF32, ActF16x3>::type;
    Act act;
    if constexpr (PREC == GZ_PV_FP32) {
        act.a = (float*)lds;
    } else {
        act.hi = (_Float16*)lds;
        act.lo = act.hi + ROWS * RS;
    }

    int count = n;
    if (d_count) {
        int c = *d_count;
        count = c < n ? c : n;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nt = wave;
    float* slab = scratch ? scratch + ((size_t)blockIdx.x * (NT / 64) + wave) * (MT * 4 * 64) : nullptr;
    act.zero_slots(tid);
    for (int i = tid; i < 3 * (ROWS - POS); i += NT) planes[(i / (ROWS - POS)) * ROWS + POS + i % (ROWS - POS)] = 0.f;

    for (int b = blockIdx.x; b < count; b += gridDim.x) {
        // ---- input planes [black, white, empty] (gomoku_board.py:239-260, absolute colours)
        const uint32_t* bd = boards + (size_t)b * 16;
        for (int p = tid; p < POS; p += NT) {
            int bit = (p / 15) * 16 + (p % 15);
            uint32_t bl = (bd[bit >> 5] >> (bit & 31)) & 1u;
            uint32_t wh = (bd[8 + (bit >> 5)] >> (bit & 31)) & 1u;
            planes[p] = (float)bl;
            planes[ROWS + p] = (float)wh;
            planes[2 * ROWS + p] = (float)(1u - (bl | wh));
        }
        __syncthreads();

        // ---- conv0 3->128 + BN + ReLU (exact f32 MFMA in both modes): K = 27 (k = tap*3+cin) -> 28
        f32x4 acc[MT];
#pragma unroll
        for (int m = 0; m < MT; m++) acc[m] = zero4();
        {
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
        }
        store_tiles(act, acc, W + C0_S, W + C0_T, (const f32x4*)nullptr, nt, lane);
        __syncthreads();

        // ---- residual tower (ResidualBlock, neural_network.py:74-91)
        for (int blk = 0; blk < 2; blk++) {
            f32x4 skip[MT];
            for (int half = 0; half < 2; half++) {
                const int layer = 2 * blk + half;
                const float* R = W + RES0 + layer * RES_STRIDE;
#pragma unroll
                for (int m = 0; m < MT; m++) acc[m] = zero4();
                if constexpr (PREC == GZ_PV_FP32) {
                    act.conv(R + RES_W, nt, lane, acc);
                } else {
                    const _Float16* wh = (const _Float16*)(W + F16_RES0 + layer * F16_STRIDE);
                    act.conv(wh, wh + K * CH, nt, lane, acc);
                }
                if (half == 0) {  // keep the block input for the skip connection
                    if constexpr (PREC == GZ_PV_FP32) slab_save(act, slab, nt, lane);
                    else load_tiles(act, skip, nt, lane);
                }
                __syncthreads();
                if (half == 0) {
                    store_tiles(act, acc, R + RES_S, R + RES_T, (const f32x4*)nullptr, nt, lane);
                } else {
                    if constexpr (PREC == GZ_PV_FP32) slab_load(slab, skip, lane);
                    store_tiles(act, acc, R + RES_S, R + RES_T, skip, nt, lane);
                }
                __syncthreads();
            }
        }

        // ---- heads: 1x1 convs (policy 128->2, value 128->1)
        if (tid < POS) {
            const int pos = tid;
            float p0 = W[P_B], p1 = W[P_B + 1], v = W[V_B];
            for (int c = 0; c < CH; c++) {
                float a = act.get(c, pos);
                p0 += W[P_W + c] * a;
                p1 += W[P_W + CH + c] * a;
                v += W[V_W + c] * a;
            }
            hp[pos] = p0;  // flatten order: channel-major (policy.view(B, -1))
            hp[POS + pos] = p1;
            hv[pos] = v;
        }
        __syncthreads();
        // policy_fc 450->225, value_fc1 225->64 (+ReLU)
        if (tid < POS) {
            const int o = tid;
            float acc1 = W[PF_B + o];
            for (int i = 0; i < 2 * POS; i++) acc1 += W[PF_WT + i * POS + o] * hp[i];
            lg[o] = acc1;
        } else if (tid >= 256 && tid < 256 + 64) {
            const int j = tid - 256;
            float acc1 = W[V1_B + j];
            for (int i = 0; i < POS; i++) acc1 += W[V1_WT + i * 64 + j] * hv[i];
            hh[j] = acc1 > 0.f ? acc1 : 0.f;
        }
        __syncthreads();
        // value_fc2 + tanh (wave 0); softmax max/sum over 225 logits (waves 0..3)
        if (wave == 0) {
            float part = W[V2_W + lane] * hh[lane];
            float tot = wave_sum(part) + W[V2_B];
            if (lane == 0) value[b] = tanhf(tot);
        }
        if (wave < 4) {
            const int o = tid;
            float x = o < POS ? lg[o] : -3.0e38f;
            float mx = wave_max(x);
            if (lane == 0) red[wave] = mx;
        }
        __syncthreads();
        if (wave < 4) {
            const int o = tid;
            const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
            float e = o < POS ? __expf(lg[o] - mx) : 0.f;
            float sm = wave_sum(e);
            if (lane == 0) red[8 + wave] = sm;
            if (o < POS) {
                logits[(size_t)b * POS + o] = lg[o];
                lg[o] = e;
            }
        }
        __syncthreads();
        if (wave < 4 && probs) {
            const int o = tid;
            const float sm = (red[8] + red[9]) + (red[10] + red[11]);
            if (o < POS) probs[(size_t)b * POS + o] = lg[o] / sm;
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" void gz_internal_set_error(const char* msg);

extern "C" size_t gz_pv_weight_floats(void) { return (size_t)TOTAL; }

static int pv_grid(int n) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
    }
    return n < cus ? n : cus;
}

extern "C" size_t gz_pv_workspace_bytes(int32_t n) {
    int grid = pv_grid(n < 1 ? 1 : n);
    return (size_t)grid * (NT / 64) * MT * 4 * 64 * sizeof(float);
}

extern "C" int gz_pv_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                             float* d_logits, float* d_value, float* d_probs, void* d_workspace, int32_t precision,
                             void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_logits || !d_value))) {
        gz_internal_set_error("gz_pv_forward: bad arguments");
        return GZ_ERR_ARG;
    }
    if (precision != GZ_PV_FP32 && precision != GZ_PV_F16X3) {
        gz_internal_set_error("gz_pv_forward: unknown precision");
        return GZ_ERR_ARG;
    }
    if (precision == GZ_PV_FP32 && !d_workspace) {
        gz_internal_set_error("gz_pv_forward: fp32 mode needs d_workspace");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    int grid = pv_grid(n);
    hipStream_t s = (hipStream_t)stream;
    if (precision == GZ_PV_FP32)
        pv_kernel<GZ_PV_FP32><<<grid, NT, 0, s>>>(d_weights, d_boards, n, d_count, d_logits, d_value, d_probs,
                                                  (float*)d_workspace);
    else
        pv_kernel<GZ_PV_F16X3><<<grid, NT, 0, s>>>(d_weights, d_boards, n, d_count, d_logits, d_value, d_probs,
                                                   nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("pv_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
