// gz_pvnet.hip -- AlphaZeroGomokuNet forward (neural_network.py:94-159) plus the
// softmax of GomokuModel.predict (neural_network.py:214-252) on gfx950.
//
// One 512-thread workgroup (8 waves) evaluates one board at a time and loops
// over boards.  The 128x225 fp32 activation map of the board stays in LDS for
// the whole tower (123 KB with a zero slot per channel row); every 3x3 conv is
// an implicit GEMM
//   C[pos][ch] = sum_k A[pos][k] * W[k][ch],  A[pos][tap*128+cin] = act[cin][pos+tap]
// on v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation).  M = 225
// positions (15 tiles of 16), N = 128 channels (8 tiles of 16): wave w owns
// N tile w for all 15 M tiles (15 accumulators of 4 VGPRs), so each weight
// (B operand, streamed from L2) is used 15 times and read once per board per
// workgroup.  Off-board neighbours read the zero slot instead of predicating.
// The residual input of a block is kept in registers while conv1's output
// overwrites the map.
#include <hip/hip_runtime.h>

#include <string>

#include "gz_pvnet.h"
#include "../../include/gzero.h"

using namespace gzpv;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;          // 8 waves: wave w owns output channels [16w, 16w+16)
constexpr int STRIDE = 240;      // per-channel row: 225 cells + 15 zero slots (cell 225 = 0)
constexpr int ZERO = POS;        // index of a zero slot: the out-of-board neighbour
constexpr int MT = 15;           // 16-position M tiles (240 >= 225)
constexpr int LDS_ACT = CH * STRIDE;
constexpr int LDS_PLANES = 3 * STRIDE;
constexpr int LDS_HP = 2 * POS;
constexpr int LDS_HV = POS;
constexpr int LDS_HH = 64;
constexpr int LDS_RED = 32;
constexpr int LDS_LG = 256;
constexpr int LDS_FLOATS = LDS_ACT + LDS_PLANES + LDS_HP + LDS_HV + LDS_HH + LDS_RED + LDS_LG;

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

// 3x3 conv 128->128 as an implicit GEMM on v_mfma_f32_16x16x4_f32.
// k = tap*128 + cin; one k-step covers 4 input channels (lane group g = lane>>4).
// Operands are double-buffered in registers: the next k-step's 15 A values
// (LDS) and the next 8 k-steps' B values (weights, L2) are in flight while the
// current 15 MFMAs issue.
__device__ __forceinline__ void conv3x3(const float* act, const float* __restrict__ Wk, int nt, int lane,
                                        f32x4 acc[MT]) {
    const int li = lane & 15, g = lane >> 4;
    const float* wbase = Wk + (size_t)g * CH + nt * 16 + li;
    float bq[8], bn[8];
#pragma unroll
    for (int s = 0; s < 8; s++) bq[s] = wbase[(size_t)(4 * s) * CH];
    for (int blk = 0; blk < 36; blk++) {  // 9 taps x 4 blocks of 8 k-steps
        const int tap = blk >> 2, sb = blk & 3;
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        // opaque copy: stops LICM from hoisting all 9x15 neighbour indices out of
        // the board loop (they would be spilled); recomputing them is cheap VALU
        int lv = li;
        asm volatile("" : "+v"(lv));
        int nb[MT];
#pragma unroll
        for (int m = 0; m < MT; m++) nb[m] = nbr(m, lv, dr, dc);
        if (blk + 1 < 36) {
            const int t2 = (blk + 1) >> 2, s2 = (blk + 1) & 3;
            const float* wp = wbase + (size_t)(t2 * CH + 32 * s2) * CH;
#pragma unroll
            for (int s = 0; s < 8; s++) bn[s] = wp[(size_t)(4 * s) * CH];
        }
        const float* ab = act + (32 * sb + g) * STRIDE;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const float* ap = ab + 4 * s * STRIDE;
            float a[MT];
#pragma unroll
            for (int m = 0; m < MT; m++) a[m] = ap[nb[m]];
#pragma unroll
            for (int m = 0; m < MT; m++) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bq[s], acc[m], 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 8; s++) bq[s] = bn[s];
    }
}

// epilogue: y = acc*S + T (+ residual), ReLU, back into the LDS map.
// C layout of 16x16x4: column (channel) = lane&15, row (position) = 4*(lane>>4) + r.
__device__ __forceinline__ void store_tiles(float* act, const f32x4 acc[MT], const float* __restrict__ S,
                                           const float* __restrict__ T, int nt, int lane) {
    const int ch = nt * 16 + (lane & 15), g = lane >> 4;
    const float s = S[ch], t = T[ch];
#pragma unroll
    for (int m = 0; m < MT; m++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int pos = m * 16 + 4 * g + r;
            if (pos < POS) {
                float y = acc[m][r] * s + t;
                act[ch * STRIDE + pos] = y > 0.f ? y : 0.f;
            }
        }
    }
}

// The block input (skip connection) of the wave's tiles is parked in a global
// scratch slab while conv1's output overwrites the LDS map: lane-contiguous, so
// each of the 60 stores / loads per lane is one coalesced 256-byte access.
__device__ __forceinline__ void save_resid(const float* act, float* __restrict__ slab, int nt, int lane) {
    const int ch = nt * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
    for (int m = 0; m < MT; m++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int pos = m * 16 + 4 * g + r;
            slab[(m * 4 + r) * 64 + lane] = pos < POS ? act[ch * STRIDE + pos] : 0.f;
        }
    }
}

__device__ __forceinline__ void store_tiles_res(float* act, const f32x4 acc[MT], const float* __restrict__ S,
                                               const float* __restrict__ T, const float* __restrict__ slab, int nt,
                                               int lane) {
    const int ch = nt * 16 + (lane & 15), g = lane >> 4;
    const float s = S[ch], t = T[ch];
#pragma unroll
    for (int m = 0; m < MT; m++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int pos = m * 16 + 4 * g + r;
            float x = slab[(m * 4 + r) * 64 + lane];
            if (pos < POS) {
                float y = acc[m][r] * s + t + x;
                act[ch * STRIDE + pos] = y > 0.f ? y : 0.f;
            }
        }
    }
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

__global__ __launch_bounds__(NT, 1) void pv_kernel(const float* __restrict__ W, const uint32_t* __restrict__ boards, int n,
                                                   const int32_t* d_count, float* __restrict__ logits,
                                                   float* __restrict__ value, float* __restrict__ probs,
                                                   float* __restrict__ scratch) {
    __shared__ float lds[LDS_FLOATS];
    float* act = lds;
    float* planes = act + LDS_ACT;
    float* hp = planes + LDS_PLANES;
    float* hv = hp + LDS_HP;
    float* hh = hv + LDS_HV;
    float* red = hh + LDS_HH;
    float* lg = red + LDS_RED;

    int count = n;
    if (d_count) {
        int c = *d_count;
        count = c < n ? c : n;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nt = wave;
    float* slab = scratch + ((size_t)blockIdx.x * (NT / 64) + wave) * (MT * 4 * 64);
    // zero slots of every channel row (never written afterwards)
    for (int i = tid; i < CH * (STRIDE - POS); i += NT) act[(i / (STRIDE - POS)) * STRIDE + POS + i % (STRIDE - POS)] = 0.f;
    for (int i = tid; i < 3 * (STRIDE - POS); i += NT) planes[(i / (STRIDE - POS)) * STRIDE + POS + i % (STRIDE - POS)] = 0.f;

    for (int b = blockIdx.x; b < count; b += gridDim.x) {
        // ---- input planes [black, white, empty] (gomoku_board.py:239-260, absolute colours)
        const uint32_t* bd = boards + (size_t)b * 16;
        for (int p = tid; p < POS; p += NT) {
            int bit = (p / 15) * 16 + (p % 15);
            uint32_t bl = (bd[bit >> 5] >> (bit & 31)) & 1u;
            uint32_t wh = (bd[8 + (bit >> 5)] >> (bit & 31)) & 1u;
            planes[p] = (float)bl;
            planes[STRIDE + p] = (float)wh;
            planes[2 * STRIDE + p] = (float)(1u - (bl | wh));
        }
        __syncthreads();

        // ---- conv0 3->128 + BN + ReLU: K = 27 (k = tap*3 + cin) padded to 28 = 7 k-steps
        f32x4 acc[MT];
#pragma unroll
        for (int m = 0; m < MT; m++) acc[m] = zero4();
        {
            int li = lane & 15;
            asm volatile("" : "+v"(li));  // keep the neighbour indices out of the hoisted set
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
                    float a = planes[(k < 27 ? cin : 0) * STRIDE + idx];
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw, acc[m], 0, 0, 0);
                }
            }
        }
        store_tiles(act, acc, W + C0_S, W + C0_T, nt, lane);
        __syncthreads();

        // ---- residual tower (ResidualBlock, neural_network.py:74-91): 4 convs in
        // one loop (one code copy): even = conv1 (+BN+ReLU), odd = conv2 (+BN, +skip, ReLU)
        for (int layer = 0; layer < 4; layer++) {
            const float* R = W + RES0 + layer * RES_STRIDE;
#pragma unroll
            for (int m = 0; m < MT; m++) acc[m] = zero4();
            conv3x3(act, R + RES_W, nt, lane, acc);
            if ((layer & 1) == 0) save_resid(act, slab, nt, lane);  // block input for the skip
            __syncthreads();
            if ((layer & 1) == 0) store_tiles(act, acc, R + RES_S, R + RES_T, nt, lane);
            else store_tiles_res(act, acc, R + RES_S, R + RES_T, slab, nt, lane);
            __syncthreads();
        }

        // ---- heads: 1x1 convs (policy 128->2, value 128->1)
        if (tid < POS) {
            const int pos = tid;
            float p0 = W[P_B], p1 = W[P_B + 1], v = W[V_B];
            for (int c = 0; c < CH; c++) {
                float a = act[c * STRIDE + pos];
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
                             float* d_logits, float* d_value, float* d_probs, void* d_workspace, void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_logits || !d_value || !d_workspace))) {
        gz_internal_set_error("gz_pv_forward: bad arguments");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    int grid = pv_grid(n);
    pv_kernel<<<grid, NT, 0, (hipStream_t)stream>>>(d_weights, d_boards, n, d_count, d_logits, d_value, d_probs,
                                                    (float*)d_workspace);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("pv_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
