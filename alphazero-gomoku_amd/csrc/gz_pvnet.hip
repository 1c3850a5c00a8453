// gz_pvnet.hip -- AlphaZeroGomokuNet forward (neural_network.py:94-159) plus the
// softmax of GomokuModel.predict (neural_network.py:214-252) on gfx950.
//
// One 512-thread workgroup (8 waves) evaluates one board at a time and loops
// over boards.  The 128x225 fp32 activation map of the board stays in LDS for
// the whole tower (115 KB); every 3x3 conv is an implicit GEMM
//   C[pos][ch] = sum_k A[pos][k] * W[k][ch],  A[pos][tap*128+cin] = act[cin][pos+tap]
// on v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation).  M = 225
// positions (8 tiles of 32), N = 128 channels (4 tiles), so each wave owns one
// N tile x four M tiles (4 accumulators of 16 VGPRs).  Weights stream from
// L2 (B operand, coalesced 2x128 B per k-step).  The residual input of a block
// is kept in registers while conv1's output overwrites the map.
#include <hip/hip_runtime.h>

#include <string>

#include "gz_pvnet.h"
#include "../../include/gzero.h"

using namespace gzpv;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 512;
constexpr int LDS_ACT = CH * POS;  // 28800
constexpr int LDS_PLANES = 3 * POS;
constexpr int LDS_HP = 2 * POS;
constexpr int LDS_HV = POS;
constexpr int LDS_HH = 64;
constexpr int LDS_RED = 32;
constexpr int LDS_LG = 256;
constexpr int LDS_FLOATS = LDS_ACT + LDS_PLANES + LDS_HP + LDS_HV + LDS_HH + LDS_RED + LDS_LG;

__device__ inline f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; i++) z[i] = 0.f;
    return z;
}

__device__ inline int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// 3x3 conv 128->128 over act (LDS), accumulating the wave's 4 tiles
__device__ __forceinline__ void conv128(const float* act, const float* __restrict__ Wk, int nt, int mt0, int lane,
                                        f32x16 acc[4]) {
    const int li = lane & 31, h = lane >> 5;
    int pr[4], pc[4];
    bool pin[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        int pos = (mt0 + m) * 32 + li;
        pin[m] = pos < POS;
        pr[m] = pos / 15;
        pc[m] = pos % 15;
    }
    for (int tap = 0; tap < 9; tap++) {
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        int nb[4];
        bool ok[4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            int rr = pr[m] + dr, cc = pc[m] + dc;
            ok[m] = pin[m] && rr >= 0 && rr < 15 && cc >= 0 && cc < 15;
            nb[m] = ok[m] ? rr * 15 + cc : 0;
        }
        const float* wrow = Wk + (size_t)(tap * CH + h) * CH + nt * 32 + li;
        const float* arow = act + h * POS;
#pragma unroll 8
        for (int s = 0; s < CH / 2; s++) {
            const float b = __builtin_nontemporal_load(wrow + (size_t)(2 * s) * CH);
            const float* ar = arow + 2 * s * POS;
#pragma unroll
            for (int m = 0; m < 4; m++) {
                float a = ar[nb[m]];
                a = ok[m] ? a : 0.f;
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m], 0, 0, 0);
            }
        }
    }
}

__device__ __forceinline__ void store_tiles(float* act, const f32x16 acc[4], const float* __restrict__ S,
                                           const float* __restrict__ T, const f32x16* res, int nt, int mt0,
                                           int lane) {
    const int li = lane & 31, h = lane >> 5;
    const int ch = nt * 32 + li;
    const float s = S[ch], t = T[ch];
#pragma unroll
    for (int m = 0; m < 4; m++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
            int pos = (mt0 + m) * 32 + acc_row(r, h);
            if (pos < POS) {
                float y = acc[m][r] * s + t;
                if (res) y += res[m][r];
                act[ch * POS + pos] = y > 0.f ? y : 0.f;
            }
        }
    }
}

__device__ __forceinline__ void load_tiles(const float* act, f32x16 out[4], int nt, int mt0, int lane) {
    const int li = lane & 31, h = lane >> 5;
    const int ch = nt * 32 + li;
#pragma unroll
    for (int m = 0; m < 4; m++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
            int pos = (mt0 + m) * 32 + acc_row(r, h);
            out[m][r] = pos < POS ? act[ch * POS + pos] : 0.f;
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
                                                   float* __restrict__ value, float* __restrict__ probs) {
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
    const int li = lane & 31, h = lane >> 5;
    const int nt = wave & 3;
    const int mt0 = (wave >> 2) * 4;

    for (int b = blockIdx.x; b < count; b += gridDim.x) {
        // ---- input planes [black, white, empty] (gomoku_board.py:239-260, absolute colours)
        const uint32_t* bd = boards + (size_t)b * 16;
        for (int p = tid; p < POS; p += NT) {
            int bit = (p / 15) * 16 + (p % 15);
            uint32_t bl = (bd[bit >> 5] >> (bit & 31)) & 1u;
            uint32_t wh = (bd[8 + (bit >> 5)] >> (bit & 31)) & 1u;
            planes[p] = (float)bl;
            planes[POS + p] = (float)wh;
            planes[2 * POS + p] = (float)(1u - (bl | wh));
        }
        __syncthreads();

        // ---- conv0 3->128 + BN + ReLU: K = 27 (k = tap*3 + cin), padded to 28
        f32x16 acc[4];
#pragma unroll
        for (int m = 0; m < 4; m++) acc[m] = zero16();
        {
            int pr[4], pc[4];
            bool pin[4];
#pragma unroll
            for (int m = 0; m < 4; m++) {
                int pos = (mt0 + m) * 32 + li;
                pin[m] = pos < POS;
                pr[m] = pos / 15;
                pc[m] = pos % 15;
            }
            for (int s = 0; s < K0 / 2; s++) {
                const int k = 2 * s + h;
                const float bw = W[C0_W + k * CH + nt * 32 + li];
                const int tap = k / 3, cin = k % 3;
                const int dr = tap / 3 - 1, dc = tap % 3 - 1;
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    int rr = pr[m] + dr, cc = pc[m] + dc;
                    bool ok = k < 27 && pin[m] && rr >= 0 && rr < 15 && cc >= 0 && cc < 15;
                    float a = planes[ok ? cin * POS + rr * 15 + cc : 0];
                    a = ok ? a : 0.f;
                    acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw, acc[m], 0, 0, 0);
                }
            }
        }
        store_tiles(act, acc, W + C0_S, W + C0_T, nullptr, nt, mt0, lane);
        __syncthreads();

        // ---- residual tower (ResidualBlock, neural_network.py:74-91)
        for (int blk = 0; blk < 2; blk++) {
            const float* R1 = W + RES0 + (2 * blk) * RES_STRIDE;
            const float* R2 = W + RES0 + (2 * blk + 1) * RES_STRIDE;
            f32x16 xs[4];
#pragma unroll
            for (int m = 0; m < 4; m++) acc[m] = zero16();
            conv128(act, R1 + RES_W, nt, mt0, lane, acc);
            load_tiles(act, xs, nt, mt0, lane);  // block input, kept for the skip connection
            __syncthreads();
            store_tiles(act, acc, R1 + RES_S, R1 + RES_T, nullptr, nt, mt0, lane);
            __syncthreads();
#pragma unroll
            for (int m = 0; m < 4; m++) acc[m] = zero16();
            conv128(act, R2 + RES_W, nt, mt0, lane, acc);
            __syncthreads();
            store_tiles(act, acc, R2 + RES_S, R2 + RES_T, xs, nt, mt0, lane);
            __syncthreads();
        }

        // ---- heads: 1x1 convs (policy 128->2, value 128->1)
        if (tid < POS) {
            const int pos = tid;
            float p0 = W[P_B], p1 = W[P_B + 1], v = W[V_B];
            for (int c = 0; c < CH; c++) {
                float a = act[c * POS + pos];
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

extern "C" int gz_pv_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                             float* d_logits, float* d_value, float* d_probs, void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_logits || !d_value))) {
        gz_internal_set_error("gz_pv_forward: bad arguments");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
    }
    int grid = n < cus ? n : cus;
    pv_kernel<<<grid, NT, 0, (hipStream_t)stream>>>(d_weights, d_boards, n, d_count, d_logits, d_value, d_probs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("pv_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
