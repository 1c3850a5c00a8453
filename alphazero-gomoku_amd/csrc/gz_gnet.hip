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
template <int NMW>
__device__ __forceinline__ void gn_tower(ActF16x3& act, const float* __restrict__ W, int np, int m0, int lane) {
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
        if (i % 2 == 0) GN_STAMP(4);
        else GN_STAMP(6);
    }
}

__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4))) void gn_kernel(
    const float* __restrict__ W, const uint32_t* __restrict__ boards, int n, const int32_t* d_count,
    float* __restrict__ rec) {
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
    for (int b = blockIdx.x; b < count; b += gridDim.x) {
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
            gn_tower<NM - 1>(act, W, np, m0, lane);
        else
            gn_tower<NM>(act, W, np, m0, lane);

        // ---- policy head conv1x1 64->2 (one thread per position), flattened
        // channel-major into the record.  The next board's first LDS write that
        // could clobber the map (its im2col) comes after a barrier, so none here.
        int tid_h = threadIdx.x;  // re-read (not kept live across the tower)
        asm volatile("" : "+v"(tid_h));
        if (tid_h < POS) {
            float p0 = W[GP_B], p1 = W[GP_B + 1];
            for (int c0 = 0; c0 < HID; c0 += 8) {
                float a[8];
                act.get8(c0, tid_h, a);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    p0 += W[GP_W + c0 + j] * a[j];
                    p1 += W[GP_W + HID + c0 + j] * a[j];
                }
            }
            rb[tid_h] = p0;
            rb[POS + tid_h] = p1;
        }
        GN_STAMP(7);
    }
}

// ============================================================ batched heads
// policy FC 450->225 + softmax (bg_planner.py:55-56, 243-246) and OpponentDQN
// (bg_planner.py:68-78) for HB = 64 boards per workgroup as fp32-MFMA GEMMs over
// the records gn_kernel left (heads_gemm_block, gz_f16conv.h).  DQN fc0 on the one-hot
// planes = base + the (colour - empty) delta rows of the stones (gz_gnet.h): a GEMM
// with K = 450 over the record's stone inputs.  Wave w: n-tiles {w, w+4, w+8, w+12}.
constexpr int HB = 64;
constexpr int NTH_H = 256;
constexpr int LG_STRIDE = 228;   // logits rows
constexpr int H_STRIDE = 260;    // DQN hidden rows (16 B apart in bank space per row)
static_assert(REC_X == 29 * 16 && REC - REC_X == 29 * 16 && REC % 4 == 0 && REC_X % 16 == 0 && H_STRIDE % 4 == 0, "16-B A loads");

template <int KB, int NTILES>
__device__ __forceinline__ void heads_gemm(const float* __restrict__ Wp, int lane, const int (&nt)[4], int ntn,
                                           f32x4 (&acc)[4][4], const float* __restrict__ arow[4]) {
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc[m][q] = zero4();
    for (int kb = 0; kb < KB; kb++) heads_gemm_block(Wp, NTILES, kb, lane, nt, ntn, acc, arow);
}

// acc + bias (ReLU if RELU) into LDS rows dst[board][n] for the wave's n-tiles
template <bool RELU>
__device__ __forceinline__ void heads_put(const f32x4 (&acc)[4][4], const float* __restrict__ bias, int nmax,
                                          const int (&nt)[4], int ntn, int lane, float* dst, int stride) {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q >= ntn) continue;
        const int o = 16 * nt[q] + li;
        if (o >= nmax) continue;
        const float bv = bias[o];
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float y = acc[m][q][r] + bv;
                if (RELU) y = y > 0.f ? y : 0.f;
                dst[(16 * m + 4 * g + r) * stride + o] = y;
            }
    }
}

__global__ __launch_bounds__(NTH_H, 1) void gn_heads_kernel(const float* __restrict__ W, const float* __restrict__ rec,
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
    const float* arow[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
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
    f32x4 acc[4][4];
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
        const float* ax[4];
#pragma unroll
        for (int m = 0; m < 4; m++) ax[m] = arow[m] + REC_X;
        heads_gemm<(REC - REC_X) / 16, 16>(W + D0_P, lane, nt, 4, acc, ax);
        heads_put<true>(acc, W + D0_BASE, DQH, nt, 4, lane, rb, H_STRIDE);
    }
    __syncthreads();  // rb complete; ra (logits) no longer read
    const float* ah[4];
    // ---- fc1 256 -> 256 + ReLU into ra
#pragma unroll
    for (int m = 0; m < 4; m++) ah[m] = rb + (16 * m + li) * H_STRIDE;
    heads_gemm<DQH / 16, 16>(W + D1_P, lane, nt, 4, acc, ah);
    heads_put<true>(acc, W + D1_B, DQH, nt, 4, lane, ra, H_STRIDE);
    __syncthreads();
    // ---- fc2 256 -> 225: q
#pragma unroll
    for (int m = 0; m < 4; m++) ah[m] = ra + (16 * m + li) * H_STRIDE;
    heads_gemm<DQH / 16, 15>(W + D2_P, lane, nt, ntn_p, acc, ah);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q >= ntn_p) continue;
        const int o = 16 * nt[q] + li;
        if (o >= POS) continue;
        const float bv = W[D2_B + o];
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int b = b0 + 16 * m + 4 * g + r;
                if (b < count) q_out[(size_t)b * POS + o] = acc[m][q][r] + bv;
            }
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

extern "C" size_t gz_gn_workspace_bytes(int32_t n) { return (size_t)(n < 1 ? 1 : n) * REC * sizeof(float); }

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
    gn_kernel<<<grid, NT, 0, s>>>(d_weights, d_boards, n, d_count, (float*)d_workspace);
    gn_heads_kernel<<<(n + HB - 1) / HB, NTH_H, 0, s>>>(d_weights, (const float*)d_workspace, n, d_count, d_p, d_q,
                                                        d_logits);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("gn_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
