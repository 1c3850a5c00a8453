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
// Heads (policy conv 1x1, FC 450->225, softmax) and the DQN MLP run on VALU.
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
constexpr int SMALL_F = 3 * PROWS + 2 * POS + 256 + 2 * 256 + 32 + 2 * DQH + 2 * DQH + 256;
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

__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4))) void gn_kernel(const float* __restrict__ W, const uint32_t* __restrict__ boards,
                                                   int n, const int32_t* d_count, float* __restrict__ p_out,
                                                   float* __restrict__ q_out, float* __restrict__ logits_out) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    ActF16x3 act;
    act.hi = (_Float16*)lds;
    act.lo = act.hi + HID * ROWS16;
    float* planes = (float*)(lds + ACT_BYTES);  // [3][240]
    float* pc = planes + 3 * PROWS;             // [450] policy conv output, channel-major
    float* lg = pc + 2 * POS;                   // [256]
    float* part = lg + 256;                     // [2][256]
    float* red = part + 2 * 256;                // [32]
    float* da = red + 32;                       // [2][256] dqn partial sums / activations
    float* dc = da + 2 * DQH;                   // [2][256]
    int* slist = (int*)(dc + 2 * DQH);          // [225] stones (delta rows), row-major

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
        // ---- input planes [black, white, empty] (bg_planner.py:225-230)
        const uint32_t* bd = boards + (size_t)b * 16;
        for (int p = tid; p < POS; p += NT) {
            int bit = (p / 15) * 16 + (p % 15);
            uint32_t bl = (bd[bit >> 5] >> (bit & 31)) & 1u;
            uint32_t wh = (bd[8 + (bit >> 5)] >> (bit & 31)) & 1u;
            planes[p] = (float)bl;
            planes[PROWS + p] = (float)wh;
            planes[2 * PROWS + p] = (float)(1u - (bl | wh));
        }
        __syncthreads();
        GN_STAMP(0);

        // ---- OpponentDQN (bg_planner.py:68-78).  fc0 on the one-hot planes =
        // base + the delta rows of the stones (gz_gnet.h), stones listed in
        // row-major order (a fixed summation order: q is reproducible)
        if (wave < 4) {
            const int pos = tid;
            int code = -1;
            if (pos < POS) code = planes[pos] != 0.f ? pos : (planes[PROWS + pos] != 0.f ? POS + pos : -1);
            const uint64_t m = __ballot(code >= 0);
            if (lane == 0) red[16 + wave] = (float)__popcll(m);
            __syncthreads();
            int off = 0;
            for (int k = 0; k < wave; k++) off += (int)red[16 + k];
            if (code >= 0) slist[off + __popcll(m & ((1ull << lane) - 1ull))] = code;
            if (tid == 0) red[24] = red[16] + red[17] + red[18] + red[19];
        } else {
            __syncthreads();
        }
        __syncthreads();
        {
            const int j = tid & 255, h = tid >> 8;
            const int ns = (int)red[24];
            float acc = h == 0 ? W[D0_BASE + j] : 0.f;
            const float* dt = W + D0_DELTA + j;
            int i = h;
            for (; i + 14 < ns; i += 16) {  // 8 independent loads in flight
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = dt[(size_t)slist[i + 2 * u] * DQH];
#pragma unroll
                for (int u = 0; u < 8; u++) acc += v[u];
            }
            for (; i < ns; i += 2) acc += dt[(size_t)slist[i] * DQH];
            da[h * DQH + j] = acc;
        }
        __syncthreads();
        if (tid < DQH) {
            float a = da[tid] + da[DQH + tid];
            dc[tid] = a > 0.f ? a : 0.f;
        }
        __syncthreads();
        {  // fc1 256->256 in two input halves
            const int j = tid & 255, h = tid >> 8;
            da[h * DQH + j] = dot_col<128, 64>(W + D1_WT + (size_t)(h * 128) * DQH + j, DQH, dc + h * 128);
        }
        __syncthreads();
        if (tid < DQH) {
            float a = W[D1_B + tid] + (da[tid] + da[DQH + tid]);
            dc[DQH + tid] = a > 0.f ? a : 0.f;
        }
        __syncthreads();
        {  // fc2 256->225 in two input halves
            const int j = tid & 255, h = tid >> 8;
            if (j < POS) da[h * DQH + j] = dot_col<128, 64>(W + D2_WT + (size_t)(h * 128) * POS + j, POS, dc + DQH + h * 128);
        }
        __syncthreads();
        if (tid < POS) q_out[(size_t)b * POS + tid] = W[D2_B + tid] + (da[tid] + da[DQH + tid]);
        GN_STAMP(1);

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

        // ---- policy head: conv1x1 64->2 (one thread per position), flatten channel-major
        if (tid < POS) {
            float p0 = W[GP_B], p1 = W[GP_B + 1];
            for (int c0 = 0; c0 < HID; c0 += 8) {
                float a[8];
                act.get8(c0, tid, a);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    p0 += W[GP_W + c0 + j] * a[j];
                    p1 += W[GP_W + HID + c0 + j] * a[j];
                }
            }
            pc[tid] = p0;
            pc[POS + tid] = p1;
        }
        __syncthreads();
        GN_STAMP(7);
        {  // Linear 450->225 in two input halves
            const int o = tid & 255, h = tid >> 8;
            if (o < POS) part[h * 256 + o] = dot_col<POS, 45>(W + GF_WT + (size_t)h * POS * POS + o, POS, pc + h * POS);
        }
        __syncthreads();
        if (tid < POS) lg[tid] = W[GF_B + tid] + (part[tid] + part[256 + tid]);
        __syncthreads();
        GN_STAMP(8);
        // ---- softmax over 225 logits (waves 0..3), torch.softmax(dim=0) semantics in fp32
        if (wave < 4) {
            float x = tid < POS ? lg[tid] : -3.0e38f;
            float mx = wave_max(x);
            if (lane == 0) red[wave] = mx;
        }
        __syncthreads();
        if (wave < 4) {
            const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
            float e = tid < POS ? __expf(lg[tid] - mx) : 0.f;
            float s = wave_sum(e);
            if (lane == 0) red[8 + wave] = s;
            if (tid < POS) {
                if (logits_out) logits_out[(size_t)b * POS + tid] = lg[tid];
                lg[tid] = e;
            }
        }
        __syncthreads();
        if (wave < 4) {
            const float s = (red[8] + red[9]) + (red[10] + red[11]);
            if (tid < POS) p_out[(size_t)b * POS + tid] = lg[tid] / s;
        }
        __syncthreads();
        GN_STAMP(9);
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

extern "C" int gz_gn_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                             float* d_p, float* d_q, float* d_logits, void* stream) {
    if (n < 0 || (n > 0 && (!d_weights || !d_boards || !d_p || !d_q))) {
        gz_internal_set_error("gz_gn_forward: bad arguments");
        return GZ_ERR_ARG;
    }
    if (n == 0) return GZ_OK;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    int grid = n < 2 * cus ? n : 2 * cus;
    gn_kernel<<<grid, NT, 0, (hipStream_t)stream>>>(d_weights, d_boards, n, d_count, d_p, d_q, d_logits);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("gn_kernel: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
