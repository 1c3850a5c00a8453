// gz_sgd.hip -- the policy-value net's residual tower in TRAINING mode (SURVEY §8f
// row 1: training.py:277-311, the forward/backward of neural_network.py:74-91 and
// 132-145 with BatchNorm on batch statistics), forward and backward on the device.
//
// The tower: a0 = relu(BN0(y0)), then two residual blocks
//     h = relu(BN1(conv1(a) + b1)),  a' = relu(BN2(conv2(h) + b2) + a)
// y0 = conv0(x) (3 -> 128 channels) and the heads stay in torch (gzero/sgd.py).
// Activations are fp32 NHWC [board][225][128].
//
// Convolutions (4 forward + 4 input-gradient): one workgroup per (board, half of
// the output channels), 8 waves; the input plane is staged into LDS as f16 hi/lo
// (gz_f16conv.h layout) with the producing BatchNorm / ReLU / skip applied on the
// fly, and gz_f16conv.h's f16x3 implicit GEMM (v_mfma_f32_16x16x32_f16, three
// products per element, fp32 accumulate) runs the 9 taps x 128 channels.  The
// input-gradient conv is the same GEMM with the weights transposed and the taps
// flipped; its operand (the BN input gradient) is scaled by a power of two chosen
// from a per-channel bound so that its hi/lo halves stay in fp16's normal range.
// Epilogues write the conv output and each board's per-channel BatchNorm partials
// (mean, centred sum of squares, max |y|; or sum g, sum g*xhat, max |g|), which a
// 128-thread kernel combines (Chan's formula, fp64) into the batch statistics,
// the running-stat update and the backward coefficients.
// Weight gradients: the same f16x3 MFMA with K = positions, one workgroup per
// (quarter of the 128 x 128 channel pairs, group of boards), all 9 taps; the saved
// NHWC activations and input gradients are staged into LDS as [position][channel]
// rows and read transposed (ds_read_b64_tr_b16); the groups' partial sums are added
// by a second kernel.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/gzero.h"
#include "gz_f16conv.h"

extern "C" void gz_internal_set_error(const char* msg);

namespace {
using namespace gzc;

constexpr int CH = 128;
constexpr int NPOS = 225;
constexpr int LAYERS = 4;   // the residual convs
constexpr int NBN = 5;      // BN0 + 4
constexpr int FRAG_HALVES = 36 * 8 * 64 * 8;  // one hi or lo plane of a conv's fragments
constexpr int CONV_THREADS = 512;

// per-BN coefficient block (floats)
constexpr int CO_S = 0, CO_T = 128, CO_MEAN = 256, CO_INV = 384, CO_K = 512, CO_MG = 640, CO_MGX = 768,
              CO_YMAX = 896, CO_SUMXH = 1024, CO_FLOATS = 1152;
// f16x3 operands are scaled by powers of two so that their largest value is just below
// 2^14: the lo halves of small values then stay out of fp16's subnormal range, where
// they would lose bits (a float64 emulation of this step put the gradient error at
// ~1e-3 without the scaling, ~1e-7 with it).  Scale = 2^(14 - e) for max < 2^e; the
// max is exact: per board for the convolutions (whose sums stay within a board), per
// group of boards for the weight gradient, per conv for the weights.
__device__ __forceinline__ int f16_scale_exp(float m) {
    int ex = 0;
    if (m > 0.f && isfinite(m)) frexpf(m, &ex);
    const int e = 14 - ex;
    return e < -100 ? -100 : (e > 100 ? 100 : e);
}
constexpr int PART = 3 * CH;  // per board partials

__host__ __device__ constexpr size_t align256(size_t x) { return (x + 255) / 256 * 256; }

// f16x3 A fragments of the four residual convs: [layer][mode][hi, lo][ks 36][n-tile 8][lane 64][8];
// element (ks, nt, lane, j): output channel n = 16 nt + lane % 16, k = 32 ks + 8 (lane / 16) + j,
// tap = k / 128, input channel c = k % 128.  mode 0 (forward): w[n][c][tap]; mode 1 (input
// gradient: conv with taps flipped, channels swapped): w[c][n][8 - tap].
struct PackArgs {
    const float* w[LAYERS];
};
// max |w| of each conv (float bits of non-negative values order as unsigned integers)
__global__ __launch_bounds__(256) void sgd_wmax_kernel(PackArgs a, unsigned* __restrict__ wmax) {
    const float* W = a.w[blockIdx.y];
    float m = 0.f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < CH * CH * 9; i += gridDim.x * 256) m = fmaxf(m, fabsf(W[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomicMax(wmax + blockIdx.y, __float_as_uint(m));
}
// wsc: [0, 4) max |w| bits (sgd_wmax_kernel), [4, 8) 1 / the weight scale of each conv
__global__ void sgd_pack_kernel(PackArgs a, float* __restrict__ wsc, _Float16* __restrict__ frag) {
    const int per = 2 * FRAG_HALVES;  // elements of one (layer, mode): hi plane index space only
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= LAYERS * 2 * FRAG_HALVES) return;
    const int lm = e / FRAG_HALVES, i = e - lm * FRAG_HALVES;
    const int layer = lm >> 1, mode = lm & 1;
    const int j = i & 7, lane = (i >> 3) & 63, nt = (i >> 9) & 7, ks = i >> 12;
    const int n = 16 * nt + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + j, tap = k >> 7, c = k & 127;
    const float* W = a.w[layer];
    const int se = f16_scale_exp(__uint_as_float(((const unsigned*)wsc)[layer]));
    if (i == 0 && mode == 0) wsc[4 + layer] = ldexpf(1.f, -se);
    const float v = ldexpf(mode == 0 ? W[(n * CH + c) * 9 + tap] : W[(c * CH + n) * 9 + (8 - tap)], se);
    const _Float16 h = (_Float16)v;
    _Float16* f = frag + (size_t)lm * per;
    f[i] = h;
    f[FRAG_HALVES + i] = (_Float16)(v - (float)h);
}

// ---------------------------------------------------------------- BN statistics
// Per-board kernels: 256 threads = 32 channel quads (float4) x 8 position strides; the
// board's 225 x 128 values are read once into registers (29 float4 per thread), then
// reduced over the 8 strides in LDS.
constexpr int PB_THREADS = 256, PB_STRIDES = PB_THREADS / 32, PB_ITEMS = (NPOS + PB_STRIDES - 1) / PB_STRIDES;
__device__ __forceinline__ f32x4 pb_reduce(f32x4 v, f32x4* sh, int q, int h, bool mx) {
    __syncthreads();
    sh[h * 32 + q] = v;
    __syncthreads();
    f32x4 t = sh[q];
#pragma unroll
    for (int k = 1; k < PB_STRIDES; k++) {
        const f32x4 u = sh[k * 32 + q];
#pragma unroll
        for (int r = 0; r < 4; r++) t[r] = mx ? fmaxf(t[r], u[r]) : t[r] + u[r];
    }
    return t;
}

// conv0 (3 -> 128 channels, 3x3, fp32 FMA) of a board's planes [3][15][15] into y0
// (NHWC), and the per-channel mean, centred sum of squares and max |y| of the board
// (the residual convs produce theirs in their epilogue).  The planes (zero-padded to
// 17 x 17) and the weights, transposed to [ci*9 + tap][co], sit in LDS.
constexpr int C0K = 27;
__device__ __forceinline__ void c0_stage(const float* __restrict__ x, int b, float* xs, int tid) {
    for (int i = tid; i < 3 * 17 * 17; i += PB_THREADS) {
        const int ci = i / 289, r = (i % 289) / 17 - 1, c = i % 17 - 1;
        xs[i] = (r >= 0 && r < 15 && c >= 0 && c < 15) ? x[((size_t)b * 3 + ci) * NPOS + r * 15 + c] : 0.f;
    }
}
__global__ __launch_bounds__(PB_THREADS) void sgd_conv0_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ w0,
                                                              const float* __restrict__ b0, float* __restrict__ y,
                                                              float* __restrict__ part) {
    __shared__ f32x4 sh[PB_THREADS];
    __shared__ float xs[3 * 17 * 17];
    __shared__ __attribute__((aligned(16))) float ws[C0K * CH];
    const int b = blockIdx.x, tid = threadIdx.x, q = tid & 31, h = tid >> 5;
    c0_stage(x, b, xs, tid);
    for (int i = tid; i < C0K * CH; i += PB_THREADS) ws[(i % C0K) * CH + i / C0K] = w0[i];  // w0[co][ci][kh][kw]
    __syncthreads();
    const f32x4 bias = *(const f32x4*)(b0 + 4 * q);
    f32x4* yb = (f32x4*)(y + (size_t)b * NPOS * CH) + q;
    // the thread's channel quad of the 27 weights in registers (read from LDS once: the
    // loop below was bound by re-reading them per position)
    f32x4 wr[C0K];
#pragma unroll
    for (int kk = 0; kk < C0K; kk++) wr[kk] = *(const f32x4*)(ws + kk * CH + 4 * q);
    f32x4 v[PB_ITEMS], s = zero4(), mx = zero4();
#pragma unroll
    for (int k = 0; k < PB_ITEMS; k++) {
        const int p = h + k * PB_STRIDES;
        v[k] = zero4();
        if (p < NPOS) {
            const int r = p / 15, c = p - (p / 15) * 15;
            f32x4 acc = bias;
#pragma unroll
            for (int kk = 0; kk < C0K; kk++) {
                const int ci = kk / 9, tap = kk % 9;
                const float xv = xs[ci * 289 + (r + tap / 3) * 17 + c + tap % 3];
                acc += xv * wr[kk];
            }
            v[k] = acc;
            yb[(size_t)p * 32] = acc;
        }
        s += v[k];
#pragma unroll
        for (int r = 0; r < 4; r++) mx[r] = fmaxf(mx[r], fabsf(v[k][r]));
    }
    const f32x4 mean = pb_reduce(s, sh, q, h, false) * (1.f / NPOS);
    f32x4 m2 = zero4();
#pragma unroll
    for (int k = 0; k < PB_ITEMS; k++)
        if (h + k * PB_STRIDES < NPOS) m2 += (v[k] - mean) * (v[k] - mean);
    m2 = pb_reduce(m2, sh, q, h, false);
    mx = pb_reduce(mx, sh, q, h, true);
    if (h == 0) {
        float* o = part + (size_t)b * PART + 4 * q;
        *(f32x4*)o = mean;
        *(f32x4*)(o + CH) = m2;
        *(f32x4*)(o + 2 * CH) = mx;
    }
}

// batch statistics from the boards' partials (equal counts: Chan's combination in
// fp64), BN scale/shift, the running-stat update (momentum, unbiased variance) --
// torch BatchNorm2d in training mode.  1024 threads: channel c = tid % 128 over the
// boards b = tid / 128 (mod 8), combined in LDS.
constexpr int RED_THREADS = 1024, RED_PARTS = RED_THREADS / CH;
__device__ __forceinline__ double red_sum(double v, double* sh, int c, int h) {
    __syncthreads();
    sh[h * CH + c] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < RED_PARTS; k++) t += sh[k * CH + c];
    return t;
}
__device__ __forceinline__ double red_max(double v, double* sh, int c, int h) {
    __syncthreads();
    sh[h * CH + c] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < RED_PARTS; k++) t = fmax(t, sh[k * CH + c]);
    return t;
}
__global__ __launch_bounds__(RED_THREADS) void sgd_bn_fwd_reduce_kernel(const float* __restrict__ part, int B,
                                                                       const float* __restrict__ gamma,
                                                                       const float* __restrict__ beta,
                                                                       float* __restrict__ run_mean,
                                                                       float* __restrict__ run_var, float momentum,
                                                                       float eps, float* __restrict__ coef) {
    __shared__ double sh[RED_THREADS];
    const int c = threadIdx.x & (CH - 1), h = threadIdx.x / CH;
    double sm = 0.0, mx = 0.0;
#pragma unroll 4
    for (int b = h; b < B; b += RED_PARTS) {
        sm += part[(size_t)b * PART + c];
        mx = fmax(mx, (double)part[(size_t)b * PART + 2 * CH + c]);
    }
    const double mean = red_sum(sm, sh, c, h) / B;
    mx = red_max(mx, sh, c, h);
    double m2 = 0.0, dev = 0.0;
#pragma unroll 4
    for (int b = h; b < B; b += RED_PARTS) {
        const double d = (double)part[(size_t)b * PART + c] - mean;
        m2 += part[(size_t)b * PART + CH + c] + (double)NPOS * d * d;
        dev += (double)NPOS * d;
    }
    m2 = red_sum(m2, sh, c, h);
    dev = red_sum(dev, sh, c, h);
    if (h) return;
    const double M = (double)NPOS * B;
    const double var = m2 / M;
    const double inv = 1.0 / sqrt(var + (double)eps);
    const float sc = (float)(gamma[c] * inv);
    coef[CO_S + c] = sc;
    coef[CO_T + c] = (float)(beta[c] - mean * (double)sc);
    coef[CO_MEAN + c] = (float)mean;
    coef[CO_INV + c] = (float)inv;
    coef[CO_YMAX + c] = (float)mx;
    coef[CO_SUMXH + c] = (float)(dev * inv);
    if (run_mean) {
        run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mean);
        run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * var * (M > 1.0 ? M / (M - 1.0) : 1.0));
    }
}

// backward of a BN + ReLU (+ skip) from the boards' partials of g = dL/d(BN output):
// mean(g), mean(g * xhat), dgamma = sum g xhat, dbeta = sum g and the conv bias gradient
// (sum of dL/dy over the rows)
__global__ __launch_bounds__(RED_THREADS) void sgd_bn_bwd_reduce_kernel(const float* __restrict__ part, int B,
                                                                       const float* __restrict__ gamma,
                                                                       float* __restrict__ coef,
                                                                       float* __restrict__ dgamma,
                                                                       float* __restrict__ dbeta,
                                                                       float* __restrict__ dbias) {
    __shared__ double sh[RED_THREADS];
    const int c = threadIdx.x & (CH - 1), h = threadIdx.x / CH;
    double sg = 0.0, sgx = 0.0;
#pragma unroll 4
    for (int b = h; b < B; b += RED_PARTS) {
        sg += part[(size_t)b * PART + c];
        sgx += part[(size_t)b * PART + CH + c];
    }
    sg = red_sum(sg, sh, c, h);
    sgx = red_sum(sgx, sh, c, h);
    if (h) return;
    const double M = (double)NPOS * B;
    const double mg = sg / M, mgx = sgx / M;
    const double inv = coef[CO_INV + c];
    const double k = (double)gamma[c] * inv;
    coef[CO_K + c] = (float)k;
    coef[CO_MG + c] = (float)mg;
    coef[CO_MGX + c] = (float)mgx;
    dgamma[c] = (float)sgx;
    dbeta[c] = (float)sg;
    // sum over rows of k (g - mg - xhat mgx) = -k mgx sum(xhat)
    if (dbias) dbias[c] = (float)(-k * mgx * (double)coef[CO_SUMXH + c]);
}

// The heads' 1x1 convs backward and the tower output's ReLU: dL/da2[p][c] =
// dpin[0][p] wp[0][c] + dpin[1][p] wp[1][c] + dvin[p] wv[c]; g4 = that [a2 > 0] and
// its BN-backward partials (sum g, sum g xhat, max |g|); the board's partial weight
// gradients of policy_conv / value_conv (sum_p dpin[k][p] a2[p][c], sum_p dvin[p] a2[p][c])
// and of their biases (sum_p dpin[k][p], sum_p dvin[p]): hpart[b][HP], HP = 3 CH + 4.
constexpr int HP = 3 * CH + 4;
__global__ __launch_bounds__(PB_THREADS) void sgd_heads_bwd_kernel(const float* __restrict__ dpin,
                                                                  const float* __restrict__ dvin,
                                                                  const float* __restrict__ act,
                                                                  const float* __restrict__ y,
                                                                  const float* __restrict__ coef,
                                                                  const float* __restrict__ wp,
                                                                  const float* __restrict__ wv,
                                                                  float* __restrict__ g, float* __restrict__ part,
                                                                  float* __restrict__ hpart) {
    __shared__ f32x4 sh[PB_THREADS];
    const int b = blockIdx.x, q = threadIdx.x & 31, h = threadIdx.x >> 5;
    const f32x4 mean = *(const f32x4*)(coef + CO_MEAN + 4 * q), inv = *(const f32x4*)(coef + CO_INV + 4 * q);
    const f32x4 w0 = *(const f32x4*)(wp + 4 * q), w1 = *(const f32x4*)(wp + CH + 4 * q), w2 = *(const f32x4*)(wv + 4 * q);
    const size_t base = (size_t)b * NPOS * 32 + q;
    const float* dp = dpin + (size_t)b * 2 * NPOS;
    const float* dv = dvin + (size_t)b * NPOS;
    f32x4 s = zero4(), sx = zero4(), mx = zero4(), h0 = zero4(), h1 = zero4(), h2 = zero4(), hb = zero4();
#pragma unroll 4
    for (int p = h; p < NPOS; p += PB_STRIDES) {
        const size_t o = base + (size_t)p * 32;
        const float d0 = dp[p], d1 = dp[NPOS + p], d2 = dv[p];
        hb[0] += d0;
        hb[1] += d1;
        hb[2] += d2;
        const f32x4 a = ((const f32x4*)act)[o], yv = ((const f32x4*)y)[o];
        const f32x4 da = d0 * w0 + d1 * w1 + d2 * w2;
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            v[r] = a[r] > 0.f ? da[r] : 0.f;
            mx[r] = fmaxf(mx[r], fabsf(v[r]));
        }
        ((f32x4*)g)[o] = v;
        s += v;
        sx += v * ((yv - mean) * inv);
        h0 += d0 * a;
        h1 += d1 * a;
        h2 += d2 * a;
    }
    s = pb_reduce(s, sh, q, h, false);
    sx = pb_reduce(sx, sh, q, h, false);
    mx = pb_reduce(mx, sh, q, h, true);
    h0 = pb_reduce(h0, sh, q, h, false);
    h1 = pb_reduce(h1, sh, q, h, false);
    h2 = pb_reduce(h2, sh, q, h, false);
    hb = pb_reduce(hb, sh, q, h, false);  // (the same in every q)
    if (h == 0) {
        float* o = part + (size_t)b * PART + 4 * q;
        *(f32x4*)o = s;
        *(f32x4*)(o + CH) = sx;
        *(f32x4*)(o + 2 * CH) = mx;
        float* oh = hpart + (size_t)b * HP + 4 * q;
        *(f32x4*)oh = h0;
        *(f32x4*)(oh + CH) = h1;
        *(f32x4*)(oh + 2 * CH) = h2;
        if (q == 0) *(f32x4*)(hpart + (size_t)b * HP + 3 * CH) = hb;
    }
}

// the heads' weight and bias gradients: the sums of the boards' partials.  Workgroup k
// takes outputs [128 k, 128 k + 128) of the HP (the last 3 = the biases), 4 threads per
// output over interleaved quarters of the boards, combined in a fixed order.
constexpr int HR_THREADS = 512;
__global__ __launch_bounds__(HR_THREADS) void sgd_heads_reduce_kernel(const float* __restrict__ hpart, int B,
                                                                     float* __restrict__ dwp, float* __restrict__ dbp,
                                                                     float* __restrict__ dwv, float* __restrict__ dbv) {
    __shared__ float sh[HR_THREADS];
    const int t = threadIdx.x, o = blockIdx.x * 128 + (t & 127), qq = t >> 7;
    float a = 0.f;
    if (o < 3 * CH + 3) {
#pragma unroll 8
        for (int b = qq; b < B; b += 4) a += hpart[(size_t)b * HP + o];
    }
    sh[t] = a;
    __syncthreads();
    if (qq || o >= 3 * CH + 3) return;
    a = (sh[t] + sh[t + 128]) + (sh[t + 256] + sh[t + 384]);
    if (o < 2 * CH) dwp[o] = a;
    else if (o < 3 * CH) dwv[o - 2 * CH] = a;
    else if (o < 3 * CH + 2) dbp[o - 3 * CH] = a;
    else dbv[0] = a;
}

// conv0's weight / bias gradient partials of a board: dy0 = k (g0 - mg - xhat mgx)
// (BN0's input gradient, never stored) times the board's planes at each tap:
// wpart0[b][co][ci*9 + tap], [27] = sum_p dy0[p][co]
__global__ __launch_bounds__(PB_THREADS) void sgd_conv0_wgrad_kernel(const float* __restrict__ g,
                                                                    const float* __restrict__ y,
                                                                    const float* __restrict__ coef,
                                                                    const float* __restrict__ x,
                                                                    float* __restrict__ wpart) {
    __shared__ f32x4 red7[7][PB_THREADS];
    __shared__ float xs[3 * 17 * 17];
    const int b = blockIdx.x, tid = threadIdx.x, q = tid & 31, h = tid >> 5;
    c0_stage(x, b, xs, tid);
    __syncthreads();
    const f32x4 mean = *(const f32x4*)(coef + CO_MEAN + 4 * q), inv = *(const f32x4*)(coef + CO_INV + 4 * q);
    const f32x4 k = *(const f32x4*)(coef + CO_K + 4 * q), mg = *(const f32x4*)(coef + CO_MG + 4 * q);
    const f32x4 mgx = *(const f32x4*)(coef + CO_MGX + 4 * q);
    const size_t base = (size_t)b * NPOS * 32 + q;
    f32x4 acc[C0K + 1];
#pragma unroll
    for (int kk = 0; kk <= C0K; kk++) acc[kk] = zero4();
    for (int p = h; p < NPOS; p += PB_STRIDES) {
        const size_t o = base + (size_t)p * 32;
        const f32x4 gv = ((const f32x4*)g)[o], yv = ((const f32x4*)y)[o];
        const f32x4 dy = k * (gv - mg - (yv - mean) * inv * mgx);
        const int r = p / 15, c = p - (p / 15) * 15;
#pragma unroll
        for (int kk = 0; kk < C0K; kk++) {
            const int ci = kk / 9, tap = kk % 9;
            acc[kk] += xs[ci * 289 + (r + tap / 3) * 17 + c + tap % 3] * dy;
        }
        acc[C0K] += dy;
    }
    // the 28 sums over the 8 position strides, 7 at a time through LDS (2 barriers per 7
    // instead of per sum), stride 0's threads adding the strides in order
    float* o = wpart + (size_t)b * CH * (C0K + 1);
    constexpr int RB = 7;
    static_assert((C0K + 1) % RB == 0, "batches");
#pragma unroll
    for (int k0 = 0; k0 <= C0K; k0 += RB) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RB; j++) red7[j][h * 32 + q] = acc[k0 + j];
        __syncthreads();
        if (h == 0)
#pragma unroll
            for (int j = 0; j < RB; j++) {
                f32x4 t = red7[j][q];
#pragma unroll
                for (int k = 1; k < PB_STRIDES; k++) t += red7[j][k * 32 + q];
#pragma unroll
                for (int r = 0; r < 4; r++) o[(4 * q + r) * (C0K + 1) + k0 + j] = t[r];
            }
    }
}

// conv0's weight ([128][3][3][3]) and bias gradients: sums of the boards' partials
__global__ void sgd_conv0_reduce_kernel(const float* __restrict__ wpart, int B, float* __restrict__ dw,
                                        float* __restrict__ db) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;  // co * 28 + kk
    if (e >= CH * (C0K + 1)) return;
    float a = 0.f;
#pragma unroll 4
    for (int b = 0; b < B; b++) a += wpart[(size_t)b * CH * (C0K + 1) + e];
    const int co = e / (C0K + 1), kk = e - co * (C0K + 1);
    if (kk < C0K) dw[co * C0K + kk] = a; else db[co] = a;
}

// the tower output a2 = relu(y4 s + t + a1) (saved) and the heads' 1x1 convs on it:
// pin[b][k*225 + p] = bp[k] + sum_c a2[p][c] wp[k][c] (policy_conv, 2 channels, in
// torch's flatten order), vin[b][p] = bv + sum_c a2[p][c] wv[c] (value_conv); one row
// (board position) per thread
__global__ __launch_bounds__(256) void sgd_out_heads_kernel(const float* __restrict__ y,
                                                           const float* __restrict__ coef,
                                                           const float* __restrict__ skip,
                                                           const float* __restrict__ wp,
                                                           const float* __restrict__ bp,
                                                           const float* __restrict__ wv,
                                                           const float* __restrict__ bv, float* __restrict__ out,
                                                           float* __restrict__ pin, float* __restrict__ vin, int rows) {
    __shared__ __attribute__((aligned(16))) float cs[5 * CH];  // s, t, wp0, wp1, wv
    for (int i = threadIdx.x; i < CH; i += 256) {
        cs[i] = coef[CO_S + i];
        cs[CH + i] = coef[CO_T + i];
        cs[2 * CH + i] = wp[i];
        cs[3 * CH + i] = wp[CH + i];
        cs[4 * CH + i] = wv[i];
    }
    __syncthreads();
    const int row = blockIdx.x * 256 + threadIdx.x;
    if (row >= rows) return;
    const f32x4* yr = (const f32x4*)(y + (size_t)row * CH);
    const f32x4* sr = (const f32x4*)(skip + (size_t)row * CH);
    f32x4* orow = (f32x4*)(out + (size_t)row * CH);
    f32x4 d0 = zero4(), d1 = zero4(), d2 = zero4();
#pragma unroll 8
    for (int c4 = 0; c4 < 32; c4++) {
        const f32x4 sv = *(const f32x4*)(cs + 4 * c4), tv = *(const f32x4*)(cs + CH + 4 * c4);
        f32x4 a = yr[c4] * sv + tv + sr[c4];
#pragma unroll
        for (int r = 0; r < 4; r++) a[r] = a[r] > 0.f ? a[r] : 0.f;
        orow[c4] = a;
        d0 += a * *(const f32x4*)(cs + 2 * CH + 4 * c4);
        d1 += a * *(const f32x4*)(cs + 3 * CH + 4 * c4);
        d2 += a * *(const f32x4*)(cs + 4 * CH + 4 * c4);
    }
    const int b = row / NPOS, p = row - b * NPOS;
    pin[(size_t)b * 2 * NPOS + p] = bp[0] + (d0[0] + d0[1] + d0[2] + d0[3]);
    pin[(size_t)b * 2 * NPOS + NPOS + p] = bp[1] + (d1[0] + d1[1] + d1[2] + d1[3]);
    vin[row] = bv[0] + (d2[0] + d2[1] + d2[2] + d2[3]);
}

// ---------------------------------------------------------------- f16x3 convolutions
struct ConvArgs {
    // stage: the conv's input plane, computed per element
    //   forward: x = relu(src s + t (+ skip)), saved to `save` (the activation)
    //   input gradient: x = k (src - mg - xhat mgx), xhat = (ysrc - mean) inv, saved to
    //   `save` (dL/dy for the weight gradient) and staged times the scale
    const float* src;
    const float* ysrc;
    const float* skip;
    const float* coef;
    float* save;
    const _Float16* frag;  // the conv's fragments (hi plane, lo plane after it), weights x 2^k
    const float* winv;     // 2^-k
    float* bmax;           // per board: max |staged input| (written by the workgroup saving it)
    // forward epilogue: y = acc + bias -> out, BN partials of y -> part
    const float* bias;
    // input-gradient epilogue: dx = acc / scale (+ eskip) -> g = dx [eact > 0] -> out,
    // BN-backward partials of g against the lower BN (ey, ecoef) -> part
    const float* eskip;
    const float* eact;
    const float* ey;
    const float* ecoef;
    float* out;
    float* part;
};

template <int MODE, int NM>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const f32x4 (&acc)[2][NM], int b, int np, int m0,
                                              int mq, int lane, float (*red)[4][CH], float scale_inv) {
    const int li = lane & 15, q = lane >> 4;
    const size_t board = (size_t)b * NPOS;
    float s[2][4], s2[2][4], mx[2][4];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int r = 0; r < 4; r++) s[n][r] = s2[n][r] = mx[n][r] = 0.f;
    if constexpr (MODE == 0) {
        f32x4 bias[2];
#pragma unroll
        for (int n = 0; n < 2; n++) bias[n] = *(const f32x4*)(a.bias + 16 * (2 * np + n) + 4 * q);
        f32x4 y[2][NM];
#pragma unroll
        for (int m = 0; m < NM; m++) {
            const int pos = 16 * (m0 + m) + li;
#pragma unroll
            for (int n = 0; n < 2; n++) {
                y[n][m] = acc[n][m] * scale_inv + bias[n];
                if (pos < NPOS) {
                    *(f32x4*)(a.out + (board + pos) * CH + 16 * (2 * np + n) + 4 * q) = y[n][m];
#pragma unroll
                    for (int r = 0; r < 4; r++) s[n][r] += y[n][m][r];
                }
            }
        }
        // board mean per channel: lanes li, then the 4 M quarters
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float v = s[n][r];
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                v += __shfl_xor(v, 8);
                if (li == 0) red[0][mq][16 * (2 * np + n) + 4 * q + r] = v;
            }
        __syncthreads();
        float mean[2][4];
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int c = 16 * (2 * np + n) + 4 * q + r;
                mean[n][r] = (red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c]) * (1.f / NPOS);
            }
#pragma unroll
        for (int m = 0; m < NM; m++) {
            const int pos = 16 * (m0 + m) + li;
            if (pos < NPOS)
#pragma unroll
                for (int n = 0; n < 2; n++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float d = y[n][m][r] - mean[n][r];
                        s2[n][r] += d * d;
                        mx[n][r] = fmaxf(mx[n][r], fabsf(y[n][m][r]));
                    }
        }
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float v = s2[n][r], w = mx[n][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    v += __shfl_xor(v, o);
                    w = fmaxf(w, __shfl_xor(w, o));
                }
                if (li == 0) {
                    red[1][mq][16 * (2 * np + n) + 4 * q + r] = v;
                    red[2][mq][16 * (2 * np + n) + 4 * q + r] = w;
                }
            }
        __syncthreads();
        if (mq == 0 && li == 0) {
            float* o = a.part + (size_t)b * PART;
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int c = 16 * (2 * np + n) + 4 * q + r;
                    o[c] = mean[n][r];
                    o[CH + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
                    o[2 * CH + c] = fmaxf(fmaxf(red[2][0][c], red[2][1][c]), fmaxf(red[2][2][c], red[2][3][c]));
                }
        }
    } else {
        f32x4 emean[2], einv[2];
#pragma unroll
        for (int n = 0; n < 2; n++) {
            emean[n] = *(const f32x4*)(a.ecoef + CO_MEAN + 16 * (2 * np + n) + 4 * q);
            einv[n] = *(const f32x4*)(a.ecoef + CO_INV + 16 * (2 * np + n) + 4 * q);
        }
#pragma unroll
        for (int m = 0; m < NM; m++) {
            const int pos = 16 * (m0 + m) + li;
            if (pos >= NPOS) continue;
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const size_t o = (board + pos) * CH + 16 * (2 * np + n) + 4 * q;
                f32x4 dx = acc[n][m] * scale_inv;
                if (a.eskip) dx += *(const f32x4*)(a.eskip + o);
                const f32x4 act = *(const f32x4*)(a.eact + o), yv = *(const f32x4*)(a.ey + o);
                f32x4 gv;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    gv[r] = act[r] > 0.f ? dx[r] : 0.f;
                    s[n][r] += gv[r];
                    s2[n][r] += gv[r] * ((yv[r] - emean[n][r]) * einv[n][r]);
                    mx[n][r] = fmaxf(mx[n][r], fabsf(gv[r]));
                }
                *(f32x4*)(a.out + o) = gv;
            }
        }
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float u = s[n][r], v = s2[n][r], w = mx[n][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    u += __shfl_xor(u, o);
                    v += __shfl_xor(v, o);
                    w = fmaxf(w, __shfl_xor(w, o));
                }
                if (li == 0) {
                    const int c = 16 * (2 * np + n) + 4 * q + r;
                    red[0][mq][c] = u;
                    red[1][mq][c] = v;
                    red[2][mq][c] = w;
                }
            }
        __syncthreads();
        if (mq == 0 && li == 0) {
            float* o = a.part + (size_t)b * PART;
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int c = 16 * (2 * np + n) + 4 * q + r;
                    o[c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
                    o[CH + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
                    o[2 * CH + c] = fmaxf(fmaxf(red[2][0][c], red[2][1][c]), fmaxf(red[2][2][c], red[2][3][c]));
                }
        }
    }
}

// grid (2, boards): workgroup (h, b) computes output channels [64 h, 64 h + 64) of board b;
// wave w: n-tile pair np = 2 h + (w & 1), M quarter w >> 1 (tiles 4 mq .. 4 mq + 3; 12..14)
template <int MODE>
__global__ __launch_bounds__(CONV_THREADS, 1) void sgd_conv_kernel(ConvArgs a) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 16 * ROWS16 * 8];
    __shared__ float red[3][4][CH];
    const int b = blockIdx.y, tid = threadIdx.x;
    ActF16x3 act;
    act.hi = lds;
    act.lo = lds + 16 * ROWS16 * 8;
    const size_t board = (size_t)b * NPOS * CH;
    const bool save = a.save && blockIdx.x == 0;
    // the board's input plane: every value computed into registers first (STG per thread),
    // the board's max |x| -> the power-of-two scale, then the scaled hi / lo into LDS
    constexpr int STG = (NPOS * 32 + CONV_THREADS - 1) / CONV_THREADS;
    f32x4 xs[STG];
    float xmax = 0.f;
#pragma unroll
    for (int k = 0; k < STG; k++) {
        const int e = tid + k * CONV_THREADS;
        if (e >= NPOS * 32) continue;
        const int p = e >> 5, c0 = (e & 31) * 4;
        const size_t o = board + (size_t)p * CH + c0;
        const f32x4 v = *(const f32x4*)(a.src + o);
        f32x4 x;
        if constexpr (MODE == 0) {
            const f32x4 sv = *(const f32x4*)(a.coef + CO_S + c0), tv = *(const f32x4*)(a.coef + CO_T + c0);
            x = v * sv + tv;
            if (a.skip) x += *(const f32x4*)(a.skip + o);
#pragma unroll
            for (int r = 0; r < 4; r++) x[r] = x[r] > 0.f ? x[r] : 0.f;
        } else {
            const f32x4 yv = *(const f32x4*)(a.ysrc + o);
            const f32x4 mean = *(const f32x4*)(a.coef + CO_MEAN + c0), inv = *(const f32x4*)(a.coef + CO_INV + c0);
            const f32x4 k = *(const f32x4*)(a.coef + CO_K + c0), mg = *(const f32x4*)(a.coef + CO_MG + c0);
            const f32x4 mgx = *(const f32x4*)(a.coef + CO_MGX + c0);
            x = k * (v - mg - (yv - mean) * inv * mgx);
        }
        if (save) *(f32x4*)(a.save + o) = x;
        xs[k] = x;
        xmax = fmaxf(xmax, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
    }
    xmax = wave_max(xmax);
    if ((tid & 63) == 0) red[0][0][tid >> 6] = xmax;
    __syncthreads();
    xmax = red[0][0][0];
#pragma unroll
    for (int w8 = 1; w8 < CONV_THREADS / 64; w8++) xmax = fmaxf(xmax, red[0][0][w8]);
    const int se = f16_scale_exp(xmax);
    const float scale = ldexpf(1.f, se);
    if (save && tid == 0) a.bmax[b] = xmax;  // the weight gradient's group scale
#pragma unroll
    for (int k = 0; k < STG; k++) {
        const int e = tid + k * CONV_THREADS;
        if (e >= NPOS * 32) continue;
        const int p = e >> 5, c0 = (e & 31) * 4;
        const f32x4 x = xs[k] * scale;
        h4 hi, lo;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const _Float16 hh = (_Float16)x[r];
            hi[r] = hh;
            lo[r] = (_Float16)(x[r] - (float)hh);
        }
        const int lo_off = ActF16x3::off(c0, p);
        *(h4*)(act.hi + lo_off) = hi;
        *(h4*)(act.lo + lo_off) = lo;
    }
    act.zero_slots(tid, CONV_THREADS, CH);
    __syncthreads();  // (also: every wave has read red[0][0] before the epilogue reuses it)
    const int wave = tid >> 6, lane = tid & 63, mq = wave >> 1;
    const int np = 2 * blockIdx.x + (wave & 1);
    const float sinv = ldexpf(1.f, -se) * *a.winv;
    // quarter 3 has tiles 12..14; its fourth tile (positions 240..255) stays zero and
    // is skipped by the epilogue (every wave runs the same epilogue and barriers)
    f32x4 acc[2][4];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int m = 0; m < 4; m++) acc[n][m] = zero4();
    if (mq < 3) {
        f16_conv<4, 4, 8, 9>(act, a.frag, np, 4 * mq, lane, acc);
    } else {
        f32x4 a3[2][3];
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int m = 0; m < 3; m++) a3[n][m] = zero4();
        f16_conv<3, 4, 8, 9>(act, a.frag, np, 12, lane, a3);
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int m = 0; m < 3; m++) acc[n][m] = a3[n][m];
    }
    conv_epilogue<MODE, 4>(a, acc, b, np, 4 * mq, mq, lane, red, sinv);
}

// ---------------------------------------------------------------- weight gradient
// dW[tap][c][n] = sum over boards and positions p of x[p + off(tap)][c] * dy[p][n]
// (x = the conv's input activation, dy = dL/d(conv output)): M = input channel c,
// N = output channel n, K = positions.  Partial sums per group of boards -> wpart
// [tap][group][c][n] (times S), added by sgd_wreduce_kernel.
constexpr int WG_THREADS = 256;
// f16x3 MFMA (v_mfma_f32_16x16x32_f16, K = 32 positions per MFMA): workgroup (c half, n half, group of boards), 4 waves; wave w takes input
// channels [16 w, 16 w + 16) of the half and all 64 output channels of its n half,
// all 9 taps (9 x 4 accumulator tiles).  A board's x (the conv input, 64 channels)
// and dy (64 output channels, times the BN-backward scale S) are staged as f16 hi/lo
// in LDS as [position][channel] rows of 128 B (225 positions + a zero row); the
// MFMA operands, 8 consecutive positions of one channel per lane, come from
// ds_read_b64_tr_b16 (4 positions x 16 channels per 16-lane group, delivered
// transposed).  A row's four 32-B channel tiles are stored XOR-swizzled by
// s(row) = bit 1 | bit 3 << 1 of the row so that the 8 rows of a half-wave's read
// (p0 + {0..3, 8..11}) hit 8 different 32-B bank slots.  Taps shift the A rows:
// x at position p + off(tap), the zero row off the board and past position 224.
constexpr int W16_ROWS = NPOS + 1;            // + the zero row
constexpr int W16_PLANE = W16_ROWS * 128;     // bytes per hi / lo plane (64 channels)
__device__ __forceinline__ int w16_off(int row, int ch) {  // byte offset of channel ch (0..63) of a row
    const int s = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    return row * 128 + 32 * ((ch >> 4) ^ s) + 2 * (ch & 15);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ h4 w16_tr(const char* lds, int byte) {
    return __builtin_bit_cast(h4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                      (__attribute__((address_space(3))) s16x4*)(lds + byte)));
}
__device__ __forceinline__ h8 w16_cat(h4 a, h4 b) {
    h8 r;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        r[j] = a[j];
        r[4 + j] = b[j];
    }
    return r;
}
__global__ __launch_bounds__(WG_THREADS, 1) void sgd_wgrad16_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ dy,
                                                                   const float* __restrict__ xmax,
                                                                   const float* __restrict__ dymax, int B, int G,
                                                                   int NG, float* __restrict__ wpart) {
    __shared__ __attribute__((aligned(16))) char lds[4 * W16_PLANE];  // x hi, x lo, dy hi, dy lo
    const int cq = blockIdx.x & 1, nq = (blockIdx.x >> 1) & 1, grp = blockIdx.x >> 2;
    const int b0 = grp * G, b1 = b0 + G < B ? b0 + G : B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, q = (lane >> 2) & 3, pc = lane & 3;
    // the group's scales from its boards' max |x|, max |dy| (the convolutions' staging)
    float mx = 0.f, md = 0.f;
    for (int b = b0; b < b1; b++) {
        mx = fmaxf(mx, xmax[b]);
        md = fmaxf(md, dymax[b]);
    }
    const int ex = f16_scale_exp(mx), ed = f16_scale_exp(md);
    const float S = ldexpf(1.f, ed), SX = ldexpf(1.f, ex), unscale = ldexpf(1.f, -ed - ex);
    f32x4 acc[9][4];
#pragma unroll
    for (int t = 0; t < 9; t++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[t][j] = zero4();
    // zero rows (both tensors, both planes), never overwritten by the staging
    if (tid < 4 * 16) *(uint64_t*)(lds + (tid >> 4) * W16_PLANE + NPOS * 128 + 8 * (tid & 15)) = 0ull;
    for (int b = b0; b < b1; b++) {
        __syncthreads();  // the previous board's reads are done
#pragma unroll 4
        for (int e = tid; e < 2 * NPOS * 16; e += WG_THREADS) {
            const int t = e >= NPOS * 16, r = e - t * NPOS * 16, p = r >> 4, c4 = (r & 15) * 4;
            const float* src = t ? dy + ((size_t)b * NPOS + p) * CH + 64 * nq + c4
                                 : x + ((size_t)b * NPOS + p) * CH + 64 * cq + c4;
            f32x4 v = *(const f32x4*)src;
            v = v * (t ? S : SX);
            h4 hi, lo;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const _Float16 h = (_Float16)v[k];
                hi[k] = h;
                lo[k] = (_Float16)(v[k] - (float)h);
            }
            char* base = lds + 2 * t * W16_PLANE + w16_off(p, c4);
            *(h4*)base = hi;
            *(h4*)(base + W16_PLANE) = lo;
        }
        __syncthreads();
        const char* xh = lds;
        const char* dh = lds + 2 * W16_PLANE;
        for (int s = 0; s < 8; s++) {
            // the lane's two rows: positions p_a (elements 0..3) and p_a + 4 (4..7)
            const int pa = 32 * s + 8 * g + q, pb = pa + 4;
            h8 bh[4], bl[4];
            {
                const int ra = pa < NPOS ? pa : NPOS, rb = pb < NPOS ? pb : NPOS;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int ch = 16 * j + 4 * pc;
                    const h4 a0 = w16_tr(dh, w16_off(ra, ch)), a1 = w16_tr(dh, w16_off(rb, ch));
                    const h4 c0 = w16_tr(dh + W16_PLANE, w16_off(ra, ch)), c1 = w16_tr(dh + W16_PLANE, w16_off(rb, ch));
                    bh[j] = w16_cat(a0, a1);
                    bl[j] = w16_cat(c0, c1);
                }
            }
            const int ya = pa / 15, xa = pa - 15 * ya, yb = pb / 15, xb = pb - 15 * yb;
#pragma unroll
            for (int tap = 0; tap < 9; tap++) {
                const int dr = tap / 3 - 1, dc = tap % 3 - 1;
                const int r1 = ya + dr, c1 = xa + dc, r2 = yb + dr, c2 = xb + dc;
                const int ra = pa < NPOS && (unsigned)r1 < 15u && (unsigned)c1 < 15u ? r1 * 15 + c1 : NPOS;
                const int rb = pb < NPOS && (unsigned)r2 < 15u && (unsigned)c2 < 15u ? r2 * 15 + c2 : NPOS;
                const int ch = 16 * wave + 4 * pc;
                const h8 ah = w16_cat(w16_tr(xh, w16_off(ra, ch)), w16_tr(xh, w16_off(rb, ch)));
                const h8 al = w16_cat(w16_tr(xh + W16_PLANE, w16_off(ra, ch)), w16_tr(xh + W16_PLANE, w16_off(rb, ch)));
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    acc[tap][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[tap][j], 0, 0, 0);
                    acc[tap][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[tap][j], 0, 0, 0);
                    acc[tap][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[tap][j], 0, 0, 0);
                }
            }
        }
    }
    // D[row = c: 4 g + r][col = n: lane % 16] of tile (tap, j), unscaled
    const int i = lane & 15;
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
        float* o = wpart + ((size_t)tap * NG + grp) * CH * CH;
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                o[(size_t)(64 * cq + 16 * wave + 4 * g + r) * CH + 64 * nq + 16 * j + i] = acc[tap][j][r] * unscale;
    }
}

// dW (torch layout [n][c][kh][kw]) = sum of the groups' partials
__global__ void sgd_wreduce_kernel(const float* __restrict__ wpart, int NG, float* __restrict__ dw) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;  // (tap, c, n), n fastest
    if (e >= 9 * CH * CH) return;
    const int tap = e / (CH * CH), rem = e - tap * CH * CH, c = rem >> 7, n = rem & 127;
    const float* p = wpart + (size_t)tap * NG * CH * CH + rem;
    float s = 0.f;
#pragma unroll 8
    for (int g = 0; g < NG; g++) s += p[(size_t)g * CH * CH];
    dw[((size_t)n * CH + c) * 9 + tap] = s;
}

// ---------------------------------------------------------------- FC heads and loss
// training.py:292-297 over neural_network.py:150-159 (PolicyValueNet's FC heads):
//   logits = policy_fc(pin),  h = relu(value_fc1(vin)),  val = tanh(value_fc2(h)),
//   loss = CrossEntropy(logits, y) + MSE(val, v)     (both means over the batch)
// and its backward down to dL/dpin, dL/dvin (the tower's backward takes it from there)
// and the six FC parameter gradients.  fp32 throughout; every sum runs over its index
// in order (deterministic).  Three launches: (1) the two forward products as tiled
// jobs (logits, value_fc1's pre-activation), (2) one workgroup per board: softmax
// cross-entropy, the value head, dlogits and dL/d(value_fc1 pre-activation), (3) the
// four backward products (dWp, dW1, dpin, dvin) as tiled jobs plus the bias / value_fc2
// gradients and the loss.
constexpr int FC_P_IN = 450, FC_P_OUT = 225, FC_V_IN = 225, FC_V_HID = 64;
// per board, in the workspace: logits / dlogits (in place), value_fc1 pre-activation /
// dpre1 (in place), h, dpre2, ce, squared error
constexpr int FC_SAVE = FC_P_OUT + 2 * FC_V_HID + 4;
constexpr int FS_H = FC_P_OUT + FC_V_HID, FS_DP2 = FS_H + FC_V_HID;

// One job: C[m][n] (+)= sum_k a(k, m) * b(k, n) (+ bias[n]), a(k, m) = A[k*sak + m*sam],
// b(k, n) = Bm[k*sbk + n*sbn], C at m*ldc + n; tiles of 16 m x 32 n (enough workgroups
// for these small products), K staged in chunks of 32 through LDS, the next chunk
// loaded into registers meanwhile; 256 threads, 2 outputs each.
struct FcJob {
    const float* A;
    const float* Bm;
    const float* bias;
    float* C;
    int sak, sam, sbk, sbn, ldc, M, N, K, tiles_n, first;  // first: this job's first workgroup
};
constexpr int FC_MAXJOBS = 4, FC_TM = 16, FC_TN = 32, FC_TK = 32;
struct FcJobs {
    FcJob j[FC_MAXJOBS];
    int n;
};
__global__ __launch_bounds__(256) void sgd_fc_gemm_kernel(FcJobs jobs) {
    __shared__ float As[FC_TK][FC_TM + 1], Bs[FC_TK][FC_TN + 1];
    int q = 0;
    while (q + 1 < jobs.n && (int)blockIdx.x >= jobs.j[q + 1].first) q++;
    const FcJob& J = jobs.j[q];
    const int tile = blockIdx.x - J.first, m0 = (tile / J.tiles_n) * FC_TM, n0 = (tile % J.tiles_n) * FC_TN;
    const int t = threadIdx.x, tm = t >> 4, tn = t & 15;
    float acc[2] = {};
    // staging: the contiguous index of each operand runs across the threads; the next
    // chunk's elements are loaded into registers while the current one is multiplied
    constexpr int NA = FC_TK * FC_TM / 256, NB = FC_TK * FC_TN / 256;
    float ra[NA], rb[NB];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int r = 0; r < NA; r++) {
            const int e = t + 256 * r;
            int kk, mm;
            if (J.sak == 1) kk = e % FC_TK, mm = e / FC_TK;
            else mm = e % FC_TM, kk = e / FC_TM;
            const int k = k0 + kk, m = m0 + mm;
            ra[r] = k < J.K && m < J.M ? J.A[(size_t)k * J.sak + (size_t)m * J.sam] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < NB; r++) {
            const int e = t + 256 * r;
            int kk, nn;
            if (J.sbk == 1) kk = e % FC_TK, nn = e / FC_TK;
            else nn = e % FC_TN, kk = e / FC_TN;
            const int k = k0 + kk, n = n0 + nn;
            rb[r] = k < J.K && n < J.N ? J.Bm[(size_t)k * J.sbk + (size_t)n * J.sbn] : 0.f;
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int r = 0; r < NA; r++) {
            const int e = t + 256 * r;
            if (J.sak == 1) As[e % FC_TK][e / FC_TK] = ra[r];
            else As[e / FC_TM][e % FC_TM] = ra[r];
        }
#pragma unroll
        for (int r = 0; r < NB; r++) {
            const int e = t + 256 * r;
            if (J.sbk == 1) Bs[e % FC_TK][e / FC_TK] = rb[r];
            else Bs[e / FC_TN][e % FC_TN] = rb[r];
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < J.K; k0 += FC_TK) {
        __syncthreads();
        put();
        __syncthreads();
        if (k0 + FC_TK < J.K) fetch(k0 + FC_TK);
        const int kn = J.K - k0 < FC_TK ? J.K - k0 : FC_TK;
#pragma unroll 8
        for (int kk = 0; kk < kn; kk++) {
            const float a0 = As[kk][tm];
            acc[0] = __builtin_fmaf(a0, Bs[kk][tn], acc[0]);
            acc[1] = __builtin_fmaf(a0, Bs[kk][tn + 16], acc[1]);
        }
    }
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int m = m0 + tm, n = n0 + tn + 16 * c;
        if (m < J.M && n < J.N) J.C[(size_t)m * J.ldc + n] = acc[c] + (J.bias ? J.bias[n] : 0.f);
    }
}

__device__ __forceinline__ float fc_wave_sum(float x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    return x;
}
// one 64-thread workgroup per board: softmax cross-entropy about the max, the value
// head, dlogits (in place of the logits) and dpre1 (in place of the pre-activation)
__global__ __launch_bounds__(64) void sgd_fc_loss_kernel(gz_sgd_fc fc, const int64_t* __restrict__ y,
                                                        const float* __restrict__ v, int B, float scale,
                                                        float* __restrict__ save) {
    const int b = blockIdx.x, lane = threadIdx.x;
    float* sb = save + (size_t)b * FC_SAVE;
    float m = -INFINITY;
    for (int i = lane; i < FC_P_OUT; i += 64) m = fmaxf(m, sb[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = fmaxf(m, __shfl_xor(m, d));
    float e = 0.f;
    for (int i = lane; i < FC_P_OUT; i += 64) e += expf(sb[i] - m);
    e = fc_wave_sum(e);
    const int64_t yt = y[b];
    // a label outside [0, 225) (torch's CrossEntropyLoss raises) poisons the loss and every
    // gradient of the step with NaN instead of training on a substituted class
    const bool bad = !(yt >= 0 && yt < FC_P_OUT);
    const int t = bad ? 0 : (int)yt;
    const float ce = m + logf(e) - sb[t], g = bad ? NAN : scale / (float)B;
    // value: h = relu(pre1), val = tanh(w2 . h + b2)
    const float pre1 = sb[FC_P_OUT + lane], h = fmaxf(pre1, 0.f);
    const float val = tanhf(fc_wave_sum(fc.value2_weight[lane] * h) + fc.value2_bias[0]), diff = val - v[b];
    const float dpre2 = 2.f * diff * g * (1.f - val * val);
    __syncthreads();  // every lane has read the logits before they are overwritten
    for (int i = lane; i < FC_P_OUT; i += 64) sb[i] = (expf(sb[i] - m) / e - (i == t ? 1.f : 0.f)) * g;
    sb[FC_P_OUT + lane] = pre1 > 0.f ? dpre2 * fc.value2_weight[lane] : 0.f;
    sb[FS_H + lane] = h;
    if (lane == 0) {
        sb[FS_DP2] = dpre2;
        sb[FS_DP2 + 1] = yt == t ? ce : NAN;
        sb[FS_DP2 + 2] = diff * diff;
    }
}
// the bias gradients, value_fc2's weight and bias gradients and the loss: one wave per
// output, lanes over the boards (fixed lane order, then a fixed shuffle tree)
__global__ __launch_bounds__(256) void sgd_fc_small_kernel(const float* __restrict__ save, int B, gz_sgd_fc_grads gr,
                                                           float* __restrict__ loss) {
    const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    float a = 0.f, c = 0.f;
    for (int b = lane; b < B; b += 64) {
        const float* sb = save + (size_t)b * FC_SAVE;
        if (e < FC_P_OUT) a += sb[e];
        else if (e < FC_P_OUT + FC_V_HID) a += sb[e];  // dpre1 (in place of the pre-activation)
        else if (e < FC_P_OUT + 2 * FC_V_HID) a = __builtin_fmaf(sb[FS_DP2], sb[FS_H + e - FC_P_OUT - FC_V_HID], a);
        else if (e == FC_P_OUT + 2 * FC_V_HID) a += sb[FS_DP2];
        else {
            a += sb[FS_DP2 + 1];
            c += sb[FS_DP2 + 2];
        }
    }
    a = fc_wave_sum(a);
    c = fc_wave_sum(c);
    if (lane) return;
    if (e < FC_P_OUT) gr.policy_bias[e] = a;
    else if (e < FC_P_OUT + FC_V_HID) gr.value1_bias[e - FC_P_OUT] = a;
    else if (e < FC_P_OUT + 2 * FC_V_HID) gr.value2_weight[e - FC_P_OUT - FC_V_HID] = a;
    else if (e == FC_P_OUT + 2 * FC_V_HID) gr.value2_bias[0] = a;
    else if (e == FC_P_OUT + 2 * FC_V_HID + 1) {  // the loss: mean cross-entropy + mean squared error
        loss[0] = a / (float)B + c / (float)B;
        loss[1] = a / (float)B;
        loss[2] = c / (float)B;
    }
}
constexpr int FC_SMALL = FC_P_OUT + 2 * FC_V_HID + 2;

// ---------------------------------------------------------------- host side
struct Ws {
    _Float16* frag;
    float* y[NBN];    // y0 (conv0's output), y1..y4
    float* act[4];    // a0, h1, a1, h2 (inputs of conv 1..4)
    float* out;       // a2, the tower output (the heads' input)
    float* g[NBN];    // dL/d(BN output) of BN 0..4
    float* dy;        // dL/dy of the current conv (weight gradient operand)
    float* coef;      // [NBN][CO_FLOATS]
    float* wsc;       // weight scales (sgd_pack_kernel)
    float* xmax;      // [4][B] max |conv input| per board (forward staging)
    float* dymax;     // [4][B] max |dL/dy| per board (input-gradient staging)
    float* fpart;     // [NBN][B][PART]
    float* bpart;     // [NBN][B][PART]
    float* wpart;     // [9][NG][CH][CH]
    float* hpart;     // [B][HP] heads' weight- and bias-gradient partials
    float* c0part;    // [B][CH][28] conv0's weight / bias gradient partials
    int NG, G;
};

size_t ws_layout(int B, Ws* w, char* base) {
    const size_t R = (size_t)B * NPOS * CH * sizeof(float);
    const int NG = B < 64 ? B : 64, G = (B + NG - 1) / NG;  // 4 NG weight-gradient workgroups
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    Ws t;
    t.frag = (_Float16*)take((size_t)LAYERS * 2 * 2 * FRAG_HALVES * sizeof(_Float16));
    for (int i = 0; i < NBN; i++) t.y[i] = (float*)take(R);
    for (int i = 0; i < 4; i++) t.act[i] = (float*)take(R);
    t.out = (float*)take(R);
    for (int i = 0; i < NBN; i++) t.g[i] = (float*)take(R);
    t.dy = (float*)take(R);
    t.coef = (float*)take((size_t)NBN * CO_FLOATS * sizeof(float));
    t.wsc = (float*)take(8 * sizeof(float));
    t.xmax = (float*)take((size_t)4 * B * sizeof(float));
    t.dymax = (float*)take((size_t)4 * B * sizeof(float));
    t.fpart = (float*)take((size_t)NBN * B * PART * sizeof(float));
    t.bpart = (float*)take((size_t)NBN * B * PART * sizeof(float));
    t.wpart = (float*)take((size_t)9 * NG * CH * CH * sizeof(float));
    t.hpart = (float*)take((size_t)B * HP * sizeof(float));
    t.c0part = (float*)take((size_t)B * CH * (C0K + 1) * sizeof(float));
    t.NG = NG;
    t.G = G;
    if (w) *w = t;
    return off;
}

int sgd_fail(int code, const std::string& msg) {
    gz_internal_set_error(msg.c_str());
    return code;
}

int sgd_check(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return sgd_fail(GZ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return GZ_OK;
}

int check_net(const gz_sgd_net* net, int B, const void* ws) {
    if (!net || B < 1 || B > GZ_SGD_MAX_BOARDS || !ws) return sgd_fail(GZ_ERR_ARG, "gz_sgd: bad arguments");
    for (int i = 0; i < NBN; i++)
        if (!net->bn_weight[i] || !net->bn_bias[i]) return sgd_fail(GZ_ERR_ARG, "gz_sgd: BatchNorm parameters are NULL");
    for (int i = 0; i < LAYERS; i++)
        if (!net->conv_weight[i] || !net->conv_bias[i]) return sgd_fail(GZ_ERR_ARG, "gz_sgd: conv parameters are NULL");
    if (!net->conv0_weight || !net->conv0_bias || !net->policy_weight || !net->policy_bias || !net->value_weight ||
        !net->value_bias)
        return sgd_fail(GZ_ERR_ARG, "gz_sgd: conv0 / head conv parameters are NULL");
    if (!(net->eps > 0.f) || !(net->momentum >= 0.f && net->momentum <= 1.f))
        return sgd_fail(GZ_ERR_ARG, "gz_sgd: eps must be > 0 and momentum in [0, 1]");
    return GZ_OK;
}

}  // namespace

// a copy of what gz_sgd_forward saved (checkers): which 0..3 = the inputs of conv 1..4
// (a0, h1, a1, h2), 4..7 = the conv outputs y1..y4, 8 = the tower output a2, 9 = y0
// (conv0's output); fp32 NHWC [boards][225][128]
extern "C" int gz_sgd_saved(const void* d_ws, int32_t B, int32_t which, float* d_out, void* stream) {
    if (!d_ws || !d_out || B < 1 || B > GZ_SGD_MAX_BOARDS || which < 0 || which > 9)
        return sgd_fail(GZ_ERR_ARG, "gz_sgd_saved: bad arguments");
    Ws w;
    ws_layout(B, &w, (char*)d_ws);
    const float* src = which < 4 ? w.act[which] : which < 8 ? w.y[which - 3] : which == 8 ? w.out : w.y[0];
    if (hipMemcpyAsync(d_out, src, (size_t)B * NPOS * CH * sizeof(float), hipMemcpyDeviceToDevice,
                       (hipStream_t)stream) != hipSuccess)
        return sgd_fail(GZ_ERR_HIP, "gz_sgd_saved: copy");
    return GZ_OK;
}

extern "C" size_t gz_sgd_workspace_bytes(int32_t boards) {
    return boards < 1 ? 0 : ws_layout(boards, nullptr, nullptr);
}

extern "C" int gz_sgd_forward(const gz_sgd_net* net, int32_t B, const float* d_x, float* d_pin, float* d_vin,
                              void* d_ws, void* stream) {
    int rc;
    if ((rc = check_net(net, B, d_ws))) return rc;
    if (!d_x || !d_pin || !d_vin) return sgd_fail(GZ_ERR_ARG, "gz_sgd_forward: x / outputs are NULL");
    hipStream_t s = (hipStream_t)stream;
    Ws w;
    ws_layout(B, &w, (char*)d_ws);
    PackArgs pa;
    for (int i = 0; i < LAYERS; i++) pa.w[i] = net->conv_weight[i];
    if (hipMemsetAsync(w.wsc, 0, 8 * sizeof(float), s) != hipSuccess)
        return sgd_fail(GZ_ERR_HIP, "gz_sgd_forward: memset");
    sgd_wmax_kernel<<<dim3(32, LAYERS), 256, 0, s>>>(pa, (unsigned*)w.wsc);
    sgd_pack_kernel<<<(LAYERS * 2 * FRAG_HALVES + 255) / 256, 256, 0, s>>>(pa, w.wsc, w.frag);
    // y0 = conv0(x) and its BN0 partials
    sgd_conv0_kernel<<<B, PB_THREADS, 0, s>>>(d_x, net->conv0_weight, net->conv0_bias, w.y[0], w.fpart);
    sgd_bn_fwd_reduce_kernel<<<1, RED_THREADS, 0, s>>>(w.fpart, B, net->bn_weight[0], net->bn_bias[0],
                                                      net->bn_running_mean[0], net->bn_running_var[0], net->momentum,
                                                      net->eps, w.coef);
    if ((rc = sgd_check("gz_sgd_forward: conv0"))) return rc;
    // conv L (1..4): input = relu(BN_{L-1}(y_{L-1}) (+ skip)), skip a0 for conv 3's input a1
    for (int L = 1; L <= LAYERS; L++) {
        ConvArgs a{};
        a.src = w.y[L - 1];
        a.coef = w.coef + (size_t)(L - 1) * CO_FLOATS;
        a.skip = L == 3 ? w.act[0] : nullptr;
        a.save = w.act[L - 1];
        a.frag = w.frag + (size_t)((L - 1) * 2 + 0) * 2 * FRAG_HALVES;
        a.winv = w.wsc + 4 + (L - 1);
        a.bmax = w.xmax + (size_t)(L - 1) * B;
        a.bias = net->conv_bias[L - 1];
        a.out = w.y[L];
        a.part = w.fpart + (size_t)L * B * PART;
        sgd_conv_kernel<0><<<dim3(2, B), CONV_THREADS, 0, s>>>(a);
        sgd_bn_fwd_reduce_kernel<<<1, RED_THREADS, 0, s>>>(a.part, B, net->bn_weight[L], net->bn_bias[L],
                                                          net->bn_running_mean[L], net->bn_running_var[L],
                                                          net->momentum, net->eps, w.coef + (size_t)L * CO_FLOATS);
        if ((rc = sgd_check("gz_sgd_forward: conv"))) return rc;
    }
    // a2 = relu(BN4(y4) + a1), then the heads' 1x1 convs
    const int rows = B * NPOS;
    sgd_out_heads_kernel<<<(rows + 255) / 256, 256, 0, s>>>(w.y[4], w.coef + 4 * CO_FLOATS, w.act[2],
                                                            net->policy_weight, net->policy_bias, net->value_weight,
                                                            net->value_bias, w.out, d_pin, d_vin, rows);
    return sgd_check("gz_sgd_forward: output");
}

extern "C" int gz_sgd_backward(const gz_sgd_net* net, int32_t B, const float* d_x, const float* d_dpin,
                               const float* d_dvin, const gz_sgd_grads* gr, void* d_ws, void* stream) {
    int rc;
    if ((rc = check_net(net, B, d_ws))) return rc;
    if (!d_x || !d_dpin || !d_dvin || !gr) return sgd_fail(GZ_ERR_ARG, "gz_sgd_backward: NULL argument");
    for (int i = 0; i < NBN; i++)
        if (!gr->bn_weight[i] || !gr->bn_bias[i]) return sgd_fail(GZ_ERR_ARG, "gz_sgd_backward: NULL gradient");
    for (int i = 0; i < LAYERS; i++)
        if (!gr->conv_weight[i] || !gr->conv_bias[i]) return sgd_fail(GZ_ERR_ARG, "gz_sgd_backward: NULL gradient");
    if (!gr->conv0_weight || !gr->conv0_bias || !gr->policy_weight || !gr->policy_bias || !gr->value_weight ||
        !gr->value_bias)
        return sgd_fail(GZ_ERR_ARG, "gz_sgd_backward: NULL gradient");
    hipStream_t s = (hipStream_t)stream;
    Ws w;
    ws_layout(B, &w, (char*)d_ws);
    // the heads' 1x1 convs backward -> g4 = dL/d(BN4 output) (also the skip gradient into a1)
    sgd_heads_bwd_kernel<<<B, PB_THREADS, 0, s>>>(d_dpin, d_dvin, w.out, w.y[4], w.coef + 4 * CO_FLOATS,
                                                  net->policy_weight, net->value_weight, w.g[4],
                                                  w.bpart + (size_t)4 * B * PART, w.hpart);
    sgd_heads_reduce_kernel<<<(HP + 127) / 128, HR_THREADS, 0, s>>>(w.hpart, B, gr->policy_weight, gr->policy_bias,
                                                                    gr->value_weight, gr->value_bias);
    for (int L = LAYERS; L >= 1; L--) {
        float* coefL = w.coef + (size_t)L * CO_FLOATS;
        sgd_bn_bwd_reduce_kernel<<<1, RED_THREADS, 0, s>>>(w.bpart + (size_t)L * B * PART, B, net->bn_weight[L],
                                                          coefL, gr->bn_weight[L], gr->bn_bias[L], gr->conv_bias[L - 1]);
        // input gradient of conv L: dy_L = k (g_L - mg - xhat mgx) staged (and saved for the
        // weight gradient); its output is dL/d(input of conv L) -> masked by that
        // activation's ReLU (+ the skip gradient: g4 into a1, g2 into a0)
        ConvArgs a{};
        a.src = w.g[L];
        a.ysrc = w.y[L];
        a.coef = coefL;
        a.save = w.dy;
        a.frag = w.frag + (size_t)((L - 1) * 2 + 1) * 2 * FRAG_HALVES;
        a.winv = w.wsc + 4 + (L - 1);
        a.bmax = w.dymax + (size_t)(L - 1) * B;
        a.eskip = L == 3 ? w.g[4] : (L == 1 ? w.g[2] : nullptr);
        a.eact = w.act[L - 1];
        a.ey = w.y[L - 1];
        a.ecoef = w.coef + (size_t)(L - 1) * CO_FLOATS;
        a.out = w.g[L - 1];
        a.part = w.bpart + (size_t)(L - 1) * B * PART;
        sgd_conv_kernel<1><<<dim3(2, B), CONV_THREADS, 0, s>>>(a);
        sgd_wgrad16_kernel<<<4 * w.NG, WG_THREADS, 0, s>>>(w.act[L - 1], w.dy, w.xmax + (size_t)(L - 1) * B,
                                                           w.dymax + (size_t)(L - 1) * B, B, w.G, w.NG, w.wpart);
        sgd_wreduce_kernel<<<(9 * CH * CH + 255) / 256, 256, 0, s>>>(w.wpart, w.NG, gr->conv_weight[L - 1]);
        if ((rc = sgd_check("gz_sgd_backward: conv"))) return rc;
    }
    // BN0, then conv0's weight and bias gradients (its input gradient is not needed)
    sgd_bn_bwd_reduce_kernel<<<1, RED_THREADS, 0, s>>>(w.bpart, B, net->bn_weight[0], w.coef, gr->bn_weight[0],
                                                      gr->bn_bias[0], nullptr);
    sgd_conv0_wgrad_kernel<<<B, PB_THREADS, 0, s>>>(w.g[0], w.y[0], w.coef, d_x, w.c0part);
    sgd_conv0_reduce_kernel<<<(CH * (C0K + 1) + 255) / 256, 256, 0, s>>>(w.c0part, B, gr->conv0_weight,
                                                                         gr->conv0_bias);
    return sgd_check("gz_sgd_backward: conv0");
}

extern "C" size_t gz_sgd_fc_workspace_bytes(int32_t boards) {
    return boards < 1 ? 0 : (size_t)boards * FC_SAVE * sizeof(float);
}

extern "C" int gz_sgd_fc_loss(const gz_sgd_fc* fc, int32_t B, const float* d_pin, const float* d_vin,
                              const int64_t* d_y, const float* d_v, float scale, float* d_dpin, float* d_dvin,
                              const gz_sgd_fc_grads* gr, float* d_loss, void* d_ws, void* stream) {
    if (!fc || !gr || B < 1 || B > GZ_SGD_MAX_BOARDS || !d_pin || !d_vin || !d_y || !d_v || !d_dpin || !d_dvin ||
        !d_loss || !d_ws)
        return sgd_fail(GZ_ERR_ARG, "gz_sgd_fc_loss: bad arguments");
    if (!fc->policy_weight || !fc->policy_bias || !fc->value1_weight || !fc->value1_bias || !fc->value2_weight ||
        !fc->value2_bias || !gr->policy_weight || !gr->policy_bias || !gr->value1_weight || !gr->value1_bias ||
        !gr->value2_weight || !gr->value2_bias)
        return sgd_fail(GZ_ERR_ARG, "gz_sgd_fc_loss: NULL parameter or gradient");
    hipStream_t s = (hipStream_t)stream;
    float* save = (float*)d_ws;
    auto job = [](const float* A, int sak, int sam, const float* Bm, int sbk, int sbn, const float* bias, float* C,
                  int ldc, int M, int N, int K) {
        FcJob j{A, Bm, bias, C, sak, sam, sbk, sbn, ldc, M, N, K, (N + FC_TN - 1) / FC_TN, 0};
        return j;
    };
    auto launch = [&](FcJobs& js) {
        int wg = 0;
        for (int q = 0; q < js.n; q++) {
            js.j[q].first = wg;
            wg += ((js.j[q].M + FC_TM - 1) / FC_TM) * js.j[q].tiles_n;
        }
        sgd_fc_gemm_kernel<<<wg, 256, 0, s>>>(js);
    };
    // (1) logits[b][i] = sum_k pin[b][k] Wp[i][k] + bp[i];  pre1[b][j] = sum_k vin[b][k] W1[j][k] + b1[j]
    FcJobs f{};
    f.j[0] = job(d_pin, 1, FC_P_IN, fc->policy_weight, 1, FC_P_IN, fc->policy_bias, save, FC_SAVE, B, FC_P_OUT,
                 FC_P_IN);
    f.j[1] = job(d_vin, 1, FC_V_IN, fc->value1_weight, 1, FC_V_IN, fc->value1_bias, save + FC_P_OUT, FC_SAVE, B,
                 FC_V_HID, FC_V_IN);
    f.n = 2;
    launch(f);
    // (2) the loss terms, dlogits, dpre1
    sgd_fc_loss_kernel<<<B, 64, 0, s>>>(*fc, d_y, d_v, B, scale, save);
    // (3) dWp[i][k] = sum_b dl[b][i] pin[b][k];  dW1[j][k] = sum_b dpre1[b][j] vin[b][k];
    //     dpin[b][k] = sum_i dl[b][i] Wp[i][k];  dvin[b][k] = sum_j dpre1[b][j] W1[j][k]
    FcJobs g{};
    g.j[0] = job(save, FC_SAVE, 1, d_pin, FC_P_IN, 1, nullptr, gr->policy_weight, FC_P_IN, FC_P_OUT, FC_P_IN, B);
    g.j[1] = job(save + FC_P_OUT, FC_SAVE, 1, d_vin, FC_V_IN, 1, nullptr, gr->value1_weight, FC_V_IN, FC_V_HID,
                 FC_V_IN, B);
    g.j[2] = job(save, 1, FC_SAVE, fc->policy_weight, FC_P_IN, 1, nullptr, d_dpin, FC_P_IN, B, FC_P_IN, FC_P_OUT);
    g.j[3] = job(save + FC_P_OUT, 1, FC_SAVE, fc->value1_weight, FC_V_IN, 1, nullptr, d_dvin, FC_V_IN, B, FC_V_IN,
                 FC_V_HID);
    g.n = 4;
    launch(g);
    sgd_fc_small_kernel<<<(FC_SMALL + 3) / 4, 256, 0, s>>>(save, B, *gr, d_loss);
    return sgd_check("gz_sgd_fc_loss");
}
