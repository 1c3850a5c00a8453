// gz_train.hip -- training-set materialisation on the device.
//
// GomokuSelfPlayDataset (training.py:104-134) turns the replay into
//   samples [0, n)           : every record as is
//   samples n + 8j + 2k + f  : record sel[j] under rot90^k then (f) a horizontal flip
//                              (augment_sample, training.py:63-71: k = 0..3, flip F/T)
// with planes [black, white, empty] float32 [3][15][15] (the model input),
// the label move index and the value float(z).  The planes follow np.rot90
// (counter-clockwise, axes (1, 2)) and np.flip(axis=2) (training.py:44-51);
// the label follows the reference's _transform_index (training.py:53-61),
// which rotates the other way -- kept bit for bit unless GZ_AUG_FIX_LABELS.
//
// HBM-bound byte work (2,712 B written per sample): one thread per output cell
// writes its three plane values; the 80-byte record of a sample is read by the
// 225 threads that cover it (L1/L2 hits).  Measured 2.85 TB/s for the whole-set
// build (nontemporal stores; plain stores 2.3 TB/s).  Slower, kept out: a
// bounded grid-stride grid (1.9), 16-byte stores over 4-sample groups (2.2), a
// wave per sample (2.2), 4 samples per thread with all loads first (2.3).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/gzero.h"

namespace {

constexpr int N = 15;
constexpr int POS = N * N;
constexpr int SAMPLE_F = 3 * POS;  // 675 floats

// source cell (row-major) of output cell (i, j) under flip(rot90^k(x));
// y = rot90(x) reads y[i][j] = x[j][N-1-i], so rot90^k reads x at
// k=0 (i, j), k=1 (j, N-1-i), k=2 (N-1-i, N-1-j), k=3 (N-1-j, i)
__device__ __forceinline__ int aug_source(int i, int j, int k, int flip) {
    if (flip) j = N - 1 - j;
    const int a = (k == 0) ? i : (k == 1) ? j : (k == 2) ? N - 1 - i : N - 1 - j;
    const int b = (k == 0) ? j : (k == 1) ? N - 1 - i : (k == 2) ? N - 1 - j : i;
    return a * N + b;
}

// label of a move under the same symmetry (training.py:53-61, or the corrected map)
__device__ __forceinline__ int aug_label(int idx, int k, int flip, int fix) {
    int r = idx / N, c = idx % N;
    for (int t = 0; t < k; t++) {
        const int a = fix ? N - 1 - c : c, b = fix ? r : N - 1 - r;
        r = a;
        c = b;
    }
    if (flip) c = N - 1 - c;
    return r * N + c;
}

struct SampleRef {
    int rec, k, flip;
};

__device__ __forceinline__ SampleRef sample_ref(long long s, int n, const int32_t* __restrict__ sel) {
    if (s < n) return {(int)s, 0, 0};
    const long long a = s - n;
    return {sel[a >> 3], (int)((a & 7) >> 1), (int)(a & 1)};
}

// one thread per (sample, output cell): the source cell's two bits give the
// three plane values, stored at cell, 225 + cell and 450 + cell of the sample
// (consecutive lanes -> consecutive cells: coalesced 4-byte stores).  NT: the
// whole-set build streams past the caches; a batch gather stays in L2 for the
// forward that reads it next.
template <bool NT>
__global__ void dataset_planes_kernel(const gz_record* __restrict__ recs, int n, const int32_t* __restrict__ sel,
                                      const int64_t* __restrict__ ids, long long n_all, long long count,
                                      float* __restrict__ x) {
    const long long total = count * POS;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const long long so = t / POS;
        const int cell = (int)(t - so * POS);
        const long long s = ids ? ids[so] : so;
        const SampleRef r =
            (unsigned long long)s < (unsigned long long)n_all ? sample_ref(s, n, sel) : SampleRef{-1, 0, 0};
        float b = 0.f, w = 0.f, e = 0.f;
        if ((unsigned)r.rec < (unsigned)n) {  // out-of-range selections give zero planes, label -1
            const int src = aug_source(cell / N, cell % N, r.k, r.flip);
            const int bit = (src / N) * 16 + src % N;
            const gz_record* rec = recs + r.rec;
            const uint32_t bb = (rec->black[bit >> 5] >> (bit & 31)) & 1u;
            const uint32_t ww = (rec->white[bit >> 5] >> (bit & 31)) & 1u;
            b = (float)bb;
            w = (float)ww;
            e = (float)(1u - (bb | ww));
        }
        float* o = x + so * SAMPLE_F + cell;
        if (NT) {
            __builtin_nontemporal_store(b, o);
            __builtin_nontemporal_store(w, o + POS);
            __builtin_nontemporal_store(e, o + 2 * POS);
        } else {
            o[0] = b;
            o[POS] = w;
            o[2 * POS] = e;
        }
    }
}

__global__ void dataset_labels_kernel(const gz_record* __restrict__ recs, int n, const int32_t* __restrict__ sel,
                                      const int64_t* __restrict__ ids, long long n_all, long long count, int fix,
                                      int64_t* __restrict__ y, float* __restrict__ val) {
    const long long so = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (so >= count) return;
    const long long s = ids ? ids[so] : so;
    const SampleRef r = (unsigned long long)s < (unsigned long long)n_all ? sample_ref(s, n, sel) : SampleRef{-1, 0, 0};
    if ((unsigned)r.rec >= (unsigned)n) {
        y[so] = -1;
        val[so] = 0.f;
        return;
    }
    const gz_record* rec = recs + r.rec;
    y[so] = aug_label(rec->move, r.k, r.flip, fix);
    val[so] = (float)rec->z;
}

}  // namespace

extern "C" void gz_internal_set_error(const char* msg);

namespace {
int launch(const gz_record* d_records, int32_t n, const int32_t* d_sel, int32_t m, const int64_t* d_ids,
           long long count, int32_t flags, float* d_x, int64_t* d_y, float* d_v, hipStream_t st, const char* who) {
    if (n < 0 || m < 0 || count < 0 || (n > 0 && !d_records) || (m > 0 && !d_sel) ||
        (count > 0 && (!d_x || !d_y || !d_v)) || (flags & ~GZ_AUG_FIX_LABELS)) {
        gz_internal_set_error((std::string(who) + ": bad arguments").c_str());
        return GZ_ERR_ARG;
    }
    if (m > 0 && n == 0) {
        gz_internal_set_error((std::string(who) + ": augmentation of an empty replay").c_str());
        return GZ_ERR_ARG;
    }
    if (count == 0) return GZ_OK;
    const long long n_all = (long long)n + 8LL * m;
    const int bs = 256;
    long long th = count * POS;
    if (th > (1LL << 30)) th = 1LL << 30;  // one thread per cell up to 4M blocks, grid-stride beyond
    if (d_ids)
        dataset_planes_kernel<false><<<(unsigned)((th + bs - 1) / bs), bs, 0, st>>>(d_records, n, d_sel, d_ids, n_all,
                                                                                   count, d_x);
    else
        dataset_planes_kernel<true><<<(unsigned)((th + bs - 1) / bs), bs, 0, st>>>(d_records, n, d_sel, d_ids, n_all,
                                                                                  count, d_x);
    dataset_labels_kernel<<<(unsigned)((count + bs - 1) / bs), bs, 0, st>>>(
        d_records, n, d_sel, d_ids, n_all, count, (flags & GZ_AUG_FIX_LABELS) ? 1 : 0, d_y, d_v);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string(who) + ": " + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
}  // namespace

extern "C" int gz_dataset_build(const gz_record* d_records, int32_t n, const int32_t* d_sel, int32_t m, int32_t flags,
                                float* d_x, int64_t* d_y, float* d_v, void* stream) {
    return launch(d_records, n, d_sel, m, nullptr, (long long)n + 8LL * (m > 0 ? m : 0), flags, d_x, d_y, d_v,
                  (hipStream_t)stream, "gz_dataset_build");
}

extern "C" int gz_dataset_gather(const gz_record* d_records, int32_t n, const int32_t* d_sel, int32_t m,
                                 const int64_t* d_ids, int64_t count, int32_t flags, float* d_x, int64_t* d_y,
                                 float* d_v, void* stream) {
    if (count > 0 && !d_ids) {
        gz_internal_set_error("gz_dataset_gather: d_ids is required");
        return GZ_ERR_ARG;
    }
    return launch(d_records, n, d_sel, m, d_ids, count, flags, d_x, d_y, d_v, (hipStream_t)stream,
                  "gz_dataset_gather");
}

// ============================================================ optimiser step
// clip_grad_norm_ + torch.optim.Adam (training.py:303-304) over the parameter tensors:
// adam_norm_kernel sums g^2 in float64 over a fixed slice of the concatenated elements per
// workgroup; adam_update_kernel re-reduces those partials in the same order in every
// workgroup (so every workgroup has the same clip factor, no grid barrier), then applies
// the clip and the Adam update to its slice.
namespace {
constexpr int ADAM_BLOCKS = 512, ADAM_THREADS = 256;

struct AdamTable {  // by value (kernel arguments)
    gz_adam_tensor t[GZ_ADAM_MAX_TENSORS];
    int64_t start[GZ_ADAM_MAX_TENSORS + 1];  // prefix of numel
    int n;
};

__device__ __forceinline__ int adam_find(const AdamTable& T, int64_t i) {
    int k = 0;
    while (k + 1 < T.n && T.start[k + 1] <= i) k++;
    return k;
}

template <class F>
__device__ __forceinline__ void adam_slice(const AdamTable& T, F&& f) {
    const int64_t total = T.start[T.n];
    const int64_t per = (total + ADAM_BLOCKS - 1) / ADAM_BLOCKS;
    const int64_t b = per * blockIdx.x, e = b + per < total ? b + per : total;
    for (int64_t i0 = b; i0 < e; i0 += ADAM_THREADS) {
        const int64_t i = i0 + threadIdx.x;
        if (i >= e) break;
        const int k = adam_find(T, i);
        f(T.t[k], i - T.start[k]);
    }
}

__device__ __forceinline__ double adam_block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int j = 0; j < ADAM_THREADS / 64; j++) s += red[j];
    __syncthreads();
    return s;
}

__global__ __launch_bounds__(ADAM_THREADS) void adam_norm_kernel(AdamTable T, double* partial) {
    __shared__ double red[ADAM_THREADS / 64];
    double s = 0.0;
    adam_slice(T, [&](const gz_adam_tensor& t, int64_t j) {
        const double g = t.grad[j];
        s += g * g;
    });
    s = adam_block_sum(s, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(ADAM_THREADS) void adam_update_kernel(AdamTable T, const double* partial, float lr,
                                                                   float beta1, float beta2, float eps, float wd,
                                                                   float bc1, float bc2s, float max_norm,
                                                                   float* norm_out) {
    __shared__ double red[ADAM_THREADS / 64];
    float clip = 1.f;
    if (max_norm > 0.f) {
        double s = 0.0;
        for (int j = threadIdx.x; j < ADAM_BLOCKS; j += ADAM_THREADS) s += partial[j];
        s = adam_block_sum(s, red);
        const float norm = (float)sqrt(s);
        const float c = max_norm / (norm + 1e-6f);
        clip = c < 1.f ? c : 1.f;
        if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) *norm_out = norm;
    }
    const float step_size = lr / bc1;
    adam_slice(T, [&](const gz_adam_tensor& t, int64_t j) {
        float g = t.grad[j];
        if (max_norm > 0.f) {
            g *= clip;
            t.grad[j] = g;
        }
        const float p = t.param[j];
        if (wd != 0.f) g = g + wd * p;
        const float m0 = t.exp_avg[j];
        const float m = m0 + (1.f - beta1) * (g - m0);  // torch's exp_avg.lerp_(grad, 1 - beta1)
        const float v = beta2 * t.exp_avg_sq[j] + (1.f - beta2) * g * g;
        t.exp_avg[j] = m;
        t.exp_avg_sq[j] = v;
        const float denom = sqrtf(v) / bc2s + eps;
        t.param[j] = p - step_size * (m / denom);
    });
}
}  // namespace

extern "C" size_t gz_adam_workspace_bytes(void) { return ADAM_BLOCKS * sizeof(double); }

extern "C" int gz_adam_step(const gz_adam_tensor* tensors, int32_t n_tensors, float lr, float beta1, float beta2,
                            float eps, float weight_decay, int64_t step, float max_norm, float* d_norm,
                            void* d_workspace, void* stream) {
    if (!tensors || n_tensors < 1 || n_tensors > GZ_ADAM_MAX_TENSORS || step < 1 || !d_workspace) {
        gz_internal_set_error("gz_adam_step: bad arguments");
        return GZ_ERR_ARG;
    }
    AdamTable T;
    T.n = n_tensors;
    T.start[0] = 0;
    for (int k = 0; k < n_tensors; k++) {
        const gz_adam_tensor& t = tensors[k];
        if (t.numel < 0 || (t.numel > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq))) {
            gz_internal_set_error("gz_adam_step: bad tensor");
            return GZ_ERR_ARG;
        }
        T.t[k] = t;
        T.start[k + 1] = T.start[k] + t.numel;
    }
    for (int k = n_tensors; k < GZ_ADAM_MAX_TENSORS; k++) T.t[k] = gz_adam_tensor{};
    if (T.start[n_tensors] == 0) return GZ_OK;
    hipStream_t st = (hipStream_t)stream;
    double* partial = (double*)d_workspace;
    // torch's bias corrections: 1 - beta^step in float64, then used in float32
    const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
    const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
    if (max_norm > 0.f) adam_norm_kernel<<<ADAM_BLOCKS, ADAM_THREADS, 0, st>>>(T, partial);
    adam_update_kernel<<<ADAM_BLOCKS, ADAM_THREADS, 0, st>>>(T, partial, lr, beta1, beta2, eps, weight_decay, bc1,
                                                             bc2s, max_norm, d_norm);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gz_internal_set_error((std::string("gz_adam_step: ") + hipGetErrorString(e)).c_str());
        return GZ_ERR_HIP;
    }
    return GZ_OK;
}
