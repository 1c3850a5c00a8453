// HBM counter calibration (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are exact only
// for some access widths): streams a known byte count through each access width the
// PV forward uses, one kernel per pattern, so rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
// can be divided by the true bytes (profiles/summarize.py applies the factors).
//   read4 / read16: 4-B / 16-B loads per lane, coalesced, summed into a sink
//   write4 / write16: 4-B / 16-B stores per lane, coalesced
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/hbm_calib tools/hbm_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read4(const float* __restrict__ a, size_t n, float* sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.f) sink[0] = s;
}
__global__ void read16(const float4* __restrict__ a, size_t n, float* sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) sink[0] = s;
}
__global__ void write4(float* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (float)i;
}
__global__ void write16(float4* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

int main() {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB: far past the 256 MiB Infinity Cache
    float *a, *b, *sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    const int grid = 256 * 8, block = 256;
    write16<<<grid, block>>>((float4*)a, bytes / 16);  // initialise a
    write16<<<grid, block>>>((float4*)b, bytes / 16);  // evict a's lines from the caches
    read4<<<grid, block>>>(a, bytes / 4, sink);
    write16<<<grid, block>>>((float4*)b, bytes / 16);
    read16<<<grid, block>>>((const float4*)a, bytes / 16, sink);
    write4<<<grid, block>>>(b, bytes / 4);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"bytes_per_kernel\": %zu}\n", bytes);
    return 0;
}
