// Diagnostic micro-benchmark (not product code): dependent-chain latency of f64 / f32 adds in
// shader cycles (s_memtime) and wall time (s_memrealtime, 100 MHz) -> effective clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename T>
__global__ void chain(T* o, T d, int n, long long* out) {
    T x = o[threadIdx.x];
    long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) x = x + d;
    }
    long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = c1 - c0; out[1] = r1 - r0; }
}

int main() {
    double* od; float* of; long long* out; long long h[2];
    CK(hipMalloc(&od, 1 << 20)); CK(hipMalloc(&of, 1 << 20)); CK(hipMalloc(&out, 64));
    CK(hipMemset(od, 0, 1 << 20)); CK(hipMemset(of, 0, 1 << 20));
    const int n = 8192;
    for (int rep = 0; rep < 2; ++rep) {
        for (int grid : {1, 1024}) {
            chain<double><<<grid, 64>>>(od, 0.1, n, out);
            CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
            printf("f64 add chain, %4d waves: %.2f cycles/add, %.2f ns/add, clock %.2f GHz\n", grid,
                   (double)h[0] / n, h[1] * 10.0 / n, (double)h[0] / (h[1] * 10.0));
            chain<float><<<grid, 64>>>(of, 0.1f, n, out);
            CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
            printf("f32 add chain, %4d waves: %.2f cycles/add, %.2f ns/add, clock %.2f GHz\n", grid,
                   (double)h[0] / n, h[1] * 10.0 / n, (double)h[0] / (h[1] * 10.0));
        }
    }
    return 0;
}
