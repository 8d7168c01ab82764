// Diagnostic micro-benchmark (not product code): what a dependent global load and cold
// instruction fetch cost inside a one-workgroup kernel that follows a whole-chip kernel, the
// situation of the window pipeline's resolve/commit kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void writer(int* a, int n) {  // every CU writes part of the chase array
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        a[i] = (int)(((long long)i * 7919 + 13) % n);
}

__global__ void chase(const int* a, int steps, long long* out) {
    if (threadIdx.x != 0) return;
    long long t0 = __builtin_amdgcn_s_memrealtime();
    int p = 0;
    for (int s = 0; s < steps; ++s) p = __builtin_nontemporal_load(a + p) ^ 0;
    long long t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = t1 - t0;
    out[1] = p;
}

// a long straight-line body: 32 independent dependent-free blocks of FMA chains
template <int N>
__device__ __forceinline__ float body(float x) {
#pragma unroll
    for (int i = 0; i < N; ++i) x = __builtin_fmaf(x, 1.0000001f, (float)i * 1e-7f);
    return x;
}
__global__ void bigcode(float* o, long long* out) {
    long long t0 = __builtin_amdgcn_s_memrealtime();
    float x = o[threadIdx.x];
    x = body<2048>(x);
    long long t1 = __builtin_amdgcn_s_memrealtime();
    o[threadIdx.x] = x;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

int main() {
    const int n = 1 << 22;
    int* a; long long* out; float* o;
    CK(hipMalloc(&a, n * sizeof(int)));
    CK(hipMalloc(&out, 16 * sizeof(long long)));
    CK(hipMalloc(&o, 1024 * sizeof(float)));
    CK(hipMemset(o, 0, 1024 * sizeof(float)));
    long long h[2];
    for (int rep = 0; rep < 3; ++rep) {
        writer<<<2048, 256>>>(a, n);
        chase<<<1, 64>>>(a, 64, out);
        CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
        printf("chase after writer: %.3f us per dependent load\n", h[0] / 100.0 / 64);
        chase<<<1, 64>>>(a, 64, out);
        CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
        printf("chase again (warm): %.3f us per dependent load\n", h[0] / 100.0 / 64);
    }
    for (int rep = 0; rep < 3; ++rep) {
        writer<<<2048, 256>>>(a, n);
        bigcode<<<1, 64>>>(o, out);
        CK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
        printf("2048-fma straight line after writer: %.3f us\n", h[0] / 100.0);
        bigcode<<<1, 64>>>(o, out);
        CK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
        printf("2048-fma straight line again:        %.3f us\n", h[0] / 100.0);
    }
    return 0;
}
