// Diagnostic micro-benchmark (not product code): cost of the first touch of a separately
// allocated buffer (TLB walk) from a one-workgroup kernel that follows a whole-chip kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr int NB = 16;
struct Bufs { int* b[NB]; };

__global__ void writer(int* a, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = i & 1;
}
// hop k loads buffer (k % nb) at an offset that depends on the previous value
__global__ void hops(Bufs B, int nb, int stride, long long* out) {
    if (threadIdx.x != 0) return;
    int v = 0;
    long long t[NB + 1];
    t[0] = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < NB; ++k) {
        v = __builtin_nontemporal_load(B.b[k % nb] + (v & 1) + k * stride);
        t[k + 1] = __builtin_amdgcn_s_memrealtime();
    }
    for (int k = 0; k < NB; ++k) out[k] = t[k + 1] - t[k];
    out[NB] = v;
}

int main() {
    const int n = 1 << 22;  // 16 MB per buffer
    Bufs B;
    for (int k = 0; k < NB; ++k) { CK(hipMalloc(&B.b[k], n * sizeof(int))); CK(hipMemset(B.b[k], 0, n * sizeof(int))); }
    int* w; long long* out; long long h[NB + 1];
    CK(hipMalloc(&w, (size_t)n * 16 * sizeof(int)));
    CK(hipMalloc(&out, (NB + 1) * sizeof(long long)));
    const char* names[3] = {"16 buffers, first touch each", "1 buffer, 16 hops 64 KB apart", "1 buffer, 16 hops 4 MB apart"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            writer<<<2048, 256>>>(w, n * 16);  // 256 MB: evicts caches and TLBs
            if (mode == 0) hops<<<1, 64>>>(B, NB, 0, out);
            else hops<<<1, 64>>>(B, 1, mode == 1 ? 16384 : (1 << 20), out);
            CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
            printf("%-34s:", names[mode]);
            for (int k = 0; k < NB; ++k) printf(" %.2f", h[k] / 100.0);
            printf(" us\n");
        }
    }
    return 0;
}
