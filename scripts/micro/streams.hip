// Diagnostic micro-benchmark (not product code): gap between the end of a kernel and the start of
// a dependent one — same stream vs another stream through hipStreamWaitEvent.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void stamp_end(long long* t, int slot) {
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0) t[slot] = __builtin_amdgcn_s_memrealtime();
}
__global__ void stamp_start(long long* t, int slot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t[slot] = __builtin_amdgcn_s_memrealtime();
}
__global__ void busy(float* o, int n) {  // ~20 us of whole-chip work
    float x = o[threadIdx.x];
    for (int i = 0; i < n; ++i) x = __builtin_fmaf(x, 1.0000001f, 1e-7f);
    if (x == 12345.f) o[threadIdx.x] = x;
}

int main() {
    long long* t; float* o;
    CK(hipMalloc(&t, 1024 * sizeof(long long)));
    CK(hipMalloc(&o, 1024 * sizeof(float)));
    CK(hipMemset(o, 0, 1024 * sizeof(float)));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t e1, e2, et;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreate(&et));
    const int R = 20;
    long long h[1024];
    for (int mode = 0; mode < 3; ++mode) {
        for (int r = 0; r < R; ++r) {
            busy<<<1024, 256, 0, a>>>(o, 2000);
            stamp_end<<<1, 64, 0, a>>>(t, 2 * r);
            if (mode == 0) {
                stamp_start<<<1, 64, 0, a>>>(t, 2 * r + 1);
            } else {
                hipEvent_t ev = mode == 1 ? e1 : et;
                CK(hipEventRecord(ev, a));
                CK(hipStreamWaitEvent(b, ev, 0));
                stamp_start<<<1, 64, 0, b>>>(t, 2 * r + 1);
                CK(hipEventRecord(e2, b));
                CK(hipStreamWaitEvent(a, e2, 0));
            }
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, t, 2 * R * sizeof(long long), hipMemcpyDeviceToHost));
        double s = 0, mn = 1e9, mx = 0;
        for (int r = 2; r < R; ++r) {
            const double g = (h[2 * r + 1] - h[2 * r]) / 100.0;
            s += g; mn = g < mn ? g : mn; mx = g > mx ? g : mx;
        }
        const char* nm[3] = {"same stream", "cross-stream event (no timing)", "cross-stream event (timing)"};
        printf("%-32s: kernel end -> dependent kernel start avg %.2f us (min %.2f max %.2f)\n", nm[mode], s / (R - 2), mn, mx);
    }
    return 0;
}
