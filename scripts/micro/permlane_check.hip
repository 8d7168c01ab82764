// Micro-check (GPU): the gfx950 lane swaps used by the wave reductions.  For every lane l,
// {r0, r1} of v_permlane16_swap(v, v) must be {v[l], v[l ^ 16]} and of v_permlane32_swap(v, v)
// {v[l], v[l ^ 32]}; wave_incl_scan (pp_device.h, DPP) must equal the serial prefix sums.  Build: hipcc --offload-arch=gfx950 -O2 -o permlane_check permlane_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../rs-pathplanning_amd/csrc/pp_device.h"
__global__ void scan_k(const int* in, int* out) { out[threadIdx.x] = ppamd::wave_incl_scan(in[threadIdx.x]); }
__global__ void k(const int* in, int* out) {
    const int l = threadIdx.x;
    const int v = in[l];
    auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    out[4 * l] = a[0];
    out[4 * l + 1] = a[1];
    out[4 * l + 2] = b[0];
    out[4 * l + 3] = b[1];
}
int main() {
    int h[64], o[256];
    for (int i = 0; i < 64; ++i) h[i] = 1000 + i;
    int *din, *dout;
    (void)hipMalloc(&din, sizeof h);
    (void)hipMalloc(&dout, sizeof o);
    (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(din, dout);
    (void)hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    int bad16 = 0, bad32 = 0;
    for (int l = 0; l < 64; ++l) {
        const int p = h[l], q16 = h[l ^ 16], q32 = h[l ^ 32];
        const int a0 = o[4 * l], a1 = o[4 * l + 1], b0 = o[4 * l + 2], b1 = o[4 * l + 3];
        if (!((a0 == p && a1 == q16) || (a0 == q16 && a1 == p))) ++bad16;
        if (!((b0 == p && b1 == q32) || (b0 == q32 && b1 == p))) ++bad32;
        if (l < 2 || l == 16 || l == 32 || l == 63)
            printf("lane %2d: swap16 (%d, %d) swap32 (%d, %d)\n", l, a0 - 1000, a1 - 1000, b0 - 1000, b1 - 1000);
    }
    printf("permlane16_swap pairs {l, l^16}: %s; permlane32_swap pairs {l, l^32}: %s\n",
           bad16 ? "NO" : "yes", bad32 ? "NO" : "yes");
    int bads = 0;
    for (int rep = 0; rep < 100; ++rep) {
        unsigned r = 12345u + 7919u * rep;
        for (int i = 0; i < 64; ++i) { r = r * 1103515245u + 12345u; h[i] = (int)((r >> 16) % 1000) - (rep % 2 ? 0 : 300); }
        (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
        scan_k<<<1, 64>>>(din, dout);
        (void)hipMemcpy(o, dout, 64 * sizeof(int), hipMemcpyDeviceToHost);
        int acc = 0;
        for (int i = 0; i < 64; ++i) { acc += h[i]; bads += o[i] != acc; }
    }
    printf("wave_incl_scan (DPP): %d of 6400 prefix sums differ\n", bads);
    return bad16 || bad32 || bads;
}
