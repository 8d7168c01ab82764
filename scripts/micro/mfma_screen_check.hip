// Micro-check for an MFMA form of the expanded NN screen: does
// v_mfma_f32_32x32x2_f32 give D[i][j] = fma(A[i][1], B[1][j], fma(A[i][0], B[0][j], C[i][j]))
// bit for bit (the VALU chain the screen uses), and which (row, column) does lane l, register r
// of D hold?  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off mfma_screen_check.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void probe(const float* A, const float* B, const float* C, float* D) {
    // A: 32 x 2 (row i, k), B: 2 x 32 (k, column j), C/D: per lane 16 registers
    const int l = threadIdx.x;
    const float a = A[(l % 32) * 2 + l / 32];   // A[i = l % 32][k = l / 32]
    const float b = B[(l / 32) * 32 + l % 32];  // B[k = l / 32][j = l % 32]
    floatx16 c;
    for (int r = 0; r < 16; ++r) c[r] = C[l * 16 + r];
    const floatx16 d = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = d[r];
}

static float frand(unsigned& s) {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
}

int main() {
    std::vector<float> A(64), B(64), C(1024, 0.0f), D(1024);
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, 256);
    hipMalloc(&dB, 256);
    hipMalloc(&dC, 4096);
    hipMalloc(&dD, 4096);
    auto run = [&]() {
        hipMemcpy(dA, A.data(), 256, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), 256, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
        probe<<<1, 64>>>(dA, dB, dC, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    };
    // 1. layout: A[i][0] = i + 1, B[0][j] = 1 -> D = i + 1 (row); then B[0][j] = j + 1, A = 1 (column)
    int row[64][16], col[64][16];
    for (int i = 0; i < 32; ++i) A[i * 2] = (float)(i + 1), A[i * 2 + 1] = 0.0f;
    for (int j = 0; j < 32; ++j) B[j] = 1.0f, B[32 + j] = 0.0f;
    run();
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) row[l][r] = (int)D[l * 16 + r] - 1;
    for (int i = 0; i < 32; ++i) A[i * 2] = 1.0f;
    for (int j = 0; j < 32; ++j) B[j] = (float)(j + 1);
    run();
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) col[l][r] = (int)D[l * 16 + r] - 1;
    bool formula = true;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int ei = (r / 4) * 8 + (l / 32) * 4 + (r % 4), ej = l % 32;
            formula &= row[l][r] == ei && col[l][r] == ej;
        }
    printf("layout: lane 0 rows %d %d %d %d %d ..., lane 32 rows %d %d ..., col(l=5)=%d; "
           "row = (r/4)*8 + (l/32)*4 + r%%4, col = l%%32: %s\n",
           row[0][0], row[0][1], row[0][2], row[0][3], row[0][4], row[32][0], row[32][1],
           col[5][0], formula ? "yes" : "NO");
    // 2. arithmetic: random operands of the screen's magnitudes, D against the VALU chain
    unsigned s = 12345;
    long long mism = 0, total = 0;
    for (int trial = 0; trial < 2000; ++trial) {
        for (int i = 0; i < 64; ++i) A[i] = frand(s) * 300.0f;
        for (int j = 0; j < 64; ++j) B[j] = frand(s) * 600.0f;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r) C[l * 16 + r] = std::fabs(frand(s)) * 90000.0f;
        run();
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r) {
                const int i = row[l][r], j = col[l][r];
                const float c = C[l * 16 + r];
                const float e = std::fmaf(A[i * 2 + 1], B[32 + j], std::fmaf(A[i * 2], B[j], c));
                float g = D[l * 16 + r];
                ++total;
                if (std::memcmp(&e, &g, 4) != 0) ++mism;
            }
    }
    printf("fma chain k=0 then k=1: %lld of %lld results differ\n", mism, total);
    return mism == 0 && formula ? 0 : 1;
}
