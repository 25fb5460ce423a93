// Probe: A = Y Y^T off-diagonal 32x32 tile with v_mfma_f32_32x32x2_f32, the
// operand/accumulator mapping used in leggedsim.hip, checked against the CPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int R = 64, K = 18;
__global__ void k(const float* Y, float* C) {  // C[32][32] = Y[32..63] * Y[0..31]^T
    const int lane = threadIdx.x, li = lane & 31, lk = lane >> 5;
    floatx16 acc;
    for (int t = 0; t < 16; ++t) acc[t] = 0.f;
    for (int st = 0; st < K / 2; ++st) {
        const int kk = 2 * st + lk;
        const float a = Y[(32 + li) * K + kk];
        const float b = Y[li * K + kk];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    for (int t = 0; t < 16; ++t) {
        const int row = (t & 3) + 8 * (t >> 2) + 4 * lk, col = li;
        C[row * 32 + col] = acc[t];
    }
}
int main() {
    float hY[R * K], hC[32 * 32];
    for (int i = 0; i < R * K; ++i) hY[i] = (float)((i * 37) % 101) / 50.f - 1.f;
    float *dY, *dC;
    hipMalloc(&dY, sizeof hY); hipMalloc(&dC, sizeof hC);
    hipMemcpy(dY, hY, sizeof hY, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dY, dC);
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    double e = 0, et = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            float s = 0.f, st = 0.f;
            for (int k2 = 0; k2 < K; ++k2) { s = fmaf(hY[(32 + i) * K + k2], hY[j * K + k2], s); st = fmaf(hY[(32 + j) * K + k2], hY[i * K + k2], st); }
            e = fmax(e, fabs(hC[i * 32 + j] - s));
            et = fmax(et, fabs(hC[i * 32 + j] - st));
        }
    printf("max |C - Y1 Y0^T| = %g   max |C - (Y1 Y0^T)^T| = %g\n", e, et);
    return 0;
}
