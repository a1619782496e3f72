// Diagnostic: single-wave ISSUE cost (independent instructions) on gfx950: v_fma_f64,
// v_mul_f64, v_cndmask_b32 pairs (f64 select), v_rcp_f64, and f64 MFMA 16x16x4 throughput
// with 4 independent accumulators; plus two waves on different SIMDs.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int W>
__global__ void k(double* io, long long* cyc) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = io[(threadIdx.x + i) & 127];
    const double y = io[threadIdx.x & 127] * 0.5;
    f64x4 a0 = {x[0], x[1], x[2], x[3]}, a1 = a0, a2 = a0, a3 = a0;
    const bool c = (threadIdx.x & 3) == 1;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; ++it) {
        if (W == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = fma(x[i], y, 0.25);
        }
        if (W == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = x[i] * y;
        }
        if (W == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = c ? x[(i + 1) & 7] : x[i];
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
        }
        if (W == 3) {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_rcp(x[i]);
        }
        if (W == 4) {
            a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], y, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], y, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], y, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], y, a3, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[4], y, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[5], y, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[6], y, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[7], y, a3, 0, 0, 0);
        }
        if (W == 5) {   // 4 MFMAs + 8 fma interleaved
            a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], y, a0, 0, 0, 0);
            x[4] = fma(x[4], y, 0.25); x[5] = fma(x[5], y, 0.25);
            a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], y, a1, 0, 0, 0);
            x[6] = fma(x[6], y, 0.25); x[7] = fma(x[7], y, 0.25);
            a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], y, a2, 0, 0, 0);
            x[4] = fma(x[4], y, 0.25); x[5] = fma(x[5], y, 0.25);
            a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], y, a3, 0, 0, 0);
            x[6] = fma(x[6], y, 0.25); x[7] = fma(x[7], y, 0.25);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = a0[0] + a1[1] + a2[2] + a3[3];
    for (int i = 0; i < 8; ++i) s += x[i];
    io[threadIdx.x & 127] = s;
    if ((threadIdx.x & 63) == 0) cyc[W * 4 + (threadIdx.x >> 6)] = (t1 - t0);
}
int main() {
    double* d; long long* c; (void)hipMalloc(&d, 128 * 8); (void)hipMalloc(&c, 512);
    double h[128]; for (int i = 0; i < 128; ++i) h[i] = 1.0 + 1e-9 * i;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const char* nm[] = {"v_fma_f64 (8 indep)", "v_mul_f64 (8 indep)", "f64 select (8 indep)", "v_rcp_f64 (8 indep)",
                        "mfma f64 16x16x4 (4 acc)", "4 mfma + 8 fma interleaved"};
    const int per[] = {8, 8, 8, 8, 8, 4};
    for (int nw = 1; nw <= 4; nw *= 4) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k<0>, 1, 64 * nw, 0, 0, d, c); hipLaunchKernelGGL(k<1>, 1, 64 * nw, 0, 0, d, c);
            hipLaunchKernelGGL(k<2>, 1, 64 * nw, 0, 0, d, c); hipLaunchKernelGGL(k<3>, 1, 64 * nw, 0, 0, d, c);
            hipLaunchKernelGGL(k<4>, 1, 64 * nw, 0, 0, d, c); hipLaunchKernelGGL(k<5>, 1, 64 * nw, 0, 0, d, c);
        }
        long long hc[64]; (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("%d wave(s) per workgroup:\n", nw);
        for (int w = 0; w < 6; ++w) printf("  %-30s %6.1f clk per instruction (wave 0)\n", nm[w], hc[w * 4] / (64.0 * per[w]));
    }
}
