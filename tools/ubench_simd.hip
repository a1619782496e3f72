// Diagnostic: fp64 VALU throughput vs number of waves in one workgroup (SIMD placement).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int ILP>
__global__ void k(double* io, long long* cyc, int* hwid) {
    double x[ILP];
    for (int j = 0; j < ILP; ++j) x[j] = io[threadIdx.x % 64] + j;
    const double y = io[64];
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 512; ++i)
#pragma unroll
        for (int j = 0; j < ILP; ++j) x[j] = fma(x[j], y, 0.5);
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0; for (int j = 0; j < ILP; ++j) s += x[j];
    io[128 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        cyc[threadIdx.x >> 6] = (t1 - t0);
        unsigned v; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v)); hwid[threadIdx.x >> 6] = v;
    }
}
int main() {
    double* d; long long* c; int* hw;
    (void)hipMalloc(&d, 2048 * 8); (void)hipMalloc(&c, 16 * 8); (void)hipMalloc(&hw, 64);
    double h[2048]; for (int i = 0; i < 2048; ++i) h[i] = 0.999;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    for (int nt : {64, 128, 256, 512}) {
        for (int ilp : {1, 8}) {
            if (ilp == 1) hipLaunchKernelGGL(k<1>, 1, nt, 0, 0, d, c, hw); else hipLaunchKernelGGL(k<8>, 1, nt, 0, 0, d, c, hw);
            long long hc[8]; int hh[8];
            (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost); (void)hipMemcpy(hh, hw, sizeof(hh), hipMemcpyDeviceToHost);
            printf("threads %3d ILP %d: clk per FMA-step per wave:", nt, ilp);
            for (int w = 0; w < nt / 64; ++w) printf(" %.1f(simd%d)", hc[w] / (512.0 * ilp), (hh[w] >> 4) & 3);
            printf("\n");
        }
    }
}
