// Diagnostic: dependent-chain latencies on gfx950 for the diagonal-factor floor (shader clocks
// per op, s_memtime): the pivot reciprocal as the factor computes it (rcp_nr1: v_rcp_f64 + one
// Newton step), gfx950's cross-row lane swaps (v_permlane16/32_swap), a DPP row broadcast, and
// the MFMA -> VALU read of its result (an accumulator block feeding the next pivot's arithmetic).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_lat3.hip -o tools/ubench_lat3
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double rcp_nr1(double a) {
    const double r = __builtin_amdgcn_rcp(a);
    return fma(r, fma(-a, r, 1.0), r);
}

template <int W>
__global__ void k(double* io, long long* cyc) {
    double x = io[threadIdx.x & 127], y = io[(threadIdx.x + 64) & 127];
    f64x4 acc = {x, y, x, y};
    long long t0 = __builtin_amdgcn_s_memtime();
    if (W == 0) { for (int i = 0; i < 256; ++i) x = rcp_nr1(x) + 1e-300; }
    if (W == 1) {   // permlane32 swap of both halves of a double, then a multiply
        for (int i = 0; i < 256; ++i) {
            long long b = __builtin_bit_cast(long long, x);
            unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
            auto p = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
            x = __builtin_bit_cast(double, ((unsigned long long)p[1] << 32) | p[0]) * y;
        }
    }
    if (W == 2) {
        for (int i = 0; i < 256; ++i) {
            long long b = __builtin_bit_cast(long long, x);
            unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
            auto p = __builtin_amdgcn_permlane16_swap(lo, hi, false, false);
            x = __builtin_bit_cast(double, ((unsigned long long)p[1] << 32) | p[0]) * y;
        }
    }
    if (W == 3) {   // DPP row_bcast-like: broadcast lane 0 of each row of 16 (row_shr chain substitute)
        for (int i = 0; i < 256; ++i) {
            long long b = __builtin_bit_cast(long long, x);
            int lo = __builtin_amdgcn_mov_dpp((int)b, 0x150, 0xf, 0xf, false);          // row_share:0
            int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x150, 0xf, 0xf, false);
            x = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) * y;
        }
    }
    if (W == 4) {   // MFMA, then a VALU op on its result, feeding the next MFMA's A operand
        for (int i = 0; i < 256; ++i) {
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
            x = acc[1] * y;
        }
        x += acc[0] + acc[2] + acc[3];
    }
    if (W == 5) { for (int i = 0; i < 256; ++i) x = __builtin_amdgcn_rcp(x) + 1e-300; }
    long long t1 = __builtin_amdgcn_s_memtime();
    io[threadIdx.x & 127] = x + acc[0];
    if (threadIdx.x == 0) cyc[W] = (t1 - t0) / 256;
}

int main() {
    double* d;
    long long* c;
    (void)hipMalloc(&d, 128 * 8);
    (void)hipMalloc(&c, 8 * 8);
    double h[128];
    for (int i = 0; i < 128; ++i) h[i] = 1.0 + 1e-9 * i;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const char* nm[] = {"rcp_nr1 chain (+add)", "permlane32_swap x1 (2 dwords) + mul_f64",
                        "permlane16_swap x1 (2 dwords) + mul_f64", "dpp row_share x2 + mul_f64",
                        "mfma_f64_16x16x4 -> mul_f64 -> next mfma", "v_rcp_f64 chain (+add)"};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d, c);
        hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d, c);
        hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, d, c);
        hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, d, c);
        hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, d, c);
        hipLaunchKernelGGL(k<5>, dim3(1), dim3(64), 0, 0, d, c);
        (void)hipDeviceSynchronize();
    }
    long long hc[8];
    (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    for (int i = 0; i < 6; ++i) printf("%-45s %lld clocks\n", nm[i], hc[i]);
    return 0;
}
