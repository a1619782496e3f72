// Diagnostic: dependent-chain latencies on gfx950 (shader clocks per op).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int W>
__global__ void k(double* io, long long* cyc) {
    double x = io[threadIdx.x], y = io[64 + threadIdx.x];
    long long t0 = __builtin_amdgcn_s_memtime();
    if (W == 0) { for (int i = 0; i < 256; ++i) x = fma(x, y, 0.5); }
    if (W == 1) { for (int i = 0; i < 256; ++i) x = __builtin_amdgcn_rcp(x) + 1e-300; }
    if (W == 2) {
        for (int i = 0; i < 256; ++i) {
            long long b = __builtin_bit_cast(long long, x);
            int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), 3);
            int hi = __builtin_amdgcn_readlane((int)(b >> 32), 3);
            x = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) * y;
        }
    }
    if (W == 3) {
        for (int i = 0; i < 256; ++i) {
            long long b = __builtin_bit_cast(long long, x);
            int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffff), 3 << 5);
            int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 3 << 5);
            x = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) * y;
        }
    }
    if (W == 4) { for (int i = 0; i < 256; ++i) x = x * y; }
    if (W == 5) { float f = (float)x, g = (float)y; for (int i = 0; i < 256; ++i) f = fmaf(f, g, 0.5f); x = f; }
    if (W == 6) {   // LDS write -> read round trip by the same wave
        __shared__ double sh[64];
        for (int i = 0; i < 256; ++i) { sh[threadIdx.x] = x; __builtin_amdgcn_s_waitcnt(0); x = sh[(threadIdx.x + 1) & 63] * y; }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    io[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[W] = (t1 - t0) / 256;
}
int main() {
    double* d; long long* c; (void)hipMalloc(&d, 128 * 8); (void)hipMalloc(&c, 64);
    double h[128]; for (int i = 0; i < 128; ++i) h[i] = 1.0 + 1e-9 * i;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const char* nm[] = {"fma_f64 chain", "rcp_f64 chain", "readlane x2 + mul_f64", "ds_swizzle x2 + mul_f64", "mul_f64 chain", "fma_f32 chain", "ds_write+wait+ds_read+mul"};
    hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, d, c); hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, d, c);
    hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, d, c); hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, d, c);
    hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, d, c); hipLaunchKernelGGL(k<5>, 1, 64, 0, 0, d, c);
    hipLaunchKernelGGL(k<6>, 1, 64, 0, 0, d, c);
    long long hc[8]; (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    for (int w = 0; w < 7; ++w) printf("%-28s %lld clk/iter\n", nm[w], hc[w]);
}
