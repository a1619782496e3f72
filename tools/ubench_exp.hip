// Diagnostic: fp64 exp cost on gfx950 (shader clocks per exp, s_memtime; and the shader clock
// against the 100 MHz s_memrealtime): one dependent chain of library exp(), four chains written
// side by side, four chains stage-pinned (exp4 form of k_gram_flow), and 8 independent FMA chains.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_exp.hip -o tools/ubench_exp
#include <hip/hip_runtime.h>
#include <stdio.h>
#define PIN4(v) asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]))
__device__ __forceinline__ double dbits(unsigned long long u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ void exp4(double (&x)[4]) {
    const double C[10] = {dbits(0x3e928af3fca7ab0cull), dbits(0x3ec71dee623fde64ull), dbits(0x3efa01997c89e6b0ull),
                          dbits(0x3f2a01a014761f6eull), dbits(0x3f56c16c1852b7b0ull), dbits(0x3f81111111122322ull),
                          dbits(0x3fa55555555502a1ull), dbits(0x3fc5555555555511ull), dbits(0x3fe000000000000bull), 1.0};
    double n[4], r[4], p[4];
    for (int u = 0; u < 4; ++u) n[u] = __builtin_rint(x[u] * dbits(0x3ff71547652b82feull));
    PIN4(n);
    for (int u = 0; u < 4; ++u) r[u] = fma(dbits(0xbfe62e42fefa39efull), n[u], x[u]);
    PIN4(r);
    for (int u = 0; u < 4; ++u) r[u] = fma(dbits(0xbc7abc9e3b39803full), n[u], r[u]);
    PIN4(r);
    for (int u = 0; u < 4; ++u) p[u] = fma(dbits(0x3e5ade156a5dcb37ull), r[u], C[0]);
    PIN4(p);
    for (int k = 1; k < 10; ++k) {
        for (int u = 0; u < 4; ++u) p[u] = fma(r[u], p[u], C[k]);
        PIN4(p);
    }
    for (int u = 0; u < 4; ++u) p[u] = fma(r[u], p[u], 1.0);
    PIN4(p);
    for (int u = 0; u < 4; ++u) {
        const double e = __builtin_ldexp(p[u], (int)n[u]);
        x[u] = x[u] > 1024.0 ? __builtin_inf() : (x[u] < -1075.0 ? 0.0 : e);
    }
}

template <int W>
__global__ void k(double* io, long long* cyc) {
    double x[4];
    for (int u = 0; u < 4; ++u) x[u] = io[(threadIdx.x + 17 * u) & 127];
    const double y = io[threadIdx.x & 127] * 1e-3;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    constexpr int IT = 128;
    if (W == 0) { for (int i = 0; i < IT; ++i) x[0] = exp(x[0] * y - 1.0); }
    if (W == 1) {
        for (int i = 0; i < IT; ++i)
            for (int u = 0; u < 4; ++u) x[u] = exp(x[u] * y - 1.0);
    }
    if (W == 2) {
        for (int i = 0; i < IT; ++i) {
            for (int u = 0; u < 4; ++u) x[u] = x[u] * y - 1.0;
            exp4(x);
        }
    }
    if (W == 3) {
        double z[8];
        for (int u = 0; u < 8; ++u) z[u] = x[u & 3] + u;
        for (int i = 0; i < IT; ++i)
            for (int rep = 0; rep < 4; ++rep)
                for (int u = 0; u < 8; ++u) z[u] = fma(z[u], y, 0.25);
        for (int u = 0; u < 4; ++u) x[u] = z[u] + z[u + 4];
    }
    if (W == 4) { for (int i = 0; i < IT; ++i) for (int rep = 0; rep < 32; ++rep) x[0] = fma(x[0], y, 0.25); }
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    io[threadIdx.x & 127] = x[0] + x[1] + x[2] + x[3];
    if (threadIdx.x == 0) { cyc[2 * W] = (t1 - t0); cyc[2 * W + 1] = (r1 - r0); }
    if (threadIdx.x == 64 * (blockDim.x / 64 - 1)) { cyc[16 + 2 * W] = (t1 - t0); }
}

int main() {
    double* d;
    long long* c;
    hipMalloc(&d, 128 * sizeof(double));
    hipMalloc(&c, 32 * sizeof(long long));
    double h[128];
    for (int i = 0; i < 128; ++i) h[i] = 0.5 + 0.001 * i;
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const char* nm[5] = {"exp chain (per exp)", "4 exp() side by side (per exp)", "exp4 pinned (per exp)",
                         "8 indep fma chains (per fma)", "1 fma chain (per fma)"};
    const double per[5] = {128, 512, 512, 128 * 32, 128 * 32};
    for (int nt : {64, 256, 512, 1024}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k<0>, dim3(1), dim3(nt), 0, 0, d, c);
            hipLaunchKernelGGL(k<1>, dim3(1), dim3(nt), 0, 0, d, c);
            hipLaunchKernelGGL(k<2>, dim3(1), dim3(nt), 0, 0, d, c);
            hipLaunchKernelGGL(k<3>, dim3(1), dim3(nt), 0, 0, d, c);
            hipLaunchKernelGGL(k<4>, dim3(1), dim3(nt), 0, 0, d, c);
            hipDeviceSynchronize();
        }
        long long hc[32];
        hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("-- one workgroup of %d threads (%d waves): first wave / last wave\n", nt, nt / 64);
        for (int w = 0; w < 5; ++w)
            printf("%-34s %8.1f / %8.1f clk   (shader clock %.0f MHz)\n", nm[w], hc[2 * w] / per[w],
                   hc[16 + 2 * w] / per[w], 100.0 * hc[2 * w] / (double)hc[2 * w + 1]);
    }
    return 0;
}
