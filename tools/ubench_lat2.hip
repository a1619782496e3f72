// Diagnostic: more dependent-chain latencies on gfx950 (shader clocks per op): the f64
// MFMA accumulator chain, f64 rsq/sqrt, a 4-wave workgroup barrier, an LDS publish ->
// barrier -> read round trip, and a single-wave LDS write -> read round trip.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int W>
__global__ void k(double* io, long long* cyc) {
    __shared__ double sh[512];
    double x = io[threadIdx.x & 127], y = io[(threadIdx.x + 64) & 127];
    f64x4 acc = {x, y, x, y};
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    if (W == 0) { for (int i = 0; i < 256; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0); }
    if (W == 1) { for (int i = 0; i < 256; ++i) x = __builtin_amdgcn_rsq(x) + 0.5; }
    if (W == 2) { for (int i = 0; i < 256; ++i) x = __builtin_sqrt(x) + 0.5; }
    if (W == 3) { for (int i = 0; i < 256; ++i) { __syncthreads(); x = x * y; } }
    if (W == 4) {   // publish by wave 0, barrier, everyone reads
        for (int i = 0; i < 256; ++i) {
            if (threadIdx.x < 64) sh[threadIdx.x] = x;
            __syncthreads();
            x = sh[(threadIdx.x + 1) & 63] * y;
            __syncthreads();
        }
    }
    if (W == 5) {   // one wave: write, wait, read another lane's word (no barrier)
        for (int i = 0; i < 256; ++i) {
            sh[threadIdx.x] = x;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            x = sh[(threadIdx.x & ~63) + ((threadIdx.x + 1) & 63)] * y;
        }
    }
    if (W == 6) {   // mfma chain where the next A operand depends on the result (acc -> operand)
        for (int i = 0; i < 256; ++i) {
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
            x = acc[0];
        }
    }
    if (W == 7) {   // ds_read_b128 broadcast (same address) round trip
        for (int i = 0; i < 256; ++i) {
            sh[threadIdx.x & 255] = x;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const double2 v = *reinterpret_cast<const double2*>(sh + 2 * (int)(x > 1e300));
            x = v.x * y + v.y;
        }
    }
    if (W == 8) { for (int i = 0; i < 256; ++i) x = __builtin_amdgcn_rcp(x) + 0.5; }
    long long t1 = __builtin_amdgcn_s_memtime();
    io[threadIdx.x & 127] = x + acc[0] + acc[1] + acc[2] + acc[3];
    if (threadIdx.x == 0) cyc[W] = (t1 - t0) / 256;
}
int main() {
    double* d; long long* c; (void)hipMalloc(&d, 128 * 8); (void)hipMalloc(&c, 128);
    double h[128]; for (int i = 0; i < 128; ++i) h[i] = 1.0 + 1e-9 * i;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const char* nm[] = {"mfma_f64_16x16x4 acc chain", "rsq_f64 chain", "sqrt_f64 chain", "barrier (4 waves)",
                        "publish+barrier+read (4w)", "1-wave lds write->read", "mfma acc->operand chain",
                        "1-wave write->b128 bcast", "rcp_f64 chain"};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, d, c); hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, d, c);
        hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, d, c); hipLaunchKernelGGL(k<3>, 1, 256, 0, 0, d, c);
        hipLaunchKernelGGL(k<4>, 1, 256, 0, 0, d, c); hipLaunchKernelGGL(k<5>, 1, 64, 0, 0, d, c);
        hipLaunchKernelGGL(k<6>, 1, 64, 0, 0, d, c); hipLaunchKernelGGL(k<7>, 1, 64, 0, 0, d, c);
        hipLaunchKernelGGL(k<8>, 1, 64, 0, 0, d, c);
    }
    long long hc[16]; (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    for (int w = 0; w < 9; ++w) printf("%-30s %lld clk/iter\n", nm[w], hc[w]);
}
