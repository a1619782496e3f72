// Diagnostic: ablations of the NB=32 pivot loop (timings only; outputs are garbage for V != 0).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"
using namespace mfgp;

template <int V>
__device__ void fac32(double* __restrict__ A, double* __restrict__ R, double* __restrict__ dg, int* bad) {
    constexpr int NB = 32, S = TileCfg<NB>::S;
    double* colb = R; double* rowb = R + 2 * NB; double* invb = R + 4 * NB;
    const int t = threadIdx.x, i = t >> 3, g = t & 7, c0 = 4 * g;
    double a[4], r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) { a[q] = A[i * S + c0 + q]; r[q] = (i == c0 + q) ? 1.0 : 0.0; }
    __syncthreads();
    if (g == 0) colb[i] = a[0];
    if (t < NB) rowb[t] = (t == 0) ? 1.0 : 0.0;
    if (t == 0) { invb[0] = 1.0 / a[0]; dg[0] = a[0]; }
    __syncthreads();
    for (int k = 0; k < NB; ++k) {
        const int cur = k & 1, nxt = cur ^ 1;
        const double inv = (V & 1) ? 1.0 : invb[cur];
        const double aik = colb[cur * NB + i];
        const double2 ca = *reinterpret_cast<const double2*>(colb + cur * NB + c0);
        const double2 cb = *reinterpret_cast<const double2*>(colb + cur * NB + c0 + 2);
        const double2 ra = *reinterpret_cast<const double2*>(rowb + cur * NB + c0);
        const double2 rb = *reinterpret_cast<const double2*>(rowb + cur * NB + c0 + 2);
        const double colv[4] = {ca.x, ca.y, cb.x, cb.y};
        const double rowv[4] = {ra.x, ra.y, rb.x, rb.y};
        const double s = aik * inv;
        if (V & 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) { a[q] -= s * colv[q]; r[q] -= s * rowv[q]; }
        } else if (i > k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int c = c0 + q;
                if (c > k && c <= i) a[q] -= s * colv[q];
                if (c <= k) r[q] -= s * rowv[q];
            }
        }
        const int k1 = k + 1;
        if ((V & 32) && k1 < NB) {   // unconditional column publish to a dump slot, no division
            double v = a[0];
#pragma unroll
            for (int q = 1; q < 4; ++q) if (q == (k1 & 3)) v = a[q];
            const bool own = ((k1 >> 2) == g) && i >= k1;
            colb[own ? nxt * NB + i : 5 * NB + 2 + t] = v;
            if (own && i == k1) { invb[nxt] = v; dg[k1] = v; }
            if (!(V & 64) && i == k1) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (c0 + q <= k1) rowb[nxt * NB + c0 + q] = (c0 + q == k1) ? 1.0 : r[q];
            }
        }
        if (!(V & 8) && !(V & 32) && k1 < NB) {
            if ((k1 >> 2) == g && i >= k1) {
                double v = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) if (q == (k1 & 3)) v = a[q];
                colb[nxt * NB + i] = v;
                if (i == k1) {
                    invb[nxt] = (V & 2) ? v : 1.0 / v;
                    dg[k1] = v;
                }
            }
            if (i == k1) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (c0 + q <= k1) rowb[nxt * NB + c0 + q] = (c0 + q == k1) ? 1.0 : r[q];
            }
        }
        if (V & 16) __builtin_amdgcn_s_barrier(); else __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) R[i * S + c0 + q] = r[q] + a[q];
    __syncthreads();
}

template <int V>
__global__ __launch_bounds__(256) void k_b(const double* Ag, double* out, long long* cyc, int reps) {
    constexpr int E = TileCfg<32>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem; double* R = A + E + 300; double* dg = R + E;
    int* bad = reinterpret_cast<int*>(dg + 32);
    long long t0 = 0, t1 = 0;
    for (int it = 0; it < reps; ++it) {
        tile_load<32>(A, Ag, 32);
        __syncthreads();
        if (it == 1) t0 = __builtin_amdgcn_s_memtime();
        fac32<V>(A, R, dg, bad);
        if (it == reps - 1) t1 = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) cyc[0] = (t1 - t0) / (reps - 2);
    tile_store<32>(out, 32, R);
}

template <int V>
void run(const char* name, const double* dA, double* dO, long long* dc) {
    size_t sm = sizeof(double) * (2 * 32 * 34 + 34 + 300);
    hipLaunchKernelGGL((k_b<V>), dim3(1), dim3(256), sm, 0, dA, dO, dc, 40);
    (void)hipDeviceSynchronize();
    long long c;
    (void)hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    printf("V=%2d %-40s %8lld clk/factor  %6.0f clk/pivot\n", V, name, c, c / 32.0);
}

int main() {
    double h[32 * 32];
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) h[i * 32 + j] = (i == j ? 32 : 0.0) + 1.0 / (1.0 + i + j);
    double *dA, *dO; long long* dc;
    (void)hipMalloc(&dA, sizeof(h)); (void)hipMalloc(&dO, sizeof(h)); (void)hipMalloc(&dc, 8);
    (void)hipMemcpy(dA, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>("full", dA, dO, dc);
    run<1>("no inv read (inv=1)", dA, dO, dc);
    run<2>("no division (publish v)", dA, dO, dc);
    run<4>("unpredicated updates", dA, dO, dc);
    run<8>("no publish", dA, dO, dc);
    run<16>("raw s_barrier", dA, dO, dc);
    run<2 | 4>("no div + unpredicated", dA, dO, dc);
    run<2 | 4 | 8>("no div/publish, unpredicated", dA, dO, dc);
    run<1 | 2 | 4 | 8 | 16>("bare: reads + 8 fma + barrier", dA, dO, dc);
    run<32>("uncond col publish + row publish", dA, dO, dc);
    run<32 | 64>("uncond col publish only", dA, dO, dc);
    run<32 | 64 | 4>("uncond col only, unpredicated", dA, dO, dc);
    run<32 | 4>("uncond col+row, unpredicated", dA, dO, dc);
    return 0;
}
