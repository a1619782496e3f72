// Diagnostic: variants of the branch-free NB=32 pivot loop (timing + max error vs. numpy-free check).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"
using namespace mfgp;

// rcp_nr: v_rcp_f64 + two Newton steps (mfgp_device.h)

template <int V>
__device__ void fac(double* __restrict__ A, double* __restrict__ R, double* __restrict__ dg) {
    constexpr int NB = 32, S = TileCfg<NB>::S;
    double* colb = R; double* rowb = R + 2 * NB;
    const int t = threadIdx.x, i = t >> 3, g = t & 7, c0 = 4 * g;
    double a[4], r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) { a[q] = A[i * S + c0 + q]; r[q] = (i == c0 + q) ? 1.0 : 0.0; }
    __syncthreads();
    if (g == 0) colb[i] = a[0];
    if (t < NB) rowb[t] = (t == 0) ? 1.0 : 0.0;
    __syncthreads();
    double dgk = 0.0;
#pragma unroll 4
    for (int k = 0; k < NB; ++k) {
        const int cur = k & 1, nxt = cur ^ 1;
        const double akk = colb[cur * NB + k];
        const double aik = colb[cur * NB + i];
        const double2 ca = *reinterpret_cast<const double2*>(colb + cur * NB + c0);
        const double2 cb = *reinterpret_cast<const double2*>(colb + cur * NB + c0 + 2);
        const double2 ra = *reinterpret_cast<const double2*>(rowb + cur * NB + c0);
        const double2 rb = *reinterpret_cast<const double2*>(rowb + cur * NB + c0 + 2);
        if (V & 4) { if (i == k) dgk = akk; } else { if (t == 0) dg[k] = akk; }
        const double sA = (V & 1) ? aik * rcp_nr(akk) : aik / akk;
        const double sR = (i > k) ? sA : 0.0;
        a[0] -= sA * ca.x; a[1] -= sA * ca.y; a[2] -= sA * cb.x; a[3] -= sA * cb.y;
        r[0] -= sR * ra.x; r[1] -= sR * ra.y; r[2] -= sR * rb.x; r[3] -= sR * rb.y;
        const int k1 = k + 1, q1 = k1 & 3;
        const double v = (q1 == 0) ? a[0] : (q1 == 1) ? a[1] : (q1 == 2) ? a[2] : a[3];
        const bool own = (k1 >> 2) == g;
        colb[own ? nxt * NB + i : 4 * NB + t] = (i >= k1) ? v : 0.0;
        if (V & 2) {
            const bool rown = (i == k1);
            *reinterpret_cast<double4*>(rowb + (rown ? nxt * NB + c0 : 4 * NB + 256 + 4 * t)) = double4{r[0], r[1], r[2], r[3]};
        } else {
            if (i == k1) *reinterpret_cast<double4*>(rowb + nxt * NB + c0) = double4{r[0], r[1], r[2], r[3]};
        }
        if (V & 8) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); }
        else __syncthreads();
    }
    if (V & 4) { if (g == 0) dg[i] = dgk; __syncthreads(); }
    const double li = sqrt(dg[i]);
    const double rli = 1.0 / li;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) R[i * S + c0 + q] = (c0 + q <= i) ? r[q] * rli : 0.0;
    __syncthreads();
}

template <int V>
__global__ __launch_bounds__(256) void k_b(const double* Ag, double* out, long long* cyc, int reps) {
    constexpr int E = TileCfg<32>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem; double* R = A + E; double* dg = R + E + 1400;
    long long t0 = 0, t1 = 0;
    for (int it = 0; it < reps; ++it) {
        tile_load<32>(A, Ag, 32);
        __syncthreads();
        if (it == 1) t0 = __builtin_amdgcn_s_memtime();
        fac<V>(A, R, dg);
        if (it == reps - 1) t1 = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) cyc[0] = (t1 - t0) / (reps - 2);
    tile_store<32>(out, 32, R);
}

double h[32 * 32], o[32 * 32];
template <int V>
void run(const char* name, const double* dA, double* dO, long long* dc) {
    size_t sm = sizeof(double) * (2 * 32 * 34 + 1400 + 40);
    hipLaunchKernelGGL((k_b<V>), dim3(1), dim3(256), sm, 0, dA, dO, dc, 40);
    (void)hipDeviceSynchronize();
    long long c;
    (void)hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(o, dO, sizeof(o), hipMemcpyDeviceToHost);
    // check: D A D^T = I
    double err = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            double s = 0;
            for (int p = 0; p < 32; ++p)
                for (int q = 0; q < 32; ++q) s += o[i * 32 + p] * h[p * 32 + q] * o[j * 32 + q];
            err = fmax(err, fabs(s - (i == j)));
        }
    printf("V=%2d %-36s %8lld clk/factor  %6.0f clk/pivot  |DAD^T-I|=%.2e\n", V, name, c, c / 32.0, err);
}

int main() {
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) h[i * 32 + j] = (i == j ? 32 : 0.0) + 1.0 / (1.0 + i + j);
    double *dA, *dO; long long* dc;
    (void)hipMalloc(&dA, sizeof(h)); (void)hipMalloc(&dO, sizeof(h)); (void)hipMalloc(&dc, 8);
    (void)hipMemcpy(dA, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>("current", dA, dO, dc);
    run<1>("rcp+2NR", dA, dO, dc);
    run<1 | 2>("rcp + uncond row publish", dA, dO, dc);
    run<1 | 4>("rcp + dg in register", dA, dO, dc);
    run<1 | 8>("rcp + raw barrier", dA, dO, dc);
    run<1 | 2 | 4 | 8>("all", dA, dO, dc);
    run<1 | 2 | 4>("rcp+row+dg", dA, dO, dc);
    return 0;
}
