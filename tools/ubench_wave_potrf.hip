// Diagnostic micro-benchmark (not part of libmfgp.so): single-wave 32x32 Cholesky with
// the pivot chain kept inside one wavefront (no LDS round trip, no barrier per pivot).
//   lane l (l < 32) owns row i = l in 32 registers (lanes 32..63 duplicate rows);
//   pivot k: a_kk = readlane(lane k), s_i = a_ik / a_kk (0 for i <= k), row k of the
//   trailing part broadcast from lane k (MODE 0: v_readlane -> SGPR operand,
//   MODE 1: ds_swizzle broadcast within each 32-lane group), a_ij -= s_i a_kj (j > k).
//   Columns are scaled at the end: L_ij = a_ij / sqrt(pivot_j).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

constexpr int NB = 32, S = NB + 2;

__device__ __forceinline__ double readlane_d(double x, int l) {
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int K>
__device__ __forceinline__ double swz_d(double x) {
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffff), K << 5);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), K << 5);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

template <int MODE, int K, int J>
__device__ __forceinline__ void upd(double (&a)[NB], double s, int k) {
    if constexpr (J < NB) {
        const double b = (MODE == 0) ? readlane_d(a[J], K) : swz_d<K>(a[J]);
        a[J] = fma(-s, b, a[J]);
        upd<MODE, K, J + 1>(a, s, k);
    }
}
__device__ __forceinline__ double rsq_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}
template <int MODE, int K>
__device__ __forceinline__ void pivots(double (&a)[NB], int i) {
    if constexpr (K < NB) {
        const double akk = readlane_d(a[K], K);
        const double r2 = rcp_nr(akk);
        const double s = (i > K) ? a[K] * r2 : 0.0;
        upd<MODE, K, K + 1>(a, s, K);
        // column K is final: L_iK = a_iK / sqrt(a_KK) (off the pivot chain)
        a[K] = (i > K) ? a[K] * rsq_nr(akk) : (i == K ? sqrt(akk) : 0.0);
        pivots<MODE, K + 1>(a, i);
    }
}

template <int MODE>
__device__ void potrf_wave(double* A, double* dg) {
    const int lane = threadIdx.x & 63, i = lane & 31;
    double a[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) a[j] = A[i * S + j];
    pivots<MODE, 0>(a, i);
    if (lane < 32) {
#pragma unroll
        for (int j = 0; j < NB; ++j) A[i * S + j] = a[j];
        dg[i] = A[i * S + i];
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_bench(const double* Ag, double* out, long long* cyc, int reps) {
    __shared__ __attribute__((aligned(16))) double A[NB * S];
    __shared__ double dg[NB];
    long long t0 = 0, t1 = 0;
    for (int it = 0; it < reps; ++it) {
        for (int e = threadIdx.x; e < NB * NB; e += 256) A[(e / NB) * S + e % NB] = Ag[e];
        __syncthreads();
        if (it == 1) t0 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x < 64) potrf_wave<MODE>(A, dg);
        __syncthreads();
        if (it == reps - 1) t1 = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) cyc[0] = (t1 - t0) / (reps - 2);
    for (int e = threadIdx.x; e < NB * NB; e += 256) out[e] = A[(e / NB) * S + e % NB];
}

template <int MODE>
void run(const char* name, const double* dA, double* dO, long long* dc, const double* h) {
    const int reps = 50;
    hipLaunchKernelGGL((k_bench<MODE>), dim3(1), dim3(256), 0, 0, dA, dO, dc, reps);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_bench<MODE>), dim3(1), dim3(256), 0, 0, dA, dO, dc, reps);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    long long c; (void)hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    static double L[NB * NB];
    (void)hipMemcpy(L, dO, sizeof(L), hipMemcpyDeviceToHost);
    // residual |L L^T - A|
    double e = 0;
    for (int i = 0; i < NB; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = 0;
            for (int m = 0; m <= j; ++m) s += L[i * NB + m] * L[j * NB + m];
            e = fmax(e, fabs(s - h[i * NB + j]));
        }
    printf("%-24s %8lld shader-clk/iter  %.3f us/iter (event)  max|LL^T-A| = %.2e\n", name, c, ms * 1e3 / reps, e);
}

int main() {
    static double h[NB * NB];
    for (int i = 0; i < NB; ++i)
        for (int j = 0; j < NB; ++j) h[i * NB + j] = (i == j ? NB : 0.0) + 1.0 / (1.0 + i + j);
    double *dA, *dO; long long* dc;
    (void)hipMalloc(&dA, sizeof(h)); (void)hipMalloc(&dO, sizeof(h)); (void)hipMalloc(&dc, 64);
    (void)hipMemcpy(dA, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>("wave potrf (readlane)", dA, dO, dc, h);
    run<1>("wave potrf (ds_swizzle)", dA, dO, dc, h);
    return 0;
}
