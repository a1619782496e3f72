// Diagnostic: the tall-panel band wave (tile_band_w1_wave, mfgp_device.h) in lock-step with the
// publishing fused factor (tile_potrf_inv_w1_wave<true>).  Reports clocks to the factor's end and
// to the band's end, with the band chasing the factor from the start ("chase") or starting only
// once every round is published ("late"), checks L(k+1,k) = B L^{-T} and S = L L^T against a
// long-double host reference and the factor's D bitwise against the non-publishing factor.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I multi_fidelity_gpflow_amd/csrc tools/ubench_band.hip -o /tmp/ubb
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "mfgp_device.h"
using namespace mfgp;
constexpr int NB = 32;

// V 0: plain factor.  V 1: publishing factor + band on wave BW (LATE: band starts after the factor).
template <int V, int BW, bool LATE>
__global__ __launch_bounds__(512) void k_band(const double* Ag, const double* Bg, double* Rg, double* dgg, double* Lg,
                                              double* Sg, long long* cyc, int* badg, int reps) {
    constexpr int S = TileCfg<NB>::S, E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* X = smem;                 // 32 x 33
    double* Bs = X + 32 * 33;         // 32 x 33
    double* Pn = Bs + 32 * 33;        // 128 panel + 128 pivots (dpv = Pn + 128, the factor's own)
    double* Yb = Pn + 256;            // 8 x 128
    double* Fb = Yb + 1024;           // 8 x 16
    double* dpv = Fb + 128;           // 128
    double* Q = dpv + 128;            // 128
    double* R = Q + 128;              // E
    double* Lb = R + E;               // E
    double* Sb = Lb + E;              // E
    double* dg = Sb + E;              // 32
    int* bad = reinterpret_cast<int*>(dg + 32);
    int* prog = bad + 2;
    int* done = bad + 3;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (threadIdx.x == 0) { *prog = 0; *done = 0; }
    long long tf = 0, tb = 0;
    for (int it = 0; it < reps; ++it) {
        for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
            X[(e >> 5) * 33 + (e & 31)] = Ag[e];
            Bs[(e >> 5) * 33 + (e & 31)] = Bg[e];
        }
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        if (V == 0) {
            if (w == 0) tile_potrf_inv_w1_wave(X, 33, Pn, R, dg, bad);
        } else {
            if (w == 0) {
                W1Pub pub{Yb, Fb, prog, 8 * it};
                tile_potrf_inv_w1_wave<true>(X, 33, Pn, R, dg, bad, pub);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (l == 0) __hip_atomic_store(done, it + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (w == BW) {
                if (LATE)
                    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < it + 1) {}
                tile_band_w1_wave(Bs, 33, Yb, Fb, Pn + 128, prog, 8 * it, Q, Lb, S, Sb, S);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (it > 0) tb += __builtin_amdgcn_s_memtime() - t0;
            }
        }
        if (w == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (it > 0) tf += __builtin_amdgcn_s_memtime() - t0;
        }
        __syncthreads();
    }
    tile_store<NB>(Rg, NB, R);
    if (V) { tile_store<NB>(Lg, NB, Lb); tile_store<NB>(Sg, NB, Sb); }
    if (threadIdx.x < NB) dgg[threadIdx.x] = dg[threadIdx.x];
    if (threadIdx.x == 0) badg[0] = *bad;
    if (w == 0 && l == 0) cyc[0] = tf / (reps - 1);
    if (w == BW && l == 0) cyc[1] = tb / (reps - 1);
}

static void host_chol(const double* A, long double (*L)[NB]) {
    for (int j = 0; j < NB; ++j) {
        long double s = A[j * NB + j];
        for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
        L[j][j] = sqrtl(s);
        for (int i = j + 1; i < NB; ++i) {
            long double t = A[i * NB + j];
            for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
            L[i][j] = t / L[j][j];
        }
        for (int i = 0; i < j; ++i) L[i][j] = 0;
    }
}

static double Rref[NB * NB];
template <int V, int BW, bool LATE>
static void run(const char* name, const double* hA, const double* hB, const double* dA, const double* dB, double* dR,
                double* dd, double* dL, double* dS, long long* dc, int* db) {
    const size_t sm = sizeof(double) * (2 * 32 * 33 + 256 + 1024 + 128 + 128 + 128 + 3 * TileCfg<NB>::ELEMS + 32 + 8);
    (void)hipMemset(dc, 0, 128);
    hipLaunchKernelGGL((k_band<V, BW, LATE>), dim3(1), dim3(512), sm, 0, dA, dB, dR, dd, dL, dS, dc, db, 50);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
    double R[NB * NB], Lb[NB * NB], Sb[NB * NB];
    long long c[16] = {};
    (void)hipMemcpy(R, dR, sizeof(R), hipMemcpyDeviceToHost);
    (void)hipMemcpy(Lb, dL, sizeof(Lb), hipMemcpyDeviceToHost);
    (void)hipMemcpy(Sb, dS, sizeof(Sb), hipMemcpyDeviceToHost);
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    bool same = true;
    if (V == 0) memcpy(Rref, R, sizeof(R));
    else same = memcmp(Rref, R, sizeof(R)) == 0;
    double eL = 0, mL = 0, eS = 0, mS = 0;
    if (V) {
        static long double L[NB][NB], Lr[NB][NB];
        host_chol(hA, L);
        // Lr = B L^{-T}: row i solves Lr[i] L^T = B[i]
        for (int i = 0; i < NB; ++i)
            for (int j = 0; j < NB; ++j) {
                long double t = hB[i * NB + j];
                for (int k = 0; k < j; ++k) t -= Lr[i][k] * L[j][k];
                Lr[i][j] = t / L[j][j];
            }
        for (int i = 0; i < NB; ++i)
            for (int j = 0; j < NB; ++j) {
                eL = fmax(eL, (double)fabsl(Lb[i * NB + j] - Lr[i][j]));
                mL = fmax(mL, (double)fabsl(Lr[i][j]));
                if (j > i || (i < 16 && j >= 16)) continue;
                long double s = 0;
                for (int k = 0; k < NB; ++k) s += Lr[i][k] * Lr[j][k];
                eS = fmax(eS, (double)fabsl(Sb[i * NB + j] - s));
                mS = fmax(mS, (double)fabsl(s));
            }
    }
    printf("%-22s factor %6lld clk  band %6lld clk  err L %.2e  S %.2e  D %s\n", name, c[0], c[1], mL ? eL / mL : 0.0,
           mS ? eS / mS : 0.0, V == 0 ? "(reference)" : (same ? "bitwise = plain factor" : "DIFFERS"));
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    static double hA[NB * NB], hB[NB * NB];
    srand(11);
    double x[2 * NB][10];
    for (int i = 0; i < 2 * NB; ++i) for (int d = 0; d < 10; ++d) x[i][d] = rand() / (double)RAND_MAX;
    auto k = [&](int i, int j) {
        double r2 = 0;
        for (int d = 0; d < 10; ++d) r2 += (x[i][d] - x[j][d]) * (x[i][d] - x[j][d]);
        return exp(-0.5 * r2);
    };
    for (int i = 0; i < NB; ++i)
        for (int j = 0; j < NB; ++j) {
            hA[i * NB + j] = k(i, j) + (i == j ? 1e-3 : 0.0);
            hB[i * NB + j] = k(NB + i, j);
        }
    double *dA, *dB, *dR, *dd, *dL, *dS;
    long long* dc;
    int* db;
    (void)hipMalloc(&dA, sizeof(hA)); (void)hipMalloc(&dB, sizeof(hB)); (void)hipMalloc(&dR, 8 * NB * NB);
    (void)hipMalloc(&dd, 8 * NB); (void)hipMalloc(&dL, 8 * NB * NB); (void)hipMalloc(&dS, 8 * NB * NB);
    (void)hipMalloc(&dc, 128); (void)hipMalloc(&db, 128);
    (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
    run<0, 1, false>("plain factor", hA, hB, dA, dB, dR, dd, dL, dS, dc, db);
    run<1, 1, false>("pub + band chase w1", hA, hB, dA, dB, dR, dd, dL, dS, dc, db);
    run<1, 2, false>("pub + band chase w2", hA, hB, dA, dB, dR, dd, dL, dS, dc, db);
    run<1, 4, false>("pub + band chase w4", hA, hB, dA, dB, dR, dd, dL, dS, dc, db);
    run<1, 2, true>("pub + band late w2", hA, hB, dA, dB, dR, dd, dL, dS, dc, db);
    return 0;
}
