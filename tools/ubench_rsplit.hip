// Diagnostic: the NB = 32 diagonal factor split over two waves (tile_elim_w1_wave on the A wave,
// tile_rinv_w1_wave on an R wave, mfgp_device.h) against the fused single-wave
// tile_potrf_inv_w1_wave.  Reports clocks from the start to the A wave's last publish and to D
// written, checks D / L_ii bitwise against the fused factor, and repeats with a load wave issuing
// f64 MFMAs on the R wave's SIMD (the flow's band helpers share it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I multi_fidelity_gpflow_amd/csrc tools/ubench_rsplit.hip -o /tmp/ubr
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "mfgp_device.h"
using namespace mfgp;
constexpr int NB = 32;

// V 0: fused (wave 0).  V 1: split, R on wave RW.  V 2: split + a load wave (LW) on the R wave's SIMD.
// V 3: split, the inverse by halves: Ra on wave RW, Rb on wave LW (D done: Rb's end).
template <int V, int RW, int LW>
__global__ __launch_bounds__(512) void k_fac(const double* Ag, double* Rg, double* dgg, long long* cyc, int* badg,
                                             int reps, int nload) {
    constexpr int S = TileCfg<NB>::S, E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* X = smem;                 // 32 x 33
    double* Pn = X + 32 * 33;         // 8 x 128 panels
    double* Zb = Pn + 1024;           // 8 x 128 round z
    double* dpv = Zb + 1024;          // 104
    double* R = dpv + 128;            // E
    double* dg = R + E;               // 32
    int* bad = reinterpret_cast<int*>(dg + 32);
    int* prog = bad + 2;
    int* tw = bad + 3;
    double* Tb = dg + 64;             // 16 x 17
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (threadIdx.x == 0) { *prog = 0; *tw = 0; }
    long long ta = 0, td = 0;
    f64x4 junk = {0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < reps; ++it) {
        for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) X[(e >> 5) * 33 + (e & 31)] = Ag[e];
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        if (V == 0) {
            if (w == 0) tile_potrf_inv_w1_wave(X, 33, Pn, R, dg, bad);
        } else {
            if (w == 0) tile_elim_w1_wave(X, 33, Pn, Zb, dpv, prog, 8 * it);
            if (w == 0 && it > 0) ta += __builtin_amdgcn_s_memtime() - t0;
            if (V != 3 && w == RW) tile_rinv_w1_wave(Zb, prog, 8 * it, dpv, R, dg, bad);
            if (V == 3 && w == RW) tile_rinv_lo_w1_wave(Zb, prog, 8 * it, dpv, R, Tb, tw, it + 1);
            if (V == 3 && w == LW) tile_rinv_hi_w1_wave(Zb, prog, 8 * it, dpv, R, Tb, tw, it + 1, dg, bad);
            if (V == 2 && w == LW) {
                for (int q = 0; q < nload; ++q)
                    junk = __builtin_amdgcn_mfma_f64_16x16x4f64((double)l, 1.0, junk, 0, 0, 0);
            }
        }
        if ((V == 0 && w == 0) || (V != 0 && V != 3 && w == RW) || (V == 3 && w == LW)) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (it > 0) td += __builtin_amdgcn_s_memtime() - t0;
        }
        __syncthreads();
    }
    if (V == 2 && junk[0] == 12345.0) cyc[15] = 1;
    tile_store<NB>(Rg, NB, R);
    if (threadIdx.x < NB) dgg[threadIdx.x] = dg[threadIdx.x];
    if (threadIdx.x == 0) { badg[0] = *bad; }
    if ((V == 0 && w == 0 && l == 0) || (V != 0 && V != 3 && w == RW && l == 0) || (V == 3 && w == LW && l == 0))
        cyc[1] = td / (reps - 1);
    if (V != 0 && w == 0 && l == 0) cyc[0] = ta / (reps - 1);
}

static void host_ref(const double* A, long double* Linv, long double* Ld) {
    long double L[NB][NB] = {};
    for (int j = 0; j < NB; ++j) {
        long double s = A[j * NB + j];
        for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
        L[j][j] = sqrtl(s);
        for (int i = j + 1; i < NB; ++i) {
            long double t = A[i * NB + j];
            for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
            L[i][j] = t / L[j][j];
        }
    }
    for (int i = 0; i < NB; ++i) Ld[i] = L[i][i];
    for (int c = 0; c < NB; ++c)
        for (int i = 0; i < NB; ++i) {
            long double s = (i == c) ? 1.0L : 0.0L;
            for (int k = c; k < i; ++k) s -= L[i][k] * Linv[k * NB + c];
            Linv[i * NB + c] = (i < c) ? 0.0L : s / L[i][i];
        }
}

static double Rref[NB * NB], dref[NB];
template <int V, int RW, int LW>
static void run(const char* name, const double* hA, const double* dA, double* dR, double* dd, long long* dc, int* db,
                int nload) {
    const size_t sm = sizeof(double) * (32 * 33 + 2048 + 128 + TileCfg<NB>::ELEMS + 64 + 16 * 17 + 8);
    (void)hipMemset(dc, 0, 128);
    hipLaunchKernelGGL((k_fac<V, RW, LW>), dim3(1), dim3(512), sm, 0, dA, dR, dd, dc, db, 50, nload);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
    double R[NB * NB], dg[NB];
    long long c[16] = {};
    int b[4];
    (void)hipMemcpy(R, dR, sizeof(R), hipMemcpyDeviceToHost);
    (void)hipMemcpy(dg, dd, sizeof(dg), hipMemcpyDeviceToHost);
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(b, db, sizeof(b), hipMemcpyDeviceToHost);
    static long double Li[NB * NB], Ld[NB];
    host_ref(hA, Li, Ld);
    long double eR = 0, mR = 0, eD = 0;
    for (int i = 0; i < NB * NB; ++i) { eR = fmaxl(eR, fabsl(R[i] - Li[i])); mR = fmaxl(mR, fabsl(Li[i])); }
    for (int i = 0; i < NB; ++i) eD = fmaxl(eD, fabsl(dg[i] - Ld[i]) / Ld[i]);
    bool same = true;
    if (V == 0) { memcpy(Rref, R, sizeof(R)); memcpy(dref, dg, sizeof(dg)); }
    else same = memcmp(Rref, R, sizeof(R)) == 0 && memcmp(dref, dg, sizeof(dg)) == 0;
    unsigned long long hsh = 1469598103934665603ull;
    for (int i = 0; i < NB * NB; ++i) { unsigned long long b; memcpy(&b, &R[i], 8); hsh = (hsh ^ b) * 1099511628211ull; }
    for (int i = 0; i < NB; ++i) { unsigned long long b; memcpy(&b, &dg[i], 8); hsh = (hsh ^ b) * 1099511628211ull; }
    printf("  [bits %016llx] ", hsh);
    printf("%-26s A done %6lld clk  D done %6lld clk  err D %.2e  L_ii %.2e  bad=%d  %s\n", name, c[0], c[1],
           (double)(eR / mR), (double)eD, b[0], V == 0 ? "(reference bits)" : (same ? "bitwise = fused" : "bits differ from fused (rounding)"));
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    double hA[2][NB * NB];
    srand(7);
    double x[NB][10];
    for (int i = 0; i < NB; ++i) for (int d = 0; d < 10; ++d) x[i][d] = rand() / (double)RAND_MAX;
    for (int i = 0; i < NB; ++i)
        for (int j = 0; j < NB; ++j) {
            double r2 = 0;
            for (int d = 0; d < 10; ++d) r2 += (x[i][d] - x[j][d]) * (x[i][d] - x[j][d]);
            hA[0][i * NB + j] = exp(-0.5 * r2) + (i == j ? 1e-3 : 0.0);
            const double t = (x[i][0] - x[j][0]) / 0.5;
            hA[1][i * NB + j] = exp(-0.5 * t * t) + (i == j ? 1e-6 : 0.0);
        }
    double *dA, *dR, *dd;
    long long* dc;
    int* db;
    (void)hipMalloc(&dA, sizeof(hA)); (void)hipMalloc(&dR, 8 * NB * NB); (void)hipMalloc(&dd, 8 * NB);
    (void)hipMalloc(&dc, 128); (void)hipMalloc(&db, 128);
    (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    for (int m = 0; m < 2; ++m) {
        printf("tile %d (%s)\n", m, m == 0 ? "10-D RBF + 1e-3 I" : "1-D RBF l=0.5 + 1e-6 I");
        const double* a = dA + m * NB * NB;
        run<0, 0, 0>("fused w1", hA[m], a, dR, dd, dc, db, 0);
        run<1, 1, 0>("split, R on wave 1", hA[m], a, dR, dd, dc, db, 0);
        run<1, 2, 0>("split, R on wave 2", hA[m], a, dR, dd, dc, db, 0);
        run<1, 4, 0>("split, R on wave 4 (SIMD 0)", hA[m], a, dR, dd, dc, db, 0);
        run<2, 1, 5>("split + 32 MFMA load", hA[m], a, dR, dd, dc, db, 32);
        run<2, 1, 5>("split + 64 MFMA load", hA[m], a, dR, dd, dc, db, 64);
        run<2, 1, 5>("split + 128 MFMA load", hA[m], a, dR, dd, dc, db, 128);
        run<3, 1, 2>("halves Ra w1 Rb w2", hA[m], a, dR, dd, dc, db, 0);
        run<3, 1, 3>("halves Ra w1 Rb w3", hA[m], a, dR, dd, dc, db, 0);
        run<3, 5, 6>("halves + SIMD sharers", hA[m], a, dR, dd, dc, db, 0);
    }
    return 0;
}
