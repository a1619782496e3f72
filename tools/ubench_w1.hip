// Diagnostic: NB = 32 diagonal-tile Cholesky + inverse, the 4-wave MFMA 4-pivot form (m4) vs
// the single-wave form (w1), both from an LDS tile and from the accumulator layout.
// Checks D = L^{-1} and L_ii against a long-double host factorisation of the same tile.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "factor_variants.h"
using namespace mfgp;
constexpr int NB = 32;

template <int V>
__global__ __launch_bounds__(256) void k_fac(const double* Ag, double* Rg, double* dgg, long long* cyc, int* badg,
                                             int reps, long long* trg) {
    constexpr int S = TileCfg<NB>::S, E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem;
    double* R = A + E;
    double* dg = R + E;
    int* bad = reinterpret_cast<int*>(dg + NB + 2);
    double* ws = dg + NB + 8;
    long long tsum = 0, atsum = 0;
    int* flag = reinterpret_cast<int*>(ws + W2_WS + 128);
    if (threadIdx.x == 0) { flag[0] = 0; flag[1] = 0; flag[2] = 0; }
    for (int it = 0; it < reps; ++it) {
        tile_load<NB>(A, Ag, NB);
        __syncthreads();
        f64x4 aA;
        {
            const int w = threadIdx.x >> 6, l = threadIdx.x & 63, bi = w >> 1, bj = w & 1;
#pragma unroll
            for (int q = 0; q < 4; ++q) aA[q] = A[(16 * bi + (l >> 4) + 4 * q) * S + 16 * bj + (l & 15)];
        }
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        if (V == 0) tile_potrf_inv_m4(A, R, dg, bad);
        if (V == 1) tile_potrf_inv_w1(A, R, dg, bad);
        if (V == 2) tile_potrf_inv_m4_acc(aA, A, R, dg, bad);
        if (V == 3) tile_potrf_inv_w1_acc(aA, A, R, dg, bad);
        if (V == 4) tile_potrf_inv_w2_acc(aA, ws, R, dg, bad);
        if (V == 5) {
            const int w = threadIdx.x >> 6;
            if (w == 0) {
                tile_potrf_inv_s2_a(A, S, A, flag, 8 * it, it == reps - 1 ? trg : nullptr);
                if (it == reps - 1 && threadIdx.x == 0) trg[24] = t0;
                const long long ta = __builtin_amdgcn_s_memtime();
                if (it > 0 && threadIdx.x == 0) atsum += ta - t0;
            }
            if (w == 1) tile_potrf_inv_s2_l(A, ws + W2_WS, flag, flag + 2, 8 * it);
            if (w == 2) tile_potrf_inv_s2_r(A, ws + W2_WS, flag + 2, flag + 1, 8 * it, ws + W2_WS + 136, R,
                                            it == reps - 1 ? trg : nullptr);
            if (w == 3) tile_potrf_inv_s2_s(ws + W2_WS, flag + 2, flag + 1, 8 * it, ws + W2_WS + 136, dg, bad);
            __syncthreads();
        }
        const long long t1 = __builtin_amdgcn_s_memtime();
        if (V == 5 && it == reps - 1 && threadIdx.x == 0) trg[25] = t1;
        if (it > 0) tsum += t1 - t0;
        __syncthreads();
    }
    tile_store<NB>(Rg, NB, R);
    if (threadIdx.x < NB) dgg[threadIdx.x] = dg[threadIdx.x];
    if (threadIdx.x == 0) { cyc[V] = tsum / (reps - 1); badg[V] = *bad; if (V == 5) cyc[6] = atsum / (reps - 1); }
    if (V == 5 && (threadIdx.x & 63) == 0) cyc[7 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
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

static long long* g_tr;
template <int V>
static void run(const char* name, const double* hA, const double* dA, double* dR, double* dd, long long* dc, int* db) {
    const size_t sm = sizeof(double) * (2 * TileCfg<NB>::ELEMS + NB + 8 + W2_WS + 176);
    hipLaunchKernelGGL(k_fac<V>, dim3(1), dim3(256), sm, 0, dA, dR, dd, dc, db, 50, g_tr);
    (void)hipDeviceSynchronize();
    double R[NB * NB], dg[NB];
    long long c[16] = {};
    int b[8];
    (void)hipMemcpy(R, dR, sizeof(R), hipMemcpyDeviceToHost);
    (void)hipMemcpy(dg, dd, sizeof(dg), hipMemcpyDeviceToHost);
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(b, db, sizeof(b), hipMemcpyDeviceToHost);
    static long double Li[NB * NB], Ld[NB];
    host_ref(hA, Li, Ld);
    long double eR = 0, mR = 0, eD = 0;
    for (int i = 0; i < NB * NB; ++i) { eR = fmaxl(eR, fabsl(R[i] - Li[i])); mR = fmaxl(mR, fabsl(Li[i])); }
    for (int i = 0; i < NB; ++i) eD = fmaxl(eD, fabsl(dg[i] - Ld[i]) / Ld[i]);
    if (V == 5) {
        long long tr[32];
        (void)hipMemcpy(tr, g_tr, sizeof(tr), hipMemcpyDeviceToHost);
        printf("    (t1 - t0 of the traced rep: %lld)\n", tr[25] - tr[24]);
        for (int k = 0; k < 8; ++k)
            printf("    round %d: A flag %6lld   R sees %6lld   R done %6lld\n", k, tr[k] - tr[24], tr[8 + k] - tr[24],
                   tr[16 + k] - tr[24]);
    }
    if (V == 5) printf("  (A wave alone: %lld clk; HW_ID simd of waves 0-3: %lld %lld %lld %lld)\n", c[6],
                       (c[7] >> 4) & 3, (c[8] >> 4) & 3, (c[9] >> 4) & 3, (c[10] >> 4) & 3);
    printf("%-10s %7lld clk  max|D-Dref|/max|Dref| = %.2e  max rel L_ii err = %.2e  bad=%d\n", name, c[V],
           (double)(eR / mR), (double)eD, b[V]);
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    // two test tiles: a 10-D RBF Gram (l = 1) + 1e-3 I, and a 1-D RBF Gram (l = 0.5) + 1e-6 I
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
    (void)hipMalloc(&dc, 128); (void)hipMalloc(&g_tr, 256); (void)hipMalloc(&db, 128);
    (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    for (int m = 0; m < 2; ++m) {
        printf("tile %d (%s)\n", m, m == 0 ? "10-D RBF + 1e-3 I" : "1-D RBF l=0.5 + 1e-6 I");
        run<0>("m4 lds", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<1>("w1 lds", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<2>("m4 acc", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<3>("w1 acc", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<4>("w2 acc", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<5>("s2 lds", hA[m], dA + m * NB * NB, dR, dd, dc, db);
    }
    return 0;
}
