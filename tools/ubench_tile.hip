// Diagnostic micro-benchmark (not part of libmfgp.so): latency of the pieces on the
// k_chol_step critical path, each run REPS times inside ONE single-workgroup launch
// and timed with s_memtime (shader clock) + hipEvents.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
static double prev[64 * 64];
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"
using namespace mfgp;


// instrumented copy of tile_potrf_inv<32>'s pivot loop: per-phase shader clocks (wave 0)
__device__ void potrf_probe(double* A, double* R, long long* ph) {
    constexpr int NB = 32;
    constexpr int S = TileCfg<NB>::S;
    double* colb = R;
    double* rowb = R + 2 * NB;
    const int t = threadIdx.x;
    const int i = t >> 3, g = t & 7, c0 = 4 * g;
    double a[4], r[4];
    for (int q = 0; q < 4; ++q) { a[q] = A[i * S + c0 + q]; r[q] = (i == c0 + q) ? 1.0 : 0.0; }
    __syncthreads();
    if (g == 0) colb[i] = a[0];
    if (t < NB) rowb[t] = (t == 0) ? 1.0 : 0.0;
    __syncthreads();
    long long acc[5] = {0, 0, 0, 0, 0};
#pragma unroll 4
    for (int k = 0; k < NB; ++k) {
        const long long t0 = __builtin_amdgcn_s_memtime();
        const int cur = k & 1, nxt = cur ^ 1;
        const double akk = colb[cur * NB + k];
        const double aik = colb[cur * NB + i];
        const double2 ca = *reinterpret_cast<const double2*>(colb + cur * NB + c0);
        const double2 cb = *reinterpret_cast<const double2*>(colb + cur * NB + c0 + 2);
        const double2 ra = *reinterpret_cast<const double2*>(rowb + cur * NB + c0);
        const double2 rb = *reinterpret_cast<const double2*>(rowb + cur * NB + c0 + 2);
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        const long long t1 = __builtin_amdgcn_s_memtime();
        const double inv = rcp_nr(akk);
        const double sA = aik * inv;
        const double sR = (i > k) ? sA : 0.0;
        a[0] -= sA * ca.x; a[1] -= sA * ca.y; a[2] -= sA * cb.x; a[3] -= sA * cb.y;
        r[0] -= sR * ra.x; r[1] -= sR * ra.y; r[2] -= sR * rb.x; r[3] -= sR * rb.y;
        const int k1 = k + 1, q1 = k1 & 3;
        const double v = (q1 == 0) ? a[0] : (q1 == 1) ? a[1] : (q1 == 2) ? a[2] : a[3];
        const bool own = (k1 >> 2) == g;
        __builtin_amdgcn_s_waitcnt(0);
        const long long t2 = __builtin_amdgcn_s_memtime();
        colb[own ? nxt * NB + i : 4 * NB + t] = (i >= k1) ? v : 0.0;
        if (i == k1) *reinterpret_cast<double4*>(rowb + nxt * NB + c0) = double4{r[0], r[1], r[2], r[3]};
        __builtin_amdgcn_s_waitcnt(0xc07f);
        const long long t3 = __builtin_amdgcn_s_memtime();
        __syncthreads();
        const long long t4 = __builtin_amdgcn_s_memtime();
        acc[0] += t1 - t0; acc[1] += t2 - t1; acc[2] += t3 - t2; acc[3] += t4 - t3;
    }
    if (t == 0) for (int q = 0; q < 4; ++q) ph[q] = acc[q];
}

template <int ABL>
__device__ __forceinline__ void k4_abl(double* A, double* R, double* dg, int* bad, long long* st) {
    constexpr int NB = 32;
    constexpr int S = TileCfg<NB>::S;
    double* colb = R;                 // [2][NB][4]
    double* rowb = R + 2 * NB * 4;    // [2][4][NB]
    double* piv = R + 4 * NB * 4;     // [NB]
    const int t = threadIdx.x;
    const int i = t >> 3, g = t & 7, c0 = 4 * g;
    double a[4], r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a[q] = A[i * S + c0 + q];
        r[q] = (i == c0 + q) ? 1.0 : 0.0;
    }
    __syncthreads();
    if (g == 0) {
        *reinterpret_cast<double2*>(colb + i * 4) = double2{a[0], a[1]};
        *reinterpret_cast<double2*>(colb + i * 4 + 2) = double2{a[2], a[3]};
    }
    if (i < 4) {
        *reinterpret_cast<double2*>(rowb + i * NB + c0) = double2{r[0], r[1]};
        *reinterpret_cast<double2*>(rowb + i * NB + c0 + 2) = double2{r[2], r[3]};
    }
    __syncthreads();
#pragma unroll 2
    for (int rd = 0; rd < NB / 4; ++rd) {
        const int k = 4 * rd, cur = rd & 1, nxt = cur ^ 1;
        const double* C = colb + cur * NB * 4;
        const double* RP = rowb + cur * 4 * NB;
        double M[4][4], Ci[4], Cj[4][4], Rp[4][4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const double2 u = *reinterpret_cast<const double2*>(C + (k + p) * 4);
            const double2 w = *reinterpret_cast<const double2*>(C + (k + p) * 4 + 2);
            M[p][0] = u.x; M[p][1] = u.y; M[p][2] = w.x; M[p][3] = w.y;
        }
        {
            const double2 u = *reinterpret_cast<const double2*>(C + i * 4);
            const double2 w = *reinterpret_cast<const double2*>(C + i * 4 + 2);
            Ci[0] = u.x; Ci[1] = u.y; Ci[2] = w.x; Ci[3] = w.y;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double2 u = *reinterpret_cast<const double2*>(C + (c0 + q) * 4);
            const double2 w = *reinterpret_cast<const double2*>(C + (c0 + q) * 4 + 2);
            Cj[q][0] = u.x; Cj[q][1] = u.y; Cj[q][2] = w.x; Cj[q][3] = w.y;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const double2 u = *reinterpret_cast<const double2*>(RP + m * NB + c0);
            const double2 w = *reinterpret_cast<const double2*>(RP + m * NB + c0 + 2);
            Rp[m][0] = u.x; Rp[m][1] = u.y; Rp[m][2] = w.x; Rp[m][3] = w.y;
        }
        long long q0 = 0, q1 = 0, q2 = 0, q3 = 0, q4 = 0;
        if (ABL == 4) { q0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_s_waitcnt(0xc07f); q1 = __builtin_amdgcn_s_memtime(); }
        // LDL^T of the pivot block (lower entries): u_ab = L_ab d_b = e_ab
        const double d0 = M[0][0];
        const double i0 = (ABL == 1 ? 0.5 : rcp_nr(d0));
        const double L10 = M[1][0] * i0, L20 = M[2][0] * i0, L30 = M[3][0] * i0;
        const double d1 = M[1][1] - L10 * M[1][0];
        const double i1 = (ABL == 1 ? 0.5 : rcp_nr(d1));
        const double e21 = M[2][1] - L20 * M[1][0];
        const double e31 = M[3][1] - L30 * M[1][0];
        const double L21 = e21 * i1, L31 = e31 * i1;
        const double d2 = M[2][2] - L20 * M[2][0] - L21 * e21;
        const double i2 = (ABL == 1 ? 0.5 : rcp_nr(d2));
        const double e32 = M[3][2] - L30 * M[2][0] - L31 * e21;
        const double L32 = e32 * i2;
        const double d3 = M[3][3] - L30 * M[3][0] - L31 * e31 - L32 * e32;
        const double i3 = (ABL == 1 ? 0.5 : rcp_nr(d3));
        // w = C_i M^{-1} = ((C_i L^{-T}) D^{-1}) L^{-1}
        const double y0 = Ci[0];
        const double y1 = Ci[1] - L10 * y0;
        const double y2 = Ci[2] - L20 * y0 - L21 * y1;
        const double y3 = Ci[3] - L30 * y0 - L31 * y1 - L32 * y2;
        const double w3 = y3 * i3;
        const double w2 = y2 * i2 - L32 * w3;
        const double w1 = y1 * i1 - L21 * w2 - L31 * w3;
        const double w0 = y0 * i0 - L10 * w1 - L20 * w2 - L30 * w3;
        // pivot rows of R: R_P <- L^{-1} R_P, i.e. v = -(L^{-1})_{p, m<p}
        const double N10 = -L10;
        const double N21 = -L21, N20 = -(L20 + L21 * N10);
        const double N32 = -L32, N31 = -(L31 + L32 * N21), N30 = -(L30 + L31 * N10 + L32 * N20);
        if (ABL == 4) { asm volatile("" :: "v"(w0), "v"(N30)); q2 = __builtin_amdgcn_s_memtime(); }
        const int pr = i - k;
        double v0 = w0, v1 = w1, v2 = w2, v3 = w3;
        if (pr >= 0 && pr < 4) {
            v0 = (pr == 1) ? -N10 : (pr == 2) ? -N20 : (pr == 3) ? -N30 : 0.0;
            v1 = (pr == 2) ? -N21 : (pr == 3) ? -N31 : 0.0;
            v2 = (pr == 3) ? -N32 : 0.0;
            v3 = 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4 && ABL != 3; ++q) {
            a[q] -= w0 * Cj[q][0] + w1 * Cj[q][1] + w2 * Cj[q][2] + w3 * Cj[q][3];
            r[q] -= v0 * Rp[0][q] + v1 * Rp[1][q] + v2 * Rp[2][q] + v3 * Rp[3][q];
        }
        if (ABL == 4) { asm volatile("" :: "v"(a[0]), "v"(a[3]), "v"(r[0]), "v"(r[3])); q3 = __builtin_amdgcn_s_memtime(); }
        if (t == 0) {
            piv[k] = d0; piv[k + 1] = d1; piv[k + 2] = d2; piv[k + 3] = d3;
        }
        if (ABL != 2 && rd + 1 < NB / 4) {
            const int kn = k + 4;
            double* Cn = colb + nxt * NB * 4;
            double* Rn = rowb + nxt * 4 * NB;
            if (g == rd + 1) {
                const bool z = i < kn;
                *reinterpret_cast<double2*>(Cn + i * 4) = double2{z ? 0.0 : a[0], z ? 0.0 : a[1]};
                *reinterpret_cast<double2*>(Cn + i * 4 + 2) = double2{z ? 0.0 : a[2], z ? 0.0 : a[3]};
            }
            if (i >= kn && i < kn + 4) {
                *reinterpret_cast<double2*>(Rn + (i - kn) * NB + c0) = double2{r[0], r[1]};
                *reinterpret_cast<double2*>(Rn + (i - kn) * NB + c0 + 2) = double2{r[2], r[3]};
            }
        }
        if (ABL == 4) { __builtin_amdgcn_s_waitcnt(0xc07f); q4 = __builtin_amdgcn_s_memtime(); }
        __syncthreads();
        if (ABL == 4 && t == 0) st[rd] = __builtin_amdgcn_s_memtime();
        if (ABL == 4 && t == 0 && rd == 3) { st[10] = q1 - q0; st[11] = q2 - q1; st[12] = q3 - q2; st[13] = q4 - q3; }
    }
    if (ABL == 4 && t == 0) st[8] = __builtin_amdgcn_s_memtime();
    const double di = piv[i];
    if (t == 0) {
        int b = 0;
        for (int k = 0; k < NB && !b; ++k)
            if (!(piv[k] > 0.0 && piv[k] < INFINITY)) b = k + 1;
        *bad = b;
    }
    __syncthreads();
    const double li = sqrt(di);
    const double rli = 1.0 / li;
    if (g == 0) dg[i] = li;
#pragma unroll
    for (int q = 0; q < 4; ++q) R[i * S + c0 + q] = (c0 + q <= i) ? r[q] * rli : 0.0;
    __syncthreads();
}


template <int NB, int WHAT>
__global__ __launch_bounds__(256) void k_bench(const double* Ag, double* out, long long* cyc, int reps) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem; double* R = A + E; double* B = R + E; double* dg = B + E;
    int& bad = *reinterpret_cast<int*>(dg + NB);
    long long t0 = 0, t1 = 0;
    Acc<NB> acc; acc_zero(acc);
    for (int it = 0; it < reps; ++it) {
        tile_load<NB>(A, Ag, NB);
        tile_load<NB>(B, Ag, NB);
        __syncthreads();
        if (it == 1) t0 = __builtin_amdgcn_s_memtime();
        if (WHAT == 0) tile_potrf_inv<NB>(A, R, dg, &bad);
        if (WHAT == 1) { tile_mma<NB, false, true>(acc, A, B, 1.0); __syncthreads(); }
        if (WHAT == 2) { __syncthreads(); }
        if (WHAT == 3) { for (int k = 0; k < NB; ++k) __syncthreads(); }
        __shared__ long long st[2];
        if (WHAT == 6 && NB == 32) { potrf_probe(A, R, (long long*)(dg + NB + 2)); if (threadIdx.x == 0 && it == reps - 1) for (int q = 0; q < 4; ++q) cyc[4 + q] = ((long long*)(dg + NB + 2))[q]; }
        if (WHAT == 7 && NB == 32) tile_potrf_inv_k4(A, R, dg, &bad);
        __shared__ long long stk[14];
        if (WHAT == 8 && NB == 32) k4_abl<1>(A, R, dg, &bad, stk);
        if (WHAT == 9 && NB == 32) k4_abl<2>(A, R, dg, &bad, stk);
        if (WHAT == 10 && NB == 32) k4_abl<3>(A, R, dg, &bad, stk);
        if (WHAT == 11 && NB == 32) { if (threadIdx.x == 0) stk[9] = __builtin_amdgcn_s_memtime(); k4_abl<4>(A, R, dg, &bad, stk);
            if (threadIdx.x == 0 && it == reps - 1) for (int q = 0; q < 14; ++q) cyc[4 + q] = stk[q]; }
        if (WHAT == 4) { tile_potrf_inv_b8<NB>(A, R, dg, &bad, st); if (threadIdx.x == 0 && it == reps - 1) { cyc[1] = st[0]; cyc[2] = st[1]; } }
        if (it == reps - 1) t1 = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) { cyc[0] = (t1 - t0) / (reps - 2); if (WHAT == 4) { cyc[3] = t1; } }
    if (WHAT == 1) acc_store(acc, out, NB);
    if (WHAT == 0 || WHAT == 4 || WHAT == 7) tile_store<NB>(out, NB, R);
}

template <int NB, int WHAT>
void run(const char* name, const double* dA, double* dO, long long* dc) {
    const int reps = 50;
    size_t sm = sizeof(double) * (3 * NB * (NB + 2) + NB + 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL((k_bench<NB, WHAT>), dim3(1), dim3(256), sm, 0, dA, dO, dc, reps);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_bench<NB, WHAT>), dim3(1), dim3(256), sm, 0, dA, dO, dc, reps);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    long long c; hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    if (WHAT == 11) { long long cc[18]; hipMemcpy(cc, dc, sizeof(cc), hipMemcpyDeviceToHost);
        printf("    k4 round ends (clk from start):"); for (int q = 0; q < 9; ++q) printf(" %lld", cc[4 + q] - cc[13]);
        printf("\n    round 3 (thread 0): reads-wait %lld | LDLt+w %lld | select+update %lld | publish+wait %lld\n", cc[14], cc[15], cc[16], cc[17]); }
    if (WHAT == 6) { long long cc[8]; hipMemcpy(cc, dc, sizeof(cc), hipMemcpyDeviceToHost);
        printf("    per-pivot phases (sum over 32 pivots): reads %lld | compute %lld | write %lld | barrier %lld clk\n", cc[4], cc[5], cc[6], cc[7]); }
    if (WHAT == 4) { long long cc[4]; hipMemcpy(cc, dc, sizeof(cc), hipMemcpyDeviceToHost);
        printf("    last iter: factor-phase end -> diag-inv end %lld clk, diag-inv end -> t1 %lld clk\n", cc[2] - cc[1], cc[3] - cc[2]); }
    if (WHAT == 0 || WHAT == 4 || WHAT == 7) {
        static double cur[64 * 64];
        hipMemcpy(cur, dO, sizeof(double) * NB * NB, hipMemcpyDeviceToHost);
        printf("    D[0][0]=%.6f D[1][0]=%.6f D[1][1]=%.6f D[31][0]=%.6e D[0][1]=%.3e D[31][31]=%.6f\n", cur[0], cur[NB], cur[NB+1], cur[31*NB], cur[1], cur[31*NB+31]);
        if (WHAT != 0) {
            double e = 0;
            for (int i = 0; i < NB * NB; ++i) e = fmax(e, fabs(cur[i] - prev[i]));
            printf("    max |D - D_pivot| = %.3e\n", e);
        } else memcpy(prev, cur, sizeof(double) * NB * NB);
    }
    printf("%-28s NB=%d  %8lld shader-clk/iter (s_memtime)   %.3f us/iter (event, incl. 2 tile loads)\n", name, NB, c,
           ms * 1e3 / reps);
}

int main() {
    const int NBm = 64;
    double* h = (double*)malloc(sizeof(double) * NBm * NBm);
    for (int nb : {32, 64}) {
        for (int i = 0; i < nb; ++i)
            for (int j = 0; j < nb; ++j) h[i * nb + j] = (i == j ? nb : 0.0) + 1.0 / (1.0 + i + j);
        double *dA, *dO; long long* dc;
        hipMalloc(&dA, sizeof(double) * nb * nb); hipMalloc(&dO, sizeof(double) * nb * nb); hipMalloc(&dc, 256);
        hipMemcpy(dA, h, sizeof(double) * nb * nb, hipMemcpyHostToDevice);
        if (nb == 32) {
            run<32, 6>("potrf probe", dA, dO, dc); run<32, 0>("tile_potrf_inv", dA, dO, dc); run<32, 4>("tile_potrf_inv_b8", dA, dO, dc); run<32, 7>("tile_potrf_inv_k4", dA, dO, dc); run<32, 8>("k4: no rcp", dA, dO, dc); run<32, 9>("k4: no publish", dA, dO, dc); run<32, 10>("k4: no update", dA, dO, dc); run<32, 11>("k4: stamps", dA, dO, dc); run<32, 1>("tile_mma (A B^T)", dA, dO, dc);
            run<32, 2>("1 barrier + loads", dA, dO, dc); run<32, 3>("NB barriers", dA, dO, dc);
        } else {
            run<64, 0>("tile_potrf_inv", dA, dO, dc); run<64, 4>("tile_potrf_inv_b8", dA, dO, dc); run<64, 1>("tile_mma (A B^T)", dA, dO, dc);
            run<64, 2>("1 barrier + loads", dA, dO, dc); run<64, 3>("NB barriers", dA, dO, dc);
        }
        hipFree(dA); hipFree(dO); hipFree(dc);
    }
    return 0;
}
