// Diagnostic micro-benchmark (not part of libmfgp.so): latency of the pieces on the
// k_chol_step critical path, each run REPS times inside ONE single-workgroup launch
// and timed with s_memtime (shader clock) + hipEvents.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
static double prev[64 * 64];
#include "factor_variants.h"
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


template <int RD, int ABL>
__device__ __forceinline__ void m4x_round(const M4Buf& B, f64x4& aA, f64x4& aR, int bi, int bj, int lc, int lr) {
    constexpr int NB = 32;
    if constexpr (RD < NB / 4) {
        constexpr int k = 4 * RD, cur = RD & 1, nxt = cur ^ 1;
        const double* C = B.colb + cur * NB * 4;
        const double* RP = B.rowb + cur * 4 * NB;
        const int ia = 16 * bi + lc;   // A-operand row of this lane
        const int cg = 16 * bj + lc;   // accumulator / B-operand column
        // ---- reads: pivot block (lower), own operand row, B operands
        const double2 r0a = *reinterpret_cast<const double2*>(C + (k + 0) * 4);
        const double2 r1a = *reinterpret_cast<const double2*>(C + (k + 1) * 4);
        const double2 r2a = *reinterpret_cast<const double2*>(C + (k + 2) * 4);
        const double2 r2b = *reinterpret_cast<const double2*>(C + (k + 2) * 4 + 2);
        const double2 r3a = *reinterpret_cast<const double2*>(C + (k + 3) * 4);
        const double2 r3b = *reinterpret_cast<const double2*>(C + (k + 3) * 4 + 2);
        const double2 cia = *reinterpret_cast<const double2*>(C + ia * 4);
        const double2 cib = *reinterpret_cast<const double2*>(C + ia * 4 + 2);
        const double bA = C[cg * 4 + lr];
        const double bR = RP[lr * NB + cg];
        const double m00 = r0a.x, m10 = r1a.x, m11 = r1a.y, m20 = r2a.x, m21 = r2a.y, m22 = r2b.x;
        const double m30 = r3a.x, m31 = r3a.y, m32 = r3b.x, m33 = r3b.y;
        // ---- M^{-1} by 2x2 blocks: P = M[0:2,0:2], Q = M[0:2,2:4], S = M[2:4,2:4]
        const double detP = fma(m00, m11, -m10 * m10);
        const double rP = rcp_nr(detP);
        const double P00 = m11 * rP, P01 = -m10 * rP, P11 = m00 * rP;
        const double X00 = fma(P00, m20, P01 * m21), X01 = fma(P00, m30, P01 * m31);
        const double X10 = fma(P01, m20, P11 * m21), X11 = fma(P01, m30, P11 * m31);
        const double S00 = m22 - fma(m20, X00, m21 * X10);
        const double S01 = m32 - fma(m20, X01, m21 * X11);
        const double S11 = m33 - fma(m30, X01, m31 * X11);
        const double detS = fma(S00, S11, -S01 * S01);
        const double rS = rcp_nr(detS);
        const double I00 = S11 * rS, I01 = -S01 * rS, I11 = S00 * rS;
        const double Y00 = fma(X00, I00, X01 * I01), Y01 = fma(X00, I01, X01 * I11);
        const double Y10 = fma(X10, I00, X11 * I01), Y11 = fma(X10, I01, X11 * I11);
        const double T00 = P00 + fma(Y00, X00, Y01 * X01);
        const double T01 = P01 + fma(Y00, X10, Y01 * X11);
        const double T11 = P11 + fma(Y10, X10, Y11 * X11);
        // ---- w = C_ia M^{-1}; this lane feeds w[lr]
        const double c0 = cia.x, c1 = cia.y, c2 = cib.x, c3 = cib.y;
        const double w0 = fma(c0, T00, fma(c1, T01, -fma(c2, Y00, c3 * Y01)));
        const double w1 = fma(c0, T01, fma(c1, T11, -fma(c2, Y10, c3 * Y11)));
        const double w2 = fma(c2, I00, fma(c3, I01, -fma(c0, Y00, c1 * Y10)));
        const double w3 = fma(c2, I01, fma(c3, I11, -fma(c0, Y01, c1 * Y11)));
        const double wl = (lr == 0) ? w0 : (lr == 1) ? w1 : (lr == 2) ? w2 : w3;
        double vl = wl;
        // ---- pivot rows of R: v = -(L_M^{-1})_{p, lr} for lr < p (wave-uniform branch)
        if (ABL != 1 && ABL != 3 && bi == (k >> 4)) {
            const int p = lc - (k & 15);
            if (p >= 0 && p < 4) {
                const double r0 = rcp_nr(m00);
                const double L10 = m10 * r0, L20 = m20 * r0, L30 = m30 * r0;
                const double id1 = m00 * rP;
                const double e21 = m21 - L20 * m10, e31 = m31 - L30 * m10;
                const double L21 = e21 * id1, L31 = e31 * id1;
                const double L32 = (m32 - L30 * m20 - L31 * e21) * rcp_nr(S00);
                const double N10 = -L10, N21 = -L21, N32 = -L32;
                const double N20 = -(L20 + L21 * N10);
                const double N31 = -(L31 + L32 * N21);
                const double N30 = -(L30 + L31 * N10 + L32 * N20);
                const double row1 = (lr == 0) ? N10 : 0.0;
                const double row2 = (lr == 0) ? N20 : (lr == 1) ? N21 : 0.0;
                const double row3 = (lr == 0) ? N30 : (lr == 1) ? N31 : (lr == 2) ? N32 : 0.0;
                vl = -((p == 1) ? row1 : (p == 2) ? row2 : (p == 3) ? row3 : 0.0);
            }
        }
        // ---- rank-4 updates on the matrix core
        aA = __builtin_amdgcn_mfma_f64_16x16x4f64(-wl, bA, aA, 0, 0, 0);
        aR = __builtin_amdgcn_mfma_f64_16x16x4f64(-vl, bR, aR, 0, 0, 0);
        if ((ABL == 0 || ABL == 1) && threadIdx.x == 0) {
            B.piv[k] = m00;
            B.piv[k + 1] = detP / m00;
            B.piv[k + 2] = S00;
            B.piv[k + 3] = detS / S00;
        }
        // ---- publish round RD+1
        if constexpr (RD + 1 < NB / 4) {
            constexpr int kn = k + 4;
            double* Cn = B.colb + nxt * NB * 4;
            double* Rn = B.rowb + nxt * 4 * NB;
            if (bj == (kn >> 4)) {
                const int m = lc - (kn & 15);
                if (m >= 0 && m < 4) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int rg = 16 * bi + lr + 4 * q;
                        Cn[rg * 4 + m] = (rg >= kn) ? aA[q] : 0.0;
                    }
                }
            }
            if (bi == (kn >> 4)) Rn[lr * NB + cg] = aR[((kn & 15) >> 2)];
        }
        __syncthreads();
        m4x_round<RD + 1, ABL>(B, aA, aR, bi, bj, lc, lr);
    }
}

template <int ABL>
__device__ __forceinline__ void m4x(double* A, double* R, double* dg, int* bad) {
    constexpr int NB = 32;
    constexpr int S = TileCfg<NB>::S;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int bi = w >> 1, bj = w & 1, lc = l & 15, lr = l >> 4;
    const int cg = 16 * bj + lc;
    f64x4 aA, aR;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int rg = 16 * bi + lr + 4 * q;
        aA[q] = A[rg * S + cg];
        aR[q] = (rg == cg) ? 1.0 : 0.0;
    }
    __syncthreads();   // A's LDS becomes the publish buffer
    const M4Buf B{A, A + 2 * NB * 4, A + 4 * NB * 4};
    if (bj == 0 && lc < 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) B.colb[(16 * bi + lr + 4 * q) * 4 + lc] = aA[q];
    }
    if (bi == 0) B.rowb[lr * NB + cg] = (lr == cg) ? 1.0 : 0.0;
    __syncthreads();
    m4x_round<0, ABL>(B, aA, aR, bi, bj, lc, lr);
    // D = diag(d)^{-1/2} L_u^{-1} (lower); dg = sqrt(d); first bad pivot by one ballot
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int rg = 16 * bi + lr + 4 * q;
        const double sc = 1.0 / sqrt(B.piv[rg]);
        R[rg * S + cg] = (cg <= rg) ? aR[q] * sc : 0.0;
    }
    if (t < 64) {
        const double d = (t < NB) ? B.piv[t] : 1.0;
        if (t < NB) dg[t] = sqrt(d);
        const unsigned long long m = __ballot(!(d > 0.0 && d < INFINITY));
        if (t == 0) *bad = m ? __ffsll((long long)m) : 0;
    }
    __syncthreads();
}



// tile product with the K loop split over two accumulators (breaks the MFMA dependency chain)
template <int NB, bool TA, bool TB>
__device__ __forceinline__ void tile_mma2(Acc<NB>& acc, const double* __restrict__ As, const double* __restrict__ Bs, double alpha) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int BPW = TileCfg<NB>::BPW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int rb = 16 * BPW * (w >> 1), cb = 16 * BPW * (w & 1);
    Acc<NB> acc2; acc_zero(acc2);
#pragma unroll
    for (int k0 = 0; k0 < NB; k0 += 8) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int k = k0 + 4 * h + lk;
            double a[BPW], b[BPW];
#pragma unroll
            for (int t = 0; t < BPW; ++t) {
                const int i = rb + 16 * t + li;
                const int j = cb + 16 * t + li;
                a[t] = alpha * (TA ? As[k * S + i] : As[i * S + k]);
                b[t] = TB ? Bs[j * S + k] : Bs[k * S + j];
            }
#pragma unroll
            for (int ti = 0; ti < BPW; ++ti)
#pragma unroll
                for (int tj = 0; tj < BPW; ++tj) {
                    f64x4& c = h ? acc2.v[ti * BPW + tj] : acc.v[ti * BPW + tj];
                    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], c, 0, 0, 0);
                }
        }
    }
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q) acc.v[q] += acc2.v[q];
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
        if (WHAT == 0) { if constexpr (NB == 32) tile_potrf_inv_pivot32(A, R, dg, &bad); else tile_potrf_inv<NB>(A, R, dg, &bad); }
        if (WHAT == 1) { tile_mma<NB, false, true>(acc, A, B, 1.0); __syncthreads(); }
        if (WHAT == 16) { tile_mma2<NB, false, true>(acc, A, B, 1.0); __syncthreads(); }
        if (WHAT == 2) { __syncthreads(); }
        if (WHAT == 3) { for (int k = 0; k < NB; ++k) __syncthreads(); }
        __shared__ long long st[2];
        if (WHAT == 6 && NB == 32) { potrf_probe(A, R, (long long*)(dg + NB + 2)); if (threadIdx.x == 0 && it == reps - 1) for (int q = 0; q < 4; ++q) cyc[4 + q] = ((long long*)(dg + NB + 2))[q]; }
        if (WHAT == 7 && NB == 32) tile_potrf_inv_k4(A, R, dg, &bad);
        if (WHAT == 12 && NB == 32) tile_potrf_inv_m4(A, R, dg, &bad);
        if (WHAT == 13 && NB == 32) m4x<1>(A, R, dg, &bad);
        if (WHAT == 14 && NB == 32) m4x<2>(A, R, dg, &bad);
        if (WHAT == 15 && NB == 32) m4x<3>(A, R, dg, &bad);
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
    if (WHAT == 1 || WHAT == 16) acc_store(acc, out, NB);
    if (WHAT == 0 || WHAT == 4 || WHAT == 7 || WHAT == 12 || WHAT == 17) tile_store<NB>(out, NB, R);
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
    if (WHAT == 0 || WHAT == 4 || WHAT == 7 || WHAT == 12 || WHAT == 17) {
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
            run<32, 6>("potrf probe", dA, dO, dc); run<32, 0>("tile_potrf_inv", dA, dO, dc); run<32, 4>("tile_potrf_inv_b8", dA, dO, dc); run<32, 7>("tile_potrf_inv_k4", dA, dO, dc); run<32, 12>("tile_potrf_inv_m4 (MFMA)", dA, dO, dc); run<32, 13>("m4: no N", dA, dO, dc); run<32, 14>("m4: raw piv", dA, dO, dc); run<32, 15>("m4: no N + raw piv", dA, dO, dc); run<32, 8>("k4: no rcp", dA, dO, dc); run<32, 9>("k4: no publish", dA, dO, dc); run<32, 10>("k4: no update", dA, dO, dc); run<32, 11>("k4: stamps", dA, dO, dc); run<32, 1>("tile_mma (A B^T)", dA, dO, dc); run<32, 16>("tile_mma2 (2 accumulators)", dA, dO, dc);
            run<32, 2>("1 barrier + loads", dA, dO, dc); run<32, 3>("NB barriers", dA, dO, dc);
        } else {
            run<64, 0>("tile_potrf_inv", dA, dO, dc); run<64, 4>("tile_potrf_inv_b8", dA, dO, dc); run<64, 1>("tile_mma (A B^T)", dA, dO, dc); run<64, 16>("tile_mma2 (2 accumulators)", dA, dO, dc);
            run<64, 2>("1 barrier + loads", dA, dO, dc); run<64, 3>("NB barriers", dA, dO, dc);
        }
        hipFree(dA); hipFree(dO); hipFree(dc);
    }
    return 0;
}
