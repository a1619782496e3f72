// Diagnostic tile-factor variants of the fp64 diagonal factor, kept for the micro-benchmarks
// under tools/ (ubench_tile.hip, ubench_w1.hip, ubench_w2st.hip): the one-barrier-per-pivot,
// 4-pivot blocked, MFMA 4-pivot and two-wave forms that lost to the product's single-wave
// factor (tile_potrf_inv_w1, csrc/mfgp_device.h).  Not part of libmfgp.so.
#pragma once
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"

namespace mfgp {

#ifndef W2_STAMP
#define W2_STAMP(i) ((void)0)
#endif

// One-pivot-per-barrier form (kept as the reference variant for tools/ubench_tile.hip).
__device__ __forceinline__ void tile_potrf_inv_pivot32(double* __restrict__ A, double* __restrict__ R,
                                                       double* __restrict__ dg, int* __restrict__ bad) {
    // Branch-free pivot loop (measured ~3x faster than the predicated form on gfx950):
    //  * the pivot column of A is published WHOLE, zero above the pivot, so the
    //    unconditional update a_ic -= s_i a_ck / a_kk is an exact no-op on finalized
    //    columns (c < k); it zeroes column k itself, which is no longer needed (its
    //    values went to LDS and dg); garbage accumulates only in the unused upper part;
    //  * the pivot row of R is published whole (zeros right of the diagonal), so the R
    //    update is a no-op for c > k; the pivot row itself is protected by s_R = 0;
    //  * every thread writes one column word per pivot (non-owners into a dump slot)
    //    and the 8 threads of row k+1 write the next R row: no divergent publish.
    constexpr int NB = 32;
    constexpr int S = TileCfg<NB>::S;
    double* colb = R;               // [2][NB]
    double* rowb = R + 2 * NB;      // [2][NB]
    double* dump = R + 4 * NB;      // [NTHREADS] (inside the R tile; R is rewritten at the end)
    const int t = threadIdx.x;
    const int i = t >> 3, g = t & 7, c0 = 4 * g;
    double a[4], r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a[q] = A[i * S + c0 + q];
        r[q] = (i == c0 + q) ? 1.0 : 0.0;
    }
    __syncthreads();
    // pivot 0: column 0 of A (rows >= 0), row 0 of R = e_0
    if (g == 0) colb[i] = a[0];
    if (t < NB) rowb[t] = (t == 0) ? 1.0 : 0.0;
    __syncthreads();
    double dgk = 0.0;   // a_ii at its pivot, kept by the owners of row i
#pragma unroll 4
    for (int k = 0; k < NB; ++k) {
        const int cur = k & 1, nxt = cur ^ 1;
        const double akk = colb[cur * NB + k];
        const double aik = colb[cur * NB + i];
        const double2 ca = *reinterpret_cast<const double2*>(colb + cur * NB + c0);
        const double2 cb = *reinterpret_cast<const double2*>(colb + cur * NB + c0 + 2);
        const double2 ra = *reinterpret_cast<const double2*>(rowb + cur * NB + c0);
        const double2 rb = *reinterpret_cast<const double2*>(rowb + cur * NB + c0 + 2);
        if (i == k) dgk = akk;
        const double sA = aik * rcp_nr(akk);
        const double sR = (i > k) ? sA : 0.0;
        a[0] -= sA * ca.x;
        a[1] -= sA * ca.y;
        a[2] -= sA * cb.x;
        a[3] -= sA * cb.y;
        r[0] -= sR * ra.x;
        r[1] -= sR * ra.y;
        r[2] -= sR * rb.x;
        r[3] -= sR * rb.y;
        // publish pivot k+1
        const int k1 = k + 1;
        const int q1 = k1 & 3;
        const double v = (q1 == 0) ? a[0] : (q1 == 1) ? a[1] : (q1 == 2) ? a[2] : a[3];
        const bool own = (k1 >> 2) == g;
        colb[own ? nxt * NB + i : 4 * NB + t] = (i >= k1) ? v : 0.0;
        if (i == k1) *reinterpret_cast<double4*>(rowb + nxt * NB + c0) = double4{r[0], r[1], r[2], r[3]};
        __syncthreads();
    }
    (void)dump;
    // L_ii = sqrt(a_ii); D = diag(1/L) R; the pivot check needs no serial scan
    pivot_check_post(dgk, bad);
    const double li = sqrt(dgk);
    const double rli = 1.0 / li;
    __syncthreads();
    if (t == 0) *bad = pivot_check_result(bad);
    if (g == 0) dg[i] = li;
#pragma unroll
    for (int q = 0; q < 4; ++q) R[i * S + c0 + q] = (c0 + q <= i) ? r[q] * rli : 0.0;
    __syncthreads();
}

// ---------------------------------------------------------------- 4-pivot blocked diag factor
// NB = 32 Cholesky + inverse by blocked LDL^T elimination, 4 pivots per barrier round
// (8 rounds instead of 32: the per-round LDS publish -> barrier -> read latency is the
// cost, not the arithmetic).  Thread t owns row i = t/8, columns 4g..4g+3 of A and R.
// Round k (= 4 rd): the 4 current columns C = A[:, k..k+3] (zero above row k) and the 4
// pivot rows R_P = R[k..k+3, :] are published; every thread factors the pivot block
// M = C[k..k+3, :] = L_M D_M L_M^T redundantly in registers (rcp only, no sqrt), then
//   A_i -= w_i C^T,            w_i = C_i M^{-1}                 (rows >= k+4; rows < k
//                                                               have C_i = 0: no-op)
//   R_i -= v_i R_P,            v_i = w_i, or -(L_M^{-1})_{p,<p} for pivot row p = i-k.
// R accumulates L_u^{-1} (unit lower); at the end D = diag(d)^{-1/2} L_u^{-1} = L^{-1}
// and dg = sqrt(d).  A is left as garbage.  Non-positive pivots report through *bad.
__device__ __forceinline__ void tile_potrf_inv_k4(double* A, double* R, double* dg, int* bad) {
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
        // LDL^T of the pivot block (lower entries): u_ab = L_ab d_b = e_ab
        const double d0 = M[0][0];
        const double i0 = rcp_nr(d0);
        const double L10 = M[1][0] * i0, L20 = M[2][0] * i0, L30 = M[3][0] * i0;
        const double d1 = M[1][1] - L10 * M[1][0];
        const double i1 = rcp_nr(d1);
        const double e21 = M[2][1] - L20 * M[1][0];
        const double e31 = M[3][1] - L30 * M[1][0];
        const double L21 = e21 * i1, L31 = e31 * i1;
        const double d2 = M[2][2] - L20 * M[2][0] - L21 * e21;
        const double i2 = rcp_nr(d2);
        const double e32 = M[3][2] - L30 * M[2][0] - L31 * e21;
        const double L32 = e32 * i2;
        const double d3 = M[3][3] - L30 * M[3][0] - L31 * e31 - L32 * e32;
        const double i3 = rcp_nr(d3);
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
        const int pr = i - k;
        double v0 = w0, v1 = w1, v2 = w2, v3 = w3;
        if (pr >= 0 && pr < 4) {
            v0 = (pr == 1) ? -N10 : (pr == 2) ? -N20 : (pr == 3) ? -N30 : 0.0;
            v1 = (pr == 2) ? -N21 : (pr == 3) ? -N31 : 0.0;
            v2 = (pr == 3) ? -N32 : 0.0;
            v3 = 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] -= w0 * Cj[q][0] + w1 * Cj[q][1] + w2 * Cj[q][2] + w3 * Cj[q][3];
            r[q] -= v0 * Rp[0][q] + v1 * Rp[1][q] + v2 * Rp[2][q] + v3 * Rp[3][q];
        }
        if (t == 0) {
            piv[k] = d0; piv[k + 1] = d1; piv[k + 2] = d2; piv[k + 3] = d3;
        }
        if (rd + 1 < NB / 4) {
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
        __syncthreads();
    }
    const double di = piv[i];
    pivot_check_post(di, bad);
    __syncthreads();
    if (t == 0) *bad = pivot_check_result(bad);
    const double li = sqrt(di);
    const double rli = 1.0 / li;
    if (g == 0) dg[i] = li;
#pragma unroll
    for (int q = 0; q < 4; ++q) R[i * S + c0 + q] = (c0 + q <= i) ? r[q] * rli : 0.0;
    __syncthreads();
}

// ---------------------------------------------------------------- MFMA 4-pivot diag factor
// NB = 32 Cholesky + inverse, 4 pivots per barrier round with the rank-4 updates on the
// matrix core.  The tile stays in MFMA accumulator layout for the whole factorization:
// wave w owns the 16x16 blocks (w>>1, w&1) of A and of R (lane l: rows 16bi + (l>>4) + 4q,
// column 16bj + (l&15)).  Round k = 4 rd publishes C = A[:, k..k+3] (zero above row k) and
// R_P = R[k..k+3, :] through LDS; every lane factors the 4x4 pivot block M = C[k..k+3, :] =
// L_M D_M L_M^T in registers (same elimination order as pivot-by-pivot, no explicit
// inverse: an explicit M^{-1} lost ill-conditioned Forrester Grams) and feeds the matrix core
//   A -= (Y D_M^{-1}) Y^T, Y = C L_M^{-T};   R -= V R_P     (one v_mfma_f64_16x16x4 each)
// with V = C M^{-1} (= Y D_M^{-1} L_M^{-1}, by substitution) for rows >= k+4 and
// V = I - L_M^{-1} on the pivot rows, so R accumulates L_u^{-1}; pivots d give D = diag(d)^{-1/2}
// L_u^{-1} = L^{-1} and dg = sqrt(d).  The A tile's LDS doubles as the publish buffer.
struct M4Buf {
    double* colb;   // [2][NB][4]
    double* rowb;   // [2][4][NB]
    double* piv;    // [NB]
};

template <int RD>
__device__ __forceinline__ void m4_round(const M4Buf& B, f64x4& aA, f64x4& aR, int bi, int bj, int lc, int lr) {
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
        const double2 cja = *reinterpret_cast<const double2*>(C + cg * 4);
        const double2 cjb = *reinterpret_cast<const double2*>(C + cg * 4 + 2);
        const double bR = RP[lr * NB + cg];
        const double m00 = r0a.x, m10 = r1a.x, m11 = r1a.y, m20 = r2a.x, m21 = r2a.y, m22 = r2b.x;
        const double m30 = r3a.x, m31 = r3a.y, m32 = r3b.x, m33 = r3b.y;
        // ---- LDL^T of the pivot block (the same elimination order as a pivot-by-pivot
        //      Cholesky; no explicit inverse, so ill-conditioned blocks stay as stable)
        const double i0 = rcp_nr(m00);
        const double L10 = m10 * i0, L20 = m20 * i0, L30 = m30 * i0;
        const double d1 = fma(-L10, m10, m11);
        const double i1 = rcp_nr(d1);
        const double e21 = fma(-L20, m10, m21), e31 = fma(-L30, m10, m31);
        const double L21 = e21 * i1, L31 = e31 * i1;
        const double d2 = fma(-L21, e21, fma(-L20, m20, m22));
        const double i2 = rcp_nr(d2);
        const double e32 = fma(-L31, e21, fma(-L30, m20, m32));
        const double L32 = e32 * i2;
        const double d3 = fma(-L32, e32, fma(-L31, e31, fma(-L30, m30, m33)));
        const double i3 = rcp_nr(d3);
        // ---- Y = C L_M^{-T} (rows ia and cg), A -= (Y D^{-1}) Y^T
        const double y0 = cia.x;
        const double y1 = fma(-L10, y0, cia.y);
        const double y2 = fma(-L21, y1, fma(-L20, y0, cib.x));
        const double y3 = fma(-L32, y2, fma(-L31, y1, fma(-L30, y0, cib.y)));
        const double z0 = y0 * i0, z1 = y1 * i1, z2 = y2 * i2, z3 = y3 * i3;
        const double u0 = cja.x;
        const double u1 = fma(-L10, u0, cja.y);
        const double u2 = fma(-L21, u1, fma(-L20, u0, cjb.x));
        const double u3 = fma(-L32, u2, fma(-L31, u1, fma(-L30, u0, cjb.y)));
        const double wl = (lr == 0) ? z0 : (lr == 1) ? z1 : (lr == 2) ? z2 : z3;
        const double bA = (lr == 0) ? u0 : (lr == 1) ? u1 : (lr == 2) ? u2 : u3;
        // ---- R multipliers against the original pivot rows: V = Z L_M^{-1} (rows >= k+4;
        //      rows < k have C = 0), and on pivot row p: -(L_M^{-1})_{p, <p}
        const double x3 = z3;
        const double x2 = fma(-L32, x3, z2);
        const double x1 = fma(-L31, x3, fma(-L21, x2, z1));
        const double x0 = fma(-L30, x3, fma(-L20, x2, fma(-L10, x1, z0)));
        double vl = (lr == 0) ? x0 : (lr == 1) ? x1 : (lr == 2) ? x2 : x3;
        if (bi == (k >> 4)) {   // wave-uniform
            const int p = lc - (k & 15);
            if (p >= 0 && p < 4) {
                const double c20 = fma(-L21, L10, L20);                      // -(N20)
                const double c31 = fma(-L32, L21, L31);                      // -(N31)
                const double c30 = fma(-L32, c20, fma(-L31, L10, L30));      // -(N30)
                const double v1 = (lr == 0) ? L10 : 0.0;
                const double v2 = (lr == 0) ? c20 : (lr == 1) ? L21 : 0.0;
                const double v3 = (lr == 0) ? c30 : (lr == 1) ? c31 : (lr == 2) ? L32 : 0.0;
                vl = (p == 1) ? v1 : (p == 2) ? v2 : (p == 3) ? v3 : 0.0;
            }
        }
        // ---- rank-4 updates on the matrix core
        aA = __builtin_amdgcn_mfma_f64_16x16x4f64(-wl, bA, aA, 0, 0, 0);
        aR = __builtin_amdgcn_mfma_f64_16x16x4f64(-vl, bR, aR, 0, 0, 0);
        if (threadIdx.x == 0) {
            B.piv[k] = m00;
            B.piv[k + 1] = d1;
            B.piv[k + 2] = d2;
            B.piv[k + 3] = d3;
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
        m4_round<RD + 1>(B, aA, aR, bi, bj, lc, lr);
    }
}

// Entry with the tile already in accumulator layout (the Acc<32> of tile_mma: wave w
// holds block (w>>1, w&1)); scratch: >= 544 doubles of LDS nobody reads concurrently.
__device__ __forceinline__ void tile_potrf_inv_m4_acc(f64x4 aA, double* scratch, double* R, double* dg, int* bad) {
    constexpr int NB = 32;
    constexpr int S = TileCfg<NB>::S;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int bi = w >> 1, bj = w & 1, lc = l & 15, lr = l >> 4;
    const int cg = 16 * bj + lc;
    f64x4 aR;
#pragma unroll
    for (int q = 0; q < 4; ++q) aR[q] = (16 * bi + lr + 4 * q == cg) ? 1.0 : 0.0;
    const M4Buf B{scratch, scratch + 2 * NB * 4, scratch + 4 * NB * 4};
    if (bj == 0 && lc < 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) B.colb[(16 * bi + lr + 4 * q) * 4 + lc] = aA[q];
    }
    if (bi == 0) B.rowb[lr * NB + cg] = (lr == cg) ? 1.0 : 0.0;
    __syncthreads();
    m4_round<0>(B, aA, aR, bi, bj, lc, lr);
    // pivots d_i of the LDL^T, dg = sqrt(d),
    // first bad pivot by one ballot; then D = diag(d)^{-1/2} L_u^{-1} (lower)
    double* dpiv = B.rowb;   // publish buffers are dead after the last round
    if (t < 64) {
        double d = 1.0;
        if (t < NB) {
            d = B.piv[t];
            dg[t] = sqrt(d);
            dpiv[t] = d;
        }
        const unsigned long long m = __ballot(!(d > 0.0 && d < INFINITY));
        if (t == 0) *bad = m ? __ffsll((long long)m) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int rg = 16 * bi + lr + 4 * q;
        const double sc = rcp_nr(dg[rg]);
        R[rg * S + cg] = (cg <= rg) ? aR[q] * sc : 0.0;
    }
    __syncthreads();
}

// Entry from an LDS tile A (row-major, stride S); A's LDS becomes the publish buffer.
__device__ __forceinline__ void tile_potrf_inv_m4(double* A, double* R, double* dg, int* bad) {
    constexpr int S = TileCfg<32>::S;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int bi = w >> 1, bj = w & 1, lc = l & 15, lr = l >> 4;
    f64x4 aA;
#pragma unroll
    for (int q = 0; q < 4; ++q) aA[q] = A[(16 * bi + lr + 4 * q) * S + 16 * bj + lc];
    __syncthreads();
    tile_potrf_inv_m4_acc(aA, A, R, dg, bad);
}


// ---------------------------------------------------------------- two-wave diag factor
// The single-wave factor is issue-bound (one wave issues every instruction of the round in
// order): the R chain (X = C M^{-1} by substitution, W_R, two MFMAs) costs ~280 of its ~1.1k
// clocks per round.  Here wave 0 runs the A chain only and hands each round's record -- the
// 4x4 factor (L_M, pivots d) and its rows' Z = C L_M^{-T} D_M^{-1} -- to wave 1 through LDS;
// wave 1 follows one round behind, runs the R chain and finishes R.  Hand-off inside the
// workgroup: a wave's DS operations are processed in issue order, so a record written before
// the round flag is complete when another wave reads the flag; Z slots are a 4-deep ring
// released by wave 1's ack counter.  Waves 2 and 3 only meet the closing barrier.
// ws: >= W2_WS doubles of LDS, not aliasing R or dg; the layout below.
constexpr int W2_ZB = 128;                  // Z ring: 4 slots x [2 rows][64 lanes][4]
constexpr int W2_REC = W2_ZB + 4 * 512;     // records: 8 rounds x 12 doubles (L10..L32, d0..d3)
constexpr int W2_FLAG = W2_REC + 8 * 12;    // two ints: round flag (wave 0), ack (wave 1)
constexpr int W2_WS = W2_FLAG + 2;

// Workgroup-scope relaxed atomics (not volatile: a volatile access is never rewritten from
// flat to ds_* by address-space inference, and the flat form costs a system-coherent round trip).
__device__ __forceinline__ int lds_ld_volatile(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st_flag(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Bounded spin on an LDS counter written by another wave of the workgroup (the bound only
// guards against a hang; the partner wave always reaches the value within the round).
__device__ __forceinline__ void w2_wait(const int* p, int v) {
    for (int it = 0; it < (1 << 20) && lds_ld_volatile(p) < v; ++it) {}
}

template <int K>
__device__ __forceinline__ void w2_round_a(double* __restrict__ ws, f64x4& a00, f64x4& a01, f64x4& a11, int l) {
    if constexpr (K < 8) {
        constexpr int bk = K >> 2, kq = K & 3;
        const int lc = l & 15, kk = l >> 4;
        double* Pn = ws;
        W2_STAMP(K);
        if constexpr (bk == 0) Pn[lc * 4 + kk] = a00[kq];
        Pn[(16 + lc) * 4 + kk] = (bk == 0) ? a01[kq] : a11[kq];
        asm volatile("" ::: "memory");   // DS order: the reads below see the panel
        const f64x2* Pm = reinterpret_cast<const f64x2*>(Pn + 16 * K);
        const f64x2 c0a = Pm[0], c0b = Pm[1], c1a = Pm[2], c1b = Pm[3], c2b = Pm[5], c3b = Pm[7];
        const f64x2* Pr = reinterpret_cast<const f64x2*>(Pn);
        f64x2 u0a = {0.0, 0.0}, u0b = {0.0, 0.0};
        if constexpr (bk == 0) { u0a = Pr[2 * lc]; u0b = Pr[2 * lc + 1]; }
        const f64x2 u1a = Pr[2 * (16 + lc)], u1b = Pr[2 * (16 + lc) + 1];
        __builtin_amdgcn_sched_barrier(0);   // all panel reads in flight before the chain
        const double m00 = c0a.x, m10 = c0a.y, m20 = c0b.x, m30 = c0b.y;
        const double m11 = c1a.y, m21 = c1b.x, m31 = c1b.y, m22 = c2b.x, m32 = c2b.y, m33 = c3b.y;
        const double i0 = rcp_nr(m00);
        const double L10 = m10 * i0, L20 = m20 * i0, L30 = m30 * i0;
        const double d1 = fma(-L10, m10, m11);
        const double i1 = rcp_nr(d1);
        const double e21 = fma(-L20, m10, m21), e31 = fma(-L30, m10, m31);
        const double L21 = e21 * i1, L31 = e31 * i1;
        const double d2 = fma(-L21, e21, fma(-L20, m20, m22));
        const double i2 = rcp_nr(d2);
        const double e32 = fma(-L31, e21, fma(-L30, m20, m32));
        const double L32 = e32 * i2;
        const double d3 = fma(-L32, e32, fma(-L31, e31, fma(-L30, m30, m33)));
        const double i3 = rcp_nr(d3);
        double zA[2], yB[2];
        f64x2 zlo[2], zhi[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h < bk) { zA[h] = 0.0; yB[h] = 0.0; zlo[h] = f64x2{0.0, 0.0}; zhi[h] = zlo[h]; continue; }
            const f64x2 ua = h ? u1a : u0a, ub = h ? u1b : u0b;
            const bool below = 16 * h + lc > 4 * K + 3;
            const double y0 = ua.x;
            const double y1 = fma(-L10, y0, ua.y);
            const double y2 = fma(-L21, y1, fma(-L20, y0, ub.x));
            const double y3 = fma(-L32, y2, fma(-L31, y1, fma(-L30, y0, ub.y)));
            const double z0 = y0 * i0, z1 = y1 * i1, z2 = y2 * i2, z3 = y3 * i3;
            zA[h] = below ? sel4(kk, z0, z1, z2, z3) : 0.0;
            yB[h] = sel4(kk, y0, y1, y2, y3);
            zlo[h] = f64x2{z0, z1};
            zhi[h] = f64x2{z2, z3};
        }
        if constexpr (bk == 0) {
            a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0], yB[0], a00, 0, 0, 0);
            a01 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0], yB[1], a01, 0, 0, 0);
            a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1], yB[1], a11, 0, 0, 0);
        } else {
            a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1], yB[1], a11, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- hand the round to wave 1 (issued under the MFMA latency)
        const int* flag = reinterpret_cast<const int*>(ws + W2_FLAG);
        if constexpr (K >= 4) {
            w2_wait(flag + 1, K - 3);   // slot K & 3 released by wave 1
            asm volatile("" ::: "memory");
        }
        f64x2* zs = reinterpret_cast<f64x2*>(ws + W2_ZB + (K & 3) * 512);
#pragma unroll
        for (int h = bk; h < 2; ++h) {
            zs[(h * 64 + l) * 2] = zlo[h];
            zs[(h * 64 + l) * 2 + 1] = zhi[h];
        }
        asm volatile("" ::: "memory");
        if (l == 0) {
            f64x2* rc = reinterpret_cast<f64x2*>(ws + W2_REC + 12 * K);
            rc[0] = f64x2{L10, L20};
            rc[1] = f64x2{L30, L21};
            rc[2] = f64x2{L31, L32};
            rc[3] = f64x2{m00, d1};
            rc[4] = f64x2{d2, d3};
            asm volatile("" ::: "memory");
            lds_st_flag(reinterpret_cast<int*>(ws + W2_FLAG), K + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        w2_round_a<K + 1>(ws, a00, a01, a11, l);
    }
}

template <int K>
__device__ __forceinline__ void w2_round_r(double* __restrict__ ws, f64x4& r00, f64x4& r10, f64x4& r11, int l) {
    if constexpr (K < 8) {
        constexpr int bk = K >> 2, kq = K & 3;
        const int lc = l & 15, kk = l >> 4, p = lc & 3;
        const int* flag = reinterpret_cast<const int*>(ws + W2_FLAG);
        w2_wait(flag, K + 1);
        asm volatile("" ::: "memory");
        W2_STAMP(8 + K);
        const f64x2* rc = reinterpret_cast<const f64x2*>(ws + W2_REC + 12 * K);
        const f64x2 q0 = rc[0], q1 = rc[1], q2 = rc[2];
        const double L10 = q0.x, L20 = q0.y, L30 = q1.x, L21 = q1.y, L31 = q2.x, L32 = q2.y;
        const f64x2* zs = reinterpret_cast<const f64x2*>(ws + W2_ZB + (K & 3) * 512);
        f64x2 zlo[2] = {f64x2{0.0, 0.0}, f64x2{0.0, 0.0}}, zhi[2] = {f64x2{0.0, 0.0}, f64x2{0.0, 0.0}};
#pragma unroll
        for (int h = bk; h < 2; ++h) {
            zlo[h] = zs[(h * 64 + l) * 2];
            zhi[h] = zs[(h * 64 + l) * 2 + 1];
        }
        asm volatile("" ::: "memory");   // DS order: the ack is processed after the reads
        if (l == 0) lds_st_flag(reinterpret_cast<int*>(ws + W2_FLAG) + 1, K + 1);
        double wR[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h < bk) { wR[h] = 0.0; continue; }
            const int row = 16 * h + lc;
            const bool piv = (row >> 2) == K;
            const bool below = row > 4 * K + 3;
            const double v0 = piv ? (p == 0 ? 1.0 : 0.0) : zlo[h].x;
            const double v1 = piv ? (p == 1 ? 1.0 : 0.0) : zlo[h].y;
            const double v2 = piv ? (p == 2 ? 1.0 : 0.0) : zhi[h].x;
            const double v3 = piv ? (p == 3 ? 1.0 : 0.0) : zhi[h].y;
            const double x3 = v3;
            const double x2 = fma(-L32, x3, v2);
            const double x1 = fma(-L31, x3, fma(-L21, x2, v1));
            const double x0 = fma(-L30, x3, fma(-L20, x2, fma(-L10, x1, v0)));
            const double xk = sel4(kk, x0, x1, x2, x3);
            wR[h] = below ? xk : piv ? ((p == kk ? 1.0 : 0.0) - xk) : 0.0;
        }
        if constexpr (bk == 0) {
            const double pR0 = r00[kq];
            r00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[0], pR0, r00, 0, 0, 0);
            r10 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1], pR0, r10, 0, 0, 0);
        } else {
            const double pR0 = r10[kq], pR1 = r11[kq];
            r10 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1], pR0, r10, 0, 0, 0);
            r11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1], pR1, r11, 0, 0, 0);
        }
        w2_round_r<K + 1>(ws, r00, r10, r11, l);
    }
}

// Entry with the tile in accumulator layout (wave w holds block (w>>1, w&1) of a symmetric
// tile whose lower triangle is valid).  ws: W2_WS doubles of LDS, not aliasing R / dg; the
// caller's reads of ws before the call are fenced here by a barrier.
__device__ __forceinline__ void tile_potrf_inv_w2_acc(f64x4 aA, double* __restrict__ ws, double* __restrict__ R,
                                                      double* __restrict__ dg, int* __restrict__ bad) {
    constexpr int LX = 33;
    constexpr int S = TileCfg<32>::S;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int bi = w >> 1, bj = w & 1, lc = l & 15, lr = l >> 4;
    __syncthreads();   // ws may alias tiles the caller's waves were still reading
    if (bj <= bi) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ws[(16 * bi + lr + 4 * q) * LX + 16 * bj + lc] = aA[q];
    }
    if (t == 0) {
        int* flag = reinterpret_cast<int*>(ws + W2_FLAG);
        flag[0] = 0;
        flag[1] = 0;
    }
    __syncthreads();
    if (w == 0) {
        f64x4 a00, a01, a11;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = lr + 4 * q;
            const int hi = r > lc ? r : lc, lo = r > lc ? lc : r;
            a00[q] = ws[hi * LX + lo];
            a11[q] = ws[(16 + hi) * LX + 16 + lo];
            a01[q] = ws[(16 + lc) * LX + r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // X read before the panel / ring overwrite it
        w2_round_a<0>(ws, a00, a01, a11, l);
        W2_STAMP(16);
    } else if (w == 1) {
        f64x4 r00, r10 = {0.0, 0.0, 0.0, 0.0}, r11;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            r00[q] = (lr + 4 * q == lc) ? 1.0 : 0.0;
            r11[q] = r00[q];
        }
        w2_round_r<0>(ws, r00, r10, r11, l);
        W2_STAMP(17);
        // L^{-1} = diag(d)^{-1/2} L_u^{-1}; L_ii = sqrt(d_i); first bad pivot by one ballot
        const double* rec = ws + W2_REC;
        double s0[4], s1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r0 = lr + 4 * q, r1 = 16 + r0;
            s0[q] = rcp_nr(sqrt(rec[12 * (r0 >> 2) + 6 + (r0 & 3)]));
            s1[q] = rcp_nr(sqrt(rec[12 * (r1 >> 2) + 6 + (r1 & 3)]));
        }
        const int li = l & 31;
        const double dl = rec[12 * (li >> 2) + 6 + (li & 3)];
        const unsigned long long m = __ballot(l < 32 && !(dl > 0.0 && dl < INFINITY));
        if (l < 32) dg[l] = sqrt(dl);
        if (l == 0) *bad = m ? __ffsll((long long)m) : 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = lr + 4 * q;
            R[r * S + lc] = (lc <= r) ? r00[q] * s0[q] : 0.0;
            R[r * S + 16 + lc] = 0.0;
            R[(16 + r) * S + lc] = r10[q] * s1[q];
            R[(16 + r) * S + 16 + lc] = (lc <= r) ? r11[q] * s1[q] : 0.0;
        }
    }
    __syncthreads();
}

// NB = 32 uses the single-wave form (9.1k shader clocks vs 12.7k for the 4-wave MFMA 4-pivot
// form and 15.5k for the pivot form: tools/ubench_w1.hip, tools/ubench_tile.hip).

// ---------------------------------------------------------------- split diag factor (lost)
// Measured round 2 (tools/ubench_w1.hip, "s2 lds"): A wave alone 5.0-5.5k clocks, but the whole
// factor 7.9k against 8.2k for w1: whoever re-derives the 4x4 LDL^T for the inverse (the L wave,
// ~950 clocks a round) trails the A wave, and the last round's LDL -> R update -> scale chain is
// a ~1.2k-clock tail.  Posting the LDL from the A wave (one lane's 14 mailbox stores) instead
// costs its chain ~200 clocks a round.  Not used by the engine.
// The w1 factor with its inverse work moved to a second wave on another SIMD: in w1 the R work
// of the 8 rounds costs ~2.9k of the ~8.2k clocks (tools/ubench_w1.hip, "A wave alone").
// The A wave runs only the elimination chain (publish the pivot rows, 4x4 LDL^T, own-row
// substitution, rank-4 MFMA update of A).  Round K's pivot rows go to their own LDS panel
// Pn + 128 K; lane 0 posts the round's LDL^T (1/d, L, d) to the mailbox mb + 16 K and then raises
// *flag to base + K + 1 (the DS operations of one wave are processed in issue order, so the
// mailbox and panel writes land before the flag).  The R wave spins on the flag, reads the
// mailbox and its own rows of the panel, forms W_R and applies R -= W_R R[P, :] with the same
// instructions as w1; a third wave (S) turns the posted pivots into L_ii, 1/L_ii and the first bad
// pivot, and the R wave scales its rows by them on the way out: D = L^{-1}, L_ii and *bad as
// tile_potrf_inv_w1_wave writes them (identical bits).
// Pn: 8 x 128 doubles of LDS that may alias X (the A wave reads X before it first writes Pn;
// the R wave never reads X).  mb: 8 x 16 doubles, sc: 32 doubles of LDS; flag, sflag: LDS ints,
// monotonic across calls (call c uses base = 8 c).
struct S2Ldl {
    double i0, i1, i2, i3, L10, L20, L30, L21, L31, L32, d0, d1, d2, d3;
};

__device__ __forceinline__ S2Ldl s2_ldl(const double* __restrict__ P, int K) {
    const f64x2* Pm = reinterpret_cast<const f64x2*>(P + 16 * K);
    const f64x2 c0a = Pm[0], c0b = Pm[1], c1a = Pm[2], c1b = Pm[3], c2b = Pm[5], c3b = Pm[7];
    S2Ldl s;
    const double m00 = c0a.x, m10 = c0a.y, m20 = c0b.x, m30 = c0b.y;
    const double m11 = c1a.y, m21 = c1b.x, m31 = c1b.y, m22 = c2b.x, m32 = c2b.y, m33 = c3b.y;
    s.d0 = m00;
    s.i0 = rcp_nr1(m00);
    s.L10 = m10 * s.i0; s.L20 = m20 * s.i0; s.L30 = m30 * s.i0;
    s.d1 = fma(-s.L10, m10, m11);
    s.i1 = rcp_nr1(s.d1);
    const double e21 = fma(-s.L20, m10, m21), e31 = fma(-s.L30, m10, m31);
    s.L21 = e21 * s.i1; s.L31 = e31 * s.i1;
    s.d2 = fma(-s.L21, e21, fma(-s.L20, m20, m22));
    s.i2 = rcp_nr1(s.d2);
    const double e32 = fma(-s.L31, e21, fma(-s.L30, m20, m32));
    s.L32 = e32 * s.i2;
    s.d3 = fma(-s.L32, e32, fma(-s.L31, e31, fma(-s.L30, m30, m33)));
    s.i3 = rcp_nr1(s.d3);
    return s;
}

// y = C L_M^{-T} for the row held in (ua, ub)
__device__ __forceinline__ void s2_y(const S2Ldl& s, f64x2 ua, f64x2 ub, double y[4]) {
    y[0] = ua.x;
    y[1] = fma(-s.L10, y[0], ua.y);
    y[2] = fma(-s.L21, y[1], fma(-s.L20, y[0], ub.x));
    y[3] = fma(-s.L32, y[2], fma(-s.L31, y[1], fma(-s.L30, y[0], ub.y)));
}

template <int K>
__device__ __forceinline__ void s2_round_a(double* __restrict__ Pn, int* flag, int base,
                                           f64x4& a00, f64x4& a01, f64x4& a11, int l, long long* tr) {
    if constexpr (K < 8) {
        constexpr int bk = K >> 2, kq = K & 3;
        const int lc = l & 15, kk = l >> 4;
        double* P = Pn + 128 * K;
        if constexpr (bk == 0) P[lc * 4 + kk] = a00[kq];
        P[(16 + lc) * 4 + kk] = (bk == 0) ? a01[kq] : a11[kq];
        asm volatile("" ::: "memory");
        const f64x2* Pr = reinterpret_cast<const f64x2*>(P);
        f64x2 u0a = {0.0, 0.0}, u0b = {0.0, 0.0};
        if constexpr (bk == 0) { u0a = Pr[2 * lc]; u0b = Pr[2 * lc + 1]; }
        const f64x2 u1a = Pr[2 * (16 + lc)], u1b = Pr[2 * (16 + lc) + 1];
        const S2Ldl s = s2_ldl(P, K);
        __builtin_amdgcn_sched_barrier(0);
        // the LDL^T consumed the panel reads, so the panel writes have landed too
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (l == 0) {
            __hip_atomic_store(flag, base + K + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (tr) tr[K] = __builtin_amdgcn_s_memtime();
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K < 7) {   // the last round's pivots leave nothing below them to update
            double zA[2], yB[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (h < bk) { zA[h] = 0.0; yB[h] = 0.0; continue; }
                const bool below = (h > bk) || ((lc >> 2) > kq);
                double y[4];
                s2_y(s, h ? u1a : u0a, h ? u1b : u0b, y);
                const double z = sel4(kk, y[0] * s.i0, y[1] * s.i1, y[2] * s.i2, y[3] * s.i3);
                zA[h] = below ? z : 0.0;
                yB[h] = sel4(kk, y[0], y[1], y[2], y[3]);
            }
            if constexpr (bk == 0) {
                if constexpr (K < 3) {
                    a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0], yB[0], a00, 0, 0, 0);
                    a01 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0], yB[1], a01, 0, 0, 0);
                }
                a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1], yB[1], a11, 0, 0, 0);
            } else {
                a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1], yB[1], a11, 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        s2_round_a<K + 1>(Pn, flag, base, a00, a01, a11, l, tr);
    }
}

template <int K>
__device__ __forceinline__ void s2_round_r(const double* __restrict__ Pn, const double* __restrict__ mb,
                                           const int* flag, int base, f64x4& r00, f64x4& r10, f64x4& r11,
                                           int l, long long* tr) {
    if constexpr (K < 8) {
        constexpr int bk = K >> 2, kq = K & 3;
        const int lc = l & 15, kk = l >> 4, p = lc & 3;
        while (__builtin_amdgcn_readfirstlane(
                   __hip_atomic_load(const_cast<int*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
               base + K + 1) {
            // the A wave's panel round trips queue behind a tight poll: sleep except for the last
            // round, when the A wave has no LDS traffic left
            if constexpr (K < 7) __builtin_amdgcn_s_sleep(1);
        }
        if (tr && l == 0) tr[8 + K] = __builtin_amdgcn_s_memtime();
        asm volatile("" ::: "memory");
        const f64x2* m = reinterpret_cast<const f64x2*>(mb + 16 * K);
        const f64x2 m0 = m[0], m1 = m[1], m2 = m[2], m3 = m[3], m4 = m[4], m5 = m[5], m6 = m[6];
        const f64x2* Pr = reinterpret_cast<const f64x2*>(Pn + 128 * K);
        f64x2 u0a = {0.0, 0.0}, u0b = {0.0, 0.0};
        if constexpr (bk == 0) { u0a = Pr[2 * lc]; u0b = Pr[2 * lc + 1]; }
        const f64x2 u1a = Pr[2 * (16 + lc)], u1b = Pr[2 * (16 + lc) + 1];
        S2Ldl s;
        s.i0 = m0.x; s.i1 = m0.y; s.i2 = m1.x; s.i3 = m1.y; s.L10 = m2.x; s.L20 = m2.y;
        s.L30 = m3.x; s.L21 = m3.y; s.L31 = m4.x; s.L32 = m4.y; s.d0 = m5.x; s.d1 = m5.y;
        s.d2 = m6.x; s.d3 = m6.y;
        double wR[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h < bk) { wR[h] = 0.0; continue; }
            const bool piv = (h == bk) && ((lc >> 2) == kq);
            const bool below = (h > bk) || ((lc >> 2) > kq);
            double y[4], v[4];
            s2_y(s, h ? u1a : u0a, h ? u1b : u0b, y);
            v[0] = y[0] * s.i0; v[1] = y[1] * s.i1; v[2] = y[2] * s.i2; v[3] = y[3] * s.i3;
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = piv ? (p == c ? 1.0 : 0.0) : v[c];
            const double x3 = v[3];
            const double x2 = fma(-s.L32, x3, v[2]);
            const double x1 = fma(-s.L31, x3, fma(-s.L21, x2, v[1]));
            const double x0 = fma(-s.L30, x3, fma(-s.L20, x2, fma(-s.L10, x1, v[0])));
            const double xk = sel4(kk, x0, x1, x2, x3);
            wR[h] = below ? xk : piv ? ((p == kk ? 1.0 : 0.0) - xk) : 0.0;
        }
        if constexpr (bk == 0) {
            const double pR0 = r00[kq];
            r00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[0], pR0, r00, 0, 0, 0);
            r10 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1], pR0, r10, 0, 0, 0);
        } else {
            const double pR0 = r10[kq], pR1 = r11[kq];
            r10 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1], pR0, r10, 0, 0, 0);
            r11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1], pR1, r11, 0, 0, 0);
        }
        if (tr && l == 0) tr[16 + K] = __builtin_amdgcn_s_memtime();
        s2_round_r<K + 1>(Pn, mb, flag, base, r00, r10, r11, l, tr);
    }
}

// A wave: X (lower triangle, stride ldx) -> elimination; returns when its last panel is out.
__device__ __forceinline__ void tile_potrf_inv_s2_a(const double* __restrict__ X, int ldx, double* __restrict__ Pn,
                                                    int* flag, int base,
                                                    long long* tr = nullptr) {
    const int l = threadIdx.x & 63, lc = l & 15, lr = l >> 4;
    f64x4 a00, a01, a11;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = lr + 4 * q;
        const int hi = r > lc ? r : lc, lo = r > lc ? lc : r;
        a00[q] = X[hi * ldx + lo];
        a11[q] = X[(16 + hi) * ldx + 16 + lo];
        a01[q] = X[(16 + lc) * ldx + r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // X fully read before Pn (may alias) is written
    s2_round_a<0>(Pn, flag, base, a00, a01, a11, l, tr);
}

// L wave: re-derives each round's 4x4 LDL^T from the A wave's panel and posts it to the mailbox
// (the A wave itself never writes the mailbox: one lane's stores there cost its chain ~200 clocks
// a round), then raises *lflag to base + K + 1.
__device__ __forceinline__ void tile_potrf_inv_s2_l(const double* __restrict__ Pn, double* __restrict__ mb,
                                                    const int* flag, int* lflag, int base) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int K = 0; K < 8; ++K) {
        while (__builtin_amdgcn_readfirstlane(
                   __hip_atomic_load(const_cast<int*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
               base + K + 1)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        const S2Ldl s = s2_ldl(Pn + 128 * K, K);
        if (l == 0) {
            double* m = mb + 16 * K;
            m[0] = s.i0; m[1] = s.i1; m[2] = s.i2; m[3] = s.i3; m[4] = s.L10; m[5] = s.L20; m[6] = s.L30;
            m[7] = s.L21; m[8] = s.L31; m[9] = s.L32; m[10] = s.d0; m[11] = s.d1; m[12] = s.d2; m[13] = s.d3;
            asm volatile("" ::: "memory");
            __hip_atomic_store(lflag, base + K + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// S wave: 1/sqrt(d) of every pivot into sc[0..31], L_ii = sqrt(d) into dg, the first bad pivot
// into *bad; then raises *sflag to base + 8.  Off both chains: its rounds are a few lanes' work.
__device__ __forceinline__ void tile_potrf_inv_s2_s(const double* __restrict__ mb, const int* flag, int* sflag,
                                                    int base, double* __restrict__ sc, double* __restrict__ dg,
                                                    int* __restrict__ bad) {
    const int l = threadIdx.x & 63;
    int first = 0;
    for (int K = 0; K < 8; ++K) {
        while (__builtin_amdgcn_readfirstlane(
                   __hip_atomic_load(const_cast<int*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
               base + K + 1)
            __builtin_amdgcn_s_sleep(1);
        const double d = mb[16 * K + 10 + (l & 3)];
        const double r = rsq_nr(d);
        if (l < 4) { sc[4 * K + l] = r; dg[4 * K + l] = d * r; }
        const unsigned long long m = __ballot(l < 4 && !(d > 0.0 && d < INFINITY));
        if (first == 0 && m) first = 4 * K + __ffsll((long long)m);
    }
    if (l == 0) *bad = first;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (l == 0) __hip_atomic_store(sflag, base + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// R wave: follows the A wave's rounds, builds L^{-1}; with the S wave's scales writes R (stride S).
__device__ __forceinline__ void tile_potrf_inv_s2_r(const double* __restrict__ Pn, const double* __restrict__ mb,
                                                    const int* flag, const int* sflag, int base,
                                                    const double* __restrict__ sc, double* __restrict__ R,
                                                    long long* tr = nullptr) {
    constexpr int S = TileCfg<32>::S;
    const int l = threadIdx.x & 63, lc = l & 15, lr = l >> 4;
    f64x4 r00, r10 = {0.0, 0.0, 0.0, 0.0}, r11;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r00[q] = (lr + 4 * q == lc) ? 1.0 : 0.0;
        r11[q] = r00[q];
    }
    s2_round_r<0>(Pn, mb, flag, base, r00, r10, r11, l, tr);
    while (__builtin_amdgcn_readfirstlane(
               __hip_atomic_load(const_cast<int*>(sflag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
           base + 8) {}
    asm volatile("" ::: "memory");
    double s0[4], s1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s0[q] = sc[lr + 4 * q];
        s1[q] = sc[16 + lr + 4 * q];
    }
    // all eight loads in flight at once (a select on a loaded value otherwise becomes a branch
    // around the load: one LDS round trip per row)
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" :: "v"(s0[q]), "v"(s1[q]));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = lr + 4 * q;
        R[r * S + lc] = (lc <= r) ? r00[q] * s0[q] : 0.0;
        R[r * S + 16 + lc] = 0.0;
        R[(16 + r) * S + lc] = r10[q] * s1[q];
        R[(16 + r) * S + 16 + lc] = (lc <= r) ? r11[q] * s1[q] : 0.0;
    }
}

}  // namespace mfgp
