// Diagnostic: the NB = 32 diagonal factor + inverse as two 16 x 16 single-wave factors (w16) and
// the 16 x 16 products between them (L21 = A21 D11^T, A22 -= L21 L21^T, D21 = -D22 L21 D11), against
// the library's single-wave 32 x 32 factor (tile_potrf_inv_w1_wave).  Timing (s_memtime clocks) and
// max error of D = L^{-1} and L_ii against a long-double host factorisation.  Also an 8-pivot-a-round
// single-wave factor (w8): its elimination (L_ii) is right, its inverse (R work) is not -- it was
// kept as a timing-only probe once it measured slower (10.5k clocks) than the library's whole
// 4-pivot factor (8.2k).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "../multi_fidelity_gpflow_amd/csrc/mfgp_device.h"
using namespace mfgp;
constexpr int NB = 32;

// R work of round K of the 16 x 16 factor (rows of one 16-block): X = V L_M^{-1}, W_R, R -= W_R R[P, :]
template <int K>
__device__ __forceinline__ void w16_rwork(const W1Pending& pd, f64x4& r00, int l) {
    const int lc = l & 15, kk = l >> 4, p = lc & 3;
    const bool piv = (lc >> 2) == K;
    const bool below = lc > 4 * K + 3;
    const double x3 = pd.v[0][3];
    const double x2 = fma(-pd.L32, x3, pd.v[0][2]);
    const double x1 = fma(-pd.L31, x3, fma(-pd.L21, x2, pd.v[0][1]));
    const double x0 = fma(-pd.L30, x3, fma(-pd.L20, x2, fma(-pd.L10, x1, pd.v[0][0])));
    const double xk = sel4(kk, x0, x1, x2, x3);
    const double wR = below ? xk : piv ? ((p == kk ? 1.0 : 0.0) - xk) : 0.0;
    r00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR, r00[K], r00, 0, 0, 0);
}

template <int K>
__device__ __forceinline__ void w16_round(double* __restrict__ Pn, double* __restrict__ dpv, f64x4& a00, f64x4& r00,
                                          W1Pending& pd, int l) {
    if constexpr (K < 4) {
        const int lc = l & 15, kk = l >> 4;
        Pn[lc * 4 + kk] = a00[K];
        asm volatile("" ::: "memory");
        const f64x2* Pm = reinterpret_cast<const f64x2*>(Pn + 16 * K);
        const f64x2 c0a = Pm[0], c0b = Pm[1], c1a = Pm[2], c1b = Pm[3], c2b = Pm[5], c3b = Pm[7];
        const f64x2* Pr = reinterpret_cast<const f64x2*>(Pn);
        const f64x2 ua = Pr[2 * lc], ub = Pr[2 * lc + 1];
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K > 0) w16_rwork<K - 1>(pd, r00, l);
        __builtin_amdgcn_sched_barrier(0);
        const double m00 = c0a.x, m10 = c0a.y, m20 = c0b.x, m30 = c0b.y;
        const double m11 = c1a.y, m21 = c1b.x, m31 = c1b.y, m22 = c2b.x, m32 = c2b.y, m33 = c3b.y;
        const double i0 = rcp_nr1(m00);
        const double L10 = m10 * i0, L20 = m20 * i0, L30 = m30 * i0;
        const double d1 = fma(-L10, m10, m11);
        const double i1 = rcp_nr1(d1);
        const double e21 = fma(-L20, m10, m21), e31 = fma(-L30, m10, m31);
        const double L21 = e21 * i1, L31 = e31 * i1;
        const double d2 = fma(-L21, e21, fma(-L20, m20, m22));
        const double i2 = rcp_nr1(d2);
        const double e32 = fma(-L31, e21, fma(-L30, m20, m32));
        const double L32 = e32 * i2;
        const double d3 = fma(-L32, e32, fma(-L31, e31, fma(-L30, m30, m33)));
        const double i3 = rcp_nr1(d3);
        const bool piv = (lc >> 2) == K;
        const bool below = lc > 4 * K + 3;
        const int p = lc & 3;
        const double y0 = ua.x;
        const double y1 = fma(-L10, y0, ua.y);
        const double y2 = fma(-L21, y1, fma(-L20, y0, ub.x));
        const double y3 = fma(-L32, y2, fma(-L31, y1, fma(-L30, y0, ub.y)));
        const double z0 = y0 * i0, z1 = y1 * i1, z2 = y2 * i2, z3 = y3 * i3;
        if constexpr (K < 3) {
            const double zA = below ? sel4(kk, z0, z1, z2, z3) : 0.0;
            const double yB = sel4(kk, y0, y1, y2, y3);
            a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA, yB, a00, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        dpv[l < 4 ? 4 * K + l : 40 + l] = sel4(l & 3, m00, d1, d2, d3);
        pd.v[0][0] = piv ? (p == 0 ? 1.0 : 0.0) : z0;
        pd.v[0][1] = piv ? (p == 1 ? 1.0 : 0.0) : z1;
        pd.v[0][2] = piv ? (p == 2 ? 1.0 : 0.0) : z2;
        pd.v[0][3] = piv ? (p == 3 ? 1.0 : 0.0) : z3;
        pd.L10 = L10; pd.L20 = L20; pd.L30 = L30; pd.L21 = L21; pd.L31 = L31; pd.L32 = L32;
        __builtin_amdgcn_sched_barrier(0);
        w16_round<K + 1>(Pn, dpv, a00, r00, pd, l);
    } else {
        w16_rwork<3>(pd, r00, l);
    }
}

// 16 x 16 factor of the symmetric block held as an accumulator (a00[q] = A[lr + 4q][lc]); on exit
// r00[q] = D[lr + 4q][lc] (lower, zero above), dg[0..15] = L_ii, *bad = first bad pivot + 1.
__device__ __forceinline__ void w16_acc(f64x4 a00, double* __restrict__ Pn, f64x4& r00, double* __restrict__ dg,
                                        int* __restrict__ bad) {
    const int l = threadIdx.x & 63, lc = l & 15, lr = l >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) r00[q] = (lr + 4 * q == lc) ? 1.0 : 0.0;
    double* dpv = Pn + 64;
    W1Pending pd;
    w16_round<0>(Pn, dpv, a00, r00, pd, l);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = lr + 4 * q;
        r00[q] = (lc <= r) ? r00[q] * rsq_nr(dpv[r]) : 0.0;
    }
    const double dl = dpv[l & 15];
    const unsigned long long m = __ballot(l < 16 && !(dl > 0.0 && dl < INFINITY));
    if (l < 16) dg[l] = dl * rsq_nr(dl);
    if (l == 0) *bad = m ? __ffsll((long long)m) : 0;
}

// accumulator <-> LDS 16 x 16 (stride ld)
__device__ __forceinline__ void acc16_to_lds(const f64x4& a, double* S, int ld) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 4; ++q) S[((l >> 4) + 4 * q) * ld + (l & 15)] = a[q];
}
// operand o[s] = M[li][4 s + lk]   (row li of M along the contraction index)
__device__ __forceinline__ void op16_rows(double o[4], const double* S, int ld) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < 4; ++s) o[s] = S[(l & 15) * ld + 4 * s + (l >> 4)];
}
// operand o[s] = M[4 s + lk][li]   (column li of M along the contraction index)
__device__ __forceinline__ void op16_cols(double o[4], const double* S, int ld) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < 4; ++s) o[s] = S[(4 * s + (l >> 4)) * ld + (l & 15)];
}
__device__ __forceinline__ void mma16(f64x4& c, const double a[4], const double b[4], bool neg) {
#pragma unroll
    for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f64_16x16x4f64(neg ? -a[s] : a[s], b[s], c, 0, 0, 0);
}

// 32 x 32 factor + inverse by one wave, recursively: X (LDS, stride ldx, lower triangle valid) ->
// R (stride S = 34) = L^{-1}, dg = L_ii.  W: >= 64 + 104 + 2 * 16 * 17 doubles of LDS scratch.
__device__ void rec32_wave(const double* __restrict__ X, int ldx, double* __restrict__ W, double* __restrict__ R,
                           double* __restrict__ dg, int* bad) {
    constexpr int S = TileCfg<32>::S, L16 = 17;
    const int l = threadIdx.x & 63, lc = l & 15, lr = l >> 4;
    double* Pn = W;
    double* Ls = W + 168;            // L21 (16 x 17)
    double* Ts = Ls + 16 * L16;      // T1 = L21 D11 (16 x 17)
    f64x4 a11, a22, a21;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = lr + 4 * q;
        const int hi = r > lc ? r : lc, lo = r > lc ? lc : r;
        a11[q] = X[hi * ldx + lo];
        a22[q] = X[(16 + hi) * ldx + 16 + lo];
    }
    double a21o[4];
    op16_rows(a21o, X + 16 * ldx, ldx);           // A21[li][4s + lk]
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int b1 = 0, b2 = 0;
    f64x4 d11, d22;
    w16_acc(a11, Pn, d11, dg, bad);
    acc16_to_lds(d11, R, S);                      // D11 -> R[0:16, 0:16]
    // L21 = A21 D11^T:  B[k][j] = D11[j][k] (row j of D11 along k)
    double d11r[4], d11c[4];
    op16_rows(d11r, R, S);
    op16_cols(d11c, R, S);
    f64x4 l21 = {0.0, 0.0, 0.0, 0.0};
    mma16(l21, a21o, d11r, false);
    acc16_to_lds(l21, Ls, L16);
    double l21o[4];
    op16_rows(l21o, Ls, L16);                     // L21[li][4s + lk]
    mma16(a22, l21o, l21o, true);                 // A22 -= L21 L21^T
    f64x4 t1 = {0.0, 0.0, 0.0, 0.0};
    mma16(t1, l21o, d11c, false);                 // T1 = L21 D11
    b1 = *bad;
    w16_acc(a22, Pn, d22, dg + 16, bad);
    b2 = *bad;
    acc16_to_lds(t1, Ts, L16);
    acc16_to_lds(d22, R + 16 * S + 16, S);
    double d22r[4], t1c[4];
    op16_rows(d22r, R + 16 * S + 16, S);
    op16_cols(t1c, Ts, L16);
    f64x4 d21 = {0.0, 0.0, 0.0, 0.0};
    mma16(d21, d22r, t1c, true);                  // D21 = -D22 T1
    acc16_to_lds(d21, R + 16 * S, S);
#pragma unroll
    for (int q = 0; q < 4; ++q) R[(lr + 4 * q) * S + 16 + lc] = 0.0;
    if (l == 0) *bad = b1 ? b1 : (b2 ? 16 + b2 : 0);
}


// ---- 8 pivots a round (4 rounds for NB = 32): the per-round fixed latency (LDS publish -> read,
// MFMA -> next publish) is paid half as often; the 8x8 LDL^T and the substitutions are 8 deep.
struct W8Pending {
    double L[8][8];
    double v[2][8];
};
template <int K>
__device__ __forceinline__ void w8_rwork(const W8Pending& pd, f64x4& r00, f64x4& r10, f64x4& r11, int l) {
    constexpr int bk = K >> 1, jj = K & 1;
    const int lc = l & 15, kk = l >> 4;
    double wR[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h < bk) { wR[h][0] = wR[h][1] = 0.0; continue; }
        const int row = 16 * h + lc;
        const bool piv = (row >> 3) == K;
        const bool below = row > 8 * K + 7;
        const int p = row & 7;
        double x[8];
#pragma unroll
        for (int t = 7; t >= 0; --t) {   // L^T x = v (back substitution)
            double acc = pd.v[h][t];
#pragma unroll
            for (int u = t + 1; u < 8; ++u) acc = fma(-pd.L[u][t], x[u], acc);
            x[t] = acc;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const double xk = sel4(kk, x[4 * c], x[4 * c + 1], x[4 * c + 2], x[4 * c + 3]);
            wR[h][c] = below ? xk : piv ? ((p == 4 * c + kk ? 1.0 : 0.0) - xk) : 0.0;
        }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if constexpr (bk == 0) {
            const double pR0 = r00[2 * jj + c];
            r00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[0][c], pR0, r00, 0, 0, 0);
            r10 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1][c], pR0, r10, 0, 0, 0);
        } else {
            const double pR0 = r10[2 * jj + c], pR1 = r11[2 * jj + c];
            r10 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1][c], pR0, r10, 0, 0, 0);
            r11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-wR[1][c], pR1, r11, 0, 0, 0);
        }
    }
}

template <int K>
__device__ __forceinline__ void w8_round(double* __restrict__ Pn, double* __restrict__ dpv, f64x4& a00, f64x4& a01,
                                         f64x4& a11, f64x4& r00, f64x4& r10, f64x4& r11, W8Pending& pd, int l) {
    if constexpr (K < 4) {
        constexpr int bk = K >> 1, jj = K & 1;
        const int lc = l & 15, kk = l >> 4;
        // publish A[8K + t][col] at Pn[col * 8 + t], t = 4e + kk
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            if constexpr (bk == 0) Pn[lc * 8 + 4 * e + kk] = a00[2 * jj + e];
            Pn[(16 + lc) * 8 + 4 * e + kk] = (bk == 0) ? a01[2 * jj + e] : a11[2 * jj + e];
        }
        asm volatile("" ::: "memory");
        double M[8][8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const f64x2* col = reinterpret_cast<const f64x2*>(Pn + (8 * K + u) * 8);
#pragma unroll
            for (int pr = u >> 1; pr < 4; ++pr) {
                const f64x2 v = col[pr];
                M[2 * pr][u] = v.x;
                M[2 * pr + 1][u] = v.y;
            }
        }
        double C[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h < bk) continue;
            const f64x2* row = reinterpret_cast<const f64x2*>(Pn + (16 * h + lc) * 8);
#pragma unroll
            for (int pr = 0; pr < 4; ++pr) {
                const f64x2 v = row[pr];
                C[h][2 * pr] = v.x;
                C[h][2 * pr + 1] = v.y;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K > 0) w8_rwork<K - 1>(pd, r00, r10, r11, l);
        __builtin_amdgcn_sched_barrier(0);
        // LDL^T of M: E[t][u] = (L D)[t][u]
        double L[8][8], E[8][8], d[8], iv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            double du = M[u][u];
#pragma unroll
            for (int w = 0; w < u; ++w) du = fma(-L[u][w], E[u][w], du);
            d[u] = du;
            iv[u] = rcp_nr1(du);
#pragma unroll
            for (int t = u + 1; t < 8; ++t) {
                double e = M[t][u];
#pragma unroll
                for (int w = 0; w < u; ++w) e = fma(-L[t][w], E[u][w], e);
                E[t][u] = e;
                L[t][u] = e * iv[u];
            }
        }
        double zA[2][2], yB[2][2], zs[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h < bk) { zA[h][0] = zA[h][1] = yB[h][0] = yB[h][1] = 0.0; continue; }
            const int row = 16 * h + lc;
            const bool below = row > 8 * K + 7;
            double y[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                double acc = C[h][t];
#pragma unroll
                for (int w = 0; w < t; ++w) acc = fma(-L[t][w], y[w], acc);
                y[t] = acc;
                zs[h][t] = y[t] * iv[t];
            }
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                zA[h][c] = below ? sel4(kk, zs[h][4 * c], zs[h][4 * c + 1], zs[h][4 * c + 2], zs[h][4 * c + 3]) : 0.0;
                yB[h][c] = sel4(kk, y[4 * c], y[4 * c + 1], y[4 * c + 2], y[4 * c + 3]);
            }
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if constexpr (bk == 0) {
                if constexpr (K == 0) {
                    a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0][c], yB[0][c], a00, 0, 0, 0);
                    a01 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0][c], yB[1][c], a01, 0, 0, 0);
                }
                a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1][c], yB[1][c], a11, 0, 0, 0);
            } else if constexpr (K == 2) {
                a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1][c], yB[1][c], a11, 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        dpv[l < 8 ? 8 * K + l : 40 + l] =
            (l & 4) ? sel4(l & 3, d[4], d[5], d[6], d[7]) : sel4(l & 3, d[0], d[1], d[2], d[3]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = 16 * h + lc;
            const bool piv = (row >> 3) == K;
            const int p = row & 7;
#pragma unroll
            for (int t = 0; t < 8; ++t) pd.v[h][t] = piv ? (p == t ? 1.0 : 0.0) : zs[h][t];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int u = 0; u < t; ++u) pd.L[t][u] = L[t][u];
        __builtin_amdgcn_sched_barrier(0);
        w8_round<K + 1>(Pn, dpv, a00, a01, a11, r00, r10, r11, pd, l);
    } else {
        w8_rwork<3>(pd, r00, r10, r11, l);
    }
}

// Drop-in for tile_potrf_inv_w1_wave (same interface; Pn: >= 256 + 104 doubles, may alias X).
__device__ __forceinline__ void tile_potrf_inv_w8_wave(const double* __restrict__ X, int ldx, double* __restrict__ Pn,
                                                       double* __restrict__ R, double* __restrict__ dg,
                                                       int* __restrict__ bad) {
    constexpr int S = TileCfg<32>::S;
    const int l = threadIdx.x & 63, lc = l & 15, lr = l >> 4;
    f64x4 a00, a01, a11, r00, r10 = {0.0, 0.0, 0.0, 0.0}, r11;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = lr + 4 * q;
        const int hi = r > lc ? r : lc, lo = r > lc ? lc : r;
        a00[q] = X[hi * ldx + lo];
        a11[q] = X[(16 + hi) * ldx + 16 + lo];
        a01[q] = X[(16 + lc) * ldx + r];
        r00[q] = (r == lc) ? 1.0 : 0.0;
        r11[q] = r00[q];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    double* dpv = Pn + 256;
    W8Pending pd;
    w8_round<0>(Pn, dpv, a00, a01, a11, r00, r10, r11, pd, l);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    double s0[4], s1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s0[q] = rsq_nr(dpv[lr + 4 * q]);
        s1[q] = rsq_nr(dpv[16 + lr + 4 * q]);
    }
    const double dl = dpv[l & 31];
    const unsigned long long m = __ballot(l < 32 && !(dl > 0.0 && dl < INFINITY));
    if (l < 32) dg[l] = dl * rsq_nr(dl);
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

template <int V>
__global__ __launch_bounds__(256) void k_fac(const double* Ag, double* Rg, double* dgg, long long* cyc, int* badg,
                                             int reps) {
    constexpr int S = TileCfg<NB>::S, E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem;
    double* R = A + E;
    double* dg = R + E;
    int* bad = reinterpret_cast<int*>(dg + NB + 2);
    double* ws = dg + NB + 8;
    long long tsum = 0;
    for (int it = 0; it < reps; ++it) {
        tile_load<NB>(A, Ag, NB);
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x < 64) {
            if (V == 0) tile_potrf_inv_w1_wave(A, S, ws, R, dg, bad);
            if (V == 1) rec32_wave(A, S, ws, R, dg, bad);
            if (V == 3) tile_potrf_inv_w8_wave(A, S, ws, R, dg, bad);
            if (V == 4) tile_potrf_inv_w8_wave(A, S, A, R, dg, bad);   // Pn aliasing X (the flow's use)
            if (V == 2) {   // one 16 x 16 factor alone (timing only)
                f64x4 a, r;
                const int l = threadIdx.x, lc = l & 15, lr = l >> 4;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = lr + 4 * q;
                    a[q] = A[(rr > lc ? rr : lc) * S + (rr > lc ? lc : rr)];
                }
                w16_acc(a, ws, r, dg, bad);
                acc16_to_lds(r, R, S);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        const long long t1 = __builtin_amdgcn_s_memtime();
        if (it > 0) tsum += t1 - t0;
        __syncthreads();
    }
    tile_store<NB>(Rg, NB, R);
    if (threadIdx.x < NB) dgg[threadIdx.x] = dg[threadIdx.x];
    if (threadIdx.x == 0) { cyc[V] = tsum / (reps - 1); badg[V] = *bad; }
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

template <int V>
static void run(const char* name, const double* hA, const double* dA, double* dR, double* dd, long long* dc, int* db) {
    const size_t sm = sizeof(double) * (2 * TileCfg<NB>::ELEMS + NB + 8 + 800);
    hipLaunchKernelGGL(k_fac<V>, dim3(1), dim3(256), sm, 0, dA, dR, dd, dc, db, 50);
    (void)hipDeviceSynchronize();
    double R[NB * NB], dg[NB];
    long long c[8] = {};
    int b[8];
    (void)hipMemcpy(R, dR, sizeof(R), hipMemcpyDeviceToHost);
    (void)hipMemcpy(dg, dd, sizeof(dg), hipMemcpyDeviceToHost);
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(b, db, sizeof(b), hipMemcpyDeviceToHost);
    static long double Li[NB * NB], Ld[NB];
    host_ref(hA, Li, Ld);
    long double eR = 0, mR = 0, eD = 0;
    const int n = V == 2 ? 16 : NB;   // V == 2: the leading 16 x 16 block only
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) { eR = fmaxl(eR, fabsl(R[i * NB + j] - Li[i * NB + j])); mR = fmaxl(mR, fabsl(Li[i * NB + j])); }
    for (int i = 0; i < n; ++i) eD = fmaxl(eD, fabsl(dg[i] - Ld[i]) / Ld[i]);
    printf("%-12s %7lld clk  max|D-Dref|/max|Dref| = %.2e  max rel L_ii err = %.2e  bad=%d\n", name, c[V],
           (double)(eR / mR), (double)eD, b[V]);
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
        run<0>("w1 (lib)", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<1>("rec32 (2xw16)", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<2>("w16 alone", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<3>("w8 rounds", hA[m], dA + m * NB * NB, dR, dd, dc, db);
        run<4>("w8 aliased", hA[m], dA + m * NB * NB, dR, dd, dc, db);
    }
    return 0;
}
