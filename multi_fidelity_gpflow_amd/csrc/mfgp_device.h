// Device-side building blocks for the MI355X (gfx950) multi-fidelity GP engine.
//
// Tiles are NB x NB fp64 blocks (NB = 32 or 64).  A workgroup is 256 threads
// (4 wave64s).  Tiles live in LDS row-major with stride S = NB + 2 (even, so a
// thread can move a 16-byte pair; the +2 pad makes the MFMA operand reads of
// the "A = M" / "B = M^T" orientation bank-conflict free and the others 2-way).
//
// Tile products use the gfx950 FP64 matrix core: v_mfma_f64_16x16x4_f64.
//   A/B operands: lane l supplies A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15]
//   C/D (4 x f64 per lane): C[row = (l>>4) + 4*r][col = l&15], r = 0..3
// (cdna_hip_programming.md §3 "f64 MFMA does NOT use these maps").  The same
// element ownership is used by the VALU fallback so epilogues are shared; the
// GPU self-test mfgp_selftest_mfma() checks the MFMA path against it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfgp {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int NTHREADS = 256;

template <int NB>
struct TileCfg {
    static constexpr int S = NB + 2;                 // LDS row stride (doubles)
    static constexpr int ELEMS = NB * S;             // doubles per LDS tile
    static constexpr int NBLK = (NB / 16) * (NB / 16) / 4;   // 16x16 blocks per wave
    static constexpr int BPW = (NB / 16) / 2;        // blocks per wave per dim (1 or 2)
};

// ---------------------------------------------------------------- ownership
// Accumulator of one thread: NBLK blocks x 4 doubles.  Block q of wave w covers
// rows 16*(BPW*(w>>1) + q/BPW) and cols 16*(BPW*(w&1) + q%BPW).
template <int NB>
struct Acc {
    f64x4 v[TileCfg<NB>::NBLK];
};

template <int NB>
__device__ __forceinline__ int acc_row(int q, int r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int BPW = TileCfg<NB>::BPW;
    return 16 * (BPW * (w >> 1) + q / BPW) + (lane >> 4) + 4 * r;
}
template <int NB>
__device__ __forceinline__ int acc_col(int q) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int BPW = TileCfg<NB>::BPW;
    return 16 * (BPW * (w & 1) + q % BPW) + (lane & 15);
}

template <int NB>
__device__ __forceinline__ void acc_zero(Acc<NB>& a) {
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q) a.v[q] = f64x4{0.0, 0.0, 0.0, 0.0};
}

// acc <- global tile (row-major, ld), rows/cols beyond (nr, nc) read as 0
template <int NB>
__device__ __forceinline__ void acc_load(Acc<NB>& a, const double* __restrict__ g, long ld) {
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) a.v[q][r] = g[(long)acc_row<NB>(q, r) * ld + acc_col<NB>(q)];
}
template <int NB>
__device__ __forceinline__ void acc_store(const Acc<NB>& a, double* __restrict__ g, long ld) {
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) g[(long)acc_row<NB>(q, r) * ld + acc_col<NB>(q)] = a.v[q][r];
}
// ---- cross-workgroup hand-off without L2 flushes.  gfx950 has one L2 per XCD, so an
// agent-scope fence (__threadfence) writes back / invalidates the whole L2
// (buffer_wbl2 / buffer_inv sc1, microseconds).  Data that another workgroup reads in
// the same launch is instead stored and loaded as agent-scope relaxed atomics
// (global_store / global_load ... sc1: coherent at the device level); a producer drains
// its stores (s_waitcnt 0) before the workgroup barrier and the counter atomic.
__device__ __forceinline__ void st_coherent(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_coherent(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { __builtin_amdgcn_s_waitcnt(0); }
// Call after drain_stores() + __syncthreads(); thread 0 only.  Returns the old count.
__device__ __forceinline__ int arrive(int* c) {
    return __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int NB>
__device__ __forceinline__ void acc_store_coherent(const Acc<NB>& a, double* __restrict__ g, long ld) {
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) st_coherent(g + (long)acc_row<NB>(q, r) * ld + acc_col<NB>(q), a.v[q][r]);
}
template <int NB>
__device__ __forceinline__ void acc_to_lds(const Acc<NB>& a, double* __restrict__ s) {
    constexpr int S = TileCfg<NB>::S;
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[acc_row<NB>(q, r) * S + acc_col<NB>(q)] = a.v[q][r];
}

// ---------------------------------------------------------------- XCD-aware block order
// For (gx, 1, gz) grids.  Workgroups are dealt round-robin over the 8 XCDs (8 private L2s), so the tiles of one batch entry
// (one SVGP latent: its K_uf, L^{-1}, C, ... shared by all its output tiles) land on every XCD and
// every L2 fetches them.  This remap hands each XCD a contiguous chunk of the logical (x, z) grid
// (cdna_hip_programming.md T1): dispatch slot b -> logical (b % 8) * cpx + b / 8 for the first
// 8 * cpx slots (cpx = nwg / 8), the remainder unchanged (a bijection for any grid).  Placement
// only: every logical block computes the same thing wherever it runs.
__device__ __forceinline__ void xcd_swizzle(int& x, int& z) {
    const int gx = gridDim.x;
    const int nwg = gx * gridDim.z;
    const int b = blockIdx.x + gx * blockIdx.z;
    const int cpx = nwg >> 3;
    const int s = b < 8 * cpx ? (b & 7) * cpx + (b >> 3) : b;
    x = s % gx;
    z = s / gx;
}

// ---------------------------------------------------------------- tile moves
// LDS tile (row-major, stride S) <- global tile (row-major, ld).  16-byte moves.
template <int NB>
__device__ __forceinline__ void tile_load(double* __restrict__ s, const double* __restrict__ g, long ld) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int PAIRS = NB * NB / 2;
#pragma unroll
    for (int p = threadIdx.x; p < PAIRS; p += NTHREADS) {
        const int r = p / (NB / 2), c = 2 * (p % (NB / 2));
        const double2 v = *reinterpret_cast<const double2*>(g + (long)r * ld + c);
        *reinterpret_cast<double2*>(s + r * S + c) = v;
    }
}
// Split tile_load for software pipelining: fetch (global -> registers, returns at
// once) and put (registers -> LDS, waits for the fetch).
// (native <2 x double>: HIP's double2 struct is not promoted to registers when it is
// carried around a loop, it lands in scratch)
typedef double f64x2 __attribute__((ext_vector_type(2)));
template <int NB>
struct TileRegs {
    f64x2 v[NB * NB / 2 / NTHREADS];
};
template <int NB>
__device__ __forceinline__ void tile_fetch(TileRegs<NB>& r, const double* __restrict__ g, long ld) {
#pragma unroll
    for (int q = 0; q < NB * NB / 2 / NTHREADS; ++q) {
        const int p = threadIdx.x + q * NTHREADS;
        const int row = p / (NB / 2), c = 2 * (p % (NB / 2));
        r.v[q] = *reinterpret_cast<const f64x2*>(g + (long)row * ld + c);
    }
}
template <int NB>
__device__ __forceinline__ void tile_put(double* __restrict__ s, const TileRegs<NB>& r) {
    constexpr int S = TileCfg<NB>::S;
#pragma unroll
    for (int q = 0; q < NB * NB / 2 / NTHREADS; ++q) {
        const int p = threadIdx.x + q * NTHREADS;
        const int row = p / (NB / 2), c = 2 * (p % (NB / 2));
        *reinterpret_cast<f64x2*>(s + row * S + c) = r.v[q];
    }
}
template <int NB>
__device__ __forceinline__ void tile_store(double* __restrict__ g, long ld, const double* __restrict__ s) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int PAIRS = NB * NB / 2;
#pragma unroll
    for (int p = threadIdx.x; p < PAIRS; p += NTHREADS) {
        const int r = p / (NB / 2), c = 2 * (p % (NB / 2));
        *reinterpret_cast<double2*>(g + (long)r * ld + c) = *reinterpret_cast<const double2*>(s + r * S + c);
    }
}

// ---------------------------------------------------------------- tile product
// acc += alpha * op(A) * op(B), A/B LDS tiles (row-major stride S).
// TA: op(A) = A^T ; TB: op(B) = B^T.
template <int NB, bool TA, bool TB>
__device__ __forceinline__ void tile_mma(Acc<NB>& acc, const double* __restrict__ As,
                                         const double* __restrict__ Bs, double alpha) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int BPW = TileCfg<NB>::BPW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int rb = 16 * BPW * (w >> 1), cb = 16 * BPW * (w & 1);
#pragma unroll 4
    for (int k0 = 0; k0 < NB; k0 += 4) {
        const int k = k0 + lk;
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
            for (int tj = 0; tj < BPW; ++tj)
                acc.v[ti * BPW + tj] =
                    __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], acc.v[ti * BPW + tj], 0, 0, 0);
    }
}

// ---------------------------------------------------------------- scalar helpers
// 1/a by v_rcp_f64 + two Newton steps (<= 1 ulp; shorter dependent chain than the
// IEEE div sequence on the pivot critical path).
__device__ __forceinline__ double rcp_nr(double a) {
    double r = __builtin_amdgcn_rcp(a);
    double e = fma(-a, r, 1.0);
    r = fma(r, e, r);
    e = fma(-a, r, 1.0);
    return fma(r, e, r);
}

// 1/a by v_rcp_f64 + ONE Newton step (v_rcp_f64 is 4.6e-8 relative, one step 2.2e-15:
// tools/ubench_rcp.hip); for the pivot chain of the diagonal factor.
__device__ __forceinline__ double rcp_nr1(double a) {
    const double r = __builtin_amdgcn_rcp(a);
    return fma(r, fma(-a, r, 1.0), r);
}
// 1/sqrt(a) by v_rsq_f64 + two Newton steps y <- y (1 + (1 - a y^2) / 2).
__device__ __forceinline__ double rsq_nr(double a) {
    double y = __builtin_amdgcn_rsq(a);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double e = fma(-a * y, y, 1.0);
        y = fma(0.5 * y, e, y);
    }
    return y;
}

// ---------------------------------------------------------------- parameter transforms
__device__ __forceinline__ double tf_softplus(double x) {
    // tensorflow/core/kernels/softplus_op.h
    const double thr = -34.04365338911715;   // log(DBL_EPSILON) + 2
    if (x > -thr) return x;
    if (x < thr) return exp(x);
    return log(exp(x) + 1.0);
}

// ---------------------------------------------------------------- pivot check
// First non-positive / non-finite pivot of an NB = 32 tile (1-based, 0 if none) without a
// serial scan (a dependent LDS walk costs ~3.8k clocks): thread (row i = t/8, g = t%8 == 0)
// flags its row, one ballot per wave, lane 0 writes the wave's first row into slot[w].
// slot[] (4 ints) must be read back after a barrier: pivot_check_result().
__device__ __forceinline__ void pivot_check_post(double d, int* slot) {
    const int t = threadIdx.x;
    const bool fl = ((t & 7) == 0) && !(d > 0.0 && d < INFINITY);
    const unsigned long long m = __ballot(fl);
    if ((t & 63) == 0) slot[t >> 6] = m ? 8 * (t >> 6) + (__ffsll((long long)m) - 1) / 8 + 1 : 0;
}
__device__ __forceinline__ int pivot_check_result(const int* slot) {
    const int s0 = slot[0], s1 = slot[1], s2 = slot[2], s3 = slot[3];
    return s0 ? s0 : s1 ? s1 : s2 ? s2 : s3;
}

// ---------------------------------------------------------------- diag factor
// Cholesky of an SPD NB x NB tile A fused with the inverse of its factor.
// On exit R holds D = L^{-1} (lower, zero above) and dg[i] = L_ii.
// Right-looking on the unscaled pivot column (LDL^T-style recurrences):
//   a_ij -= a_ik a_jk / a_kk   (i >= j > k),     r_ic -= a_ik r_kc / a_kk   (c <= k < i)
// and at the end L_ii = sqrt(a_ii), D_ic = r_ic / L_ii.
//
// NB = 32 (the latency-critical case): every thread owns row i = t/8 and columns
// 4g..4g+3 (g = t%8) of BOTH A and R in registers.  Each pivot costs one barrier:
// the owners of the next pivot column of A / row of R publish them (unscaled) into a
// ping-pong LDS buffer together with 1/a_kk computed by the diagonal owner; everyone
// else reads 1 + 2 + 2 LDS words (b128) and applies <= 8 FMAs.
// Non-positive or non-finite pivots report through *bad (first local index + 1).
template <int NB>
__device__ void tile_potrf_inv(double* __restrict__ A, double* __restrict__ R, double* __restrict__ dg,
                               int* __restrict__ bad);

// ---------------------------------------------------------------- single-wave diag factor
// NB = 32 Cholesky + inverse by ONE wavefront, no workgroup barrier on the pivot chain
// (a 4-wave publish -> barrier -> read round trip costs ~160 clocks, an in-wave LDS round trip
// ~120 and an f64 MFMA accumulator hop 64: tools/ubench_lat2.hip).  Wave 0 holds the whole
// symmetric tile as three 16x16 MFMA accumulator blocks A00, A01 (= A10^T), A11 and the inverse
// as R00, R10, R11 (lane l: rows 16bi + (l>>4) + 4q, column 16bj + (l&15)).  Round K = 0..7
// eliminates pivots P = 4K..4K+3 (block LDL^T, un-normalised pivot rows):
//   * lanes publish the pivot rows A[P, :] (= the pivot columns) into an LDS panel, then every
//     lane reads the 4x4 pivot block M = L_M D_M L_M^T (factored redundantly in registers, the
//     m4 elimination order) and its own rows C_i = A[i, P];
//   * row i below P: W_i = C_i M^{-1} = ((C_i L_M^{-T}) D_M^{-1}) L_M^{-1} by substitution;
//     pivot row p: W_R = I - T with T = D_M^{-1/2} L_M^{-1} (row p of L_M^{-1} by the same
//     back substitution on e_p); rows above P: 0;
//   * A -= W A[P, :] and R -= W_R R[P, :]: one v_mfma_f64_16x16x4 per block, with the pivot
//     rows of A and R as the B operand exactly as they sit in the accumulator (register K&3),
//     and W in A-operand layout straight from the lane's own substitution.
// R then holds L^{-1} = blockdiag(T) L_u^{-1}.  Input: a symmetric tile whose lower triangle is
// valid, in LDS (X, stride ldx); the upper triangle is never read.  Pn: 128 doubles of LDS that
// may alias X (wave 0 has read X before it first writes Pn).  All waves must call; waves 1..3
// only meet the closing barrier.
// The panel is published and read back by the same wave: its DS operations are processed in
// issue order, so only the compiler has to be kept from reordering them (no lgkmcnt wait).
// 4-way select on the low two bits of s as two levels of v_cndmask (an equality chain
// compiles to exec-mask branches, which break the scheduling region of the pivot chain)
__device__ __forceinline__ double sel4(int s, double v0, double v1, double v2, double v3) {
    const bool b0 = (s & 1) != 0, b1 = (s & 2) != 0;
    const double lo = b0 ? v1 : v0, hi = b0 ? v3 : v2;
    return b1 ? hi : lo;
}

// R work of round K, deferred into round K+1 (after its LDS reads are issued) so that the
// in-order issue of the A chain is never held behind it: X = V L_M^{-1}, W_R, R -= W_R R[P, :].
// The lane-constant selections of the single-wave factor (component kk = l >> 4 of a row's four
// values, the unit vector e_p of pivot row p = l & 3) are one-hot products / selects of per-lane
// constants formed once, instead of v_cndmask trees rebuilt every round (8.1k -> 7.65k clocks for
// the NB = 32 factor, bit-identical; tools/ubench_rsplit.hip)
struct W1Pending {
    double L10, L20, L30, L21, L31, L32;
    double v[2][4];   // rows h = 0, 1: Z (rows below) or e_p (pivot rows)
    double u[4];      // u[c] = (kk == c)
    double e[4];      // e[c] = (p == c)
    double ekk;       // (p == kk)
};
__device__ __forceinline__ void w1_consts(W1Pending& pd, int l) {
    const int kk = l >> 4, p = l & 3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        pd.u[c] = (kk == c) ? 1.0 : 0.0;
        pd.e[c] = (p == c) ? 1.0 : 0.0;
    }
    pd.ekk = (p == kk) ? 1.0 : 0.0;
}
// component kk of (a0, a1, a2, a3): exact for finite values (one term is 1 x a_kk, the rest 0 x a_c)
__device__ __forceinline__ double w1_pick(const W1Pending& pd, int kk, double a0, double a1, double a2, double a3) {
    (void)kk;
    return fma(pd.u[3], a3, fma(pd.u[2], a2, fma(pd.u[1], a1, pd.u[0] * a0)));
}

template <int K>
__device__ __forceinline__ void w1_rwork(const W1Pending& pd, f64x4& r00, f64x4& r10, f64x4& r11, int l) {
    constexpr int bk = K >> 2, kq = K & 3;
    const int lc = l & 15, kk = l >> 4, p = lc & 3;
    double wR[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h < bk) { wR[h] = 0.0; continue; }
        const int row = 16 * h + lc;
        const bool piv = (row >> 2) == K;
        const bool below = row > 4 * K + 3;
        const double x3 = pd.v[h][3];
        const double x2 = fma(-pd.L32, x3, pd.v[h][2]);
        const double x1 = fma(-pd.L31, x3, fma(-pd.L21, x2, pd.v[h][1]));
        const double x0 = fma(-pd.L30, x3, fma(-pd.L20, x2, fma(-pd.L10, x1, pd.v[h][0])));
        const double xk = w1_pick(pd, kk, x0, x1, x2, x3);
        wR[h] = below ? xk : piv ? (pd.ekk - xk) : 0.0;
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
}

template <int K>
__device__ __forceinline__ void w1_round(double* __restrict__ Pn, double* __restrict__ dpv, f64x4& a00, f64x4& a01,
                                         f64x4& a11, f64x4& r00, f64x4& r10, f64x4& r11, W1Pending& pd, int l) {
    if constexpr (K < 8) {
        constexpr int bk = K >> 2, kq = K & 3;
        const int lc = l & 15, kk = l >> 4;
        // ---- publish A[4K + kk][col] at Pn[col * 4 + kk]
        if constexpr (bk == 0) Pn[lc * 4 + kk] = a00[kq];
        Pn[(16 + lc) * 4 + kk] = (bk == 0) ? a01[kq] : a11[kq];
        asm volatile("" ::: "memory");   // keep the compiler from reordering publish / read
        // ---- pivot block (column j of M at Pn[(4K + j) * 4 .. + 3])
        const f64x2* Pm = reinterpret_cast<const f64x2*>(Pn + 16 * K);
        const f64x2 c0a = Pm[0], c0b = Pm[1], c1a = Pm[2], c1b = Pm[3], c2b = Pm[5], c3b = Pm[7];
        // ---- own rows C_i, i = 16h + lc (h = 1 always, h = 0 while bk == 0)
        const f64x2* Pr = reinterpret_cast<const f64x2*>(Pn);
        f64x2 u0a = {0.0, 0.0}, u0b = {0.0, 0.0};
        if constexpr (bk == 0) { u0a = Pr[2 * lc]; u0b = Pr[2 * lc + 1]; }
        const f64x2 u1a = Pr[2 * (16 + lc)], u1b = Pr[2 * (16 + lc) + 1];
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K > 0) w1_rwork<K - 1>(pd, r00, r10, r11, l);
        __builtin_amdgcn_sched_barrier(0);
        const double m00 = c0a.x, m10 = c0a.y, m20 = c0b.x, m30 = c0b.y;
        const double m11 = c1a.y, m21 = c1b.x, m31 = c1b.y, m22 = c2b.x, m32 = c2b.y, m33 = c3b.y;
        // ---- LDL^T of M
#define W1RCP(x) rcp_nr1(x)
        const double i0 = W1RCP(m00);
        const double L10 = m10 * i0, L20 = m20 * i0, L30 = m30 * i0;
        const double d1 = fma(-L10, m10, m11);
        const double i1 = W1RCP(d1);
        const double e21 = fma(-L20, m10, m21), e31 = fma(-L30, m10, m31);
        const double L21 = e21 * i1, L31 = e31 * i1;
        const double d2 = fma(-L21, e21, fma(-L20, m20, m22));
        const double i2 = W1RCP(d2);
        const double e32 = fma(-L31, e21, fma(-L30, m20, m32));
        const double L32 = e32 * i2;
        const double d3 = fma(-L32, e32, fma(-L31, e31, fma(-L30, m30, m33)));
        const double i3 = W1RCP(d3);
#undef W1RCP
        // ---- per row: Y = C L_M^{-T}, Z = Y D_M^{-1}; A -= Z Y^T (symmetric form)
        double zA[2], yB[2], zs[2][4] = {};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h < bk) { zA[h] = 0.0; yB[h] = 0.0; continue; }
            const f64x2 ua = h ? u1a : u0a, ub = h ? u1b : u0b;
            const int row = 16 * h + lc;
            const bool piv = (row >> 2) == K;
            const bool below = row > 4 * K + 3;
            const int p = lc & 3;
            const double y0 = ua.x;
            const double y1 = fma(-L10, y0, ua.y);
            const double y2 = fma(-L21, y1, fma(-L20, y0, ub.x));
            const double y3 = fma(-L32, y2, fma(-L31, y1, fma(-L30, y0, ub.y)));
            const double z0 = y0 * i0, z1 = y1 * i1, z2 = y2 * i2, z3 = y3 * i3;
            zA[h] = below ? w1_pick(pd, kk, z0, z1, z2, z3) : 0.0;
            yB[h] = w1_pick(pd, kk, y0, y1, y2, y3);
            zs[h][0] = z0; zs[h][1] = z1; zs[h][2] = z2; zs[h][3] = z3;
        }
        // ---- rank-4 update of A on the matrix core (an f64 MFMA holds the SIMD for 64 clocks,
        //      f64 VALU included: after round 3 rows 0..15 are final, so A00 / A01 are skipped)
        if constexpr (bk == 0) {
            if constexpr (K < 3) {
                a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0], yB[0], a00, 0, 0, 0);
                a01 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[0], yB[1], a01, 0, 0, 0);
            }
            a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1], yB[1], a11, 0, 0, 0);
        } else {
            a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(-zA[1], yB[1], a11, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- off the A chain (issued under the MFMA latency): pivots to LDS, R-work inputs
        dpv[l < 4 ? 4 * K + l : 40 + l] = sel4(l & 3, m00, d1, d2, d3);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool piv = ((16 * h + lc) >> 2) == K;
#pragma unroll
            for (int c = 0; c < 4; ++c) pd.v[h][c] = piv ? pd.e[c] : zs[h][c];
        }
        pd.L10 = L10; pd.L20 = L20; pd.L30 = L30; pd.L21 = L21; pd.L31 = L31; pd.L32 = L32;
        __builtin_amdgcn_sched_barrier(0);
        w1_round<K + 1>(Pn, dpv, a00, a01, a11, r00, r10, r11, pd, l);
    } else {
        w1_rwork<7>(pd, r00, r10, r11, l);
    }
}

// Body run by ONE wave (any wave of the workgroup; no workgroup barrier inside).
__device__ __forceinline__ void tile_potrf_inv_w1_wave(const double* __restrict__ X, int ldx, double* __restrict__ Pn,
                                                       double* __restrict__ R, double* __restrict__ dg,
                                                       int* __restrict__ bad) {
    constexpr int S = TileCfg<32>::S;
    {
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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // X fully read before Pn (may alias) is written
        double* dpv = Pn + 128;                                // [32] pivots + dump slots
        W1Pending pd;
        w1_consts(pd, l);
        w1_round<0>(Pn, dpv, a00, a01, a11, r00, r10, r11, pd, l);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // L^{-1} = diag(d)^{-1/2} L_u^{-1}; L_ii = sqrt(d_i); first bad pivot by one ballot
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
}

__device__ __forceinline__ void tile_potrf_inv_w1_core(const double* __restrict__ X, int ldx, double* __restrict__ Pn,
                                                       double* __restrict__ R, double* __restrict__ dg,
                                                       int* __restrict__ bad) {
    if (threadIdx.x < 64) tile_potrf_inv_w1_wave(X, ldx, Pn, R, dg, bad);
    __syncthreads();
}

// Entry from an LDS tile A (row-major, stride S, lower triangle valid); A doubles as the panel.
__device__ __forceinline__ void tile_potrf_inv_w1(double* A, double* R, double* dg, int* bad) {
    tile_potrf_inv_w1_core(A, TileCfg<32>::S, A, R, dg, bad);
}

// Entry with the tile in accumulator layout (the Acc<32> of tile_mma: wave w holds block
// (w>>1, w&1)); scratch: >= 32 * 33 doubles of LDS nobody reads concurrently.
__device__ __forceinline__ void tile_potrf_inv_w1_acc(f64x4 aA, double* scratch, double* R, double* dg, int* bad) {
    constexpr int LX = 33;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int bi = w >> 1, bj = w & 1;
    if (bj <= bi) {
#pragma unroll
        for (int q = 0; q < 4; ++q) scratch[(16 * bi + (l >> 4) + 4 * q) * LX + 16 * bj + (l & 15)] = aA[q];
    }
    __syncthreads();
    tile_potrf_inv_w1_core(scratch, LX, scratch, R, dg, bad);
}

template <>
__device__ __forceinline__ void tile_potrf_inv<32>(double* __restrict__ A, double* __restrict__ R,
                                                   double* __restrict__ dg, int* __restrict__ bad) {
    tile_potrf_inv_w1(A, R, dg, bad);
}

// ---------------------------------------------------------------- blocked diag factor
// Cholesky + inverse of an NB x NB SPD tile in 8-column blocks (NB = 32 or 64).
// Per 8-block b (unrolled):
//   1. EVERY thread loads the 8x8 pivot block and factors it redundantly in registers
//      (no cross-lane communication on the pivot chain);
//   2. one thread per row below forward-substitutes its panel row: L_rb = A_rb L_bb^{-T};
//   3. barrier; all threads apply the rank-8 trailing update; barrier.
// Then D = L^{-1}: 8x8 diagonal inverses (one wave per block, redundant per lane),
// and the off-diagonal blocks by the level recurrence
//   D_ib = -D_ii sum_{m=b}^{i-1} L_im D_mb   (level = i - b), two barriers per level.
// On exit: R = D (lower, zero above), dg[i] = L_ii, *bad = first non-positive pivot + 1.
// A holds L in its lower part (upper part garbage).
template <int NB>
__device__ void tile_potrf_inv_b8(double* __restrict__ A, double* __restrict__ R, double* __restrict__ dg,
                                  int* __restrict__ bad, long long* stamps = nullptr) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int NBLK8 = NB / 8;
    const int t = threadIdx.x;
    int badloc = 0;
#pragma unroll
    for (int b = 0; b < NBLK8; ++b) {
        const int r0 = 8 * b;
        // 1. redundant 8x8 potrf in registers
        double l[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) l[i][j] = A[(r0 + i) * S + r0 + j];
        double rinv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double akk = l[k][k];
            if (badloc == 0 && !(akk > 0.0 && akk < INFINITY)) badloc = r0 + k + 1;
            const double lkk = sqrt(akk);
            const double rk = 1.0 / lkk;
            l[k][k] = lkk;
            rinv[k] = rk;
#pragma unroll
            for (int i = k + 1; i < 8; ++i) l[i][k] *= rk;
#pragma unroll
            for (int j = k + 1; j < 8; ++j)
#pragma unroll
                for (int i = j; i < 8; ++i) l[i][j] -= l[i][k] * l[j][k];
        }
        // 2. panel rows below (one thread per row) + publish L_bb and dg
        constexpr int dummy = 0;
        (void)dummy;
        const int rows = NB - r0 - 8;
        if (t < rows) {
            const int r = r0 + 8 + t;
            double x[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) x[c] = A[r * S + r0 + c];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                double v = x[c];
#pragma unroll
                for (int m = 0; m < c; ++m) v -= x[m] * l[c][m];
                x[c] = v * rinv[c];
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) A[r * S + r0 + c] = x[c];
        }
        __syncthreads();   // every wave has read the pivot block before it is overwritten
        if (t == NTHREADS - 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                dg[r0 + i] = l[i][i];
#pragma unroll
                for (int j = 0; j <= i; ++j) A[(r0 + i) * S + r0 + j] = l[i][j];
            }
        }
        // 3. trailing rank-8 update of the lower part (square index space, upper skipped)
        if (rows > 0) {
            for (int e = t; e < rows * rows; e += NTHREADS) {
                const int ii = e / rows, jj = e - (e / rows) * rows;
                if (jj > ii) continue;
                const int i = r0 + 8 + ii, j = r0 + 8 + jj;
                const double2* pi = reinterpret_cast<const double2*>(A + i * S + r0);
                const double2* pj = reinterpret_cast<const double2*>(A + j * S + r0);
                double acc = A[i * S + j];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const double2 u = pi[m], v = pj[m];
                    acc -= u.x * v.x;
                    acc -= u.y * v.y;
                }
                A[i * S + j] = acc;
            }
        }
        __syncthreads();
    }
    if (t == 0) *bad = badloc;
    if (stamps && t == 0) stamps[0] = __builtin_amdgcn_s_memtime();
    // ---- D = L^{-1}
    // (a) diagonal 8x8 inverses: wave w handles blocks b = w, w+4, ...
    const int w = t >> 6, lane = t & 63;
    for (int b = w; b < NBLK8; b += NTHREADS / 64) {
        const int r0 = 8 * b;
        double l[8][8], d[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) l[i][j] = A[(r0 + i) * S + r0 + j];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double ri = 1.0 / l[i][i];
            d[i][i] = ri;
#pragma unroll
            for (int j = 0; j < i; ++j) {
                double s = 0.0;
#pragma unroll
                for (int m = j; m < i; ++m) s += l[i][m] * d[m][j];
                d[i][j] = -s * ri;
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) R[(r0 + i) * S + r0 + j] = (j <= i) ? d[i][j] : 0.0;
        }
    }
    __syncthreads();
    if (stamps && t == 0) stamps[1] = __builtin_amdgcn_s_memtime();
    // (b) off-diagonal blocks by level; the temporary T_ib = sum_m L_im D_mb lives in the
    //     (still unused) upper block (b, i) of R.
#pragma unroll
    for (int lev = 1; lev < NBLK8; ++lev) {
        const int nblk = NBLK8 - lev;
        for (int e = t; e < nblk * 64; e += NTHREADS) {
            const int b = e >> 6, rc = e & 63, r = rc >> 3, c = rc & 7;
            const int i = b + lev;
            double s = 0.0;
            for (int m = b; m < i; ++m) {
#pragma unroll
                for (int q = 0; q < 8; ++q) s += A[(8 * i + r) * S + 8 * m + q] * R[(8 * m + q) * S + 8 * b + c];
            }
            R[(8 * b + r) * S + 8 * i + c] = s;   // T_ib[r][c] in the upper block (b, i)
        }
        __syncthreads();
        for (int e = t; e < nblk * 64; e += NTHREADS) {
            const int b = e >> 6, rc = e & 63, r = rc >> 3, c = rc & 7;
            const int i = b + lev;
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) s += R[(8 * i + r) * S + 8 * i + q] * R[(8 * b + q) * S + 8 * i + c];
            R[(8 * i + r) * S + 8 * b + c] = -s;
        }
        __syncthreads();
    }
    // zero the upper part of R (D is lower triangular)
    for (int e = t; e < NB * NB; e += NTHREADS) {
        const int i = e / NB, c = e - (e / NB) * NB;
        if ((c >> 3) > (i >> 3)) R[i * S + c] = 0.0;
    }
    __syncthreads();
}

// NB = 64 uses the blocked form: 8 blocks of 8 pivots (measured 63k vs 216k shader clocks
// for the one-barrier-per-pivot form, tools/ubench_tile.hip).
template <>
__device__ __forceinline__ void tile_potrf_inv<64>(double* __restrict__ A, double* __restrict__ R,
                                                   double* __restrict__ dg, int* __restrict__ bad) {
    tile_potrf_inv_b8<64>(A, R, dg, bad);
}


// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum over each quad of lanes (xor 1, xor 2) with quad_perm DPP moves: no LDS crossbar
// traffic, a few cycles per step (a __shfl_xor of a double is two ds_bpermute).
template <int CTRL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double quad_sum(double v) {
    v += dpp_mov_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    return v;
}

// Sum v over the 256-thread workgroup; result valid in every thread.
// scratch: >= 4 doubles of LDS.  Contains two barriers.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) scratch[w] = v;
    __syncthreads();
    const double s = (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
    __syncthreads();
    return s;
}

// ---------------------------------------------------------------- MF kernel math
// theta (constrained, fp64): [vL, lL(D), vD, lD(D), rho0, noise]
struct MFTheta {
    const double* t;
    int D;
    __device__ double vL() const { return t[0]; }
    __device__ double lL(int d) const { return t[1 + d]; }
    __device__ double vD() const { return t[1 + D]; }
    __device__ double lD(int d) const { return t[2 + D + d]; }
    __device__ double rho() const { return t[2 + 2 * D]; }
    __device__ double noise() const { return t[3 + 2 * D]; }
};

__host__ __device__ constexpr int theta_size(int D) { return 2 * D + 4; }

// GraphMultiFidelityKernel (mfgpflow/graph.py:7-115) with m LF sources: theta layout
//   [v_0, l_0(D), .., v_{m-1}, l_{m-1}(D), v_delta, l_delta(D), rho_0..rho_{m-1},
//    rhoLF (m x m, row-major; diagonal unused), noise]
constexpr int MFGP_MAX_LF = 4;
struct GraphTheta {
    const double* t;
    int D, m;
    __device__ double v(int s) const { return t[s * (1 + D)]; }            // s = m: delta
    __device__ double l(int s, int d) const { return t[s * (1 + D) + 1 + d]; }
    __device__ double rho(int i) const { return t[(m + 1) * (1 + D) + i]; }
    __device__ double rhoLF(int i, int j) const { return t[(m + 1) * (1 + D) + m + i * m + j]; }
};
__host__ __device__ constexpr int graph_theta_size(int m, int D) { return (m + 1) * (1 + D) + m + m * m + 1; }
__host__ __device__ constexpr int kernel_theta_size(int nlf, int D) {
    return nlf ? graph_theta_size(nlf, D) : theta_size(D);
}
// fidelity flag -> source index (0..m-1 LF, m HF), -1 for anything else (graph.py:47-50 masks)
__device__ __forceinline__ int graph_source(double f, int m) {
    for (int i = 0; i <= m; ++i)
        if (f == (double)i) return i;
    return -1;
}
// one RBF term of source s between raw rows xa, xb
// graph_k with the source's inverse squared lengthscales il2[0..D) precomputed
__device__ __forceinline__ double graph_k_il2(const double* xa, const double* xb, int s, const GraphTheta& th,
                                              const double* il2) {
    double r2 = 0.0;
    for (int d = 0; d < th.D; ++d) {
        const double q = xa[d] - xb[d];
        r2 += q * q * il2[d];
    }
    return th.v(s) * exp(-0.5 * r2);
}
__device__ __forceinline__ double graph_k(const double* xa, const double* xb, int s, const GraphTheta& th) {
    double r2 = 0.0;
    for (int d = 0; d < th.D; ++d) {
        const double q = (xa[d] - xb[d]) / th.l(s, d);
        r2 += q * q;
    }
    return th.v(s) * exp(-0.5 * r2);
}
// K(a, b) of graph.py:55-97 (row a with source sa, column b with source sb).  The LF-LF
// block uses the ROW source's kernel (graph.py:61-63), so K is not symmetric for
// rhoLF[i][j] != rhoLF[j][i]; the Cholesky reads the lower triangle like TF's.
__device__ __forceinline__ double graph_entry(const double* xa, const double* xb, int sa, int sb,
                                              const GraphTheta& th) {
    if (sa < 0 || sb < 0) return 0.0;
    const int m = th.m;
    if (sa < m && sb < m) return (sa == sb ? 1.0 : th.rhoLF(sa, sb)) * graph_k(xa, xb, sa, th);
    if (sa < m) return graph_k(xa, xb, sa, th) * th.rho(sa);
    if (sb < m) return graph_k(xa, xb, sb, th) * th.rho(sb);
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += graph_k(xa, xb, i, th) * (th.rho(i) * th.rho(i));
    return s + graph_k(xa, xb, m, th);
}

// ---------------------------------------------------------------- cached schedule tables
// A schedule table (k_grad task order, k_chol_flow owner table) is a pure function of a few
// shape parameters, so the workgroup that builds it keeps it in the workspace with a key
// {magic, p0, p1, p2, hash of the contents} at tab[n .. n + 5) and skips the rebuild when a
// later call finds both the key and the hash intact.  The hash is what makes this safe: the
// workspace is shared with every other entry point, which may have overwritten any part of it.
constexpr int SCHED_KEY = 5;
__device__ inline unsigned sched_hash(const int* tab, int n, unsigned* sh) {
    if (threadIdx.x == 0) *sh = 0u;
    __syncthreads();
    auto mix = [](int v, int e) {
        unsigned t = (unsigned)v * 0x9E3779B1u + (unsigned)e * 0x85EBCA77u + 0x165667B1u;
        t ^= t >> 15;
        t *= 0x2C1B3C6Du;
        return t ^ (t >> 12);
    };
    // 16-B loads, 8 in flight per thread: one memory round trip per 8 K ints (tab is 256-B
    // aligned by the workspace carve)
    unsigned h = 0u;
    const int4* t4 = reinterpret_cast<const int4*>(tab);
    const int n4 = n / 4;
    for (int e0 = threadIdx.x; e0 < n4; e0 += 8 * blockDim.x) {
        int4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * blockDim.x;
            v[u] = e < n4 ? t4[e] : make_int4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * blockDim.x;
            if (e < n4) h += mix(v[u].x, 4 * e) + mix(v[u].y, 4 * e + 1) + mix(v[u].z, 4 * e + 2) + mix(v[u].w, 4 * e + 3);
        }
    }
    for (int e = 4 * n4 + threadIdx.x; e < n; e += blockDim.x) h += mix(tab[e], e);
    atomicAdd(sh, h);
    __syncthreads();
    const unsigned r = *sh;
    __syncthreads();
    return r;
}
__device__ inline bool sched_cached(const int* tab, int n, int magic, int p0, int p1, int p2, unsigned* sh) {
    const unsigned h = sched_hash(tab, n, sh);
    const int* k = tab + n;
    return k[0] == magic && k[1] == p0 && k[2] == p1 && k[3] == p2 && (unsigned)k[4] == h;
}
__device__ inline void sched_seal(int* tab, int n, int magic, int p0, int p1, int p2, unsigned* sh) {
    __syncthreads();   // the table's stores (same CU: workgroup scope suffices)
    const unsigned h = sched_hash(tab, n, sh);
    if (threadIdx.x == 0) {
        tab[n] = magic; tab[n + 1] = p0; tab[n + 2] = p1; tab[n + 3] = p2; tab[n + 4] = (int)h;
    }
}

// exp of four independent arguments, stage by stage across the four (the compiler lays out
// four exp() calls as four back-to-back dependent chains, which a wave issues in order).  The
// same operations and constants as the device library's exp (range reduction by ln 2, degree-11
// polynomial, ldexp, overflow / underflow selects), so each result is bitwise the library's.
__device__ __forceinline__ double dbits(unsigned long long u) { return __longlong_as_double((long long)u); }
#define MFGP_PIN4(v) asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]))
__device__ __forceinline__ void exp4(double (&x)[4]) {
    const double C[10] = {dbits(0x3e928af3fca7ab0cull), dbits(0x3ec71dee623fde64ull), dbits(0x3efa01997c89e6b0ull),
                          dbits(0x3f2a01a014761f6eull), dbits(0x3f56c16c1852b7b0ull), dbits(0x3f81111111122322ull),
                          dbits(0x3fa55555555502a1ull), dbits(0x3fc5555555555511ull), dbits(0x3fe000000000000bull), 1.0};
    double n[4], r[4], p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) n[u] = __builtin_rint(x[u] * dbits(0x3ff71547652b82feull));
    MFGP_PIN4(n);
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = fma(dbits(0xbfe62e42fefa39efull), n[u], x[u]);
    MFGP_PIN4(r);
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = fma(dbits(0xbc7abc9e3b39803full), n[u], r[u]);
    MFGP_PIN4(r);
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = fma(dbits(0x3e5ade156a5dcb37ull), r[u], C[0]);
    MFGP_PIN4(p);
#pragma unroll
    for (int k = 1; k < 10; ++k) {
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = fma(r[u], p[u], C[k]);
        MFGP_PIN4(p);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = fma(r[u], p[u], 1.0);
    MFGP_PIN4(p);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const double e = __builtin_ldexp(p[u], (int)n[u]);
        x[u] = x[u] > 1024.0 ? __builtin_inf() : (x[u] < -1075.0 ? 0.0 : e);
    }
}

// exp(x) for the kernels' exp(-r2/2) weights, bitwise the device library's exp (the same range
// reduction, degree-11 polynomial and ldexp; the overflow select is moot for x <= 1024 and the
// underflow one is what ldexp does below -1075).  Every polynomial step is ONE v_fma_f64 with its
// coefficient in an SGPR pair: the library form accumulates into a VGPR copy of each coefficient
// (a v_mov_b64 per step), and in a loop the compiler keeps all eleven copies live (~24 VGPRs,
// ~12 extra instructions an exp).
__device__ __forceinline__ double fma_s(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}
__device__ __forceinline__ double exp_lib(double x) {
    const double n = __builtin_rint(x * dbits(0x3ff71547652b82feull));
    double r = fma_s(n, dbits(0xbfe62e42fefa39efull), x);
    r = fma_s(n, dbits(0xbc7abc9e3b39803full), r);
    double p = fma_s(r, dbits(0x3e5ade156a5dcb37ull), dbits(0x3e928af3fca7ab0cull));
    p = fma_s(r, p, dbits(0x3ec71dee623fde64ull));
    p = fma_s(r, p, dbits(0x3efa01997c89e6b0ull));
    p = fma_s(r, p, dbits(0x3f2a01a014761f6eull));
    p = fma_s(r, p, dbits(0x3f56c16c1852b7b0ull));
    p = fma_s(r, p, dbits(0x3f81111111122322ull));
    p = fma_s(r, p, dbits(0x3fa55555555502a1ull));
    p = fma_s(r, p, dbits(0x3fc5555555555511ull));
    p = fma_s(r, p, dbits(0x3fe000000000000bull));
    p = fma_s(r, p, 1.0);
    p = fma_s(r, p, 1.0);
    return __builtin_ldexp(p, (int)n);
}

}  // namespace mfgp
