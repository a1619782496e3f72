// K2f k_chol_flow: the LML-path tile Cholesky, its inverse factor L^{-1}, the forward solve
// Z = L^{-1} Y and alpha = L^{-T} Z as ONE persistent dataflow launch (gfx950, NB = 32).
//
// Same arithmetic as the launch-per-step k_chol_step sequence (mfgpflow/linear.py:138-153 ->
// GPflow GPR.log_marginal_likelihood: L = chol(K + s2 I), then the triangular solves), without
// the T step boundaries: at Goku (T = 37) each step launch costs ~9.4 us although the dependent
// chain inside it (the next diagonal tile's update and its factor) is ~4 us.
//
// Roles.  One workgroup per CU (the dynamic LDS is sized so that two never share one), so every
// workgroup of the grid is resident and a wait never depends on an unscheduled workgroup.
//   * workgroup 0 ("diag", 8 waves) runs the chain, see diag_chain below;
//   * every wave of workgroups 1.. ("workers") owns up to FLOW_MAXOWN output tiles (table built
//     by k_gram's extra workgroup: tiles sorted by item count, snake-dealt over the waves) and
//     runs their items level by level -- at level l first the finalize items (need D_l), then
//     the update items (need panel l):
//       A(i,j)  : A -= L(i,l) L(j,l)^T for l < j, then L(i,j) = A D_j^T at level j; the tiles
//                 (k,k), (k,k-1), (k,k-2) stop after level k-3 and hand A' to diag;
//       R(i,c)  : R -= L(i,l) X(l,c) for c <= l < i, then X(i,c) = D_i R at level i
//                 (c < T: rows of L^{-1};  c >= T: Y column tiles, X = Z);
//       al(c,y) : alpha(c,y) += X(l,c)^T Z(l,y) for l >= c.
//   A wave keeps its running tile in the global array it lives in (only it touches it).
//
// Hand-offs: the data is the flag.  Every tile another wave reads is published ONCE per launch
// into its own slot of the publication area (FlowPub), which k_gram fills with a signalling-NaN
// sentinel before this launch.  A producer stores the tile with agent-scope relaxed atomics
// (8-B global_store ... sc1: untorn, write-through) and moves on -- no drain, no flag; a
// consumer loads it with sc1 loads until no element is the sentinel (wave ballot).  Computed
// NaNs are quiet, so the signalling pattern never occurs as data.  One memory round trip per
// hop instead of three (flag poll, payload, producer drain); cdna_hip_programming.md
// Guideline 16, R2 (data-tagged granules).
// Published X tiles are stored transposed (X^T) so that every MFMA operand is a row-major read
// along the contraction index: lane (li, lq) loads 8 consecutive doubles of row 16b + li,
// contraction indices 8 lq .. 8 lq + 7 (the k order inside an MFMA sum is free).
// Every wait is bounded (FlowArgs::timeout ticks of the 100 MHz realtime clock, counted from the start
// of that wait; default FLOW_TIMEOUT_TICKS, mfgp_set_flow_timeout_us): on expiry the wave
// raises the abort word, writes info = MFGP_FLOW_TIMEOUT and runs on, so the grid drains.
#include "../../include/mfgp.h"
#include "mfgp_device.h"
#include "mfgp_internal.h"
#include "mfgp_flow.h"

namespace mfgp {

#ifndef FLOW_SLEEP
#define FLOW_SLEEP 1
#endif
constexpr int WLD = 33;                              // per-wave LDS tile stride (doubles)

__device__ __forceinline__ long long flow_clock() { return __builtin_amdgcn_s_memrealtime(); }

// ---------------------------------------------------------------- single-wave 32x32 tiles
// Accumulator: c[bi][bj][r] = C[16 bi + lq + 4 r][16 bj + li]   (li = lane & 15, lq = lane >> 4)
struct WTile {
    f64x4 v[2][2];
};
// MFMA operand: o[b][s] = M[16 b + li][8 lq + s]  (row-major M read along the contraction index)
struct WOp {
    double v[2][8];
};

__device__ __forceinline__ void wt_zero(WTile& t) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) t.v[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
}
// Plain tile traffic of the worker items (A / R / alpha tiles, runtime leading dimension): the
// row group's base (16a + 4r) * ld is wave-uniform (SGPR pair, global_load's saddr form) and the
// lane's row / column is ONE 32-bit VGPR.  With per-lane 64-bit addresses the compiler hoists
// the eight row addresses of every tile shape out of the item loop and spills them; their
// reloads carry s_waitcnt vmcnt(0), which also waits for every older store of the wave.  The
// empty asm keeps the lane offset opaque, so nothing derived from it is hoisted.
__device__ __forceinline__ unsigned wt_lane_off(long ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
    unsigned v = (unsigned)((lq * (int)ld + li) * 8);
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ void wt_load_u(WTile& t, const double* P, long ld) {
    const unsigned lo = wt_lane_off(ld);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const char* row = reinterpret_cast<const char*>(P + (long)(16 * a + 4 * r) * ld);
#pragma unroll
            for (int b = 0; b < 2; ++b) t.v[a][b][r] = *reinterpret_cast<const double*>(row + lo + 128 * b);
        }
}
__device__ __forceinline__ void wt_store_u(const WTile& t, double* P, long ld) {
    const unsigned lo = wt_lane_off(ld);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            char* row = reinterpret_cast<char*>(P + (long)(16 * a + 4 * r) * ld);
#pragma unroll
            for (int b = 0; b < 2; ++b) *reinterpret_cast<double*>(row + lo + 128 * b) = t.v[a][b][r];
        }
}

template <bool SC1>
__device__ __forceinline__ void wt_load(WTile& t, const double* P, long ld) {
    if constexpr (!SC1) {
        wt_load_u(t, P, ld);
        return;
    }
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double* q = P + (long)(16 * a + lq + 4 * r) * ld + 16 * b + li;
                t.v[a][b][r] = SC1 ? ld_coherent(q) : *q;
            }
}
template <bool SC1>
__device__ __forceinline__ void wt_store(const WTile& t, double* P, long ld) {
    if constexpr (!SC1) {
        wt_store_u(t, P, ld);
        return;
    }
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double* q = P + (long)(16 * a + lq + 4 * r) * ld + 16 * b + li;
                if (SC1) st_coherent(q, t.v[a][b][r]);
                else *q = t.v[a][b][r];
            }
}
// P[col][row] = C[row][col], sc1
__device__ __forceinline__ void wt_store_t_sc1(const WTile& t, double* P, long ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) st_coherent(P + (long)(16 * b + li) * ld + 16 * a + lq + 4 * r, t.v[a][b][r]);
}
template <bool SC1>
__device__ __forceinline__ void op_load(WOp& o, const double* P, long ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const double* q = P + (long)(16 * b + li) * ld + 8 * lq;
        if (SC1) {
#pragma unroll
            for (int s = 0; s < 8; ++s) o.v[b][s] = ld_coherent(q + s);
        } else {
#pragma unroll
            for (int s = 0; s < 8; s += 2) {
                const f64x2 x = *reinterpret_cast<const f64x2*>(q + s);
                o.v[b][s] = x.x;
                o.v[b][s + 1] = x.y;
            }
        }
    }
}
// C (+)= sgn * A B with A[i][k] = a(i,k), B[k][j] = b(j,k) in operand form
template <bool NEG>
__device__ __forceinline__ void wt_mma(WTile& c, const WOp& a, const WOp& b) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
                c.v[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(NEG ? -a.v[bi][s] : a.v[bi][s], b.v[bj][s],
                                                                   c.v[bi][bj], 0, 0, 0);
}
// accumulator -> per-wave LDS tile (row-major, stride WLD)
__device__ __forceinline__ void wt_to_lds(const WTile& t, double* S) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) S[(16 * a + lq + 4 * r) * WLD + 16 * b + li] = t.v[a][b][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
}
// operand o[b][s] = M[16 b + li][8 lq + s] from the LDS tile M  (M as the A side)
__device__ __forceinline__ void op_rows_lds(WOp& o, const double* S) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s) o.v[b][s] = S[(16 * b + li) * WLD + 8 * lq + s];
}
// operand o[b][s] = M[8 lq + s][16 b + li] from the LDS tile M  (M as the B side, untransposed)
__device__ __forceinline__ void op_cols_lds(WOp& o, const double* S) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s) o.v[b][s] = S[(8 * lq + s) * WLD + 16 * b + li];
}
// C += A B with the B side read from the per-wave LDS tile M untransposed (B[k][j] = M[k][j])
__device__ __forceinline__ void wt_mma_lds_b(WTile& c, const WOp& a, const double* S) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const double b0 = S[(8 * lq + s) * WLD + li], b1 = S[(8 * lq + s) * WLD + 16 + li];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
            c.v[bi][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.v[bi][s], b0, c.v[bi][0], 0, 0, 0);
            c.v[bi][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.v[bi][s], b1, c.v[bi][1], 0, 0, 0);
        }
    }
}
__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------- the Gram inside the launch
// Tile (ti, tj) of the padded K + s2 I of the LML (mfgpflow/linear.py:55-104 via GPflow's
// SquaredExponential.K: k = v exp(-r^2 / 2), expanded r^2 = -2 a.b + |a|^2 + |b|^2 on a = x / l,
// no clamp; K = (s s^T) o K_L + (h h^T) o K_delta with rho[0]; exact fidelity masks; the noise on
// the diagonal; identity on the padded diagonal, zero elsewhere in the padding), formed by ONE wave
// and stored to dst (row stride ld; global or LDS) in the accumulator layout (lane (li, lq): rows
// 16 bi + lq + 4 r, columns 16 bj + li), so the same wave reads its own entries back.
// The dot products a_i . a_j run on the matrix core (the v_mfma_f64_16x16x4 operand layout IS
// (row 16 b + li, dimension 4 s + lq)), the norms as partial sums over the lane's dimensions
// reduced across the four lq lanes; the HF x HF part (K_delta) only when the tile holds such a pair.
// Replaces the Gram launch in front of the flow (k_gram_flow, ~14 us at Goku): an owner forms its
// tile before its first item, while the chain factors D_0.
// One 16-row half of the tile at a time, dimensions in chunks of 16 (four MFMA k-steps of 4):
// every global load of a chunk (with the fidelity flags and theta) is issued before the first is
// used -- one memory round trip per half and chunk (a dependent load per k-step cost ~5 us a
// tile), in ~120 VGPRs (the kernel's allocation stays at its roles' 183, so small kernels of
// other streams still fit beside the flow's waves on a CU).
// SC1: publish (sc1 stores, for another wave); row halves [b0, b1) and the column halves in
// cmask (bit b: columns 16 b ..) of the tile only.
template <bool SC1>
__device__ __forceinline__ void flow_gram_tile(const double* __restrict__ X, long ldx, const double* __restrict__ th,
                                               int n, int D, int ti, int tj, double* dst, long ld, int b0 = 0,
                                               int b1 = 2, int cmask = 3) {
    constexpr int FS = 4;
    const int l = threadIdx.x & 63, li = l & 15, lq = l >> 4;
    int rj[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) rj[b] = 32 * tj + 16 * b + li;
#pragma unroll 1
    for (int bi = b0; bi < b1; ++bi) {
        const int ri = 32 * ti + 16 * bi + li;
        double fi = X[(long)min(ri, n - 1) * ldx + D];
        double fj[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) fj[b] = X[(long)min(rj[b], n - 1) * ldx + D];
        const double vL = th[0], vD = th[1 + D], rho = th[2 + 2 * D], noise = th[3 + 2 * D];
        f64x4 dl[2], dd[2];
        double ni = 0.0, nid = 0.0, nj[2] = {0.0, 0.0}, njd[2] = {0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            dl[q] = f64x4{0.0, 0.0, 0.0, 0.0};
            dd[q] = f64x4{0.0, 0.0, 0.0, 0.0};
        }
        bool hh = false;
        for (int c0 = 0; c0 < D; c0 += 4 * FS) {
            double xi[FS], xj[2][FS], lL[FS], lD[FS];
#pragma unroll
            for (int k = 0; k < FS; ++k) {   // loads only (clamped in-range addresses)
                const int d = min(c0 + 4 * k + lq, D - 1);
                lL[k] = th[1 + d];
                lD[k] = th[2 + D + d];
                xi[k] = X[(long)min(ri, n - 1) * ldx + d];
#pragma unroll
                for (int b = 0; b < 2; ++b) xj[b][k] = X[(long)min(rj[b], n - 1) * ldx + d];
            }
            if (c0 == 0) {   // the flags arrived with the first chunk
                if (ri >= n) fi = -1.0;
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    if (rj[b] >= n) fj[b] = -1.0;
                hh = __ballot(fj[0] == 1.0 || fj[1] == 1.0) != 0 && __ballot(fi == 1.0) != 0;   // HF x HF pairs
            }
#pragma unroll
            for (int k = 0; k < FS; ++k) {
                const int d = c0 + 4 * k;
                if (d >= D) break;
                const bool dv = d + lq < D;
                const double il = dv ? rcp_nr(lL[k]) : 0.0, ild = dv ? rcp_nr(lD[k]) : 0.0;   // a = x rcp_nr(l)
                const double x1 = (dv && ri < n) ? xi[k] : 0.0;
                const double ai = x1 * il, aid = x1 * ild;
                ni = fma(ai, ai, ni);
                nid = fma(aid, aid, nid);
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (!((cmask >> q) & 1)) continue;
                    const double x2 = (dv && rj[q] < n) ? xj[q][k] : 0.0;
                    const double aj = x2 * il, ajd = x2 * ild;
                    nj[q] = fma(aj, aj, nj[q]);
                    njd[q] = fma(ajd, ajd, njd[q]);
                    dl[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, aj, dl[q], 0, 0, 0);
                    if (hh) dd[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(aid, ajd, dd[q], 0, 0, 0);
                }
            }
        }
        // full norms of rows 16 b + li (the four lq lanes' partial sums)
        ni += __shfl_xor(ni, 16, 64); ni += __shfl_xor(ni, 32, 64);
        nid += __shfl_xor(nid, 16, 64); nid += __shfl_xor(nid, 32, 64);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            nj[q] += __shfl_xor(nj[q], 16, 64); nj[q] += __shfl_xor(nj[q], 32, 64);
            njd[q] += __shfl_xor(njd[q], 16, 64); njd[q] += __shfl_xor(njd[q], 32, 64);
        }
        double nr[4], nrd[4], fr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // row 16 bi + lq + 4 r: held by lane lq + 4 r
            nr[r] = __shfl(ni, lq + 4 * r, 64);
            nrd[r] = __shfl(nid, lq + 4 * r, 64);
            fr[r] = __shfl(fi, lq + 4 * r, 64);
        }
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
            if (!((cmask >> bj) & 1)) continue;
            const bool L2 = fj[bj] == 0.0, H2 = fj[bj] == 1.0;
            double kl[4], kd[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                kl[r] = -0.5 * (-2.0 * dl[bj][r] + (nr[r] + nj[bj]));
                kd[r] = -0.5 * (-2.0 * dd[bj][r] + (nrd[r] + njd[bj]));
            }
            exp4(kl);
            if (hh) exp4(kd);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * bi + lq + 4 * r;
                const int gi = 32 * ti + row, gj = rj[bj];
                double v;
                if (gi < n && gj < n) {
                    const double k1 = vL * kl[r];
                    const bool L1 = fr[r] == 0.0, H1 = fr[r] == 1.0;
                    const double kD = (H1 && H2) ? vD * kd[r] : 0.0;
                    v = (L1 && L2) ? k1 : (!(H1 && H2) ? k1 * rho : k1 * (rho * rho) + kD);
                    if (!(L1 || H1) || !(L2 || H2)) v = 0.0;   // linear.py:67-70 exact masks
                    if (gi == gj) v = v + noise;
                } else {
                    v = (gi == gj) ? 1.0 : 0.0;                // identity padding
                }
                if constexpr (SC1) st_coherent(dst + (long)row * ld + 16 * bj + li, v);
                else dst[(long)row * ld + 16 * bj + li] = v;   // the accumulator layout of wt_store_u
            }
        }
    }
}

// Y column tile cy of R's row block i (rows >= n, columns >= p zero), accumulator layout: the
// initial value of an R tile of the Z columns (the flow reads Y itself; no copy into R)
__device__ __forceinline__ void flow_y_tile(const FlowArgs& a, int i, int cy, WTile& t) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 32 * i + 16 * bi + lq + 4 * r, col = 32 * cy + 16 * bj + li;
                t.v[bi][bj][r] = (row < a.n && col < a.p) ? a.Y[(long)row * a.ldy + col] : 0.0;
            }
}


// ---------------------------------------------------------------- publication area
// Tiles (32 x 32 row-major) in one sentinel-filled region: L(i,j) i > j | D_k | X^T(i,c)
// (c <= i < T, then the T x Tp Y column tiles) | hand-offs A'(k,k-1), A'(k,k), A'(k,k-2).
struct FlowPub {
    double* base;
    int T, Tp;
    __device__ double* tile(long idx) const { return base + idx * 1024; }
    __device__ int nL() const { return T * (T - 1) / 2; }
    __device__ int nX() const { return T * (T + 1) / 2 + T * Tp; }
    __device__ double* L(int i, int j) const { return tile(i * (i - 1) / 2 + j); }
    __device__ double* D(int k) const { return tile(nL() + k); }
    __device__ double* X(int i, int c) const {
        return tile(nL() + T + (c < T ? i * (i + 1) / 2 + c : T * (T + 1) / 2 + i * Tp + (c - T)));
    }
    __device__ double* H(int kind, int k) const { return tile(nL() + T + nX() + 3 * k + kind); }   // 0: (k,k-1) 1: (k,k) 2: (k,k-2)
};

struct FlowCtx {
    FlowArgs a;
    FlowPub P;
    long long t0;
    long long waited;   // worker: ticks spent re-polling (trace only)
    __device__ double* At(int i, int j) const { return a.A + (long)i * 32 * a.lda + (long)j * 32; }
    __device__ double* Rt(int i, int c) const { return a.R + (long)i * 32 * a.ldr + (long)c * 32; }
    __device__ double* Xt(int i, int c) const { return a.Xo + (long)i * 32 * a.ldx + (long)c * 32; }
};

__device__ __forceinline__ bool is_sent(double v) {
    return (unsigned long long)__double_as_longlong(v) == FLOW_SENTINEL;
}
// Give-up path of every poll: abort word + info after `lim` ticks of this wait (or someone else's abort).
__device__ __noinline__ bool flow_give_up(int* abortw, int* info, long long t0, long long lim) {
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
        return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > lim) {
        if ((threadIdx.x & 63) == 0) {
            __hip_atomic_store(abortw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(info, MFGP_FLOW_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return true;
    }
    return false;
}
// Wait for a published tile (row-major, ld 32): probe its first line until no element is the
// sentinel, then the caller's full load re-checks every element.
__device__ __forceinline__ bool pub_probe_ok(const double* P) {
    // one 128-B line (16 doubles) per probe: a poll costs one line of traffic, not 64
    const int l = threadIdx.x & 63;
    return __ballot(is_sent(ld_coherent(P + (l & 15)))) == 0;
}
// Every wait's bound counts from the start of THAT wait (a long but progressing factorization
// never trips it; only a hand-off that stalls for FlowArgs::timeout ticks does).
__device__ __noinline__ void pub_wait(const double* P, int* abortw, int* info, long long lim) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int spin = 0;; ++spin) {
        if (pub_probe_ok(P)) return;
        if ((spin & 7) == 7 && flow_give_up(abortw, info, t0, lim)) return;
        __builtin_amdgcn_s_sleep(FLOW_SLEEP);
    }
}
// Probe first: one 128-B line of each operand before the 16-KB loads.  Most items start before
// their operands are out; fetching the whole operands just to find the sentinel was most of the
// launch's traffic (and the fabric's load is what every hand-off waits on): 3316 -> 3717 evals/s.
__device__ __forceinline__ void pub_probe2(const double* Px, const double* Py, FlowCtx& C) {
    const int l = threadIdx.x & 63;
    const double px = ld_coherent(Px + (l & 15));
    const double py = Py ? ld_coherent(Py + (l & 15)) : 0.0;
    const bool okx = __ballot(is_sent(px)) == 0, oky = __ballot(is_sent(py)) == 0;
    if (!okx || !oky) {
        const long long tw = flow_clock();
        if (!okx) pub_wait(Px, C.a.flags, C.a.info, C.a.timeout);
        if (!oky) pub_wait(Py, C.a.flags, C.a.info, C.a.timeout);
        C.waited += flow_clock() - tw;
    }
}
// 16-B sc1 loads of an operand from a published tile (buffer_load_dwordx4 ... sc1)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double bits_d(unsigned lo, unsigned hi) {
    return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}
__device__ __forceinline__ void op_load_pub(WOp& o, const double* P) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(P), (short)0, 8192, 0x00020000);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((16 * b + li) * 32 + 8 * lq + 2 * q) * 8, 0, 16);
            o.v[b][2 * q] = bits_d(v.x, v.y);
            o.v[b][2 * q + 1] = bits_d(v.z, v.w);
        }
}
__device__ __forceinline__ bool op_missing(const WOp& o) {
    bool miss = false;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s) miss |= is_sent(o.v[b][s]);
    return __ballot(miss) != 0;
}
// operand of a published tile, re-read until complete
__device__ __forceinline__ void pub_retry(WOp& o, const double* P, FlowCtx& C) {
    const long long tw = flow_clock();
    for (;;) {
        if (flow_give_up(C.a.flags, C.a.info, tw, C.a.timeout)) break;
        pub_wait(P, C.a.flags, C.a.info, C.a.timeout);
        op_load_pub(o, P);
        if (!op_missing(o)) break;
    }
    C.waited += flow_clock() - tw;
}
__device__ __forceinline__ void pub_op(WOp& o, const double* P, FlowCtx& C) {
    op_load_pub(o, P);
    if (op_missing(o)) pub_retry(o, P, C);
}
// the same re-read in full per poll (no probe round trip once the tile lands)
__device__ __forceinline__ void pub_op_direct(WOp& o, const double* P, FlowCtx& C) {
    op_load_pub(o, P);
    if (!op_missing(o)) return;
    const long long tw = flow_clock();
    for (int spin = 0;; ++spin) {
        __builtin_amdgcn_s_sleep(FLOW_SLEEP);
        op_load_pub(o, P);
        if (!op_missing(o)) break;
        if ((spin & 7) == 7 && flow_give_up(C.a.flags, C.a.info, tw, C.a.timeout)) break;
    }
    C.waited += flow_clock() - tw;
}
// two operands in one round trip
__device__ __forceinline__ void pub_op2(WOp& x, const double* Px, WOp& y, const double* Py, FlowCtx& C) {
    pub_probe2(Px, Py, C);
    op_load_pub(x, Px);
    op_load_pub(y, Py);
    if (op_missing(x)) pub_retry(x, Px, C);
    if (op_missing(y)) pub_retry(y, Py, C);
}
// the same in accumulator layout
__device__ __forceinline__ void pub_wt(WTile& t, const double* P, FlowCtx& C) {
    long long tw = 0;
    for (int spin = 0;; ++spin) {
        wt_load<true>(t, P, 32);
        bool miss = false;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) miss |= is_sent(t.v[a][b][r]);
        if (__ballot(miss) == 0) break;
        if (spin == 0) tw = flow_clock();
        if (flow_give_up(C.a.flags, C.a.info, tw, C.a.timeout)) break;
        pub_wait(P, C.a.flags, C.a.info, C.a.timeout);
    }
    if (tw) C.waited += flow_clock() - tw;
}

// The diag helpers' inputs (waves 5-7): both re-read in full until complete, one round trip
// per poll instead of probe + reload (only three waves of the launch poll this way)
__device__ __forceinline__ void pub_wt_op_direct(WTile& t, const double* Pt, WOp& o, const double* Po,
                                                 FlowCtx& C) {
    const long long tw = flow_clock();
    for (int spin = 0;; ++spin) {
        wt_load<true>(t, Pt, 32);
        op_load_pub(o, Po);
        bool miss = false;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) miss |= is_sent(t.v[a][b][r]);
        if (__ballot(miss) == 0 && !op_missing(o)) break;
        if ((spin & 7) == 7 && flow_give_up(C.a.flags, C.a.info, tw, C.a.timeout)) break;
        __builtin_amdgcn_s_sleep(FLOW_SLEEP);
    }
}

// a published accumulator tile and a published operand in ONE round trip (the diag helpers'
// inputs of a step: the band tile from its owner and the owner's L(j,j-3))
__device__ __forceinline__ void pub_wt_op(WTile& t, const double* Pt, WOp& o, const double* Po, FlowCtx& C) {
    wt_load<true>(t, Pt, 32);
    op_load_pub(o, Po);
    bool miss = false;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) miss |= is_sent(t.v[a][b][r]);
    if (__ballot(miss) != 0) pub_wt(t, Pt, C);
    if (op_missing(o)) pub_retry(o, Po, C);
}

// ---- worker items (one wave)
// Finalize from the accumulator in registers; dop: D_j (A tiles) / D_i (R tiles) in operand form.
//   A(i,j): L(i,j) = A'(i,j) D_j^T;   R(i,c): X(i,c) = D_i R(i,c) (row block i of [L^{-1} | Z])
__device__ __forceinline__ void flow_finalize_acc(FlowCtx& C, const FlowTile& t, const WTile& acc, const WOp& dop,
                                                  double* S) {
    // L(i,j) = A'(i,j) D_j^T
    WTile out;
    WOp x;
    wt_to_lds(acc, S);
    op_rows_lds(x, S);
    wt_zero(out);
    wt_mma<false>(out, x, dop);                          // B[k][j'] = D_j[j'][k]
    wt_store<true>(out, C.P.L(t.i, t.j), 32);
}

// A finalize with no update before it (tiles (i,0))
__device__ __forceinline__ void flow_finalize(FlowCtx& C, const FlowTile& t, double* S) {
    WTile acc;
    WOp d;
    wt_load<false>(acc, C.At(t.i, t.j), C.a.lda);
    pub_op(d, C.P.D(t.fin), C);
    flow_finalize_acc(C, t, acc, d, S);
}

// X(i,c) = D_i R'''(i,c): row block i of [L^{-1} | Z] from R''' (every panel < i applied) in
// registers; published transposed first (it feeds the next row's last update and alpha), then
// stored to Xo; a Z tile also leaves its sum of squares.
__device__ __forceinline__ void flow_finish_r(FlowCtx& C, const FlowTile& t, const WTile& acc, const WOp& d,
                                              double* S) {
    const FlowArgs& a = C.a;
    const int T = a.T;
    const int i = t.i;
    wt_to_lds(acc, S);
    WTile out;
    wt_zero(out);
    wt_mma_lds_b(out, d, S);                             // D_i R'''   (B[k][j] = R'''[k][j])
    wt_store_t_sc1(out, C.P.X(i, t.j), 32);              // X^T (published first: it feeds others)
    wt_store<false>(out, C.Xt(i, t.j), a.ldx);
    if (t.j >= T) {
        // sum of Z^2 over the valid (n x p) part of this tile
        const int cy = t.j - T;
        const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
        double z2 = 0.0;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = i * 32 + 16 * bi + lq + 4 * r, col = cy * 32 + 16 * bj + li;
                    const double z = out.v[bi][bj][r];
                    if (row < a.n && col < a.p) z2 += z * z;
                }
        z2 = wave_sum64(z2);
        if ((threadIdx.x & 63) == 0) a.zpart[i * a.Tp + cy] = z2;
    }
}

// The R tiles without an update: Z's row block 0, X(0,c) = D_0 Y(0,c)
__device__ __forceinline__ void flow_finalize_r(FlowCtx& C, const FlowTile& t, double* S) {
    WTile acc;
    WOp d;
    flow_y_tile(C.a, t.i, t.j - C.a.T, acc);
    pub_op(d, C.P.D(t.i), C);
    flow_finish_r(C, t, acc, d, S);
}

// Update at level l; a tile's last update runs straight into its finalize (same registers,
// D prefetched with the panel operands), so a row of L advances one hop per level.
__device__ __forceinline__ void flow_update(FlowCtx& C, const FlowTile& t, int l, double* S) {
    const FlowArgs& a = C.a;
    const int T = a.T;
    WTile acc;
    WOp x, y, d;
    const bool fin = (t.type == FT_A) && (l == t.hi) && (t.fin == l + 1);
    if (t.type == FT_A) {
        double* dst = C.At(t.i, t.j);
        wt_load<false>(acc, dst, a.lda);
        if (t.j != t.i) {
            pub_op2(x, C.P.L(t.i, l), y, C.P.L(t.j, l), C);
        } else {
            pub_op(x, C.P.L(t.i, l), C);
            y = x;
        }
        wt_mma<true>(acc, x, y);                         // A(i,j) -= L(i,l) L(j,l)^T
        if (fin) {
            // D_{l+1} is loaded only now: it is published ~one factor after L(j,l) (so an early
            // load would nearly always miss), and holding it across the update spills registers
            pub_op_direct(d, C.P.D(t.fin), C);   // ~one wave per tile of the column polls it
            flow_finalize_acc(C, t, acc, d, S);
        } else if (t.pub && l == t.hi) {
            wt_store<true>(acc, C.P.H(t.i == t.j ? 1 : t.i == t.j + 1 ? 0 : 2, t.i), 32);
        } else {
            wt_store<false>(acc, dst, a.lda);
        }
    } else if (t.type == FT_R) {
        double* dst = C.Rt(t.i, t.j);
        // first update: from the initial value -- zero (identity block, i > j + 1) or Y (Z columns)
        if (t.j < T && l == t.j) wt_zero(acc);
        else if (t.j >= T && l == t.lo) flow_y_tile(a, t.i, t.j - T, acc);
        else wt_load<false>(acc, dst, a.ldr);
        pub_op2(x, C.P.L(t.i, l), y, C.P.X(l, t.j), C);  // L(i,l), X(l,c)^T (B[k][j] = X(l,c)[k][j])
        wt_mma<true>(acc, x, y);                         // R(i,c) -= L(i,l) X(l,c)
        if (l == t.hi) {                                 // panel i-1: the finalize follows (D_i is
            pub_op_direct(d, C.P.D(t.fin), C);           // published about when L(i,i-1) X(i-1,c) is)
            flow_finish_r(C, t, acc, d, S);
        } else {
            wt_store<false>(acc, dst, a.ldr);
        }
    } else {
        const int c = t.i, cy = t.j;
        double* al = a.alpha + (long)c * 32 * a.ldal + (long)cy * 32;
        if (l == c) wt_zero(acc);
        else wt_load<false>(acc, al, a.ldal);
        pub_op2(x, C.P.X(l, c), y, C.P.X(l, T + cy), C); // A[i][k] = X(l,c)[k][i], B[k][j] = Z(l,cy)[k][j]
        wt_mma<false>(acc, x, y);                        // alpha(c) += X(l,c)^T Z(l)
        wt_store<false>(acc, al, a.ldal);
        if (l == T - 1) {
            // alpha^T rows under [L^{-1} | Z] for k_grad: -alpha^T / P (A side), alpha^T (B side)
            const double sA = -1.0 / (double)a.p;
            double* xa = a.Xo + (long)(T + cy) * 32 * a.ldx + (long)c * 32;
            double* xb = a.Xo + (long)(T + a.Tp + cy) * 32 * a.ldx + (long)c * 32;
            const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int bj = 0; bj < 2; ++bj)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const long o = (long)(16 * bj + li) * a.ldx + 16 * bi + lq + 4 * r;
                        xa[o] = sA * acc.v[bi][bj][r];
                        xb[o] = acc.v[bi][bj][r];
                    }
        }
    }
}

// item log (diagnostic): per worker wave FLOW_LOG items x {code << 8 | level, begin, ready, end}
constexpr int FLOW_LOG = 40;
__device__ __forceinline__ void flow_item_log(const FlowCtx& C, int wid, int n, int code, int l, long long i0,
                                              long long w0) {
    if (!C.a.trace || n >= FLOW_LOG || (threadIdx.x & 63) != 0) return;
    long long* e = C.a.trace + 8 * C.a.T + 3 * C.a.nwaves + ((long)wid * FLOW_LOG + n) * 4;
    const long long t1 = flow_clock();
    e[0] = ((long long)code << 8) | l;
    e[1] = i0 - C.t0;
    e[2] = i0 + (C.waited - w0) - C.t0;
    e[3] = t1 - C.t0;
}

// Slot order of a worker wave: A tiles (they feed the chain), nearest the diagonal first; then
// the R / Y tiles, then alpha.  Items run level by level in this order (a merged finalize at level
// l waits for D_{l+1}: everything of level l that the chain needs must come before it).
__device__ __forceinline__ int flow_prio(int code) {
    if (code < 0) return 1 << 30;
    const FlowTile t = flow_tile(code, 1024);
    return (t.type << 16) | (t.i << 8) | t.j;
}

__device__ __forceinline__ void flow_worker(FlowCtx& C, int wid, double* S) {
    const int T = C.a.T;
    const int* own = C.a.own + wid * FLOW_MAXOWN;
    int code[FLOW_MAXOWN];
#pragma unroll
    for (int s = 0; s < FLOW_MAXOWN; ++s) code[s] = __builtin_amdgcn_readfirstlane(own[s]);
#pragma unroll
    for (int a = 0; a < FLOW_MAXOWN; ++a)       // tiny sorting network on the priority key
#pragma unroll
        for (int b = 0; b + 1 < FLOW_MAXOWN - a; ++b)
            if (flow_prio(code[b]) > flow_prio(code[b + 1])) { const int x = code[b]; code[b] = code[b + 1]; code[b + 1] = x; }
    int last = -1;
#pragma unroll
    for (int s = 0; s < FLOW_MAXOWN; ++s) {
        if (code[s] < 0) continue;
        const FlowTile t = flow_tile(code[s], T);
        last = max(last, max(t.hi, t.fin));
    }
    const long long tb = flow_clock();
    C.waited = 0;
    int nitem = 0;
    static_assert(FLOW_MAXOWN == 4, "slot select below");
    auto pick = [&](int s) { return s == 0 ? code[0] : s == 1 ? code[1] : s == 2 ? code[2] : code[3]; };
    for (int l = 0; l <= last; ++l) {
#pragma unroll 1
        for (int s = 0; s < FLOW_MAXOWN; ++s) {
            const int cs = pick(s);
            if (cs < 0) continue;
            const FlowTile t = flow_tile(cs, T);
            if (t.fin == l && t.hi < t.lo) {
                const long long i0 = flow_clock(), w0 = C.waited;
                if (t.type == FT_R) flow_finalize_r(C, t, S);
                else flow_finalize(C, t, S);
                flow_item_log(C, wid, nitem++, cs, l, i0, w0);
            }
        }
#pragma unroll 1
        for (int s = 0; s < FLOW_MAXOWN; ++s) {
            const int cs = pick(s);
            if (cs < 0) continue;
            const FlowTile t = flow_tile(cs, T);
            if (t.lo <= l && l <= t.hi) {
                const long long i0 = flow_clock(), w0 = C.waited;
                flow_update(C, t, l, S);
                flow_item_log(C, wid, nitem++, cs, l, i0, w0);
            }
        }
    }
    if (C.a.trace && (threadIdx.x & 63) == 0) {
        long long* tr = C.a.trace + 8 * T + 3 * wid;
        tr[0] = tb - C.t0;
        tr[1] = flow_clock() - C.t0;
        tr[2] = C.waited;
    }
}

// ---- the chain (workgroup 0, 8 waves)
// Waves 0-3 ("chain") run step k: L(k,k-1) = A''(k,k-1) D_{k-1}^T, A''(k,k) -= L L^T, then
// wave 0 factors D_k.  Everything around the chain is taken off it by the other waves, which
// talk to the chain through LDS progress words (a wave's DS operations complete in issue
// order, so data written before a word's store is visible to whoever reads the word):
//   wave 4: publishes L(k,k-1), then D_k, X^T(k,k) = D_k^T, Xo(k,k), diag(L), info;
//   wave 5: L(j,j-2) = A'(j,j-2) D_{j-2}^T as soon as D_{j-2} is in LDS (the owner applied
//     every panel < j-2), into LDS for waves 6 / 7, then published;
//   waves 6, 7: prefetch step j while the chain factors step j-1: the owners' A'(j,j-1),
//     A'(j,j) (panels < j-2 applied) minus panel j-2:
//     A''(j,j-1) = A'(j,j-1) - L(j,j-2) L(j-1,j-2)^T,  A''(j,j) = A'(j,j) - L(j,j-2) L(j,j-2)^T.
// Buffers are double-buffered by step parity.
struct DiagLds {
    // LDS carve (doubles): Db[2] | Ls[2] | Ap[2] | Cp[2] | L2[2] (NB x S each) | fsc (32 x 33) | dg[2][32]
    // | bad[2] | words.  Parity-indexed buffers are computed, not held in pointer arrays (a
    // dynamically indexed pointer array lands in scratch).
    double* base;
    static constexpr int E = TileCfg<32>::ELEMS;
    __device__ double* Db(int q) const { return base + q * E; }        // D_k (stride S)
    __device__ double* Ls(int q) const { return base + (2 + q) * E; }  // L(k,k-1)
    __device__ double* Ap(int q) const { return base + (4 + q) * E; }  // A''(k,k-1)
    __device__ double* Cp(int q) const { return base + (6 + q) * E; }  // A''(k,k)
    __device__ double* L2(int q) const { return base + (8 + q) * E; }  // L(k,k-2)
    __device__ double* fsc() const { return base + 10 * E; }           // factor input (32 x 33)
    __device__ double* dg(int q) const { return base + 10 * E + 32 * 33 + 32 * q; }
    __device__ int* bad() const { return reinterpret_cast<int*>(base + 10 * E + 32 * 33 + 64); }
    __device__ int* w() const { return bad() + 2; }
    static constexpr size_t BYTES = sizeof(double) * (10 * E + 32 * 33 + 64 + 16);
};
static_assert(DiagLds::BYTES <= FLOW_LDS_BYTES, "diag workgroup LDS carve");
enum { DW_LS = 0, DW_D, DW_LPUB, DW_DPUB, DW_PRE6, DW_PRE7, DW_BAR, DW_L2, DW_P2, DW_G0, DW_N };
static_assert(DW_N <= 28, "progress words fit in the carve");

__device__ __forceinline__ int lds_get(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_put(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const int* p, int v) {
    while (__builtin_amdgcn_readfirstlane(lds_get(p)) < v) __builtin_amdgcn_s_sleep(1);
}
// barrier of waves 0-3 only (monotonic LDS counter)
__device__ __forceinline__ void chain_bar(int* cnt, int& epoch) {
    epoch += 4;
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__builtin_amdgcn_readfirstlane(lds_get(cnt)) < epoch) {}   // spin: a sleep's wake-up
                                                                        // is on the chain (+1%)
}

// wave-level tile (accumulator layout) <-> LDS tile of stride ld
__device__ __forceinline__ void wt_to_lds_ld(const WTile& t, double* S, int ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) S[(16 * a + lq + 4 * r) * ld + 16 * b + li] = t.v[a][b][r];
}
__device__ __forceinline__ void lds_to_wt_ld(WTile& t, const double* S, int ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) t.v[a][b][r] = S[(16 * a + lq + 4 * r) * ld + 16 * b + li];
}
__device__ __forceinline__ void op_rows_lds_ld(WOp& o, const double* S, int ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s) o.v[b][s] = S[(16 * b + li) * ld + 8 * lq + s];
}

__device__ __forceinline__ void op_cols_lds_ld(WOp& o, const double* S, int ld) {
    const int li = threadIdx.x & 15, lq = (threadIdx.x >> 4) & 3;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s) o.v[b][s] = S[(8 * lq + s) * ld + 16 * b + li];
}

// the chain waves (0-3) spin on their LDS words: a sleep's wake-up would sit on the critical
// path (the waits of waves 4-7 keep sleeping: wave 4 shares SIMD 0 with the factor)
__device__ __forceinline__ void lds_spin_ge(const int* p, int v) {
    while (__builtin_amdgcn_readfirstlane(lds_get(p)) < v) {}
}
__device__ __forceinline__ void diag_chain(FlowCtx& C, const DiagLds& B) {
    constexpr int S = TileCfg<32>::S;
    const FlowArgs& a = C.a;
    const int T = a.T;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    int epoch = 0;
    if (w == 0) {   // D_0: wave 0 forms tile (0,0) of K + s2 I and factors it
        // tile (0,0): flow_gram_phase's (waves 0 and 1 formed it in fsc), or the graph kernel's k_gram
        if (!a.gram) {
            for (int e = l; e < 32 * 32; e += 64) B.fsc()[(e >> 5) * 33 + (e & 31)] = a.A[(long)(e >> 5) * a.lda + (e & 31)];
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        } else {
            if (a.trace && l == 0) a.trace[0] = flow_clock() - C.t0;
            lds_spin_ge(&B.w()[DW_G0], 2);   // the blocks of waves 1 and 4
            if (a.trace && l == 0) a.trace[T] = flow_clock() - C.t0;
        }
        tile_potrf_inv_w1_wave(B.fsc(), 33, B.fsc(), B.Db(0), B.dg(0), &B.bad()[0]);
        if (l == 0) lds_put(&B.w()[DW_D], 0);
    }
    for (int k = 1; k < T; ++k) {
        const int pk = k & 1;
        if (a.trace && threadIdx.x == 0) a.trace[k] = flow_clock() - C.t0;
        lds_spin_ge(&B.w()[DW_PRE6], k);
        lds_spin_ge(&B.w()[DW_PRE7], k);
        lds_spin_ge(&B.w()[DW_D], k - 1);         // D_{k-1} in Db[pk ^ 1]
        lds_spin_ge(&B.w()[DW_LPUB], k - 2);      // wave 4 is done with Ls[pk] (L(k-2,k-3))
        if (a.trace && threadIdx.x == 0) a.trace[T + k] = flow_clock() - C.t0;
        Acc<32> pl, cij;
#pragma unroll
        for (int r = 0; r < 4; ++r) cij.v[0][r] = B.Cp(pk)[acc_row<32>(0, r) * S + acc_col<32>(0)];   // (under the product)
        acc_zero(pl);
        tile_mma<32, false, true>(pl, B.Ap(pk), B.Db(pk ^ 1), 1.0);   // L(k,k-1) = A'' D_{k-1}^T
        acc_to_lds(pl, B.Ls(pk));
        chain_bar(&B.w()[DW_BAR], epoch);
        if (threadIdx.x == 0) lds_put(&B.w()[DW_LS], k);
        // only the lower blocks of A''(k,k) feed the factor: wave 1 (block (0,1)) skips the
        // product and leaves SIMD 1 to wave 5 from the end of the first product on
        if (w != 1)
        tile_mma<32, false, true>(cij, B.Ls(pk), B.Ls(pk), -1.0);   // A''(k,k) -= L L^T
        {
            const int bi = w >> 1, bj = w & 1;
            if (bj <= bi) {
#pragma unroll
                for (int q = 0; q < 4; ++q) B.fsc()[(16 * bi + (l >> 4) + 4 * q) * 33 + 16 * bj + (l & 15)] = cij.v[0][q];
            }
        }
        chain_bar(&B.w()[DW_BAR], epoch);
        if (threadIdx.x == 0) lds_put(&B.w()[DW_P2], k);  // tile products of step k done
        if (w == 0) {
            lds_spin_ge(&B.w()[DW_DPUB], k - 2);    // wave 4 is done with Db[pk] (D_{k-2})
            if (a.trace && threadIdx.x == 0) a.trace[2 * T + k] = flow_clock() - C.t0;
            tile_potrf_inv_w1_wave(B.fsc(), 33, B.fsc(), B.Db(pk), B.dg(pk), &B.bad()[pk]);
            if (l == 0) lds_put(&B.w()[DW_D], k);
        }
    }
}


__device__ __forceinline__ void diag_publisher(FlowCtx& C, const DiagLds& B) {
    constexpr int S = TileCfg<32>::S;
    const FlowArgs& a = C.a;
    const int T = a.T;
    const int l = threadIdx.x & 63;
    for (int k = 0; k < T; ++k) {
        const int pk = k & 1;
        if (k == 0) lds_wait_ge(&B.w()[DW_D], 0);
        if (k > 0) {
            lds_wait_ge(&B.w()[DW_LS], k);
            double* dst = C.P.L(k, k - 1);
            const double* src = B.Ls(pk);
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int e = l + 64 * q;
                st_coherent(dst + e, src[(e >> 5) * S + (e & 31)]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (l == 0) lds_put(&B.w()[DW_LPUB], k);
            lds_wait_ge(&B.w()[DW_D], k);
        }
        const double* D = B.Db(pk);
        double* dp = C.P.D(k);
        double* xt = C.P.X(k, k);
        double* xo = C.Xt(k, k);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int e = l + 64 * q;
            st_coherent(dp + e, D[(e >> 5) * S + (e & 31)]);
        }
        if (a.trace && l == 0) a.trace[3 * T + k] = flow_clock() - C.t0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int e = l + 64 * q;
            const int r = e >> 5, c = e & 31;
            const double v = D[r * S + c];
            st_coherent(xt + c * 32 + r, v);             // X^T(k,k) = D_k^T
            xo[(long)r * a.ldx + c] = v;
        }
        {
            if (l < 32) a.ldiag[k * 32 + l] = B.dg(pk)[l];
            if (l == 0 && B.bad()[pk] && a.info[0] == 0) a.info[0] = k * 32 + B.bad()[pk];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (l == 0) lds_put(&B.w()[DW_DPUB], k);
    }
}

// wave 5 shares SIMD 1 with chain wave 1, whose last MFMA of a step is its block of the first
// product (L(k,k-1)): its MFMA work waits for that product (W5_GATE)
#define W5_GATE DW_LS
__device__ __forceinline__ void diag_second(FlowCtx& C, const DiagLds& B) {
    constexpr int S = TileCfg<32>::S;
    const FlowArgs& a = C.a;
    const int T = a.T;
    for (int j = 2; j < T; ++j) {
        WTile acc;
        WOp x, y;
        if (j >= 4) {
            pub_wt_op_direct(acc, C.P.H(2, j), x, C.P.L(j, j - 3), C);
        } else {
            // A(2,0), A(3,1): their initial values (Gram phase: A(2,0) this wave's, in L2[0];
            // A(3,1) a worker wave's FT_G)
            if (a.gram && j == 2) lds_to_wt_ld(acc, B.L2(0), S);
            else if (a.gram) pub_wt(acc, C.P.H(2, j), C);
            else wt_load<true>(acc, C.At(j, j - 2), a.lda);
            if (j == 3) pub_op(x, C.P.L(j, j - 3), C);
        }
        if (a.trace && (threadIdx.x & 63) == 0) a.trace[4 * T + j] = flow_clock() - C.t0;
        if (j >= 3) {
            // panel j-3: A(j,j-2) -= L(j,j-3) L(j-2,j-3)^T  (the worker's L, the chain's Ls of step j-2)
            lds_wait_ge(&B.w()[W5_GATE], j - 1);          // MFMA only once the chain's step j-1 products
            lds_wait_ge(&B.w()[DW_LS], j - 2);            // on SIMD 1 are done (an earlier window in the
                                                          // factor, or none, measured slower)
            if (a.trace && (threadIdx.x & 63) == 0) a.trace[8 * T + 3 * a.nwaves + 4 * FLOW_LOG * a.nwaves + j] = flow_clock() - C.t0;
            op_rows_lds_ld(y, B.Ls((j - 2) & 1), S);
            wt_mma<true>(acc, x, y);
        }
        lds_wait_ge(&B.w()[DW_D], j - 2);
        lds_wait_ge(&B.w()[W5_GATE], j - 1);
        lds_wait_ge(&B.w()[DW_PRE6], j - 1);              // L2[j & 1] = L(j-2,j-4): last read by
        lds_wait_ge(&B.w()[DW_PRE7], j - 2);              // wave 6 at j-1, wave 7 at j-2
        if (a.trace && (threadIdx.x & 63) == 0) a.trace[8 * T + 3 * a.nwaves + 4 * FLOW_LOG * a.nwaves + T + j] = flow_clock() - C.t0;
        wt_to_lds_ld(acc, B.L2(j & 1), S);               // staging: A'(j,j-2) as the A operand
        asm volatile("" ::: "memory");
        op_rows_lds_ld(x, B.L2(j & 1), S);
        op_rows_lds_ld(y, B.Db((j - 2) & 1), S);         // B[k][c] = D_{j-2}[c][k]
        wt_zero(acc);
        wt_mma<false>(acc, x, y);
        asm volatile("" ::: "memory");
        wt_to_lds_ld(acc, B.L2(j & 1), S);
        if ((threadIdx.x & 63) == 0) lds_put(&B.w()[DW_L2], j);
        if (a.trace && (threadIdx.x & 63) == 0) a.trace[7 * T + j] = flow_clock() - C.t0;
        wt_store<true>(acc, C.P.L(j, j - 2), 32);
    }
}

__device__ __forceinline__ void diag_prefetch(FlowCtx& C, const DiagLds& B, bool sub) {
    constexpr int S = TileCfg<32>::S;
    const FlowArgs& a = C.a;
    const int T = a.T;
    int* done = &B.w()[sub ? DW_PRE6 : DW_PRE7];
    // Gram phase: step 1's tiles came from chain waves 2 / 3, step 2's are in dst (this wave's)
    for (int j = a.gram ? 2 : 1; j < T; ++j) {
        const int pj = j & 1;
        double* dst = sub ? B.Ap(pj) : B.Cp(pj);
        WTile acc;
        WOp x, y;
        if (j >= 4) {
            pub_wt_op_direct(acc, C.P.H(sub ? 0 : 1, j), x, C.P.L(j, j - 3), C);
        } else {
            // initial values of the rows <= 3
            if (a.gram && j == 2) lds_to_wt_ld(acc, dst, S);
            else if (a.gram) pub_wt(acc, C.P.H(sub ? 0 : 1, j), C);   // a worker wave's FT_G
            else wt_load<true>(acc, sub ? C.At(j, j - 1) : C.At(j, j), a.lda);
            if (j == 3) pub_op(x, C.P.L(j, j - 3), C);
        }
        if (a.trace && (threadIdx.x & 63) == 0) a.trace[(sub ? 5 : 6) * T + j] = flow_clock() - C.t0;
        if (j >= 3) {
            // panel j-3 from the worker's L(j,j-3) and L(j-1,j-3) (wave 5, step j-1)
            lds_wait_ge(&B.w()[DW_P2], j - 1);
            if (sub) {
                lds_wait_ge(&B.w()[DW_L2], j - 1);
                op_rows_lds_ld(y, B.L2((j - 1) & 1), S);
            } else {
                y = x;
            }
            wt_mma<true>(acc, x, y);
        }
        long long* tw = a.trace ? a.trace + 8 * T + 3 * a.nwaves + 4 * FLOW_LOG * a.nwaves + (sub ? 2 : 4) * T : nullptr;
        if (j >= 2) {
            WOp x, y;
            lds_wait_ge(&B.w()[DW_P2], j - 1);
            lds_wait_ge(&B.w()[DW_L2], j);
            op_rows_lds_ld(x, B.L2(pj), S);
            lds_wait_ge(&B.w()[DW_LS], j - 1);
            if (tw && (threadIdx.x & 63) == 0) tw[j] = flow_clock() - C.t0;
            if (sub) op_rows_lds_ld(y, B.Ls(pj ^ 1), S);
            else y = x;
            wt_mma<true>(acc, x, y);
        }
        wt_to_lds_ld(acc, dst, S);
        if ((threadIdx.x & 63) == 0) lds_put(done, j);
        if (tw && (threadIdx.x & 63) == 0) tw[T + j] = flow_clock() - C.t0;
    }
}

// The diag workgroup's Gram phase (FlowArgs::gram): each wave forms the initial value of what its
// role starts from, straight into LDS: waves 0 / 4 / 1 the lower 16 x 16 blocks (0,0) / (1,0) /
// (1,1) of tile (0,0) into the factor's input (waves 4 and 1 count into DW_G0; the factor reads
// the lower blocks only), chain waves 2 / 3 step 1's A(1,0) / A(1,1) into Ap[1] / Cp[1] (in place
// of waves 6 / 7's j = 1, signalled through their words), wave 5 A(2,0) into L2[0], waves 6 / 7
// A(2,1) / A(2,2) into their j = 2 destinations.  Row 3's band tiles are FT_G worker tiles; the
// rest of the rows <= 3 are FT_A worker tiles.  Measured (tools/flow_trace.py, one call): block
// (0,0) formed 0.5 -> 5.7 us into the launch (kernel arguments 0.5, X / theta round trip 1.3,
// dots 1.2, norms 0.6, exp and stores ~1.5), D_0 at ~10-12 us (the first factor runs with a cold
// instruction cache: ~5 us against ~3.9 in the chain); the base build's chain started at 2.4 us
// with D_0 from the Gram launch before it.
__device__ __forceinline__ void diag_gram_phase(const FlowArgs& a, const DiagLds& B, long long t0) {
    constexpr int S = TileCfg<32>::S;
    const int w = threadIdx.x >> 6, T = a.T;
    auto tile = [&](int i, int j, double* dst, int ld, int b0, int b1) {
        flow_gram_tile<false>(a.X, a.ldxi, a.theta, a.n, a.D, i, j, dst, ld, b0, b1);
    };
    auto signal = [&](int word, int v) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if ((threadIdx.x & 63) == 0) lds_put(&B.w()[word], v);
    };
    if (w < 2 || w == 4) {
        // the factor reads the lower blocks only: (0,0) wave 0, (1,0) wave 4, (1,1) wave 1
        flow_gram_tile<false>(a.X, a.ldxi, a.theta, a.n, a.D, 0, 0, B.fsc(), 33, w == 0 ? 0 : 1, w == 0 ? 1 : 2,
                              w == 1 ? 2 : 1);
        if (w != 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(&B.w()[DW_G0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else if (w < 4) {
        if (T > 1) {
            tile(1, w - 2, w == 2 ? B.Ap(1) : B.Cp(1), S, 0, 2);
            signal(w == 2 ? DW_PRE6 : DW_PRE7, 1);
            if (a.trace && (threadIdx.x & 63) == 0 && w == 2) a.trace[2 * T] = flow_clock() - t0;
        }
    } else if (T > 2) {
        tile(2, w - 5, w == 5 ? B.L2(0) : w == 6 ? B.Ap(0) : B.Cp(0), S, 0, 2);
    }
}

__device__ __forceinline__ void flow_diag(FlowCtx& C, double* smem) {
    DiagLds B;
    B.base = smem;
    if (threadIdx.x < DW_N)
        B.w()[threadIdx.x] = (threadIdx.x == DW_LPUB || threadIdx.x == DW_DPUB || threadIdx.x == DW_D) ? -1 : 0;
    if (threadIdx.x < 2) B.bad()[threadIdx.x] = 0;
    if (threadIdx.x == 0) C.a.info[0] = 0;   // first writer of info in the evaluation
    __syncthreads();
    if (C.a.gram) diag_gram_phase(C.a, B, C.t0);
    const int w = threadIdx.x >> 6;
    if (w < 4) diag_chain(C, B);
    else if (w == 4) diag_publisher(C, B);
    else if (w == 5) diag_second(C, B);
    else diag_prefetch(C, B, w == 6);
}

// The Gram phase (FlowArgs::gram), run by every wave before its role, where no role state is live
// (the tile code inlined into the roles set the kernel's allocation to 254 VGPRs, so no other
// kernel's wave fit beside the flow on a CU; as a call, 248): each worker wave forms its owned A
// tiles (read back only by itself, the stores drained first) and publishes its FT_G band tiles of
// row 3 to FlowPub::H for the diag waves 5-7 (the catalogue puts those on otherwise idle waves).
// The diag workgroup has its own (diag_gram_phase).  Forming all band tiles of the rows <= 3 in
// waves 0 / 5 / 6 / 7 (two or three each) delayed the chain's start by ~25 us a launch; the eight
// as FT_G worker tiles, ~9.5 us (published ~11 us into the launch: their waves share SIMDs with
// waves forming their own tiles).
__device__ __forceinline__ void flow_gram_phase(const FlowArgs& a) {
    const int w = threadIdx.x >> 6;
    {
        const int* own = a.own + ((blockIdx.x - 1) * FLOW_WAVES + w) * FLOW_MAXOWN;
#pragma unroll 1
        for (int s = 0; s < FLOW_MAXOWN; ++s) {
            const int code = __builtin_amdgcn_readfirstlane(own[s]);
            if (code < 0) continue;
            const FlowTile t = flow_tile(code, a.T);
            double* at = a.A + (long)t.i * 32 * a.lda + (long)t.j * 32;
            if (t.type == FT_A) flow_gram_tile<false>(a.X, a.ldxi, a.theta, a.n, a.D, t.i, t.j, at, a.lda);
            if (t.type == FT_G) {
                const FlowPub P{a.pub, a.T, a.Tp};
                flow_gram_tile<true>(a.X, a.ldxi, a.theta, a.n, a.D, t.i, t.j,
                                     P.H(t.j == t.i ? 1 : t.j == t.i - 1 ? 0 : 2, t.i), 32);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
}

__global__ __launch_bounds__(FLOW_THREADS) void k_chol_flow(FlowArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    FlowCtx C;
    C.t0 = flow_clock();
    if (a.gram && blockIdx.x != 0) flow_gram_phase(a);
    C.a = a;
    C.P.base = a.pub;
    C.P.T = a.T;
    C.P.Tp = a.Tp;
    if (blockIdx.x == 0) {
        flow_diag(C, smem);
        return;
    }
    const int w = threadIdx.x >> 6;
    flow_worker(C, (blockIdx.x - 1) * FLOW_WAVES + w, smem + w * 32 * WLD);
}

long flow_npub(int T, int Tp) { return 1024L * (T * (T - 1) / 2 + T + T * (T + 1) / 2 + T * Tp + 3 * T); }
int flow_nflags(int T, int Tp) { (void)T; (void)Tp; return 1; }   // the abort word
// layout: chain / helper stamps [8T] | worker summaries + item logs | wave-5 detail [2T] | wave-6 / 7 detail
// [2T each: last waits done, published] | k_gram timeline [flow_gram_dbg_count(T)] (the last region)
int flow_trace_count(int T, int nwg) { return 8 * T + (3 + 4 * FLOW_LOG) * FLOW_WAVES * (nwg - 1) + 6 * T + flow_gram_dbg_count(T); }

void launch_chol_flow(const FlowArgs& a, int nwg, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_chol_flow),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)FLOW_LDS_BYTES);
        attr = true;
    }
    hipLaunchKernelGGL(k_chol_flow, dim3(nwg), dim3(FLOW_THREADS), FLOW_LDS_BYTES, s, a);
}

}  // namespace mfgp
