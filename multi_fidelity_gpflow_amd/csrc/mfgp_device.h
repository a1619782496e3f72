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
template <int NB>
__device__ __forceinline__ void acc_to_lds(const Acc<NB>& a, double* __restrict__ s) {
    constexpr int S = TileCfg<NB>::S;
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[acc_row<NB>(q, r) * S + acc_col<NB>(q)] = a.v[q][r];
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
#ifndef MFGP_VALU_TILES
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
#else
    // VALU fallback with the identical element ownership (diagnostic builds only)
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q) {
        const int j = acc_col<NB>(q);
        for (int k = 0; k < NB; ++k) {
            const double bv = TB ? Bs[j * S + k] : Bs[k * S + j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = acc_row<NB>(q, r);
                const double av = TA ? As[k * S + i] : As[i * S + k];
                acc.v[q][r] += alpha * av * bv;
            }
        }
    }
#endif
}

// ---------------------------------------------------------------- diag factor
// In-LDS Cholesky of an SPD NB x NB tile A (lower part used) fused with the
// inverse of its factor: on exit R holds D = L^{-1} (lower, zero above), and
// dg[i] = L_ii.  Right-looking, one barrier per pivot:
//   a_ij -= l_ik l_jk (i >= j > k),   r_ic -= l_ik x_kc (i > k >= c),  x_k = r_k / l_kk.
// Non-positive or non-finite pivots report through *bad (first local index + 1).
template <int NB>
__device__ void tile_potrf_inv(double* __restrict__ A, double* __restrict__ R, double* __restrict__ dg,
                               int* __restrict__ bad) {
    constexpr int S = TileCfg<NB>::S;
    for (int p = threadIdx.x; p < NB * NB; p += NTHREADS) {
        const int i = p / NB, c = p % NB;
        R[i * S + c] = (i == c) ? 1.0 : 0.0;
    }
    if (threadIdx.x == 0) *bad = 0;
    __syncthreads();
    for (int k = 0; k < NB; ++k) {
        const double akk = A[k * S + k];
        const double lkk = sqrt(akk);
        const double rl = 1.0 / lkk;
        if (threadIdx.x == 0) {
            dg[k] = lkk;
            if (!(akk > 0.0) || !(akk < INFINITY)) { if (*bad == 0) *bad = k + 1; }
        }
        // trailing A (lower triangle only) and R update; rows i > k
        const int rows = NB - k - 1;
        for (int p = threadIdx.x; p < rows * NB; p += NTHREADS) {
            const int i = k + 1 + p / NB, c = p % NB;
            const double lik = A[i * S + k] * rl;
            if (c > k) {
                if (c <= i) A[i * S + c] -= lik * (A[c * S + k] * rl);
            } else {
                R[i * S + c] -= lik * (R[k * S + c] * rl);
            }
        }
        __syncthreads();
    }
    // D = diag(1/l) * R  (row k of L^{-1} is r_k / l_kk)
    for (int p = threadIdx.x; p < NB * NB; p += NTHREADS) {
        const int i = p / NB, c = p % NB;
        R[i * S + c] = (c <= i) ? R[i * S + c] / dg[i] : 0.0;
    }
    __syncthreads();
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
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

}  // namespace mfgp
