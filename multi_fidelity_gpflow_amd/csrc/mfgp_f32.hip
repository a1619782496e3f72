// mfgp_f32.hip — the fp32 instance of the GPR hot path (BASELINE configs[4], "Synth":
// N_L = 16384, N_H = 2048, D = 10, P = 512).  The reference forces fp64
// (mfgpflow/linear.py:63-64); fp32 is this engine's added capability, with the same
// semantics as the fp64 path (linear.py:55-136 kernel, GPflow GPR LML / gradient / predict).
//
// At N = 18432 the factorization is 2.1 TFLOP (N^3/3): MFMA-throughput-bound, not
// chain-latency-bound like Goku's 1164.  Everything is therefore ONE tall matrix M (fp32,
// row-major, ld = Npad, 128 x 128 tiles) factored by a right-looking blocked Cholesky whose
// every stage is an NT GEMM (both operands read along the contraction index):
//
//   row tiles [0, T)                  A = K + s2 I   (lower tiles)          -> L
//   row tiles [T, T+Tp)               Y^T                                  -> Z^T = (L^-1 Y)^T
//   row tiles [T+Tp, T+Tp+Ts)         K(X*, X)  (predict only)             -> (L^-1 Kmn)^T
//   row tiles [T+Tp+Ts, +Ti)          I         (gradient only)            -> L^-T
//
// Factoring the first N columns of [K; B] gives B L^-T in the bottom rows, so the solves and
// the explicit inverse come out of the same sweep as the factor.  L^-T's rows are exactly the
// operands K^-1 = L^-T L^-1 needs in NT form, and alpha = K^-1 Y = L^-T Z the same.
//
// Sweep: outer panels of W tiles (W*128 columns).  Inside a panel, per tile column k: factor
// the 128 x 128 diagonal block in registers (k32_diag, also D_k = L_kk^-1), form the panel
// L(r,k) = M(r,k) D_k^T for every live row tile (k32_panel), update the remaining panel columns
// (k32_update, K = 128).  Then ONE trailing update of everything right of the panel with
// K = W*128 (k32_update): the C tile read-modify-write is paid once per panel, not per column.
//
// GEMM core: 128 x 128 output per 256-thread workgroup, 4 waves of 64 x 64 (2 x 2 blocks of
// v_mfma_f32_32x32x2_f32), BK = 32, LDS double buffer with register staging.  LDS rows are
// [row][k] with a 36-float stride: each lane reads 4 consecutive k of its row with one
// ds_read_b128 (the k order inside an MFMA sum is free as long as A and B agree), and the
// 16-lane groups of ds_read_b128 land on distinct banks.
#include "mfgp_device.h"
#include "mfgp_internal.h"

namespace mfgp {
namespace f32 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TB = F32_TILE;          // 128
constexpr int BK = 32;
constexpr int LDL = BK + 4;           // LDS row stride (floats)
constexpr int GT = 256;               // threads of the GEMM-shaped kernels
constexpr int STAGE = 2 * TB * LDL;   // floats per LDS stage (A + B)
constexpr size_t GEMM_SMEM = 2 * STAGE * sizeof(float);   // 73,728 B: two workgroups per CU

// ---------------------------------------------------------------- GEMM core
struct Acc {
    f32x16 c[2][2];
};

__device__ __forceinline__ void acc_zero(Acc& a) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) a.c[m][n][r] = 0.0f;
}

// Output element (m, n, reg) of this lane: MFMA 32x32 C/D map (col = lane & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)) inside the wave's 64 x 64 quarter.
__device__ __forceinline__ int acc_row(int m, int reg) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    return (w >> 1) * 64 + m * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col(int n) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    return (w & 1) * 64 + n * 32 + (lane & 31);
}

struct StageRegs {
    f32x4 a[4], b[4];
};

// thread t moves rows t/8 + 32q, floats 4(t%8) .. +3 of the 128 x 32 A and B slabs
__device__ __forceinline__ void stage_fetch(StageRegs& s, const float* __restrict__ A, long lda,
                                            const float* __restrict__ B, long ldb, int k) {
    const int r = threadIdx.x >> 3, c4 = (threadIdx.x & 7) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s.a[q] = *reinterpret_cast<const f32x4*>(A + (long)(r + 32 * q) * lda + k + c4);
        s.b[q] = *reinterpret_cast<const f32x4*>(B + (long)(r + 32 * q) * ldb + k + c4);
    }
}
__device__ __forceinline__ void stage_put(float* sm, const StageRegs& s) {
    const int r = threadIdx.x >> 3, c4 = (threadIdx.x & 7) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        *reinterpret_cast<f32x4*>(sm + (r + 32 * q) * LDL + c4) = s.a[q];
        *reinterpret_cast<f32x4*>(sm + TB * LDL + (r + 32 * q) * LDL + c4) = s.b[q];
    }
}
__device__ __forceinline__ void stage_mma(Acc& acc, const float* sm) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float* sa = sm + ((w >> 1) * 64 + (lane & 31)) * LDL + 4 * (lane >> 5);
    const float* sb = sm + TB * LDL + ((w & 1) * 64 + (lane & 31)) * LDL + 4 * (lane >> 5);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 8) {
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(sa + kk);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(sa + 32 * LDL + kk);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(sb + kk);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(sb + 32 * LDL + kk);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            acc.c[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc.c[0][0], 0, 0, 0);
            acc.c[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b1[s], acc.c[0][1], 0, 0, 0);
            acc.c[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b0[s], acc.c[1][0], 0, 0, 0);
            acc.c[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc.c[1][1], 0, 0, 0);
        }
    }
}

// acc += A[0:128, 0:32 nk] * B[0:128, 0:32 nk]^T (row-major, 16-B aligned rows).  Ends with a
// barrier, so two calls may follow each other on the same LDS.  Global loads run TWO K-steps
// ahead of the MFMAs (two register stages, the loop unrolled by two so each stage is a
// compile-time register set): at ~4k MFMA cycles per K-step, one step of lead did not cover the
// L2 / Infinity Cache latency under load.  Cpre (optional): the C tile this workgroup will
// update, loaded into *cv during the last K-step, so the epilogue does not start with a
// round trip to memory.
__device__ __forceinline__ void c_tile_load(float (&cv)[2][2][16], const float* __restrict__ C, long ld) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) cv[m][n][r] = C[(long)acc_row(m, r) * ld + acc_col(n)];
}

__device__ __forceinline__ void gemm_nt(Acc& acc, const float* __restrict__ A, long lda, const float* __restrict__ B,
                                        long ldb, int nk, float* smem, const float* Cpre = nullptr, long ldc = 0,
                                        float (*cv)[2][16] = nullptr) {
    StageRegs s0, s1;
    stage_fetch(s0, A, lda, B, ldb, 0);
    if (nk > 1) stage_fetch(s1, A, lda, B, ldb, BK);
    stage_put(smem, s0);
    if (nk > 2) stage_fetch(s0, A, lda, B, ldb, 2 * BK);
    __syncthreads();
    // invariant at even kt: buffer 0 holds step kt, s1 step kt+1, s0 step kt+2
    for (int kt = 0; kt < nk; kt += 2) {
        if (Cpre && kt + 1 >= nk) c_tile_load(*reinterpret_cast<float(*)[2][2][16]>(cv), Cpre, ldc);
        stage_mma(acc, smem);
        if (kt + 1 < nk) {
            stage_put(smem + STAGE, s1);
            if (kt + 3 < nk) stage_fetch(s1, A, lda, B, ldb, (kt + 3) * BK);
        }
        __syncthreads();
        if (kt + 1 < nk) {
            if (Cpre && kt + 2 >= nk) c_tile_load(*reinterpret_cast<float(*)[2][2][16]>(cv), Cpre, ldc);
            stage_mma(acc, smem + STAGE);
            if (kt + 2 < nk) {
                stage_put(smem, s0);
                if (kt + 4 < nk) stage_fetch(s0, A, lda, B, ldb, (kt + 4) * BK);
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ void acc_store(const Acc& a, float* __restrict__ C, long ld) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) C[(long)acc_row(m, r) * ld + acc_col(n)] = a.c[m][n][r];
}
// C -= acc, one 32 x 32 block at a time (16 loads in flight, then 16 stores: the registers the
// loads need stay within the GEMM loop's budget)
__device__ __forceinline__ void acc_sub_into(const Acc& a, float* __restrict__ C, long ld) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            float v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = C[(long)acc_row(m, r) * ld + acc_col(n)];
#pragma unroll
            for (int r = 0; r < 16; ++r) C[(long)acc_row(m, r) * ld + acc_col(n)] = v[r] - a.c[m][n][r];
        }
}

// ---------------------------------------------------------------- geometry
__host__ __device__ inline int rows_B(const F32Args& a, int k1) {   // live bottom row tiles after k1 columns
    return a.Tp + a.Ts + (k1 < a.Ti ? k1 : a.Ti);
}
__host__ __device__ inline long row_off(const F32Args& a, int rt) { return (long)rt * TB * a.ld; }
__host__ __device__ inline int id0(const F32Args& a) { return a.T + a.Tp + a.Ts; }   // first identity row tile

// identity-region tiles the gram launch initialises: row tile c, columns from the start of c's
// panel (earlier columns are never read)
__host__ __device__ inline long ident_tiles(const F32Args& a) {
    long s = 0;
    for (int c = 0; c < a.Ti; ++c) s += a.T - (c / a.W) * a.W;
    return s;
}

// ---------------------------------------------------------------- MF kernel tile (fp32)
// SquaredExponential in direct-difference form (the expanded
// |a|^2 + |b|^2 - 2 a.b of GPflow cancels catastrophically in fp32; in fp64 the two agree to
// ~1e-14, in fp32 the difference form keeps K's diagonal exact and PD-ness intact).
// Rows are staged transposed, [d][row], scaled by 1/l: xs1L, xs1D (tile rows), xs2L, xs2D (tile
// columns); flags f (0 LF, 1 HF, 2 any other value -> zero row, -1 beyond n).
struct GramSmem {
    float* x1L; float* x1D; float* x2L; float* x2D; float* f1; float* f2;
};
__device__ __forceinline__ GramSmem gram_smem(float* base, int D) {
    GramSmem g;
    g.x1L = base; g.x1D = g.x1L + D * TB; g.x2L = g.x1D + D * TB; g.x2D = g.x2L + D * TB;
    g.f1 = g.x2D + D * TB; g.f2 = g.f1 + TB;
    return g;
}
size_t gram_smem_bytes32(int D) { return sizeof(float) * (4 * (size_t)D * TB + 2 * TB); }

__device__ __forceinline__ float fid_code(float f) { return f == 0.0f ? 0.0f : (f == 1.0f ? 1.0f : 2.0f); }

__device__ void gram_stage(const GramSmem& g, const float* X1, long ldx1, int n1, int r1,
                           const float* X2, long ldx2, int n2, int r2, int D, const double* theta) {
    for (int e = threadIdx.x; e < TB * D; e += blockDim.x) {
        const int r = e % TB, d = e / TB;   // consecutive threads: consecutive rows of one dim
        const float il = (float)(1.0 / theta[1 + d]);
        const float ild = (float)(1.0 / theta[2 + D + d]);
        const float x1 = (r1 + r < n1) ? X1[(long)(r1 + r) * ldx1 + d] : 0.0f;
        const float x2 = (r2 + r < n2) ? X2[(long)(r2 + r) * ldx2 + d] : 0.0f;
        g.x1L[d * TB + r] = x1 * il; g.x1D[d * TB + r] = x1 * ild;
        g.x2L[d * TB + r] = x2 * il; g.x2D[d * TB + r] = x2 * ild;
    }
    for (int r = threadIdx.x; r < TB; r += blockDim.x) {
        g.f1[r] = (r1 + r < n1) ? fid_code(X1[(long)(r1 + r) * ldx1 + D]) : -1.0f;
        g.f2[r] = (r2 + r < n2) ? fid_code(X2[(long)(r2 + r) * ldx2 + D]) : -1.0f;
    }
}

// 128 x 128 tile of LinearMultiFidelityKernel.K (linear.py:55-104) from staged rows; thread t
// owns rows (t >> 4) + 16 i and columns 4 (t & 15) + 64 jj + q (i < 8, jj < 2, q < 4).
__device__ void gram_tile_vals(const GramSmem& g, int D, const double* theta, float v[8][8]) {
    const int t = threadIdx.x;
    const int rb = t >> 4, cb = (t & 15) * 4;
    float s2[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) s2[i][j] = 0.0f;
    for (int d = 0; d < D; ++d) {
        float a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = g.x1L[d * TB + rb + 16 * i];
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.x2L + d * TB + cb);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.x2L + d * TB + cb + 64);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float u0 = a[i] - b0[q], u1 = a[i] - b1[q];
                s2[i][q] = fmaf(u0, u0, s2[i][q]);
                s2[i][4 + q] = fmaf(u1, u1, s2[i][4 + q]);
            }
    }
    const float vL = (float)theta[0], vD = (float)theta[1 + D], rho = (float)theta[2 + 2 * D];
    bool hh = false;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float f1 = g.f1[rb + 16 * i], f2 = g.f2[cb + (j & 3) + 64 * (j >> 2)];
            const float kL = vL * __expf(-0.5f * s2[i][j]);
            float val = 0.0f;
            if (f1 == 0.0f && f2 == 0.0f) val = kL;
            else if ((f1 == 0.0f && f2 == 1.0f) || (f1 == 1.0f && f2 == 0.0f)) val = kL * rho;
            else if (f1 == 1.0f && f2 == 1.0f) { val = kL * (rho * rho); hh = true; }
            v[i][j] = val;
        }
    if (__syncthreads_or(hh)) {   // HF x HF entries also get K_delta (linear.py:96); tile-uniform
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) s2[i][j] = 0.0f;
        for (int d = 0; d < D; ++d) {
            float a[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = g.x1D[d * TB + rb + 16 * i];
            const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.x2D + d * TB + cb);
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.x2D + d * TB + cb + 64);
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float u0 = a[i] - b0[q], u1 = a[i] - b1[q];
                    s2[i][q] = fmaf(u0, u0, s2[i][q]);
                    s2[i][4 + q] = fmaf(u1, u1, s2[i][4 + q]);
                }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float f1 = g.f1[rb + 16 * i], f2 = g.f2[cb + (j & 3) + 64 * (j >> 2)];
                if (f1 == 1.0f && f2 == 1.0f) v[i][j] += vD * __expf(-0.5f * s2[i][j]);
            }
    }
}

__device__ __forceinline__ void tri_decode32(long t, int& i, int& j) {
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((long)(r + 1) * (r + 2) / 2 <= t) ++r;
    while ((long)r * (r + 1) / 2 > t) --r;
    i = r;
    j = (int)(t - (long)r * (r + 1) / 2);
}

// ---------------------------------------------------------------- K1: gram + RHS rows + identity
// blockIdx ranges: [A lower tiles][Y^T tiles Tp x T][K(X*,X) tiles Ts x T][identity fill]
__global__ __launch_bounds__(GT) void k32_gram(F32Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    long b = blockIdx.x;
    const long nA = (long)a.T * (a.T + 1) / 2, nY = (long)a.Tp * a.T, nS = (long)a.Ts * a.T;
    if (b == 0) {
        if (threadIdx.x == 0) *a.info = 0;
        if (a.cnt && threadIdx.x == 0) *a.cnt = 0;
    }
    const int t = threadIdx.x;
    if (b < nA || (b >= nA + nY && b < nA + nY + nS)) {
        // kernel tile: A (ti, tj) of K(X, X) + s2 I, or (st, tj) of K(X*, X)
        int ti, tj;
        const bool isA = b < nA;
        const float* X1;
        long ldx1;
        int n1, rt;
        if (isA) {
            tri_decode32(b, ti, tj);
            X1 = a.X; ldx1 = a.ldx; n1 = a.n; rt = ti;
        } else {
            const long s = b - nA - nY;
            ti = (int)(s / a.T); tj = (int)(s % a.T);
            X1 = a.Xs; ldx1 = a.ldxs; n1 = a.ns; rt = a.T + a.Tp + ti;
        }
        const GramSmem g = gram_smem(smem, a.D);
        gram_stage(g, X1, ldx1, n1, ti * TB, a.X, a.ldx, a.n, tj * TB, a.D, a.theta);
        __syncthreads();
        float v[8][8];
        gram_tile_vals(g, a.D, a.theta, v);
        const float noise = (float)a.theta[2 * a.D + 3];
        const int rb = t >> 4, cb = (t & 15) * 4;
        float* out = a.M + row_off(a, rt) + (long)tj * TB;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = rb + 16 * i;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                f32x4 w;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = cb + 64 * jj + q;
                    float x = v[i][4 * jj + q];
                    if (isA && ti == tj && r == c) x = (ti * TB + r < a.n) ? x + noise : 1.0f;   // identity padding
                    w[q] = x;
                }
                *reinterpret_cast<f32x4*>(out + (long)r * a.ld + cb + 64 * jj) = w;
            }
        }
        return;
    }
    if (b < nA + nY) {   // Y^T tile (pt, it): M[T + pt][it] = Y[it rows][pt cols]^T
        const long s = b - nA;
        const int pt = (int)(s / a.T), it = (int)(s % a.T);
        float* tile = smem;   // [i][p], stride TB + 1
        for (int e = t; e < TB * TB; e += GT) {
            const int i = e / TB, p = e % TB;
            const int gi = it * TB + i, gp = pt * TB + p;
            tile[i * (TB + 1) + p] = (gi < a.n && gp < a.p) ? a.Y[(long)gi * a.ldy + gp] : 0.0f;
        }
        __syncthreads();
        float* out = a.M + row_off(a, a.T + pt) + (long)it * TB;
        for (int e = t; e < TB * TB; e += GT) {
            const int p = e / TB, i = e % TB;
            out[(long)p * a.ld + i] = tile[i * (TB + 1) + p];
        }
        return;
    }
    // identity fill: row tile c, column tiles from the start of c's panel
    long s = b - nA - nY - nS;
    int c = 0;
    for (; c < a.Ti; ++c) {
        const long cnt = a.T - (c / a.W) * a.W;
        if (s < cnt) break;
        s -= cnt;
    }
    if (c >= a.Ti) return;
    const int j = (c / a.W) * a.W + (int)s;
    float* out = a.M + row_off(a, id0(a) + c) + (long)j * TB;
    for (int e = t; e < TB * TB / 4; e += GT) {
        const int r = e / (TB / 4), c4 = (e % (TB / 4)) * 4;
        f32x4 w = {0.0f, 0.0f, 0.0f, 0.0f};
        if (j == c && r >= c4 && r < c4 + 4) w[r - c4] = 1.0f;
        *reinterpret_cast<f32x4*>(out + (long)r * a.ld + c4) = w;
    }
}

// ---------------------------------------------------------------- K2a: diagonal block factor
// L_kk = chol(M(k,k)) and D_k = L_kk^-1 of one 128 x 128 block: ONE workgroup of 4 waves, the
// block and its inverse staged in LDS, blocked by 32:
//   for s = 0..3:  wave 0 factors the 32 x 32 diagonal sub-block in fp64 (factor32_w1, below) ->
//                  D_ss, L_ii;  L_is = A_is D_ss^T (i >= s) and A_ij -= L_is L_js^T (s < j <= i)
//                  on the MFMA (v_mfma_f32_32x32x2_f32, one 32 x 32 x 32 product per wave at a time);
//   then the inverse's off-diagonal blocks D_ij = -D_ii sum_{m=j}^{i-1} L_im D_mj, row by row.
constexpr int DIAG_THREADS = 256;
constexpr int DLD = TB + 4;   // LDS row stride of the staged block / inverse (floats)
constexpr int DIAG_R64 = 32 * TileCfg<32>::S;   // fp64 inverse of a 32 x 32 sub-block (w1 layout)
constexpr size_t DIAG_SMEM = sizeof(float) * (2 * (size_t)TB * DLD + 3 * 32 * 33 + TB) + 16 +
                             sizeof(double) * (DIAG_R64 + 32);

// acc += A[0:32, 0:32] B[0:32, 0:32]^T (row-major LDS tiles, ld multiple of 4)
__device__ __forceinline__ void mma32_nt(f32x16& acc, const float* A, int lda, const float* B, int ldb) {
    const int l = threadIdx.x & 63;
    const float* pa = A + (l & 31) * lda + 4 * (l >> 5);
    const float* pb = B + (l & 31) * ldb + 4 * (l >> 5);
#pragma unroll
    for (int kk = 0; kk < 32; kk += 8) {
        const f32x4 a4 = *reinterpret_cast<const f32x4*>(pa + kk);
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(pb + kk);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[s], b4[s], acc, 0, 0, 0);
    }
}
// acc += A[0:32, 0:32] B[0:32, 0:32] (B read along its rows)
__device__ __forceinline__ void mma32_nn(f32x16& acc, const float* A, int lda, const float* B, int ldb) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int k2 = 0; k2 < 32; k2 += 2) {
        const int kk = k2 + (l >> 5);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[(l & 31) * lda + kk], B[kk * ldb + (l & 31)], acc, 0, 0, 0);
    }
}
// LDS tile <- scale * acc (32 x 32 C/D layout: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5))
__device__ __forceinline__ void acc32_store(float* C, int ldc, const f32x16& acc, float scale) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * ldc + (l & 31)] = scale * acc[r];
}
__device__ __forceinline__ void acc32_load(f32x16& acc, const float* C, int ldc) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * ldc + (l & 31)];
}

// One wave: the 32 x 32 sub-block at (S, S) through the fp64 single-wave factor of the fp64 path
// (tile_potrf_inv_w1_wave, mfgp_device.h: 4 pivots a round on v_mfma_f64_16x16x4): the
// lower triangle widened into X (fp64, stride 33; also its panel scratch), D = L^-1 rounded into
// Ds, L_ii straight to ldiag.  (An fp32 one-wave factor that broadcast every pivot row with
// v_readlane took ~10 us a sub-block: tools/ubench_f32diag.hip.)  L_ss itself is formed by the
// panel step as A_ss D_ss^T.
__device__ __forceinline__ void factor32_w1(float* As, float* Ds, int S, double* X, double* R, double* dg, int* badw,
                                            int* bad, double* ldiag) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int e = l + 64 * q, r = e >> 5, c = e & 31;
        X[r * 33 + c] = (double)As[(S + r) * DLD + S + c];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tile_potrf_inv_w1_wave(X, 33, X, R, dg, badw);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int e = l + 64 * q, r = e >> 5, c = e & 31;
        Ds[(S + r) * DLD + S + c] = (float)R[r * TileCfg<32>::S + c];   // w1 writes zeros above
    }
    if (l < 32) ldiag[S + l] = dg[l];
    if (l == 0 && *badw && *bad == 0) *bad = S + *badw;
}

__global__ __launch_bounds__(DIAG_THREADS) void k32_diag(F32Args a, int k) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* As = smem;                 // [128][DLD]  A -> L (lower)
    float* Ds = As + TB * DLD;        // [128][DLD]  D = L^-1 (lower), zero above
    float* Ts = Ds + TB * DLD;        // 3 x [32][33] scratch for the inverse
    float* piv = Ts + 3 * 32 * 33;    // [128]
    int* bad = reinterpret_cast<int*>(piv + TB);
    int* badw = bad + 1;
    double* R64 = reinterpret_cast<double*>(smem + 2 * TB * DLD + 3 * 32 * 33 + TB + 4);   // 16-B aligned
    double* dg64 = R64 + DIAG_R64;
    double* X64 = reinterpret_cast<double*>(Ts);   // the inverse's scratch, free until the inverse
    const int w = threadIdx.x >> 6;
    float* Mkk = a.M + row_off(a, k) + (long)k * TB;
    {
        // all 16 loads of a thread in flight before the first LDS store (one memory round trip)
        constexpr int NQ = TB * TB / 4 / DIAG_THREADS;
        f32x4 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = threadIdx.x + q * DIAG_THREADS, r = e / (TB / 4), c4 = (e % (TB / 4)) * 4;
            v[q] = *reinterpret_cast<const f32x4*>(Mkk + (long)r * a.ld + c4);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = threadIdx.x + q * DIAG_THREADS, r = e / (TB / 4), c4 = (e % (TB / 4)) * 4;
            *reinterpret_cast<f32x4*>(As + r * DLD + c4) = v[q];
            *reinterpret_cast<f32x4*>(Ds + r * DLD + c4) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    }
    if (threadIdx.x == 0) *bad = 0;
    __syncthreads();
    auto T32 = [&](float* base, int i, int j) { return base + 32 * i * DLD + 32 * j; };
    for (int s = 0; s < 4; ++s) {
        if (w == 0) factor32_w1(As, Ds, 32 * s, X64, R64, dg64, badw, bad, a.ldiag + k * TB);
        __syncthreads();
        // panel: L_is = A_is D_ss^T (i >= s: the diagonal sub-block's L too, from the full
        // symmetric A_ss), one sub-block per wave
        for (int i = s + w; i < 4; i += 4) {
            f32x16 acc = {};
            mma32_nt(acc, T32(As, i, s), DLD, T32(Ds, s, s), DLD);
            acc32_store(T32(As, i, s), DLD, acc, 1.0f);   // the wave read its whole input first
        }
        __syncthreads();
        // trailing: A_ij -= L_is L_js^T, s < j <= i < 4
        int t = 0;
        for (int i = s + 1; i < 4; ++i)
            for (int j = s + 1; j <= i; ++j, ++t) {
                if (t % 4 != w) continue;
                f32x16 acc;
                acc32_load(acc, T32(As, i, j), DLD);
                f32x16 p = {};
                mma32_nt(p, T32(As, i, s), DLD, T32(As, j, s), DLD);
                acc -= p;
                acc32_store(T32(As, i, j), DLD, acc, 1.0f);
            }
        __syncthreads();
    }
    // inverse, row block i = 1..3: T_ij = sum_{m=j}^{i-1} L_im D_mj, then D_ij = -D_ii T_ij
    for (int i = 1; i < 4; ++i) {
        if (w < i) {
            const int j = w;
            f32x16 acc = {};
            for (int m = j; m < i; ++m) mma32_nn(acc, T32(As, i, m), DLD, T32(Ds, m, j), DLD);
            acc32_store(Ts + j * 32 * 33, 33, acc, 1.0f);
        }
        __syncthreads();
        if (w < i) {
            const int j = w;
            f32x16 acc = {};
            mma32_nn(acc, T32(Ds, i, i), DLD, Ts + j * 32 * 33, 33);
            acc32_store(T32(Ds, i, j), DLD, acc, -1.0f);
        }
        __syncthreads();
    }
    float* Dk = a.Dd + (long)k * TB * TB;
    for (int e = threadIdx.x; e < TB * TB / 4; e += DIAG_THREADS) {
        const int r = e / (TB / 4), c4 = (e % (TB / 4)) * 4;
        const f32x4 lv = *reinterpret_cast<const f32x4*>(As + r * DLD + c4);
        float* dst = Mkk + (long)r * a.ld + c4;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (c4 + q <= r) dst[q] = lv[q];
        *reinterpret_cast<f32x4*>(Dk + r * TB + c4) = *reinterpret_cast<const f32x4*>(Ds + r * DLD + c4);
    }
    if (a.LT) {   // refinement: D_k^T as tile (k, k) of L^T
        float* lt = a.LT + row_off(a, k) + (long)k * TB;
        for (int e = threadIdx.x; e < TB * TB; e += DIAG_THREADS) {
            const int r = e / TB, c = e % TB;   // lt row r = column r of D_k
            lt[(long)r * a.ld + c] = Ds[c * DLD + r];
        }
    }
    if (threadIdx.x == 0 && *bad && k * TB + *bad - 1 < a.n && *a.info == 0) *a.info = k * TB + *bad;
}

// ---------------------------------------------------------------- K2b: panel  M(r,k) <- M(r,k) D_k^T
// row tiles: A rows k+1 .. T-1, then the live bottom rows (Y^T, K(X*,X), identity rows <= k)
__global__ __launch_bounds__(GT, 2) void k32_panel(F32Args a, int k) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.x;
    const int nA = a.T - k - 1;
    const int rt = (b < nA) ? k + 1 + b : a.T + (b - nA);
    float* Mr = a.M + row_off(a, rt) + (long)k * TB;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, Mr, a.ld, a.Dd + (long)k * TB * TB, TB, TB / BK, smem);
    acc_store(acc, Mr, a.ld);
    if (a.LT && rt < a.T) {   // refinement: L(rt,k)^T as tile (k, rt) of L^T
        float* lt = a.LT + row_off(a, k) + (long)rt * TB;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int r = 0; r < 16; ++r) lt[(long)acc_col(n) * a.ld + acc_row(m, r)] = acc.c[m][n][r];
    }
}

// ---------------------------------------------------------------- K2c: update
// M(r, j) -= sum_{k in [k0,k1)} L(r,k) L(j,k)^T for columns j in [jb, je): A rows r >= j, then
// every live bottom row.  Inside a panel (k1 = k0 + 1) and the trailing update (K = W*128).
__host__ __device__ inline long update_tiles(const F32Args& a, int k1, int jb, int je) {
    long s = 0;
    for (int j = jb; j < je; ++j) s += a.T - j;
    return s + (long)rows_B(a, k1) * (je - jb);
}

// ntile > gridDim.x: a capped (persistent) grid, each workgroup walks tiles blockIdx.x + i * gridDim.x
// (the lookahead leaves CUs free for the next panel's factorization on the side stream).
__global__ __launch_bounds__(GT, 2) void k32_update(F32Args a, int k0, int k1, int jb, int je, int ntile) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int nB = rows_B(a, k1);
    const long koff = (long)k0 * TB;
    for (long t = blockIdx.x; t < ntile; t += gridDim.x) {
        long b = t;
        int rt = -1, jt = jb;
        for (int j = jb; j < je; ++j) {
            const int cnt = a.T - j;
            if (b < cnt) { rt = j + (int)b; jt = j; break; }
            b -= cnt;
        }
        if (rt < 0) {
            rt = a.T + (int)(b % nB);
            jt = jb + (int)(b / nB);
        }
        Acc acc;
        acc_zero(acc);
        gemm_nt(acc, a.M + row_off(a, rt) + koff, a.ld, a.M + row_off(a, jt) + koff, a.ld, (k1 - k0) * (TB / BK),
                smem);
        acc_sub_into(acc, a.M + row_off(a, rt) + (long)jt * TB, a.ld);
    }
}

// ---------------------------------------------------------------- K3: alpha = K^-1 Y = L^-T Z
// alpha[a][p] = sum_{i >= a} L^-T[a][i] Z^T[p][i]   (tile (at, pt), contraction from tile at)
__global__ __launch_bounds__(GT, 2) void k32_alpha(F32Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int at = blockIdx.x / a.Tp, pt = blockIdx.x % a.Tp;
    const long koff = (long)at * TB;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, a.M + row_off(a, id0(a) + at) + koff, a.ld, a.M + row_off(a, a.T + pt) + koff, a.ld,
            (a.T - at) * (TB / BK), smem);
    acc_store(acc, a.alpha + (long)at * TB * a.ldal + (long)pt * TB, a.ldal);
}

// ---------------------------------------------------------------- K5: gradient
// Lower tile (I, J): W = alpha_I alpha_J^T - P sum_{l >= I} L^-T(I,l) L^-T(J,l)^T, contracted
// with dK/dtheta recomputed from X (the fp64 k_grad epilogue in fp32; per-tile sums in fp64).
// gpart[q][task] = 1/2 sum W dK/dtheta_q over the tile (x2 for the mirrored upper tile).
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int DT>   // compile-time bound on D (DT >= D): per-dimension sums stay in registers
__global__ __launch_bounds__(GT, 2) void k32_grad(F32Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int task = blockIdx.x;
    int I, J;
    tri_decode32(task, I, J);
    {
        Acc acc;
        acc_zero(acc);
        const long koff = (long)I * TB;
        gemm_nt(acc, a.M + row_off(a, id0(a) + I) + koff, a.ld, a.M + row_off(a, id0(a) + J) + koff, a.ld,
                (a.T - I) * (TB / BK), smem);
        const float negP = -(float)a.p;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc.c[m][n][r] *= negP;
        gemm_nt(acc, a.alpha + (long)I * TB * a.ldal, a.ldal, a.alpha + (long)J * TB * a.ldal, a.ldal,
                a.Tp * (TB / BK), smem);
        // W tile (x 1/2 on the diagonal tile; x 1 off it: the mirrored upper tile) into LDS
        const float wscale = (I == J) ? 0.5f : 1.0f;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int r = 0; r < 16; ++r) smem[acc_row(m, r) * (TB + 1) + acc_col(n)] = acc.c[m][n][r] * wscale;
    }
    // raw inputs of the two row tiles [d][row], flags, inverse squared lengthscales, reduction slots
    const int D = a.D;
    float* xi = smem + TB * (TB + 1);
    float* xj = xi + D * TB;
    float* fi = xj + D * TB;
    float* fj = fi + TB;
    float* il2 = fj + TB;   // [2][D]
    double* red = reinterpret_cast<double*>(il2 + 2 * MAXD_HOST);   // [G][4]
    for (int e = threadIdx.x; e < TB * D; e += GT) {
        const int r = e % TB, d = e / TB;
        const int gi = I * TB + r, gj = J * TB + r;
        xi[d * TB + r] = gi < a.n ? a.X[(long)gi * a.ldx + d] : 0.0f;
        xj[d * TB + r] = gj < a.n ? a.X[(long)gj * a.ldx + d] : 0.0f;
    }
    for (int r = threadIdx.x; r < TB; r += GT) {
        const int gi = I * TB + r, gj = J * TB + r;
        fi[r] = gi < a.n ? fid_code(a.X[(long)gi * a.ldx + D]) : -1.0f;
        fj[r] = gj < a.n ? fid_code(a.X[(long)gj * a.ldx + D]) : -1.0f;
    }
    if (threadIdx.x < 2 * D) {
        const int src = threadIdx.x / D, d = threadIdx.x % D;
        const double l = a.theta[src == 0 ? 1 + d : 2 + D + d];
        il2[threadIdx.x] = (float)(1.0 / (l * l));
    }
    __syncthreads();
    const float vL = (float)a.theta[0], vD = (float)a.theta[1 + D], rho = (float)a.theta[2 + 2 * D];
    // thread: column c = t & 127, rows (t >> 7) + 2 i (a wave shares its row: broadcast reads)
    const int c = threadIdx.x & (TB - 1);
    float xc[DT], il[DT], ild[DT], tl[DT], td[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) {
        const bool on = d < D;
        xc[d] = on ? xj[d * TB + c] : 0.0f;
        il[d] = on ? il2[d] : 0.0f;
        ild[d] = on ? il2[D + d] : 0.0f;
        tl[d] = 0.0f;
        td[d] = 0.0f;
    }
    const float f2 = fj[c];
    const bool L2 = f2 == 0.0f, H2 = f2 == 1.0f;
    const float sj = L2 ? 1.0f : (H2 ? rho : 0.0f), hj = H2 ? 1.0f : 0.0f;
    float gvL = 0.0f, gvD = 0.0f, grho = 0.0f, gno = 0.0f;
    for (int r = threadIdx.x >> 7; r < TB; r += 2) {
        const float f1 = fi[r];
        const bool L1 = f1 == 0.0f, H1 = f1 == 1.0f;
        const float w = smem[r * (TB + 1) + c];
        if (!((L1 || H1) && (L2 || H2))) continue;
        float df2[DT];
        float s2 = 0.0f, s2d = 0.0f;
#pragma unroll
        for (int d = 0; d < DT; ++d) {
            const float df = (d < D ? xi[d * TB + r] : 0.0f) - xc[d];
            df2[d] = df * df;
            s2 = fmaf(df2[d], il[d], s2);
            s2d = fmaf(df2[d], ild[d], s2d);
        }
        const float eL = __expf(-0.5f * s2);   // dk/dv in TF's autodiff form (finite at v = 0)
        const float eD = (H1 && H2) ? __expf(-0.5f * s2d) : 0.0f;
        const float kL = vL * eL, kD = vD * eD;
        const float si = L1 ? 1.0f : rho, hi = H1 ? 1.0f : 0.0f;
        const float cL = w * si * sj * kL, cD = w * hi * hj * kD;
        gvL += w * si * sj * eL;
        gvD += w * hi * hj * eD;
        grho += w * (hi * sj + si * hj) * kL;
        if (I == J && r == c && I * TB + r < a.n) gno += w;
#pragma unroll
        for (int d = 0; d < DT; ++d) {
            tl[d] = fmaf(cL, df2[d], tl[d]);
            td[d] = fmaf(cD, df2[d], td[d]);
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int G = theta_size(D);
    auto put = [&](int q, float v) {
        const double s = wave_sum_d((double)v);
        if (lane == 0) red[q * 4 + wv] = s;
    };
    put(0, gvL);
    put(1 + D, gvD);
    put(2 + 2 * D, grho);
    put(3 + 2 * D, gno);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
        if (d < D) {
            put(1 + d, tl[d]);
            put(2 + D + d, td[d]);
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < G; q += GT) {
        double v = (red[q * 4] + red[q * 4 + 1]) + (red[q * 4 + 2] + red[q * 4 + 3]);
        if ((q >= 1 && q <= D) || (q >= 2 + D && q <= 1 + 2 * D)) { const double l = a.theta[q]; v /= l * l * l; }
        a.gpart[(long)q * gridDim.x + task] = v;
    }
}

size_t grad_smem_bytes32(int D) {
    const size_t epi = sizeof(float) * ((size_t)TB * (TB + 1) + 2 * (size_t)D * TB + 2 * TB + 2 * MAXD_HOST) +
                       sizeof(double) * 4 * (size_t)theta_size(D);
    return GEMM_SMEM > epi ? GEMM_SMEM : epi;
}

// ---------------------------------------------------------------- K4 input: sum Z^2 partials
__global__ __launch_bounds__(GT) void k32_zsum(F32Args a) {
    __shared__ double red[4];
    const f32x4* Z = reinterpret_cast<const f32x4*>(a.M + row_off(a, a.T));
    const long total = (long)a.Tp * TB * a.ld / 4;
    double s = 0.0;
    for (long e = blockIdx.x * (long)GT + threadIdx.x; e < total; e += (long)gridDim.x * GT) {
        const f32x4 v = Z[e];
        s += (double)(v[0] * v[0]) + (double)(v[1] * v[1]) + (double)(v[2] * v[2]) + (double)(v[3] * v[3]);
    }
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) a.zpart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---------------------------------------------------------------- K6: predict
// mean[s][p] = sum_i (L^-1 Kmn)^T[s][i] Z^T[p][i]
__global__ __launch_bounds__(GT, 2) void k32_pred_mean(F32Args a, float* mean, long ldm) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int st = blockIdx.x / a.Tp, pt = blockIdx.x % a.Tp;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, a.M + row_off(a, a.T + a.Tp + st), a.ld, a.M + row_off(a, a.T + pt), a.ld, a.T * (TB / BK), smem);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gs = st * TB + acc_row(m, r), gp = pt * TB + acc_col(n);
                if (gs < a.ns && gp < a.p) mean[(long)gs * ldm + gp] = acc.c[m][n][r];
            }
}

// full_cov: cov[s][s'] -= sum_i A[i][s] A[i][s'] on top of K(X*, X*) already in cov (GPflow
// base_conditional(full_cov=True): Knn - A^T A); both operands are rows of the A^T region of M
__global__ __launch_bounds__(GT, 2) void k32_pred_cov(F32Args a, float* cov, long ldc) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int st = blockIdx.x / a.Ts, st2 = blockIdx.x % a.Ts;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, a.M + row_off(a, a.T + a.Tp + st), a.ld, a.M + row_off(a, a.T + a.Tp + st2), a.ld,
            a.T * (TB / BK), smem);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gs = st * TB + acc_row(m, r), gs2 = st2 * TB + acc_col(n);
                if (gs < a.ns && gs2 < a.ns) cov[(long)gs * ldc + gs2] -= acc.c[m][n][r];
            }
}

// var[s] = K_diag(x*_s) - sum_i A[i][s]^2 (linear.py:106-136 for K_diag); one wave per row
__global__ __launch_bounds__(GT) void k32_pred_var(F32Args a, float* var) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (s >= a.ns) return;
    const f32x4* row = reinterpret_cast<const f32x4*>(a.M + row_off(a, a.T + a.Tp) + (long)s * a.ld);
    double acc = 0.0;
    for (long e = lane; e < a.ld / 4; e += 64) {
        const f32x4 v = row[e];
        acc += (double)(v[0] * v[0] + v[1] * v[1]) + (double)(v[2] * v[2] + v[3] * v[3]);
    }
    acc = wave_sum_d(acc);
    if (lane == 0) {
        const float f = a.Xs[(long)s * a.ldxs + a.D];
        const double vL = a.theta[0], vD = a.theta[1 + a.D], rho = a.theta[2 + 2 * a.D];
        const double kd = f == 0.0f ? vL : (f == 1.0f ? rho * rho * vL + vD : 0.0);
        var[s] = (float)(kd - acc);
    }
}

// ---------------------------------------------------------------- dense gram (mfgp_mf_gram_ex f32)
__global__ __launch_bounds__(GT) void k32_gram_dense(const float* X1, long ldx1, int n1, const float* X2, long ldx2,
                                                     int n2, int D, const double* theta, float diag_add, float* K,
                                                     long ldk, int tc) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int ti = blockIdx.x / tc, tj = blockIdx.x % tc;
    const GramSmem g = gram_smem(smem, D);
    gram_stage(g, X1, ldx1, n1, ti * TB, X2, ldx2, n2, tj * TB, D, theta);
    __syncthreads();
    float v[8][8];
    gram_tile_vals(g, D, theta, v);
    const int t = threadIdx.x, rb = t >> 4, cb = (t & 15) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int gi = ti * TB + rb + 16 * i, gj = tj * TB + cb + (j & 3) + 64 * (j >> 2);
            if (gi < n1 && gj < n2) K[(long)gi * ldk + gj] = v[i][j] + (gi == gj ? diag_add : 0.0f);
        }
}

// ---------------------------------------------------------------- fp64 refinement of the solve
// One step of iterative refinement with the residual in fp64 (value-only LML, predict mean):
//   alpha0 = L~^-T L~^-1 Y (fp32 factor), R = Y - K alpha0 (fp64, K recomputed in fp64),
//   W = L~^-1 R;  LML quad term q = Y.alpha0 + alpha0.R + |W|^2  (exact identity
//   Y^T K^-1 Y = Y^T a0 + a0^T R + R^T K^-1 R, with K^-1 ~ K~^-1 only in the second-order term);
//   predict: alpha1 = alpha0 + L~^-T W, mean = K(X*, X) alpha1 (fp64).
// The triangular solves run on rows [P x Npad] (right solves X L^T = B and X L = B) with the NT
// GEMM core: the forward solve reads L's rows, the backward one the rows of L^T (stored by the
// sweep's panel / diagonal kernels when a.LT is set).

// B(pt, k) <- B(pt, k) Dop^T (in place; Dop row-major, ld ldd)
__global__ __launch_bounds__(GT, 2) void k32_sdiag(float* B, long ldb, int k, const float* Dop, long ldd) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Bt = B + (long)blockIdx.x * TB * ldb + (long)k * TB;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, Bt, ldb, Dop, ldd, TB / BK, smem);
    acc_store(acc, Bt, ldb);
}

// B(pt, j) -= sum_{kk in [k0, k1)} B(pt, kk) Lr(j, kk)^T for j in [jb, je) (tile t: pt = t % np)
__global__ __launch_bounds__(GT, 2) void k32_supd(float* B, long ldb, int np, int k0, int k1, int jb,
                                                  const float* Lr, long ldl) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int pt = blockIdx.x % np, j = jb + blockIdx.x / np;
    float* Brow = B + (long)pt * TB * ldb;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, Brow + (long)k0 * TB, ldb, Lr + (long)j * TB * ldl + (long)k0 * TB, ldl, (k1 - k0) * (TB / BK), smem);
    acc_sub_into(acc, Brow + (long)j * TB, ldb);
}

// One column step of a right-looking solve (one launch per tile column): for j in [jb, jb + nj),
// B(pt, j) -= B(pt, k) Lr(j, k)^T; the tile of column jf (the next diagonal) is then finalised in
// the same workgroup, B(pt, jf) <- B(pt, jf) Dop^T (its only writer: the update went through
// global memory, read back by the same workgroup after a barrier).
__global__ __launch_bounds__(GT, 2) void k32_sstep(float* B, long ldb, int np, int k, int jb, const float* Lr,
                                                   long ldl, int jf, const float* Dop, long ldd) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int pt = blockIdx.x % np, j = jb + blockIdx.x / np;
    float* Brow = B + (long)pt * TB * ldb;
    Acc acc;
    acc_zero(acc);
    gemm_nt(acc, Brow + (long)k * TB, ldb, Lr + (long)j * TB * ldl + (long)k * TB, ldl, TB / BK, smem);
    acc_sub_into(acc, Brow + (long)j * TB, ldb);
    if (j != jf) return;
    __threadfence_block();
    __syncthreads();
    acc_zero(acc);
    gemm_nt(acc, Brow + (long)j * TB, ldb, Dop, ldd, TB / BK, smem);
    acc_store(acc, Brow + (long)j * TB, ldb);
}

// out[i][q] = (Y ? Y[i][q] - (K C)[i][q] : (K C)[i][q]), fp64.  K entries recomputed in fp64 from
// the fp32 inputs, in GPflow's expanded form with the exact fidelity masks (the fp64 path's
// gram_entry, mfgp_kernels.hip; linear.py:55-104), plus s2 on i == j when add_noise
// (K(X, X) + s2 I).  64 rows x 256 columns a workgroup (K recomputed once per 256 columns of C),
// 16 columns of K a step: the K tile (64 x 16) and the C slab (16 x 256) through LDS, the next
// step's inputs prefetched into registers during this step's products; v_mfma_f64_16x16x4,
// a wave 16 rows x 256 columns (16 accumulators).  C must have >= ceil16(n2) readable rows and
// tq * 256 readable columns (the refinement's fp64 buffers: Npad x Ppad, zero padded).
struct KmatArgs {
    const float* X1; long ldx1; int n1;
    const float* X2; long ldx2; int n2;
    int D; const double* theta; int add_noise;
    const double* C; long ldc;
    const float* Y; long ldy;
    double* out; long ldo; float* out32; long ldo32; int p;
    int tq;   // column blocks of 256
};
constexpr int KM_R = 64, KM_Q = 256, KM_J = 16, KM_XS = MAXD_HOST + 1, KM_CS = KM_Q + 2;
constexpr size_t KMAT_SMEM = sizeof(double) * (KM_R * KM_XS + KM_R + 2 * KM_J * KM_XS + 3 * KM_J +
                                               KM_R * (KM_J + 1) + KM_J * KM_CS + 2 * MAXD_HOST);

template <int D4>
__global__ __launch_bounds__(256, 2) void k64_kmat(KmatArgs a) {
    extern __shared__ __attribute__((aligned(16))) double sm64[];
    double* rD = sm64;                       // [64][XS] row side, HF-scaled (K_HH pairs)
    double* rnd = rD + KM_R * KM_XS;         // [64] |rD|^2
    double* cL = rnd + KM_R;                 // [16][D4] column side, LF-scaled (zero padded)
    double* cD = cL + KM_J * KM_XS;          // [16][XS] column side, HF-scaled
    double* cn = cD + KM_J * KM_XS;
    double* cnd = cn + KM_J;
    double* cf = cnd + KM_J;
    double* Ks = cf + KM_J;                  // [64][17]
    double* Cs = Ks + KM_R * (KM_J + 1);     // [16][KM_CS]
    double* il = Cs + KM_J * KM_CS;          // [2][MAXD]
    const int t = threadIdx.x, D = a.D;
    const int i0 = (blockIdx.x / a.tq) * KM_R, q0 = (blockIdx.x % a.tq) * KM_Q;
    const double vL = a.theta[0], vD = a.theta[1 + D], rho = a.theta[2 + 2 * D];
    const double s2 = a.add_noise ? a.theta[3 + 2 * D] : 0.0;
    if (t < D) {
        il[t] = 1.0 / a.theta[1 + t];
        il[MAXD_HOST + t] = 1.0 / a.theta[2 + D + t];
    }
    __syncthreads();
    // row side in registers: thread t's row r = t / 4 for the whole launch (the LF-scaled row, its
    // norm and flag; the HF-scaled row in LDS for the rare K_HH pairs)
    const int r = t >> 2, gi = i0 + r;
    const bool rin = gi < a.n1;
    double ra[D4], rn, rf;
    {
        float xr[D4 + 1];
        const int gc = min(gi, a.n1 - 1);
#pragma unroll
        for (int d = 0; d < D4 + 1; ++d) xr[d] = a.X1[(long)gc * a.ldx1 + min(d, D)];   // unconditional
        double sl = 0.0, sd = 0.0;
#pragma unroll
        for (int d = 0; d < D4; ++d) {
            const double x = (rin && d < D) ? (double)xr[d] : 0.0;
            ra[d] = d < D ? x * il[d] : 0.0;
            sl += ra[d] * ra[d];
            if ((t & 3) == 0 && d < D) {
                const double h = x * il[MAXD_HOST + d];
                rD[r * KM_XS + d] = h;
                sd += h * h;
            }
        }
        rn = sl;
        rf = rin ? (double)xr[D] : -1.0;   // xr[D]: the flag column (min(d, D) at d = D)
        if ((t & 3) == 0) rnd[r] = sd;
        if (D4 == D) rf = rin ? (double)a.X1[(long)gc * a.ldx1 + D] : -1.0;
    }
    // column-side prefetch: thread t < 16 loads row j0 + t of X2; every thread 16 C values
    float xc[D4 + 1];
    double cv[KM_J];
    auto prefetch = [&](int j0) {
        if (t < KM_J) {
            const int gj = min(j0 + t, a.n2 - 1);
#pragma unroll
            for (int d = 0; d < D4 + 1; ++d) xc[d] = a.X2[(long)gj * a.ldx2 + min(d, D)];
        }
#pragma unroll
        for (int u = 0; u < KM_J; ++u) cv[u] = a.C[(long)(j0 + u) * a.ldc + q0 + t];
    };
    const int lane = t & 63, w = t >> 6, li = lane & 15, lk = lane >> 4;
    f64x4 acc[KM_Q / 16];
#pragma unroll
    for (int b = 0; b < KM_Q / 16; ++b) acc[b] = f64x4{0.0, 0.0, 0.0, 0.0};
    prefetch(0);
    for (int j0 = 0; j0 < a.n2; j0 += KM_J) {
        // commit the prefetched step
        if (t < KM_J) {
            const bool in = j0 + t < a.n2;
            double sl = 0.0, sd = 0.0;
#pragma unroll
            for (int d = 0; d < D4; ++d) {
                const double x = (in && d < D) ? (double)xc[d] : 0.0;
                const double l = x * (d < D ? il[d] : 0.0), h = x * (d < D ? il[MAXD_HOST + d] : 0.0);
                cL[t * D4 + d] = l;
                cD[t * KM_XS + d] = h;
                sl += l * l;
                sd += h * h;
            }
            cn[t] = sl;
            cnd[t] = sd;
            cf[t] = in ? (double)(D4 == D ? a.X2[(long)min(j0 + t, a.n2 - 1) * a.ldx2 + D] : xc[D]) : -1.0;
        }
#pragma unroll
        for (int u = 0; u < KM_J; ++u) Cs[u * KM_CS + t] = cv[u];
        __syncthreads();
        if (j0 + KM_J < a.n2) prefetch(j0 + KM_J);
        // 4 entries a thread: row r, columns 4 (t % 4) + u, side by side (dot4 order per entry)
        double kl[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int d = 0; d < D4; ++d) {
#pragma unroll
            for (int u = 0; u < 4; ++u) kl[u] += ra[d] * cL[(4 * (t & 3) + u) * D4 + d];
            MFGP_PIN4(kl);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) kl[u] = -0.5 * (-2.0 * kl[u] + (rn + cn[4 * (t & 3) + u]));
        exp4(kl);
        MFGP_PIN4(kl);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = 4 * (t & 3) + u, gj = j0 + c;
            const double f2 = cf[c];
            double v = 0.0;
            if (rin && gj < a.n2) {
                const double kL = vL * kl[u];
                const bool L1 = rf == 0.0, H1 = rf == 1.0, L2 = f2 == 0.0, H2 = f2 == 1.0;
                if (!(L1 || H1) || !(L2 || H2)) v = 0.0;   // linear.py:67-70 exact masks
                else if (L1 && L2) v = kL;
                else if (!(H1 && H2)) v = kL * rho;
                else {   // K_HH (linear.py:96)
                    double dd = 0.0;
                    for (int d = 0; d < D; ++d) dd += rD[r * KM_XS + d] * cD[c * KM_XS + d];
                    v = kL * (rho * rho) + vD * exp(-0.5 * (-2.0 * dd + (rnd[r] + cnd[c])));
                }
                if (gi == gj) v += s2;
            }
            Ks[r * (KM_J + 1) + c] = v;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KM_J / 4; ++ks) {
            const double av = Ks[(16 * w + li) * (KM_J + 1) + 4 * ks + lk];
#pragma unroll
            for (int b = 0; b < KM_Q / 16; ++b) {
                const double bv = Cs[(4 * ks + lk) * KM_CS + 16 * b + li];
                acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[b], 0, 0, 0);
            }
        }
        __syncthreads();   // K / C slabs consumed before the next commit
    }
#pragma unroll
    for (int b = 0; b < KM_Q / 16; ++b)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int gi2 = i0 + 16 * w + lk + 4 * rr, gq = q0 + 16 * b + li;
            if (gi2 >= a.n1 || gq >= a.p) continue;
            const double v = a.Y ? (double)a.Y[(long)gi2 * a.ldy + gq] - acc[b][rr] : acc[b][rr];
            if (a.out) a.out[(long)gi2 * a.ldo + gq] = v;
            if (a.out32) a.out32[(long)gi2 * a.ldo32 + gq] = (float)v;
        }
}

// fp32 rows [P][N] (ld ldr) <-> fp64 [N][P] (ld ld64); zero outside n x p.  mode 0: to64 (out = rows^T),
// 1: to32 (rows = in^T), 2: add (out += rows^T).  32 x 32 tiles through LDS.
__global__ __launch_bounds__(256) void k_tr3264(float* rows, long ldr, double* m64, long ld64, int n, int p,
                                               int npad, int ppad, int mode) {
    __shared__ double tl[32][33];
    const int tn = npad / 32;
    const int bi = blockIdx.x % tn, bq = blockIdx.x / tn;   // tile: i in 32 bi.., q in 32 bq..
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int yy = ty; yy < 32; yy += 8) {
        const int i = 32 * bi + yy, q = 32 * bq + tx;   // read m64 coalesced along q, rows along i
        if (mode == 1) tl[yy][tx] = (i < n && q < p) ? m64[(long)i * ld64 + q] : 0.0;
        else tl[yy][tx] = (double)rows[(long)(32 * bq + yy) * ldr + 32 * bi + tx];   // rows: q row, i col
    }
    __syncthreads();
    for (int yy = ty; yy < 32; yy += 8) {
        if (mode == 1) {
            const int q = 32 * bq + yy, i = 32 * bi + tx;
            rows[(long)q * ldr + i] = (float)tl[tx][yy];
        } else {
            const int i = 32 * bi + yy, q = 32 * bq + tx;
            const double v = (i < n && q < p) ? tl[tx][yy] : 0.0;
            if (mode == 0) m64[(long)i * ld64 + q] = v;
            else if (i < n && q < p) m64[(long)i * ld64 + q] += v;
        }
    }
}

// q partials: sum_{i<n, q<p} (Y a0 + a0 R)[i][q] + sum W^2 over the fp32 rows (P x Npad)
__global__ __launch_bounds__(256) void k_refine_q(const float* Y, long ldy, const double* A64, const double* R64,
                                                 long ld64, const float* Wr, long ldw, int n, int p, double* part) {
    __shared__ double red[4];
    double s = 0.0;
    const long tot = (long)n * p;
    for (long e = blockIdx.x * 256L + threadIdx.x; e < tot; e += (long)gridDim.x * 256) {
        const int i = (int)(e / p), q = (int)(e % p);
        const double a = A64[(long)i * ld64 + q];
        s += ((double)Y[(long)i * ldy + q] + R64[(long)i * ld64 + q]) * a;
        const double wv = (double)Wr[(long)q * ldw + i];
        s += wv * wv;
    }
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace f32

// ---------------------------------------------------------------- host launchers
using namespace f32;

size_t f32_gemm_smem() { return GEMM_SMEM; }

int f32_ident_fill_tiles(const F32Args& a) { return (int)ident_tiles(a); }

// The whole sweep: gram (+ RHS rows, identity), then per panel of W tile columns: factor,
// panel, in-panel updates; then the trailing update.  want_grad: alpha and gradient partials;
// always: sum Z^2 partials (a.nz workgroups).
// Dynamic LDS above 64 KB must be allowed per kernel (once per process; not a stream operation,
// so it is safe before or during graph capture).
static void f32_lds_attributes() {
    static bool done = false;
    if (done) return;
    done = true;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k32_diag), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)DIAG_SMEM);
    const void* gemms[] = {reinterpret_cast<const void*>(&k32_panel), reinterpret_cast<const void*>(&k32_update),
                           reinterpret_cast<const void*>(&k32_alpha), reinterpret_cast<const void*>(&k32_pred_mean),
                           reinterpret_cast<const void*>(&k32_pred_cov),
                           reinterpret_cast<const void*>(&k32_grad<4>), reinterpret_cast<const void*>(&k32_grad<8>),
                           reinterpret_cast<const void*>(&k32_grad<12>), reinterpret_cast<const void*>(&k32_grad<16>),
                           reinterpret_cast<const void*>(&k32_grad<32>)};
    for (const void* f : gemms)
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static void f32_gram(const F32Args& a, hipStream_t s, F32Marks* mk) {
    f32_lds_attributes();
    const long nA = (long)a.T * (a.T + 1) / 2;
    const long ngram = nA + (long)a.Tp * a.T + (long)a.Ts * a.T + ident_tiles(a);
    const size_t glds = gram_smem_bytes32(a.D) > (size_t)TB * (TB + 1) * 4 ? gram_smem_bytes32(a.D)
                                                                           : (size_t)TB * (TB + 1) * 4;
    if (mk) mk->begin(s, F32_GRAM);
    hipLaunchKernelGGL(k32_gram, dim3((unsigned)ngram), dim3(GT), glds, s, a);
    if (mk) mk->end(s, 0.0);
}

constexpr double TILE_FL = 2.0 * TB * TB;   // flops of one 128 x 128 output tile per unit of K

// F(panel): per tile column k of [k0, k1): diagonal factor, panel, update of the panel's
// remaining columns
static void f32_panel_factor(const F32Args& a, int k0, int k1, hipStream_t s, F32Marks* mk) {
    for (int k = k0; k < k1; ++k) {
        if (mk) mk->begin(s, F32_DIAG);
        hipLaunchKernelGGL(k32_diag, dim3(1), dim3(DIAG_THREADS), DIAG_SMEM, s, a, k);
        if (mk) mk->end(s, (double)TB * TB * TB * 2.0 / 3.0);
        const int np = (a.T - k - 1) + rows_B(a, k + 1);
        if (np > 0) {
            if (mk) mk->begin(s, F32_PANEL);
            hipLaunchKernelGGL(k32_panel, dim3(np), dim3(GT), GEMM_SMEM, s, a, k);
            if (mk) mk->end(s, TILE_FL * TB * np);
        }
        if (k + 1 < k1) {
            const long nt = update_tiles(a, k + 1, k + 1, k1);
            if (mk) mk->begin(s, F32_UPD_IN);
            hipLaunchKernelGGL(k32_update, dim3((unsigned)nt), dim3(GT), GEMM_SMEM, s, a, k, k + 1, k + 1, k1, (int)nt);
            // useful work: every tile but the strictly upper half of the diagonal tiles
            if (mk) mk->end(s, TILE_FL * TB * (nt - 0.5 * (k1 - k - 1) * (TB - 1) / TB));
        }
    }
}

// U(panel, [jb, je)): columns jb .. je-1 updated with the panel's K = (k1 - k0) * 128
static void f32_trailing(const F32Args& a, int k0, int k1, int jb, int je, hipStream_t s, F32Marks* mk,
                         int slots = 0) {
    if (jb >= je) return;
    const long nt = update_tiles(a, k1, jb, je);
    const long grid = (slots > 0 && nt > slots) ? slots : nt;
    if (mk) mk->begin(s, F32_UPD_OUT);
    hipLaunchKernelGGL(k32_update, dim3((unsigned)grid), dim3(GT), GEMM_SMEM, s, a, k0, k1, jb, je, (int)nt);
    if (mk) mk->end(s, TILE_FL * TB * (k1 - k0) * (nt - 0.5 * (je - jb) * (TB - 1) / TB));
}

// The sweep.  With a side stream (and no timing marks): one-panel lookahead -- the next panel's
// columns are updated first, then the rest of the trailing update (main stream) runs beside the
// next panel's factorization (side stream, high priority), which is the critical path; both
// read panel K's columns only and write disjoint column ranges.  Fork / join through events,
// so the sequence stays hipGraph-capturable.
void launch_f32_sweep(const F32Args& a, hipStream_t s, F32Marks* mk, hipStream_t side, hipEvent_t fork,
                      hipEvent_t join) {
    f32_gram(a, s, mk);
    const bool ahead = side && fork && join && !mk;
    const int W = a.W;
    auto pend = [&](int k0) { return (k0 + W < a.T) ? k0 + W : a.T; };
    f32_panel_factor(a, 0, pend(0), s, mk);
    for (int k0 = 0; k0 < a.T; k0 += W) {
        const int k1 = pend(k0);
        if (k1 >= a.T) break;
        const int k2 = pend(k1);
        if (!ahead) {
            f32_trailing(a, k0, k1, k1, a.T, s, mk);
            f32_panel_factor(a, k1, k2, s, mk);
            continue;
        }
        f32_trailing(a, k0, k1, k1, k2, s, mk);
        if (k2 < a.T) {
            (void)hipEventRecord(fork, s);
            (void)hipStreamWaitEvent(side, fork, 0);
            f32_trailing(a, k0, k1, k2, a.T, s, mk, a.upd_slots);
            f32_panel_factor(a, k1, k2, side, mk);
            (void)hipEventRecord(join, side);
            (void)hipStreamWaitEvent(s, join, 0);
        } else {
            f32_panel_factor(a, k1, k2, s, mk);
        }
    }
}

void launch_f32_grad(const F32Args& a, hipStream_t s, F32Marks* mk) {
    const double tile_fl = TILE_FL;
    if (mk) mk->begin(s, F32_ALPHA);
    hipLaunchKernelGGL(k32_alpha, dim3(a.T * a.Tp), dim3(GT), GEMM_SMEM, s, a);
    if (mk) mk->end(s, tile_fl * TB * a.Tp * (double)a.T * (a.T + 1) / 2);
    const dim3 g(a.T * (a.T + 1) / 2);
    const size_t lds = grad_smem_bytes32(a.D);
    if (mk) mk->begin(s, F32_GRAD);
    if (a.D <= 4) hipLaunchKernelGGL(k32_grad<4>, g, dim3(GT), lds, s, a);
    else if (a.D <= 8) hipLaunchKernelGGL(k32_grad<8>, g, dim3(GT), lds, s, a);
    else if (a.D <= 12) hipLaunchKernelGGL(k32_grad<12>, g, dim3(GT), lds, s, a);
    else if (a.D <= 16) hipLaunchKernelGGL(k32_grad<16>, g, dim3(GT), lds, s, a);
    else hipLaunchKernelGGL(k32_grad<32>, g, dim3(GT), lds, s, a);
    if (mk) {   // sum over lower tiles (I, J) of K = (T - I) tiles + Ppad
        double kt = 0.0;
        for (int I = 0; I < a.T; ++I) kt += (double)(I + 1) * ((a.T - I) * TB + a.Tp * TB);
        mk->end(s, tile_fl * kt);
    }
}

void launch_f32_zsum(const F32Args& a, hipStream_t s) {
    hipLaunchKernelGGL(k32_zsum, dim3(a.nz), dim3(GT), 0, s, a);
}

void launch_f32_predict(const F32Args& a, float* mean, long ldm, float* var, hipStream_t s) {
    hipLaunchKernelGGL(k32_pred_mean, dim3(a.Ts * a.Tp), dim3(GT), GEMM_SMEM, s, a, mean, ldm);
    hipLaunchKernelGGL(k32_pred_var, dim3((a.ns + 3) / 4), dim3(GT), 0, s, a, var);
}

void launch_f32_predict_cov(const F32Args& a, float* cov, long ldc, hipStream_t s) {
    launch_f32_gram_dense(a.Xs, a.ldxs, a.ns, a.Xs, a.ldxs, a.ns, a.D, a.theta, 0.0f, cov, ldc, s);
    hipLaunchKernelGGL(k32_pred_cov, dim3(a.Ts * a.Ts), dim3(GT), GEMM_SMEM, s, a, cov, ldc);
}

// ---- refinement (see k32_sdiag .. k_refine_q)
// rows B [np x 128 tiles][Npad]: X L~^T = B  (forward: X = B L~^-T, i.e. (L~^-1 B^T)^T); one launch
// per tile column (k32_sstep), K = 128 each
static void f32_fsolve(const F32Args& a, float* B, long ldb, int np, hipStream_t s) {
    hipLaunchKernelGGL(k32_sdiag, dim3(np), dim3(GT), GEMM_SMEM, s, B, ldb, 0, (const float*)a.Dd, (long)TB);
    for (int k = 0; k + 1 < a.T; ++k)
        hipLaunchKernelGGL(k32_sstep, dim3(np * (a.T - k - 1)), dim3(GT), GEMM_SMEM, s, B, ldb, np, k, k + 1,
                           (const float*)a.M, a.ld, k + 1, (const float*)(a.Dd + (long)(k + 1) * TB * TB), (long)TB);
}
// X L~ = B  (backward: X = B L~^-1, i.e. (L~^-T B^T)^T), with the L^T tiles
static void f32_bsolve(const F32Args& a, float* B, long ldb, int np, hipStream_t s) {
    auto dT = [&](int k) { return (const float*)(a.LT + row_off(a, k) + (long)k * TB); };
    hipLaunchKernelGGL(k32_sdiag, dim3(np), dim3(GT), GEMM_SMEM, s, B, ldb, a.T - 1, dT(a.T - 1), a.ld);
    for (int k = a.T - 1; k > 0; --k)
        hipLaunchKernelGGL(k32_sstep, dim3(np * k), dim3(GT), GEMM_SMEM, s, B, ldb, np, k, 0, (const float*)a.LT,
                           a.ld, k - 1, dT(k - 1), a.ld);
}

static void refine_lds_attributes() {
    static bool done = false;
    if (done) return;
    done = true;
    for (const void* f : {reinterpret_cast<const void*>(&k32_sdiag), reinterpret_cast<const void*>(&k32_supd),
                          reinterpret_cast<const void*>(&k32_sstep)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (const void* f : {reinterpret_cast<const void*>(&k64_kmat<4>), reinterpret_cast<const void*>(&k64_kmat<8>),
                          reinterpret_cast<const void*>(&k64_kmat<12>), reinterpret_cast<const void*>(&k64_kmat<16>),
                          reinterpret_cast<const void*>(&k64_kmat<20>), reinterpret_cast<const void*>(&k64_kmat<24>),
                          reinterpret_cast<const void*>(&k64_kmat<28>), reinterpret_cast<const void*>(&k64_kmat<32>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)KMAT_SMEM);
}

static void kmat(const float* X1, long ldx1, int n1, const float* X2, long ldx2, int n2, int D, const double* theta,
                 int add_noise, const double* C, long ldc, const float* Y, long ldy, double* out, long ldo,
                 float* out32, long ldo32, int p, hipStream_t s) {
    KmatArgs k{X1, ldx1, n1, X2, ldx2, n2, D, theta, add_noise, C, ldc, Y, ldy, out, ldo, out32, ldo32, p,
               (p + KM_Q - 1) / KM_Q};
    const dim3 g(((n1 + KM_R - 1) / KM_R) * k.tq);
    switch ((D + 3) & ~3) {
        case 4: hipLaunchKernelGGL(k64_kmat<4>, g, dim3(256), KMAT_SMEM, s, k); break;
        case 8: hipLaunchKernelGGL(k64_kmat<8>, g, dim3(256), KMAT_SMEM, s, k); break;
        case 12: hipLaunchKernelGGL(k64_kmat<12>, g, dim3(256), KMAT_SMEM, s, k); break;
        case 16: hipLaunchKernelGGL(k64_kmat<16>, g, dim3(256), KMAT_SMEM, s, k); break;
        case 20: hipLaunchKernelGGL(k64_kmat<20>, g, dim3(256), KMAT_SMEM, s, k); break;
        case 24: hipLaunchKernelGGL(k64_kmat<24>, g, dim3(256), KMAT_SMEM, s, k); break;
        case 28: hipLaunchKernelGGL(k64_kmat<28>, g, dim3(256), KMAT_SMEM, s, k); break;
        default: hipLaunchKernelGGL(k64_kmat<32>, g, dim3(256), KMAT_SMEM, s, k); break;
    }
}

// after the sweep with a.LT set: alpha0 (r.A64), R (r.R64), W^T rows (r.XB) and the q partials
// (a.zpart, a.nz workgroups); the Z^T rows of M become alpha0^T
static void f32_refine_core(const F32Args& a, const F32Refine& r, hipStream_t s) {
    refine_lds_attributes();
    const int npad = a.T * TB, ppad = a.Tp * TB;
    float* Zr = a.M + row_off(a, a.T);
    f32_bsolve(a, Zr, a.ld, a.Tp, s);                                                  // alpha0^T
    const dim3 tg((npad / 32) * (ppad / 32));
    hipLaunchKernelGGL(k_tr3264, tg, dim3(256), 0, s, Zr, a.ld, r.A64, r.ld64, a.n, a.p, npad, ppad, 0);
    kmat(a.X, a.ldx, a.n, a.X, a.ldx, a.n, a.D, a.theta, 1, r.A64, r.ld64, a.Y, a.ldy, r.R64, r.ld64, nullptr, 0,
         a.p, s);                                                                          // R = Y - K alpha0
    hipLaunchKernelGGL(k_tr3264, tg, dim3(256), 0, s, r.XB, a.ld, r.R64, r.ld64, a.n, a.p, npad, ppad, 1);
    f32_fsolve(a, r.XB, a.ld, a.Tp, s);                                                  // W^T = (L~^-1 R)^T
}

void launch_f32_refine_lml(const F32Args& a, const F32Refine& r, hipStream_t s) {
    f32_refine_core(a, r, s);
    hipLaunchKernelGGL(k_refine_q, dim3(a.nz), dim3(256), 0, s, a.Y, a.ldy, (const double*)r.A64,
                       (const double*)r.R64, r.ld64, (const float*)r.XB, a.ld, a.n, a.p, a.zpart);
}

void launch_f32_refine_mean(const F32Args& a, const F32Refine& r, float* mean, long ldm, int steps, hipStream_t s) {
    f32_refine_core(a, r, s);
    const int npad = a.T * TB, ppad = a.Tp * TB;
    const dim3 tg((npad / 32) * (ppad / 32));
    for (int it = 0;; ++it) {
        f32_bsolve(a, r.XB, a.ld, a.Tp, s);                                              // delta^T = (L~^-T W)^T
        hipLaunchKernelGGL(k_tr3264, tg, dim3(256), 0, s, r.XB, a.ld, r.A64, r.ld64, a.n, a.p, npad, ppad,
                           2);                                                             // alpha += delta
        if (it + 1 >= steps) break;
        // the next step: R = Y - K alpha (fp64), W^T = (L~^-1 R)^T
        kmat(a.X, a.ldx, a.n, a.X, a.ldx, a.n, a.D, a.theta, 1, r.A64, r.ld64, a.Y, a.ldy, r.R64, r.ld64, nullptr, 0,
             a.p, s);
        hipLaunchKernelGGL(k_tr3264, tg, dim3(256), 0, s, r.XB, a.ld, r.R64, r.ld64, a.n, a.p, npad, ppad, 1);
        f32_fsolve(a, r.XB, a.ld, a.Tp, s);
    }
    kmat(a.Xs, a.ldxs, a.ns, a.X, a.ldx, a.n, a.D, a.theta, 0, r.A64, r.ld64, nullptr, 0, nullptr, 0, mean, ldm,
         a.p, s);                                                                          // mean = K(X*, X) alpha1
}

void launch_f32_gram_dense(const float* X1, long ldx1, int n1, const float* X2, long ldx2, int n2, int D,
                           const double* theta, float diag_add, float* K, long ldk, hipStream_t s) {
    const int tr = (n1 + TB - 1) / TB, tc = (n2 + TB - 1) / TB;
    hipLaunchKernelGGL(k32_gram_dense, dim3(tr * tc), dim3(GT), gram_smem_bytes32(D), s, X1, ldx1, n1, X2, ldx2, n2,
                       D, theta, diag_add, K, ldk, tc);
}

}  // namespace mfgp
