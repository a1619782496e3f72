// SVGP ELBO gradient (whitened, Gaussian likelihood) on the MI355X engine.
//
// Reference: the GradientTape of LatentMFCoregionalizationSVGP.optimize
// (mfgpflow/linear_svgp.py:181-191) and SingleBinSVGP.optimize (singlebin_svgp.py:81-86):
// d(-ELBO) w.r.t. q_mu, q_sqrt (FillTriangular), Z (inducing points, fidelity column
// included), every latent kernel's (vL, lL, vD, lD, rho), W and the Gaussian noise.
//
// Per latent (Li = chol(Kuu)^{-1}, A = Li Kuf, B = Lq^T A = C Kuf, C = Lq^T Li, m = q_mu[:, l]),
// with upstream alpha = dE/dg_mu and beta = dE/dg_var (E = the ELBO):
//   gA        = dE/dA = m alpha^T + 2 (Lq B - A) diag(beta)
//   dE/dm     = A alpha - m
//   dE/dLq    = tril(2 A diag(beta) B^T) - Lq + diag(1 / Lq_ii)
//   dE/dKuf   = Li^T gA
//   dE/dLi    = tril(gA Kuf^T)
//   dE/dKuu   = -Li^T Psi(tril(dE/dLi) Li^T) Li,  Psi(H) = (tril H + tril H^T - diag H) / 2
//               (the adjoint of Li = chol(Kuu)^{-1}: dLi = -Phi(Li dKuu Li^T) Li)
//   dE/dKff   = beta
// A and B are the forward's own products (k_svgp_cond keeps them).  Every adjoint is associated
// around them rather than around Li Q (Q = Kuf diag(beta) Kuf^T) or Lq C - Li: at the Goku state
// cond(Kuu) ~ 1e9 and Li's entries reach 3e4, and applying Li to the smooth Q cancels ~8 digits
// (dE/dKuu off by 3.9e-8 relative against the reference's autodiff; 3e-12 in this form).
// The kernel / inducing-point gradients are the weighted derivative sums
//   sum_ab dE/dK_ab dk(a, b)/dtheta  over (Z, Z) and (Z, X), plus the K_diag term.
// All products are batched over latents and run on v_mfma_f64_16x16x4 tiles (k_bgemm).
#include <algorithm>

#include <type_traits>

#include "mfgp_device.h"
#include "mfgp_internal.h"

namespace mfgp {

static inline int cdv(int a, int b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- batched GEMM (BgemmArgs: mfgp_internal.h)
template <int NB, bool TA, bool TB>
__global__ __launch_bounds__(NTHREADS) void k_bgemm(BgemmArgs a) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* As = smem;
    double* Bs = As + E;
    int bx, b;
    xcd_swizzle(bx, b);
    const int ti = bx / a.Nt, tj = bx % a.Nt;
    if (a.tril && tj > ti) {   // strictly-upper output tile of a lower-masked product: zeros
        Acc<NB> z;
        acc_zero(z);
        acc_store(z, a.D + b * a.sD + (long)ti * NB * a.ldd + (long)tj * NB, a.ldd);
        return;
    }
    const double* A = a.A + b * a.sA;
    const double* B = a.B + b * a.sB;
    const double* s = a.s ? a.s + b * a.ss : nullptr;
    Acc<NB> acc;
    acc_zero(acc);
    int k0 = 0, k1 = a.Kt;
    if (a.amask == 1) k1 = min(k1, ti + 1);
    else if (a.amask == 2) k0 = max(k0, ti);
    if (a.bmask == 1) k0 = max(k0, tj);
    else if (a.bmask == 2) k1 = min(k1, tj + 1);
    for (int kt = k0; kt < k1; ++kt) {
        tile_load<NB>(As, TA ? A + (long)kt * NB * a.lda + (long)ti * NB : A + (long)ti * NB * a.lda + (long)kt * NB,
                      a.lda);
        tile_load<NB>(Bs, TB ? B + (long)tj * NB * a.ldb + (long)kt * NB : B + (long)kt * NB * a.ldb + (long)tj * NB,
                      a.ldb);
        if (s) {
            __syncthreads();
            for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
                const int r = e / NB, c = e % NB;
                Bs[r * S + c] *= s[(long)kt * NB + (TB ? c : r)];
            }
        }
        __syncthreads();
        tile_mma<NB, TA, TB>(acc, As, Bs, a.alpha);
        __syncthreads();
    }
    double* Dt = a.D + b * a.sD;
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = ti * NB + acc_row<NB>(q, r), j = tj * NB + acc_col<NB>(q);
            double v = acc.v[q][r];
            if (a.Cin) v += a.beta * a.Cin[b * a.sC + (long)i * a.ldc + j];
            if (a.colscale) v *= a.colscale[b * a.scs + j];
            if (a.x) v += a.x[b * a.sx + i] * a.y[b * a.sy + j];
            if (a.tril && j > i) v = 0.0;
            Dt[(long)i * a.ldd + j] = v;
        }
}

size_t bgemm_smem(int nb) { return 2 * sizeof(double) * (size_t)nb * (nb + 2); }

// The same products on NB = 32 operands, a 64 x 64 output block per workgroup: wave w computes
// the 32 x 32 tile (2 bi + (w >> 1), 2 bj + (w & 1)) as 2 x 2 independent 16 x 16 accumulators
// (k_bgemm: one 16 x 16 chain per wave), and each k-tile's two A tiles and two B tiles are staged
// in LDS once for all four waves (twice k_bgemm's operand reuse), one buffer, the next k-tile's
// global loads issued into registers before the current products.  Every 16 x 16 block
// runs the same MFMA sequence as tile_mma<32> (k-tiles ascending, 4-deep steps ascending; alpha, a
// power of two, on the accumulated tile instead of the A operand: the same bits), so the results
// are bitwise k_bgemm's.  Edge blocks (odd Mt / Nt) load a
// clamped in-range tile for the missing half and store nothing from it.
constexpr int BG2_E = 32 * 34;   // one 32-tile in LDS (TileCfg<32>)
size_t bgemm2_smem() { return 4 * sizeof(double) * (size_t)BG2_E; }

template <bool TA, bool TB>
__global__ __launch_bounds__(NTHREADS) void k_bgemm2(BgemmArgs a) {
    constexpr int S = 34, NB = 32;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    int bx, b;
    xcd_swizzle(bx, b);
    const int Nb = (a.Nt + 1) >> 1, Mb = (a.Mt + 1) >> 1;
    // longest blocks first (placement only): a lower-masked A (k < ti + 1) or upper-masked B
    // (k < tj + 1) gives the last row / column blocks the longest k-ranges, so those are dealt first
    // and the launch does not end on them
#ifndef MFGP_BG2_LPT
#define MFGP_BG2_LPT 1
#endif
    int bi = bx / Nb, bj = bx % Nb;
    if (MFGP_BG2_LPT && a.amask == 1) bi = Mb - 1 - bi;
    if (MFGP_BG2_LPT && a.bmask == 2) bj = Nb - 1 - bj;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ti = 2 * bi + (w >> 1), tj = 2 * bj + (w & 1);   // this wave's output tile
    const bool live = ti < a.Mt && tj < a.Nt;
    // k-range of a tile (ri, cj) under the operand masks
    auto krange = [&](int ri, int cj, int& k0, int& k1) {
        k0 = 0;
        k1 = a.Kt;
        if (a.amask == 1) k1 = min(k1, ri + 1);
        else if (a.amask == 2) k0 = max(k0, ri);
        if (a.bmask == 1) k0 = max(k0, cj);
        else if (a.bmask == 2) k1 = min(k1, cj + 1);
        if (a.tril && cj > ri) k1 = k0;   // strictly upper output tile of a lower-masked product
    };
    int kw0, kw1;
    krange(ti, tj, kw0, kw1);
    if (!live) kw1 = kw0;
    // the workgroup's k-range: the union over its live tiles
    int kb0 = a.Kt, kb1 = 0;
    for (int q = 0; q < 4; ++q) {
        const int r = 2 * bi + (q >> 1), c = 2 * bj + (q & 1);
        if (r >= a.Mt || c >= a.Nt) continue;
        int k0, k1;
        krange(r, c, k0, k1);
        if (k1 > k0) { kb0 = min(kb0, k0); kb1 = max(kb1, k1); }
    }
    const double* A = a.A + b * a.sA;
    const double* B = a.B + b * a.sB;
    const double* s = a.s ? a.s + b * a.ss : nullptr;
    const int ra0 = min(2 * bi, a.Mt - 1), ra1 = min(2 * bi + 1, a.Mt - 1);
    const int cb0 = min(2 * bj, a.Nt - 1), cb1 = min(2 * bj + 1, a.Nt - 1);
    auto atile = [&](int ri, int kt) {
        return TA ? A + (long)kt * NB * a.lda + (long)ri * NB : A + (long)ri * NB * a.lda + (long)kt * NB;
    };
    auto btile = [&](int cj, int kt) {
        return TB ? B + (long)cj * NB * a.ldb + (long)kt * NB : B + (long)kt * NB * a.ldb + (long)cj * NB;
    };
    TileRegs<32> rg[4];
    auto fetch = [&](int kt) {
        tile_fetch<32>(rg[0], atile(ra0, kt), a.lda);
        tile_fetch<32>(rg[1], atile(ra1, kt), a.lda);
        tile_fetch<32>(rg[2], btile(cb0, kt), a.ldb);
        tile_fetch<32>(rg[3], btile(cb1, kt), a.ldb);
    };
    auto put = [&](double* buf, int kt) {
        tile_put<32>(buf, rg[0]);
        tile_put<32>(buf + BG2_E, rg[1]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            TileRegs<32>& r = rg[2 + h];
            if (s) {   // k scaling of the B side (k_bgemm's Bs[r][c] *= s[k])
#pragma unroll
                for (int q = 0; q < 32 * 32 / 2 / NTHREADS; ++q) {
                    const int p = threadIdx.x + q * NTHREADS;
                    const int row = p / 16, c = 2 * (p % 16);
                    r.v[q].x *= s[(long)kt * NB + (TB ? c : row)];
                    r.v[q].y *= s[(long)kt * NB + (TB ? c + 1 : row)];
                }
            }
            tile_put<32>(buf + (2 + h) * BG2_E, r);
        }
    };
    f64x4 acc[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[p][q] = f64x4{0.0, 0.0, 0.0, 0.0};
    auto mma_tile = [&](const double* cur) {
        const double* As = cur + (w >> 1) * BG2_E;
        const double* Bs = cur + (2 + (w & 1)) * BG2_E;
#pragma unroll 4
        for (int k0 = 0; k0 < NB; k0 += 4) {
            const int k = k0 + lk;
            double av[2], bv[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int i = 16 * t + li, j = 16 * t + li;
                av[t] = TA ? As[k * S + i] : As[i * S + k];
                bv[t] = TB ? Bs[j * S + k] : Bs[k * S + j];
            }
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    acc[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[p], bv[q], acc[p][q], 0, 0, 0);
        }
    };
    if (kb1 > kb0) {
        // one LDS buffer, the next k-tile's loads in registers meanwhile: 35 KB of LDS, four
        // workgroups per CU (the double-buffered form's 70 KB held two: these GEMMs have 5-37
        // k-tiles, so a workgroup's load prologue and store epilogue need company to hide;
        // Goku SVGP step 2.626 -> 2.370 ms)
        fetch(kb0);
        for (int kt = kb0; kt < kb1; ++kt) {
            put(smem, kt);
            if (kt + 1 < kb1) fetch(kt + 1);
            __syncthreads();
            if (kt >= kw0 && kt < kw1) mma_tile(smem);   // wave-uniform
            __syncthreads();
        }
    }
    if (!live) return;
    // alpha on the accumulated tile, not on every A operand (a VALU multiply feeding each MFMA):
    // every caller's alpha is a power of two (1, -1, 2), so the scaled sums are bit for bit those
    // of scaled operands
    if (a.alpha != 1.0) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = 0; q < 2; ++q) acc[p][q] *= a.alpha;
    }
    double* Dt = a.D + b * a.sD;
    if (a.sym) {   // tiles ti >= tj only (tril): v (Psi: 0.5 v) at (i, j) and (j, i)
        if (tj > ti) return;
        const double hs = a.sym == 1 ? 0.5 : 1.0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = ti * NB + 16 * p + lk + 4 * r, j = tj * NB + 16 * q + li;
                    const double v = hs * acc[p][q][r];
                    if (j <= i) Dt[(long)i * a.ldd + j] = v;
                    if (j < i) Dt[(long)j * a.ldd + i] = v;
                }
        return;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = ti * NB + 16 * p + lk + 4 * r, j = tj * NB + 16 * q + li;
                double v = acc[p][q][r];
                if (a.Cin) v += a.beta * a.Cin[b * a.sC + (long)i * a.ldc + j];
                if (a.colscale) v *= a.colscale[b * a.scs + j];
                if (a.x) v += a.x[b * a.sx + i] * a.y[b * a.sy + j];
                if (a.tril && j > i) v = 0.0;
                Dt[(long)i * a.ldd + j] = v;
            }
    if (a.csq) {   // column partials of the tile: rows 0-15 then 16-31, as k_svgp_cond2's
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            double ta = 0.0, tm = 0.0;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                double sa = 0.0, sm = 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int gr = ti * NB + 16 * p + lk + 4 * r;
                    const double v = acc[p][q][r];
                    sa += v * v;
                    if (a.csq2) sm += v * ((gr < a.qn) ? a.qv[(long)gr * a.qs + b] : 0.0);
                }
                sa += __shfl_xor(sa, 16, 64); sa += __shfl_xor(sa, 32, 64);
                sm += __shfl_xor(sm, 16, 64); sm += __shfl_xor(sm, 32, 64);
                ta += sa;
                tm += sm;
            }
            if (lk == 0) {
                const long o = ((long)b * a.Mt + ti) * a.ldcs + (long)tj * NB + 16 * q + li;
                a.csq[o] = ta;
                if (a.csq2) a.csq2[o] = tm;
            }
        }
    }
}

template <int NB>
static void bgemm(hipStream_t st, int ta, int tb, const BgemmArgs& a, int batch) {
    if (NB == 32) {
        static bool attr = false;
        if (!attr) {
            for (const void* f : {reinterpret_cast<const void*>(&k_bgemm2<false, false>),
                                  reinterpret_cast<const void*>(&k_bgemm2<false, true>),
                                  reinterpret_cast<const void*>(&k_bgemm2<true, false>),
                                  reinterpret_cast<const void*>(&k_bgemm2<true, true>)})
                (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bgemm2_smem());
            attr = true;
        }
        dim3 g(((a.Mt + 1) >> 1) * ((a.Nt + 1) >> 1), 1, batch);
        const size_t sm = bgemm2_smem();
        if (!ta && !tb) hipLaunchKernelGGL((k_bgemm2<false, false>), g, dim3(NTHREADS), sm, st, a);
        else if (!ta && tb) hipLaunchKernelGGL((k_bgemm2<false, true>), g, dim3(NTHREADS), sm, st, a);
        else if (ta && !tb) hipLaunchKernelGGL((k_bgemm2<true, false>), g, dim3(NTHREADS), sm, st, a);
        else hipLaunchKernelGGL((k_bgemm2<true, true>), g, dim3(NTHREADS), sm, st, a);
        return;
    }
    dim3 g(a.Mt * a.Nt, 1, batch);
    const size_t sm = bgemm_smem(NB);
    if (!ta && !tb) hipLaunchKernelGGL((k_bgemm<NB, false, false>), g, dim3(NTHREADS), sm, st, a);
    else if (!ta && tb) hipLaunchKernelGGL((k_bgemm<NB, false, true>), g, dim3(NTHREADS), sm, st, a);
    else if (ta && !tb) hipLaunchKernelGGL((k_bgemm<NB, true, false>), g, dim3(NTHREADS), sm, st, a);
    else hipLaunchKernelGGL((k_bgemm<NB, true, true>), g, dim3(NTHREADS), sm, st, a);
}

void launch_bgemm(int nb, hipStream_t st, int ta, int tb, const BgemmArgs& a, int batch) {
    if (nb == 64) bgemm<64>(st, ta, tb, a, batch);
    else bgemm<32>(st, ta, tb, a, batch);
}

// plain square product helper on Mpad x Mpad batched matrices
template <int NB>
static void sq(hipStream_t st, int Tm, int L, long mm, long ld, int ta, const double* A, int tb, const double* B,
               double* D, double alpha = 1.0, const double* Cin = nullptr, double beta = 0.0, int tril = 0,
               const double* x = nullptr, const double* y = nullptr, long sxy = 0, int amask = 0, int bmask = 0) {
    BgemmArgs a{};
    a.amask = amask; a.bmask = bmask;
    a.A = A; a.lda = ld; a.sA = mm;
    a.B = B; a.ldb = ld; a.sB = mm;
    a.Cin = Cin; a.ldc = ld; a.sC = mm; a.beta = beta;
    a.x = x; a.sx = sxy; a.y = y; a.sy = sxy;
    a.D = D; a.ldd = ld; a.sD = mm;
    a.alpha = alpha;
    a.Mt = Tm; a.Nt = Tm; a.Kt = Tm; a.tril = tril;
    bgemm<NB>(st, ta, tb, a, L);
}

// ---------------------------------------------------------------- matvec (batched)
// y[b][r] = alpha * sum_c op(A)[r][c] x[b][c] + beta * z[b][r]      (one wave per output row)
__global__ __launch_bounds__(NTHREADS) void k_bmatvec(const double* A, long lda, long sA, int trans,
                                                      const double* x, long sx, int rows, int cols,
                                                      double alpha, const double* z, long sz, double beta,
                                                      double* y, long sy) {
    const int b = blockIdx.z;
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * (NTHREADS / 64) + (threadIdx.x >> 6);
    if (r >= rows) return;
    const double* Ab = A + b * sA;
    const double* xb = x + b * sx;
    double acc = 0.0;
    if (!trans && (lda & 1) == 0 && ((sA | sx) & 1) == 0 && (((uintptr_t)A | (uintptr_t)x) & 15) == 0) {
        // 16-B loads, two chains: a wave reads 1 KB of its row per step (the 8-B form ran at ~1 TB/s)
        const double* row = Ab + (long)r * lda;
        double acc1 = 0.0;
        const int c2 = cols & ~1;
        int c = 2 * lane;
        for (; c + 128 < c2; c += 256) {
            const f64x2 a0 = *reinterpret_cast<const f64x2*>(row + c);
            const f64x2 x0 = *reinterpret_cast<const f64x2*>(xb + c);
            const f64x2 a1 = *reinterpret_cast<const f64x2*>(row + c + 128);
            const f64x2 x1 = *reinterpret_cast<const f64x2*>(xb + c + 128);
            acc = fma(a0.x, x0.x, acc);
            acc = fma(a0.y, x0.y, acc);
            acc1 = fma(a1.x, x1.x, acc1);
            acc1 = fma(a1.y, x1.y, acc1);
        }
        for (; c < c2; c += 128) {
            const f64x2 a0 = *reinterpret_cast<const f64x2*>(row + c);
            const f64x2 x0 = *reinterpret_cast<const f64x2*>(xb + c);
            acc = fma(a0.x, x0.x, acc);
            acc = fma(a0.y, x0.y, acc);
        }
        if ((cols & 1) && lane == 0) acc = fma(row[cols - 1], xb[cols - 1], acc);
        acc += acc1;
    } else {
        for (int c = lane; c < cols; c += 64) acc += (trans ? Ab[(long)c * lda + r] : Ab[(long)r * lda + c]) * xb[c];
    }
    acc = wave_sum(acc);
    if (lane == 0) y[b * sy + r] = alpha * acc + (z ? beta * z[b * sz + r] : 0.0);
}

// ---------------------------------------------------------------- elementwise pieces
// Psi(H) = (tril H + tril H^T - diag H) / 2 (symmetric), padded square batch
__global__ void k_psi(const double* H, double* P, int mpad, long mm) {
    const int b = blockIdx.z;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < mm; e += (long)gridDim.x * blockDim.x) {
        const int i = (int)(e / mpad), j = (int)(e % mpad);
        const double* h = H + b * mm;
        double v;
        if (i > j) v = 0.5 * h[e];
        else if (i < j) v = 0.5 * h[(long)j * mpad + i];
        else v = 0.5 * h[e];
        P[b * mm + e] = v;
    }
}

// dE/dLq := G - klm (Lq - diag(1/Lq_ii)) on the m x m lower part; zero elsewhere.  Out: [L][m][m],
// or (packed) the lower triangles [L][m (m + 1) / 2], (i, j <= i) at i (i + 1) / 2 + j
__global__ void k_glq_final(const double* G, const double* Lq, int m, int mpad, long mm, double klm, double* out,
                            int packed) {
    const int b = blockIdx.z;
    const long tot = (long)m * m, tri = (long)m * (m + 1) / 2;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
        const int i = (int)(e / m), j = (int)(e % m);
        double v = 0.0;
        if (j <= i) {
            const double lq = Lq[b * mm + (long)i * mpad + j];
            v = G[b * mm + (long)i * mpad + j] - klm * lq;
            if (i == j) v += klm / lq;
        }
        if (!packed) out[(long)b * tot + e] = v;
        else if (j <= i) out[(long)b * tri + (long)i * (i + 1) / 2 + j] = v;
    }
}

// q_mu [m][L] -> padded per-latent vectors [L][mpad]
__global__ void k_qmu_pad(const double* q_mu, int m, int L, int mpad, double* qm) {
    const int l = blockIdx.z;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < mpad; r += gridDim.x * blockDim.x)
        qm[(long)l * mpad + r] = (r < m) ? q_mu[(long)r * L + l] : 0.0;
}

// gq_mu[m][L] from the padded per-latent vectors
__global__ void k_qmu_unpad(const double* g, int m, int L, int mpad, double* out) {
    const int l = blockIdx.z;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < m; r += gridDim.x * blockDim.x)
        out[(long)r * L + l] = g[(long)l * mpad + r];
}

// ---------------------------------------------------------------- VE backward
// r[n][p] = scale (y - f_mu) / s2 ; alpha[l][n] = sum_p r W[p][l] ; beta[l][n] = -scale/(2 s2) sum_p W[p][l]^2
// (W == nullptr: identity mixing, L == P).  Also dE/dnoise partials (one per block).
__global__ __launch_bounds__(NTHREADS) void k_ve_bwd(const double* g_mu, const double* g_var, const double* W,
                                                     const double* Y, long ldy, int n, int p, int L,
                                                     const double* noise, double scale, int npad, double* r,
                                                     double* alpha, double* beta, double* gnoise_part) {
    __shared__ double red[4];
    const double s2 = noise[0];
    const double inv = 1.0 / s2;
    double gs = 0.0;
    const long tot = (long)n * p;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
        const int i = (int)(e / p), c = (int)(e % p);
        double fm, fv;
        if (W) {
            fm = 0.0;
            fv = 0.0;
            for (int l = 0; l < L; ++l) {
                const double w = W[(long)c * L + l];
                fm += g_mu[(long)l * n + i] * w;
                fv += g_var[(long)l * n + i] * (w * w);
            }
        } else {
            fm = g_mu[(long)c * n + i];
            fv = g_var[(long)c * n + i];
        }
        const double dy = Y[(long)i * ldy + c] - fm;
        r[e] = scale * dy * inv;
        gs += -0.5 * inv + 0.5 * (dy * dy + fv) * inv * inv;
    }
    gs = block_sum(gs, red);
    if (threadIdx.x == 0) gnoise_part[blockIdx.x] = scale * gs;
    (void)alpha; (void)beta; (void)npad;
}

// alpha / beta per latent (padded to npad with zeros)
__global__ void k_ab(const double* r, const double* W, int n, int p, int L, const double* noise, double scale,
                     int npad, double* alpha, double* beta) {
    const int l = blockIdx.z;
    const double inv = 1.0 / noise[0];
    double wsq = 0.0;
    if (W)
        for (int c = 0; c < p; ++c) wsq += W[(long)c * L + l] * W[(long)c * L + l];
    else
        wsq = 1.0;
    const double bconst = -0.5 * scale * inv * wsq;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npad; i += gridDim.x * blockDim.x) {
        double a = 0.0;
        if (i < n) {
            if (W)
                for (int c = 0; c < p; ++c) a += r[(long)i * p + c] * W[(long)c * L + l];
            else
                a = r[(long)i * p + l];
        }
        alpha[(long)l * npad + i] = a;
        beta[(long)l * npad + i] = (i < n) ? bconst : 0.0;
    }
}

// dE/dW[c][l] = sum_n r[n][c] g_mu[l][n] - (scale / s2) W[c][l] sum_n g_var[l][n]   (one wave per entry)
__global__ __launch_bounds__(NTHREADS) void k_gw(const double* r, const double* g_mu, const double* g_var,
                                                 const double* W, int n, int p, int L, const double* noise,
                                                 double scale, double* gW) {
    const int lane = threadIdx.x & 63;
    const int e = blockIdx.x * (NTHREADS / 64) + (threadIdx.x >> 6);
    if (e >= p * L) return;
    const int c = e / L, l = e % L;
    double s1 = 0.0, s2 = 0.0;
    for (int i = lane; i < n; i += 64) {
        s1 += r[(long)i * p + c] * g_mu[(long)l * n + i];
        s2 += g_var[(long)l * n + i];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) gW[e] = s1 - scale / noise[0] * W[e] * s2;
}

// ---------------------------------------------------------------- kernel derivative sums
// For pairs (a in P1 = Z rows, b in P2), weight Wt[a][b] (padded row-major):
//   gth[q] += sum Wt dk/dtheta_q     (q over [vL, lL(D), vD, lD(D), rho])
//   gz[a][d] += zf * sum_b Wt dk(a, b)/dz_a[d]
// With wl = Wt sa sb kL (the LF part of k) the dimension sums expand in moments of the b side:
//   sum_b wl (za_d - xb_d)^2 = za_d^2 S0 - 2 za_d S1_d + S2_d,   sum_b wl (za_d - xb_d) = za_d S0 - S1_d
// with [S0 | S1 | S2](a) = sum_b wl(a, b) [1 | xb | xb^2]: a GEMM of the pair weights with the
// augmented b rows, on the matrix core (v_mfma_f64_16x16x4: lane (i, k) forms the weight of pair
// (a_i, b_k) straight into its A operand; B = [1 | x | x^2] of b_k).  Likewise T for
// wd = Wt kD (HF x HF pairs, only when the wave holds one).  Coordinates are taken relative to
// the block's first Z row, which keeps the expansion's cancellation at the data's spread.
// The per-pair work left on the VALU is r^2 and one exp (two for HF x HF pairs).
// Workgroup: 32 a rows x cpb <= KG_COLS b columns; wave w: rows 16 (w & 1) .., b half w >> 1; the b rows
// go through LDS KG_CHUNK per half at a time, W is loaded one step ahead.
constexpr int KG_ROWS = 32, KG_COLS = 256, KG_CHUNK = 32;
#ifndef MFGP_KG_EQUAL
#define MFGP_KG_EQUAL 1
#endif
// Registers held to three waves per SIMD for D <= 12 (168 VGPRs; unbounded the allocator took 148
// VGPRs + AGPRs, two waves): 2.714 -> 2.672 ms a Goku SVGP step; four waves (10 spills) 2.675.
// Wider rows (DC 16 / 32) get two / one waves per SIMD: held to three they spill 21 / 194 VGPRs.
constexpr int KG_WAVES = 3;
template <int DC>
constexpr int kg_ncb() { return (2 * DC + 1 + 15) / 16; }

template <int DC>
__global__ __launch_bounds__(NTHREADS) __attribute__((amdgpu_waves_per_eu(DC <= 12 ? KG_WAVES : (DC <= 16 ? 2 : 1)))) void k_kgrad(const double* P1, long ld1, int n1, const double* P2, long ld2,
                                                    int n2, const double* Wt, long ldw, long sW, const double* thetas,
                                                    int G, int D, double zf, int nbc, int cpb, double* gth_part,
                                                    double* gz_part) {
    constexpr int NCB = kg_ncb<DC>(), SC = NCB * 16 + 1, XS = DC + 1, NS = DC / 4;
    static_assert(DC % 4 == 0, "dimension chunks of the distance MFMA");
    constexpr int SACC = (NTHREADS / 64) * 16 * SC, XST = 2 * KG_CHUNK * (XS + 2);
    __shared__ double il[DC], id[DC];
    // the workgroup's 32 Z rows ([row][XS]: coordinates, the fidelity at DC), loaded once for the
    // prologue and the epilogue; coordinates are centred on row 0 (cz = zsm[0][d])
    __shared__ double zsm[KG_ROWS * XS];
    // the b rows of a chunk during the pair loop -- [half][row][XS] centred coordinates (column DC
    // the fidelity), [half][row][2] their scaled squared norms -- and the moment accumulators after it
    __shared__ double lds_buf[SACC > XST ? SACC : XST];
    auto sacc = reinterpret_cast<double(*)[16][SC]>(lds_buf);
    __shared__ double wred[NTHREADS / 64][4];
    __shared__ double dsum[2][DC];
    int bx, lat;
    xcd_swizzle(bx, lat);
    const int at = bx / nbc, bc = bx % nbc;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int li = l & 15, lk = l >> 4;
    const MFTheta th{thetas + (long)lat * G, D};
    const double vL = th.vL(), vD = th.vD(), rho = th.rho();
    for (int e = t; e < KG_ROWS * XS; e += NTHREADS) {
        const int r = e / XS, d = e % XS, ag = at * KG_ROWS + r;
        double v = (d == DC) ? -1.0 : 0.0;
        if (ag < n1) {
            if (d < D) v = P1[(long)ag * ld1 + d];
            else if (d == DC) v = P1[(long)ag * ld1 + D];
        }
        zsm[e] = v;
    }
    if (t < DC) {
        il[t] = (t < D) ? 1.0 / th.lL(t) : 0.0;
        id[t] = (t < D) ? 1.0 / th.lD(t) : 0.0;
        dsum[0][t] = 0.0;
        dsum[1][t] = 0.0;
    }
    __syncthreads();
    const double* cz = zsm;   // row 0 (at * KG_ROWS < n1 always)
    const int ar = 16 * (w & 1) + li, a = at * KG_ROWS + ar;
    const double fa = zsm[ar * XS + DC];
    const bool La = (fa == 0.0), Ha = (fa == 1.0), aval = La || Ha;
    double za[DC];
#pragma unroll
    for (int d = 0; d < DC; ++d) za[d] = (aval && d < D) ? zsm[ar * XS + d] - cz[d] : 0.0;
    f64x4 accL[NCB], accD[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) { accL[c] = f64x4{0.0, 0.0, 0.0, 0.0}; accD[c] = accL[c]; }
    double gvL = 0.0, gvD = 0.0, grho = 0.0;
    const double sa = La ? 1.0 : rho;
    const int half = w >> 1;
    const int bbase = bc * cpb;
    const int bend = min(n2, bbase + cpb);
    const double* wrow = Wt + lat * sW + (long)a * ldw;
    // Pairs in 16 x 16 blocks (16 a rows of the wave x 16 b rows of its half): the distances
    // |za - xb|^2 / l^2 = |za/l|^2 + |xb/l|^2 - 2 (za/l).(xb/l) with the dot products on the matrix
    // core (NS = DC / 4 steps of v_mfma_f64_16x16x4; lane (li, lq) then holds the pairs (a = li,
    // b = lq + 4 r)), which are exactly the A-operand positions of the moment GEMM's step r: the
    // VALU keeps one exp per pair (two for HF x HF pairs) and the weights.  (The direct-difference
    // loop spent ~157 VALU instructions per 64 pairs; k_kgrad was 12.9% of a Goku SVGP step.)
    // b rows are staged one chunk of KG_CHUNK rows per half at a time: iteration i gives chunk 2 i + h
    // of the workgroup's columns to half h, and the loop stops after the last chunk that holds a
    // column (a workgroup over the last 44 of 300 columns runs one iteration, not four, and both
    // halves share the columns of a ragged last block).  The next block's pair weights are loaded
    // (into registers) while this block's pairs are processed.
    const int nit = (bend - bbase + 2 * KG_CHUNK - 1) / (2 * KG_CHUNK);
    auto bstart = [&](int i) { return bbase + (2 * i + half) * KG_CHUNK; };
    // the 4 weights (b = b0 + 4 r + lk) of a block: unconditional loads (W is padded), then the mask
    auto wload = [&](int b0, double* wv) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int b = b0 + 4 * r + lk;
            const double w = wrow[min(b, bend - 1)];
            wv[r] = (aval && b < bend) ? w : 0.0;
        }
    };
    double zl[NS], zd[NS];
    double na = 0.0, nad = 0.0;
#pragma unroll
    for (int d = 0; d < DC; ++d) {
        const double u = za[d] * il[d], v = za[d] * id[d];
        na = fma(u, u, na);
        nad = fma(v, v, nad);
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        zl[q] = za[4 * q + lk] * il[4 * q + lk];
        zd[q] = za[4 * q + lk] * id[4 * q + lk];
    }
    double* xsb = lds_buf;                                  // [2][KG_CHUNK][XS]
    double* nrm = xsb + 2 * KG_CHUNK * XS;                  // [2][KG_CHUNK][2]
    // The moment GEMM's B operand [1 | x | x^2] of b row k, column j = 16 c + li of the lane, is
    // formed from the staged row (j = 0: 1, whatever the row: its weights are 0 where it is not a
    // pair; 1 <= j <= D: x_{j-1}; D < j <= 2D: x_{j-1-D}^2; above: 0).  (A staged [1 | x | x^2]
    // copy cost a pass over the chunk and a barrier: 1.6 us of a 5 us chunk.)
    int bkind[NCB], bdim[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
        const int j = 16 * c + li;
        bkind[c] = (j == 0) ? 0 : (j <= D ? 1 : (j <= 2 * D ? 2 : 3));
        bdim[c] = (bkind[c] == 1) ? j - 1 : (bkind[c] == 2 ? j - 1 - D : 0);
    }
    auto bval = [&](const double* xrow, int c) {
        const double v = xrow[bdim[c]];
        return bkind[c] == 0 ? 1.0 : (bkind[c] == 1 ? v : (bkind[c] == 2 ? v * v : 0.0));
    };
    double wc[4], wn[4];
    wload(bstart(0), wc);
    for (int it = 0; it < nit; ++it) {
        __syncthreads();   // the previous chunk is consumed
        if (t < 2 * KG_CHUNK) {   // wave 0: the two chunks' 64 b rows (centred) and their scaled squared norms
            const int hf = t / KG_CHUNK, r = t % KG_CHUNK;
            const int b = bbase + (2 * it + hf) * KG_CHUNK + r;
            double* xq = xsb + t * XS;
            double nl = 0.0, nd = 0.0;
#pragma unroll 4
            for (int d = 0; d < DC; ++d) {
                const double v = (b < bend && d < D) ? P2[(long)b * ld2 + d] - cz[d] : 0.0;
                xq[d] = v;
                const double u = v * il[d], q = v * id[d];
                nl = fma(u, u, nl);
                nd = fma(q, q, nd);
            }
            xq[DC] = (b < bend) ? P2[(long)b * ld2 + D] : -1.0;
            nrm[t * 2] = nl;
            nrm[t * 2 + 1] = nd;
        }
        __syncthreads();
        const double* xs = xsb + half * KG_CHUNK * XS;
        const double* nr = nrm + half * KG_CHUNK * 2;
        const int b0 = bstart(it);
#pragma unroll
        for (int blk = 0; blk < KG_CHUNK / 16; ++blk) {
            const int rb = 16 * blk;
            if (b0 + rb >= bend) break;                      // wave-uniform: past the last b row
            wload(rb + 16 < KG_CHUNK ? b0 + rb + 16 : bstart(it + 1), wn);   // the next block's weights, in flight meanwhile
            f64x4 dl = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < NS; ++q)
                dl = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[(rb + li) * XS + 4 * q + lk] * il[4 * q + lk], zl[q], dl, 0, 0, 0);
            // step r: the lane's pair (a = li, b = rb + 4 r + lk); its weight is the A operand of
            // the moment GEMM's step r, B = [1 | x | x^2] of b
            // the four pairs' exps as four interleaved chains (exp4: each polynomial step issued
            // for all four before the next; one exp_lib chain at a time left the 13 dependent
            // f64 FMAs of each exp exposed), then the accumulations in r order
            double eL[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) eL[r] = -0.5 * fmax(na + nr[2 * (rb + lk + 4 * r)] - 2.0 * dl[r], 0.0);
            exp4(eL);   // dk/dvL (TF form: finite where vL underflows); bitwise exp_lib for x <= 0
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int bl = rb + lk + 4 * r;
                const double fb = xs[bl * XS + DC];
                const bool Lb = (fb == 0.0), Hb = (fb == 1.0);
                const double wv = (Lb || Hb) ? wc[r] : 0.0;
                const double sb = Lb ? 1.0 : rho;
                const double kL = vL * eL[r];
                const double wl = wv * sa * sb * kL;
                gvL += wv * sa * sb * eL[r];
                grho += wv * ((Ha ? sb : 0.0) + (Hb ? sa : 0.0)) * kL;
#pragma unroll
                for (int c = 0; c < NCB; ++c)
                    accL[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(wl, bval(xs + bl * XS, c), accL[c], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) wc[r] = wn[r];
        }
        // HF x HF pairs (the delta kernel), in a pass of their own: few blocks hold any (Goku: X's
        // HF rows are its last 36), and the hot pass above keeps its accumulators in place
#pragma unroll
        for (int blk = 0; blk < KG_CHUNK / 16; ++blk) {
            const int rb = 16 * blk;
            if (b0 + rb >= bend) break;
            bool hany = false;
#pragma unroll
            for (int r = 0; r < 4; ++r) hany |= Ha && xs[(rb + lk + 4 * r) * XS + DC] == 1.0;
            if (__ballot(hany) == 0) continue;   // wave-uniform
            double wh[4];
            wload(b0 + rb, wh);
            f64x4 dd = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < NS; ++q)
                dd = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[(rb + li) * XS + 4 * q + lk] * id[4 * q + lk], zd[q], dd, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int bl = rb + lk + 4 * r;
                const bool hh = Ha && xs[bl * XS + DC] == 1.0 && wh[r] != 0.0;
                const double rD = fmax(nad + nr[2 * bl + 1] - 2.0 * dd[r], 0.0);
                const double we = hh ? wh[r] * exp_lib(-0.5 * rD) : 0.0;
                gvD += we;
#pragma unroll
                for (int c = 0; c < NCB; ++c)
                    accD[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(we * vD, bval(xs + bl * XS, c), accD[c], 0, 0, 0);
            }
        }
    }
    __syncthreads();   // lds_buf becomes the moment buffer
    // scalar theta partials: one LDS slot per wave
    {
        const double r0 = wave_sum(gvL), r1 = wave_sum(gvD), r2 = wave_sum(grho);
        if (l == 0) { wred[w][0] = r0; wred[w][1] = r1; wred[w][2] = r2; }
    }
    // moments -> dimension sums, LF part (ph = 0) then HF part (ph = 1)
    double gzv[(KG_ROWS * DC + NTHREADS - 1) / NTHREADS];
#pragma unroll
    for (int i = 0; i < (KG_ROWS * DC + NTHREADS - 1) / NTHREADS; ++i) gzv[i] = 0.0;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) sacc[w][lk + 4 * r][16 * c + li] = ph ? accD[c][r] : accL[c][r];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < (KG_ROWS * DC + NTHREADS - 1) / NTHREADS; ++i) {
            const int e = t + NTHREADS * i;
            const int r = e & (KG_ROWS - 1), d = e / KG_ROWS;   // a half-wave per dimension
            double term = 0.0;
            if (d < D) {
                const int hw = r >> 4, rr = r & 15;
                const int ag = at * KG_ROWS + r;
                auto S = [&](int col) { return sacc[hw][rr][col] + sacc[2 + hw][rr][col]; };
                const double s0 = S(0), s1 = S(1 + d), s2 = S(1 + D + d);
                const double z = (ag < n1) ? zsm[r * XS + d] - cz[d] : 0.0;
                const double ic = ph ? id[d] : il[d];
                const double ic2 = ic * ic;
                term = (z * z * s0 - 2.0 * z * s1 + s2) * ic2 * ic;   // d k / d l = k (za - xb)^2 / l^3
                gzv[i] -= (z * s0 - s1) * ic2;
            }
            // sum over the 32 rows: the half-wave of this dimension
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) term += __shfl_xor(term, o, 64);
            if (r == 0 && d < D) dsum[ph][d] += term;   // one writer per (ph, d)
        }
        __syncthreads();
    }
    for (int q = t; q < G; q += NTHREADS) {
        double v = 0.0;
        if (q == 0) v = (wred[0][0] + wred[1][0]) + (wred[2][0] + wred[3][0]);
        else if (q <= D) v = dsum[0][q - 1];
        else if (q == D + 1) v = (wred[0][1] + wred[1][1]) + (wred[2][1] + wred[3][1]);
        else if (q <= 2 * D + 1) v = dsum[1][q - D - 2];
        else if (q == 2 * D + 2) v = (wred[0][2] + wred[1][2]) + (wred[2][2] + wred[3][2]);
        gth_part[((long)lat * gridDim.x + bx) * G + q] = v;   // noise slot (G - 1): 0
    }
#pragma unroll
    for (int i = 0; i < (KG_ROWS * DC + NTHREADS - 1) / NTHREADS; ++i) {
        const int e = t + NTHREADS * i;
        const int r = e & (KG_ROWS - 1), d = e / KG_ROWS;
        const int ag = at * KG_ROWS + r;
        if (d < D) gz_part[(((long)lat * gridDim.x + bx) * KG_ROWS + r) * D + d] = (ag < n1) ? zf * gzv[i] : 0.0;
    }
}

// K_diag term: dE/dtheta from dE/dKff = beta  (vL: L + rho^2 H ; vD: H ; rho: 2 rho vL H)
__global__ __launch_bounds__(NTHREADS) void k_kff_grad(const double* X, long ldx, int n, const double* beta,
                                                       int npad, const double* thetas, int G, int D,
                                                       double* gth_kff) {
    __shared__ double red[4];
    const int l = blockIdx.x;
    const MFTheta th{thetas + (long)l * G, D};
    double sL = 0.0, sH = 0.0;
    for (int i = threadIdx.x; i < n; i += NTHREADS) {
        const double f = X[(long)i * ldx + D];
        const double bb = beta[(long)l * npad + i];
        if (f == 0.0) sL += bb;
        else if (f == 1.0) sH += bb;
    }
    sL = block_sum(sL, red);
    sH = block_sum(sH, red);
    if (threadIdx.x == 0) {
        const double rho = th.rho();
        double* g = gth_kff + (long)l * G;
        for (int q = 0; q < G; ++q) g[q] = 0.0;
        g[0] = sL + rho * rho * sH;
        g[1 + D] = sH;
        g[2 + 2 * D] = 2.0 * rho * th.vL() * sH;
    }
}

// Final reductions: gtheta[l][q] (kff + Kuu + Kuf partials), gZ[m][D+1] (sum over latents and
// column blocks; fidelity column 0), gnoise.  GR_LANES lanes per output, lane j summing the
// partials b = j mod GR_LANES, combined by a fixed xor tree (a thread per output walking its
// partials in one dependent chain took 93 us at L = 64: 19 workgroups of 448-load chains; 8
// lanes, 56-load chains, 31 us).
constexpr int GR_LANES = 32;   // 8: 2.118 ms a Goku single-bin step, 32: 2.098, 64: 2.10
__global__ void k_grad_reduce(const double* gth_uu, int nb_uu, const double* gth_uf, int nb_uf, const double* gth_kff,
                              const double* gz_uu, const double* gz_uf, int n_at, int nbc_uu, int nbc_uf, int L,
                              int G, int D, int m, const double* gnoise_part, int nnoise, double* gtheta, double* gZ,
                              double* gnoise) {
    const long gt = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const int tid = (int)(gt / GR_LANES), j = (int)(gt % GR_LANES);
    const int nth = L * G;
    double s = 0.0;
    if (tid < nth) {
        const int l = tid / G, q = tid % G;
        const double* pu = gth_uu + (long)l * nb_uu * G + q;
        const double* pf = gth_uf + (long)l * nb_uf * G + q;
        for (int b = j; b < nb_uu + nb_uf; b += GR_LANES) s += (b < nb_uu) ? pu[(long)b * G] : pf[(long)(b - nb_uu) * G];
    } else if (tid < nth + m * (D + 1)) {
        const int e = tid - nth;
        const int a = e / (D + 1), d = e % (D + 1);
        if (d < D) {
            const int at = a / KG_ROWS, r = a % KG_ROWS;
            const int per = nbc_uu + nbc_uf;            // partials per latent
            for (int b = j; b < L * per; b += GR_LANES) {
                const int l = b / per, bc = b % per;
                s += (bc < nbc_uu) ? gz_uu[(((long)l * nb_uu + at * nbc_uu + bc) * KG_ROWS + r) * D + d]
                                   : gz_uf[(((long)l * nb_uf + at * nbc_uf + (bc - nbc_uu)) * KG_ROWS + r) * D + d];
            }
        }
    } else if (tid == nth + m * (D + 1)) {
        for (int i = j; i < nnoise; i += GR_LANES) s += gnoise_part[i];
    }
#pragma unroll
    for (int o = 1; o < GR_LANES; o <<= 1) s += __shfl_xor(s, o, 64);
    if (j != 0) return;
    if (tid < nth) gtheta[tid] = s + gth_kff[tid];
    else if (tid < nth + m * (D + 1)) gZ[tid - nth] = s;
    else if (tid == nth + m * (D + 1)) gnoise[0] = s;
    (void)n_at;
}

// ---------------------------------------------------------------- driver
struct SvgpGradLayout {
    double *qm, *alpha, *beta, *A, *B, *gA, *Gb, *H, *P, *Sig, *Kbar, *T1, *gLq, *gqm, *r, *gnp, *gth_uu, *gth_uf,
        *gth_kff, *gz_uu, *gz_uf;
    int nbc_uu, nbc_uf, n_at, nb_uu, nb_uf, nnoise;
    size_t bytes;
};

static SvgpGradLayout grad_layout(int nb, int n, int m, int L, int p, int d, size_t base_off, void* ws) {
    SvgpGradLayout g;
    const int mpad = cdv(m, nb) * nb, npad = cdv(n, nb) * nb;
    const size_t mm = (size_t)mpad * mpad;
    const int G = theta_size(d);
    g.n_at = cdv(m, KG_ROWS);
    g.nbc_uu = cdv(m, KG_COLS);
    g.nbc_uf = cdv(n, KG_COLS);
    g.nb_uu = g.n_at * g.nbc_uu;
    g.nb_uf = g.n_at * g.nbc_uf;
    g.nnoise = 256;
    size_t off = base_off;
    char* base = (char*)ws;
    auto take = [&](size_t count) {
        off = (off + 255) & ~(size_t)255;
        double* ptr = base ? reinterpret_cast<double*>(base + off) : nullptr;
        off += count * sizeof(double);
        return ptr;
    };
    g.qm = take((size_t)L * mpad);
    g.alpha = take((size_t)L * npad);
    g.beta = take((size_t)L * npad);
    g.gqm = take((size_t)L * mpad);
    g.Gb = take(mm * L);
    g.H = take(mm * L);
    g.P = take(mm * L);
    g.Sig = take(mm * L);
    g.T1 = take(mm * L);
    g.A = take((size_t)mpad * npad * L);
    g.B = take((size_t)mpad * npad * L);
    g.gA = take((size_t)mpad * npad * L);
    g.gLq = take(mm * L);
    g.Kbar = take((size_t)mpad * npad * L);
    g.r = take((size_t)n * p + 8);
    g.gnp = take(g.nnoise);
    g.gth_uu = take((size_t)L * g.nb_uu * G);
    g.gth_uf = take((size_t)L * g.nb_uf * G);
    g.gth_kff = take((size_t)L * G);
    g.gz_uu = take((size_t)L * g.nb_uu * KG_ROWS * d + 8);
    g.gz_uf = take((size_t)L * g.nb_uf * KG_ROWS * d + 8);
    g.bytes = off + 256;
    return g;
}

size_t svgp_workspace_bytes(int nb, int n, int m, int l, int p, int d);

size_t svgp_grad_workspace_bytes(int nb, int n, int m, int l, int p, int d) {
    return grad_layout(nb, n, m, l, p, d, svgp_workspace_bytes(nb, n, m, l, p, d), nullptr).bytes;
}

int svgp_elbo_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx,
                   const double* Y, int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                   const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                   size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info, const double* noise_dev);
int svgp_elbo_keep_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx,
                        const double* Y, int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                        const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                        size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info, const double* noise_dev,
                        double* Aout, double* Bout);
int svgp_predict_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* Xs, int ldx,
                      const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                      const double* W, double jitter, void* ws, size_t ws_bytes, double* g_mu, double* g_var,
                      double* f_mu, double* f_var, int* info);
// forward intermediates of svgp_run (mfgp_svgp.hip)
void svgp_forward_buffers(int nb, int n, int m, int l, int p, int d, void* ws, double** Xo, double** C, double** Kuf,
                          double** Lq, int* mpad, int* npad);

template <int DC>
static void launch_kgrad(hipStream_t s, const double* P1, long ld1, int n1, const double* P2, long ld2, int n2,
                         const double* Wt, long ldw, long sW, const double* thetas, int G, int D, double zf, int nat,
                         int nbc, int L, double* gth, double* gz) {
    // the nbc = ceil(n2 / KG_COLS) column blocks of a row tile cut EQUAL (to a multiple of KG_CHUNK):
    // K_uu's 300 columns as 160 + 140, not 256 + 44 (the long blocks set the (Z, Z) sums' length)
    const int cpb = std::min(KG_COLS, cdv(cdv(n2, nbc), KG_CHUNK) * KG_CHUNK);
    hipLaunchKernelGGL(k_kgrad<DC>, dim3(nat * nbc, 1, L), dim3(NTHREADS), 0, s, P1, ld1, n1, P2, ld2, n2, Wt, ldw,
                       sW, thetas, G, D, zf, nbc, MFGP_KG_EQUAL ? cpb : KG_COLS, gth, gz);
}

template <int NB>
static int svgp_grad_run(hipStream_t s, int n, int m, int L, int p, int d, const double* X, int ldx, const double* Y,
                         int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                         const double* q_sqrt, const double* W, const double* noise_dev, double scale, double jitter,
                         void* ws, size_t ws_bytes, double* out, double* g_mu, double* g_var, double* gZ,
                         double* gtheta, double* gq_mu, double* gq_sqrt, double* gW, double* gnoise, int* info,
                         double noise_host, double kl_mult) {
    const size_t base = svgp_workspace_bytes(NB, n, m, L, p, d);
    const SvgpGradLayout g = grad_layout(NB, n, m, L, p, d, base, ws);
    if (ws_bytes < g.bytes) return -2;
    // forward (fills Xo = Li, C = Lq^T Li, Kuf, Lq, A, B; g_mu / g_var; out = [elbo, KL, VE])
    int rc = svgp_elbo_keep_impl(s, NB, n, m, L, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise_host,
                                 scale, jitter, ws, ws_bytes, out, g_mu, g_var, info, noise_dev, g.A, g.B);
    if (rc) return rc;
    double *Li, *C, *Kuf, *Lq;
    int mpad, npad;
    svgp_forward_buffers(NB, n, m, L, p, d, ws, &Li, &C, &Kuf, &Lq, &mpad, &npad);
    const int Tm = mpad / NB, Tn = npad / NB;
    const long mm = (long)mpad * mpad, mn = (long)mpad * npad;
    const int G = theta_size(d);
    // 1. VE backward
    hipLaunchKernelGGL(k_ve_bwd, dim3(g.nnoise), dim3(NTHREADS), 0, s, g_mu, g_var, W, Y, (long)ldy, n, p, L,
                       noise_dev, scale, npad, g.r, g.alpha, g.beta, g.gnp);
    hipLaunchKernelGGL(k_ab, dim3(cdv(npad, 256), 1, L), dim3(256), 0, s, g.r, W, n, p, L, noise_dev, scale, npad,
                       g.alpha, g.beta);
    if (W) hipLaunchKernelGGL(k_gw, dim3(cdv(p * L, NTHREADS / 64)), dim3(NTHREADS), 0, s, g.r, g_mu, g_var, W, n, p, L,
                              noise_dev, scale, gW);
    hipLaunchKernelGGL(k_qmu_pad, dim3(cdv(mpad, 256), 1, L), dim3(256), 0, s, q_mu, m, L, mpad, g.qm);
    // Two branches after gA (ONE fork, one join): the side takes dE/dm, dE/dLq, Kbar -> the (Z, X)
    // derivative sums and the K_diag term; the caller's stream Gb -> Sigma_bar -> the (Z, Z) sums.
    // (Forking before gA to run dE/dm / dE/dLq beside it, then handing Kbar to the side after gA
    // with a second edge, measured 2.11 ms alone but 2.76 in a process holding more streams than
    // the 4 hardware queues: that graph's cross-queue waits stalled ~40 us at a time; this one
    // edge pair: 2.15 -> 2.08 alone, 2.18 -> 2.09 in the default bench process.)
    // 3. gA = (2 Lq B - 2 A) diag(beta) + m alpha^T
    {
        BgemmArgs a{};
        a.amask = 1;   // Lq lower
        a.A = Lq; a.lda = mpad; a.sA = mm;
        a.B = g.B; a.ldb = npad; a.sB = mn;
        a.Cin = g.A; a.ldc = npad; a.sC = mn; a.beta = -2.0;
        a.colscale = g.beta; a.scs = npad;
        a.x = g.qm; a.sx = mpad; a.y = g.alpha; a.sy = npad;
        a.D = g.gA; a.ldd = npad; a.sD = mn;
        a.alpha = 2.0;
        a.Mt = Tm; a.Nt = Tn; a.Kt = Tm;
        bgemm<NB>(s, 0, 0, a, L);
    }
    hipStream_t sb = svgp_fork(s);
    // 2. dE/dm = A alpha - m  (folding its row products into step 3's epilogue, which reads A as
    //    Cin, measured slower: +45 us there and an 18 us partial reduction against this 51 us pass)
    hipLaunchKernelGGL(k_bmatvec, dim3(cdv(mpad, NTHREADS / 64), 1, L), dim3(NTHREADS), 0, sb, g.A, (long)npad, mn, 0,
                       g.alpha, (long)npad, mpad, npad, 1.0, g.qm, (long)mpad, -kl_mult, g.gqm, (long)mpad);
    hipLaunchKernelGGL(k_qmu_unpad, dim3(cdv(m, 256), 1, L), dim3(256), 0, sb, g.gqm, m, L, mpad, gq_mu);
    // 7. dE/dLq = tril(2 A diag(beta) B^T) - Lq + diag(1/Lq_ii)
    {
        BgemmArgs a{};
        a.A = g.A; a.lda = npad; a.sA = mn;
        a.B = g.B; a.ldb = npad; a.sB = mn;
        a.s = g.beta; a.ss = npad;
        a.D = g.gLq; a.ldd = mpad; a.sD = mm;
        a.alpha = 2.0;
        a.Mt = Tm; a.Nt = Tm; a.Kt = Tn; a.tril = 1;
        bgemm<NB>(sb, 0, 1, a, L);
    }
    // 6. Kbar = dE/dKuf = Li^T gA (side)
    {
        BgemmArgs a{};
        a.amask = 2;   // Li^T upper
        a.A = Li; a.lda = mpad; a.sA = mm;
        a.B = g.gA; a.ldb = npad; a.sB = mn;
        a.D = g.Kbar; a.ldd = npad; a.sD = mn;
        a.alpha = 1.0;
        a.Mt = Tm; a.Nt = Tn; a.Kt = Tm;
        bgemm<NB>(sb, 1, 0, a, L);
    }
    // 4. dE/dLi = tril(gA Kuf^T)
    {
        BgemmArgs a{};
        a.A = g.gA; a.lda = npad; a.sA = mn;
        a.B = Kuf; a.ldb = npad; a.sB = mn;
        a.D = g.Gb; a.ldd = mpad; a.sD = mm;
        a.alpha = 1.0;
        a.Mt = Tm; a.Nt = Tm; a.Kt = Tn; a.tril = 1;
        bgemm<NB>(s, 0, 1, a, L);
    }
    // 5. Sigma_bar = -Li^T Psi(Gb Li^T) Li
    //    (NB = 32: Psi in the first product's epilogue, only its lower tiles formed)
    if (NB == 32) {
        BgemmArgs a{};
        a.amask = 1; a.bmask = 2;   // Gb lower, Li^T upper
        a.A = g.Gb; a.lda = mpad; a.sA = mm;
        a.B = Li; a.ldb = mpad; a.sB = mm;
        a.D = g.P; a.ldd = mpad; a.sD = mm;
        a.alpha = 1.0;
        a.Mt = Tm; a.Nt = Tm; a.Kt = Tm; a.tril = 1; a.sym = 1;
        bgemm<NB>(s, 0, 1, a, L);
    } else {
        sq<NB>(s, Tm, L, mm, mpad, 0, g.Gb, 1, Li, g.H, 1.0, nullptr, 0.0, 0, nullptr, nullptr, 0, 1, 2);   // Gb lower, Li^T upper
        hipLaunchKernelGGL(k_psi, dim3(std::min<long>(cdv((int)mm, 256), 1024), 1, L), dim3(256), 0, s, g.H, g.P, mpad,
                           mm);
    }
    sq<NB>(s, Tm, L, mm, mpad, 0, g.P, 0, Li, g.T1, 1.0, nullptr, 0.0, 0, nullptr, nullptr, 0, 0, 1);   // Li lower
    if (NB == 32) {   // Sigma_bar is symmetric: its lower tiles (the cheap ones under Li^T's mask), mirrored
        BgemmArgs a{};
        a.amask = 2;   // Li^T upper
        a.A = Li; a.lda = mpad; a.sA = mm;
        a.B = g.T1; a.ldb = mpad; a.sB = mm;
        a.D = g.Sig; a.ldd = mpad; a.sD = mm;
        a.alpha = -1.0;
        a.Mt = Tm; a.Nt = Tm; a.Kt = Tm; a.tril = 1; a.sym = 2;
        bgemm<NB>(s, 1, 0, a, L);
    } else {
        sq<NB>(s, Tm, L, mm, mpad, 1, Li, 0, g.T1, g.Sig, -1.0, nullptr, 0.0, 0, nullptr, nullptr, 0, 2, 0);   // Li^T upper
    }
    // 8. kernel / inducing-point derivative sums: (Z, X) on the side, (Z, Z) here
    // compile-time bound on d: the per-dimension accumulators stay in registers
    auto kgrad = [&](auto dc) {
        constexpr int DC = decltype(dc)::value;
        launch_kgrad<DC>(sb, Z, ldz, m, X, ldx, n, g.Kbar, npad, mn, thetas, G, d, 1.0, g.n_at, g.nbc_uf, L, g.gth_uf,
                         g.gz_uf);
        launch_kgrad<DC>(s, Z, ldz, m, Z, ldz, m, g.Sig, mpad, mm, thetas, G, d, 2.0, g.n_at, g.nbc_uu, L, g.gth_uu,
                         g.gz_uu);
    };
    if (d <= 4) kgrad(std::integral_constant<int, 4>{});
    else if (d <= 8) kgrad(std::integral_constant<int, 8>{});
    else if (d <= 12) kgrad(std::integral_constant<int, 12>{});
    else if (d <= 16) kgrad(std::integral_constant<int, 16>{});
    else kgrad(std::integral_constant<int, 32>{});
    // the side's short tail
    hipLaunchKernelGGL(k_glq_final, dim3(std::min(cdv(m * m, 256), 1024), 1, L), dim3(256), 0, sb, g.gLq, Lq, m, mpad,
                       mm, kl_mult, gq_sqrt, svgp_side().qs_packed);
    hipLaunchKernelGGL(k_kff_grad, dim3(L), dim3(NTHREADS), 0, sb, X, (long)ldx, n, g.beta, npad, thetas, G, d,
                       g.gth_kff);
    svgp_join(s);
    const int tot = L * G + m * (d + 1) + 1;
    hipLaunchKernelGGL(k_grad_reduce, dim3(cdv(tot * GR_LANES, 256)), dim3(256), 0, s, g.gth_uu, g.nb_uu, g.gth_uf, g.nb_uf,
                       g.gth_kff, g.gz_uu, g.gz_uf, g.n_at, g.nbc_uu, g.nbc_uf, L, G, d, m, g.gnp, g.nnoise, gtheta,
                       gZ, gnoise);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int svgp_grad_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx, const double* Y,
                   int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                   const double* W, const double* noise_dev, double noise_host, double scale, double kl_mult,
                   double jitter, void* ws, size_t ws_bytes, double* out, double* g_mu, double* g_var, double* gZ,
                   double* gtheta, double* gq_mu, double* gq_sqrt, double* gW, double* gnoise, int* info) {
    if (nb == 64)
        return svgp_grad_run<64>(s, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise_dev, scale,
                                 jitter, ws, ws_bytes, out, g_mu, g_var, gZ, gtheta, gq_mu, gq_sqrt, gW, gnoise, info,
                                 noise_host, kl_mult);
    return svgp_grad_run<32>(s, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise_dev, scale,
                             jitter, ws, ws_bytes, out, g_mu, g_var, gZ, gtheta, gq_mu, gq_sqrt, gW, gnoise, info,
                             noise_host, kl_mult);
}

// ---------------------------------------------------------------- predict with covariances
// GPflow SVGP.predict_f(Xnew, full_cov, full_output_cov) beyond the diagonal
// (posteriors.IndependentPosteriorMultiOutput -> base_conditional_with_lm(full_cov=True, white)
// per latent, then mix_latent_gp): G_l = Knn_l - A^T A + (Lq^T A)^T (Lq^T A), A = Li Kuf,
// written as G_l = Knn_l + Kuf^T F Kuf with F = C^T C - Li^T Li (C = Lq^T Li) -- the same F the
// ELBO gradient forms.  Mixing (W = NULL: independent outputs, P = L):
//   mode 1 full_cov            f_cov[p][a][b]    = sum_l W_pl^2 G_l[a][b]
//   mode 2 full_output_cov     f_cov[a][p][q]    = sum_l W_pl W_ql g_var[l][a]
//   mode 3 both                f_cov[a][p][b][q] = sum_l W_pl W_ql G_l[a][b]
__global__ void k_svgp_mix_cov(int mode, int ns, int p, int L, const double* W, const double* g_var, const double* G,
                               long ldg, long sG, double* out) {
    const long nn = (long)ns * ns, pp2 = (long)p * p;
    const long tot = mode == 1 ? p * nn : (mode == 2 ? ns * pp2 : nn * pp2);
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
        int a, b, pa, qa;
        if (mode == 1) {
            pa = (int)(e / nn);
            const long r = e % nn;
            a = (int)(r / ns); b = (int)(r % ns); qa = pa;
        } else if (mode == 2) {
            a = (int)(e / pp2);
            const long r = e % pp2;
            pa = (int)(r / p); qa = (int)(r % p); b = a;
        } else {   // [a][pa][b][qa]
            long r = e;
            qa = (int)(r % p); r /= p;
            b = (int)(r % ns); r /= ns;
            pa = (int)(r % p); a = (int)(r / p);
        }
        double v = 0.0;
        if (!W) {
            if (pa == qa) v = (mode == 2) ? g_var[(long)pa * ns + a] : G[pa * sG + a * ldg + b];
        } else {
            for (int l = 0; l < L; ++l) {
                const double w = W[(long)pa * L + l] * W[(long)qa * L + l];
                v = fma(w, (mode == 2) ? g_var[(long)l * ns + a] : G[l * sG + a * ldg + b], v);
            }
        }
        out[e] = v;
    }
}

static size_t pcov_extra(int nb, int ns, int m, int L) {
    const size_t mpad = (size_t)cdv(m, nb) * nb, npad = (size_t)cdv(ns, nb) * nb;
    return sizeof(double) * L * (2 * mpad * mpad + mpad * npad + 2 * npad * npad) + 5 * 256;
}

size_t svgp_predict_cov_workspace_bytes(int nb, int ns, int m, int l, int p, int d) {
    return svgp_workspace_bytes(nb, ns, m, l, p, d) + pcov_extra(nb, ns, m, l) + 256;
}

template <int NB>
static int svgp_predict_cov_run(hipStream_t s, int mode, int ns, int m, int L, int p, int d, const double* Xs,
                                int ldx, const double* Z, int ldz, const double* thetas, const double* q_mu,
                                const double* q_sqrt, const double* W, double jitter, void* ws, size_t ws_bytes,
                                double* g_mu, double* g_var, double* f_mu, double* f_var, double* f_cov, int* info) {
    if (ws_bytes < svgp_predict_cov_workspace_bytes(NB, ns, m, L, p, d)) return -2;
    int rc = svgp_predict_impl(s, NB, ns, m, L, p, d, Xs, ldx, Z, ldz, thetas, q_mu, q_sqrt, W, jitter, ws, ws_bytes,
                               g_mu, g_var, f_mu, f_var, info);
    if (rc) return rc;
    double *Li, *C, *Kuf, *Lq;
    int mpad, npad;
    svgp_forward_buffers(NB, ns, m, L, p, d, ws, &Li, &C, &Kuf, &Lq, &mpad, &npad);
    const int Tm = mpad / NB, Tn = npad / NB;
    const long mm = (long)mpad * mpad, mn = (long)mpad * npad, nn = (long)npad * npad;
    size_t off = (svgp_workspace_bytes(NB, ns, m, L, p, d) + 255) & ~(size_t)255;
    auto take = [&](size_t count) {
        off = (off + 255) & ~(size_t)255;
        double* q = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + off);
        off += count * sizeof(double);
        return q;
    };
    double* F1 = take((size_t)L * mm);
    double* F = take((size_t)L * mm);
    double* Tk = take((size_t)L * mn);
    double* Knn = take((size_t)L * nn);
    double* G = take((size_t)L * nn);
    if (mode != 2) {
        sq<NB>(s, Tm, L, mm, mpad, 1, C, 0, C, F1);                   // C^T C
        sq<NB>(s, Tm, L, mm, mpad, 1, Li, 0, Li, F, -1.0, F1, 1.0, 0, nullptr, nullptr, 0, 2, 1);   // F = C^T C - Li^T Li
        {
            BgemmArgs a{};
            a.A = F; a.lda = mpad; a.sA = mm;
            a.B = Kuf; a.ldb = npad; a.sB = mn;
            a.D = Tk; a.ldd = npad; a.sD = mn;
            a.alpha = 1.0;
            a.Mt = Tm; a.Nt = Tn; a.Kt = Tm;
            bgemm<NB>(s, 0, 0, a, L);                                 // F Kuf
        }
        GramArgs g{};
        g.X1 = Xs; g.ldx1 = ldx; g.sx1 = 0; g.n1 = ns;
        g.X2 = Xs; g.ldx2 = ldx; g.sx2 = 0; g.n2 = ns;
        g.theta = thetas; g.stheta = theta_size(d); g.D = d; g.rbf_only = 0;
        g.out = Knn; g.ldo = npad; g.so = nn; g.padded = 0; g.diag_add = 0.0;
        launch_gram_dense(g, L, npad, npad, s);                       // Knn_l (GPflow adds no jitter)
        {
            BgemmArgs a{};
            a.A = Kuf; a.lda = npad; a.sA = mn;
            a.B = Tk; a.ldb = npad; a.sB = mn;
            a.Cin = Knn; a.ldc = npad; a.sC = nn; a.beta = 1.0;
            a.D = G; a.ldd = npad; a.sD = nn;
            a.alpha = 1.0;
            a.Mt = Tn; a.Nt = Tn; a.Kt = Tm;
            bgemm<NB>(s, 1, 0, a, L);                                 // G = Knn + Kuf^T F Kuf
        }
    }
    const long tot = mode == 1 ? (long)p * ns * ns : (mode == 2 ? (long)ns * p * p : (long)ns * ns * p * p);
    hipLaunchKernelGGL(k_svgp_mix_cov, dim3((unsigned)std::min<long>(cdv((int)std::min<long>(tot, 1L << 30), 256), 4096)),
                       dim3(256), 0, s, mode, ns, p, L, W, g_var, G, (long)npad, nn, f_cov);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int svgp_predict_cov_impl(hipStream_t s, int nb, int mode, int ns, int m, int l, int p, int d, const double* Xs,
                          int ldx, const double* Z, int ldz, const double* thetas, const double* q_mu,
                          const double* q_sqrt, const double* W, double jitter, void* ws, size_t ws_bytes,
                          double* g_mu, double* g_var, double* f_mu, double* f_var, double* f_cov, int* info) {
    if (nb == 64)
        return svgp_predict_cov_run<64>(s, mode, ns, m, l, p, d, Xs, ldx, Z, ldz, thetas, q_mu, q_sqrt, W, jitter, ws,
                                        ws_bytes, g_mu, g_var, f_mu, f_var, f_cov, info);
    return svgp_predict_cov_run<32>(s, mode, ns, m, l, p, d, Xs, ldx, Z, ldz, thetas, q_mu, q_sqrt, W, jitter, ws,
                                    ws_bytes, g_mu, g_var, f_mu, f_var, f_cov, info);
}

// ---------------------------------------------------------------- packed Adam (training step)
// One Keras-2.10 (legacy) Adam step on a packed parameter vector: u unconstrained,
// c constrained (c = u, softplus(u) or softplus(u) + 1e-6 by transform[q] = 0 / 1 / 2),
// g = d(+objective)/dc  (the loss is its negative), learning rate lr_sched[*step].
// TF's SoftplusGrad division form g / (exp(-u) + 1) carries the gradient to u.
__global__ void k_adam_packed(int n, double* u, double* c, const double* g, double* m, double* v,
                              const unsigned char* trainable, const unsigned char* transform,
                              const unsigned char* span, const int* step, const double* lr_sched, double b1,
                              double b2, double eps, const int* info, int ninfo) {
    // once a block: the info gate (a failed evaluation: no update, the step counter stays) and
    // the step size (two pow)
    __shared__ double s_alpha;
    __shared__ int s_ok;
    if (threadIdx.x < 64) {   // wave 0: the info words a lane each (one round trip, not ninfo)
        int bad = 0;
        for (int i = threadIdx.x; i < ninfo; i += 64) bad |= info[i] != 0;
        const bool ok = __ballot(bad) == 0;
        if (threadIdx.x == 0) {
            const int s = *step;
            const double t = (double)(s + 1);
            s_alpha = lr_sched[s] * sqrt(1.0 - pow(b2, t)) / (1.0 - pow(b1, t));
            s_ok = ok ? 1 : 0;
        }
    }
    __syncthreads();
    if (!s_ok) return;
    const double alpha = s_alpha;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        const int k = span ? span[q] : 1;   // 0: follower of a tied variable (written by its leader)
        if (!trainable[q] || k == 0) continue;
        const int tr = transform[q];
        const double uq = u[q];
        double gc = 0.0;
        for (int j = 0; j < k; ++j) gc += g[q + j];
        const double gl = -gc;   // d loss / d c
        double gu;
        if (tr == 0) gu = gl;
        else if (tr == 3) {   // tfp Sigmoid: SigmoidGrad dy * y * (1 - y)
            const double y = 1.0 / (1.0 + exp(-uq));
            gu = gl * y * (1.0 - y);
        } else gu = gl / (exp(-uq) + 1.0);   // Softplus: TF SoftplusGrad form
        const double mq = m[q] + (gu - m[q]) * (1.0 - b1);
        const double vq = v[q] + (gu * gu - v[q]) * (1.0 - b2);
        const double un = uq - (mq * alpha) / (sqrt(vq) + eps);
        const double cn = (tr == 0) ? un : (tr == 3) ? 1.0 / (1.0 + exp(-un)) : tf_softplus(un) + (tr == 2 ? 1e-6 : 0.0);
        m[q] = mq;
        v[q] = vq;
        for (int j = 0; j < k; ++j) {
            u[q + j] = un;
            c[q + j] = cn;
        }
    }
}

// loss_hist[step] = -out[0] + (klm - 1) out[1] (the optimised objective), kl_hist[step] = out[1]; ++step
// (info gate: with a nonzero info word the counter stays, so the next step rewrites this entry)
__global__ void k_step_record(const double* out, double klm, double* loss_hist, double* kl_hist, int* step,
                              const int* info, int ninfo) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int s = *step;
    if (loss_hist) loss_hist[s] = -out[0] + (klm - 1.0) * out[1];
    if (kl_hist) kl_hist[s] = out[1];
    bool ok = true;
    for (int i = 0; i < ninfo; ++i) ok = ok && info[i] == 0;
    if (ok) *step = s + 1;
}

int adam_packed_impl(hipStream_t st, int n, double* u, double* c, const double* g, double* m, double* v,
                     const unsigned char* trainable, const unsigned char* transform, const unsigned char* span,
                     int* step, const double* lr_sched, double b1, double b2, double eps, const double* out,
                     double klm, double* loss_hist, double* kl_hist, const int* info, int ninfo) {
    if (!info) ninfo = 0;
    // 2.9M parameters at Goku single-bin (q_sqrt): up to four elements a thread (with the info
    // gate and the step size once a block, not once a thread: 60 us at 1024 blocks before)
    hipLaunchKernelGGL(k_adam_packed, dim3(std::min(cdv(n, 1024), 16384)), dim3(256), 0, st, n, u, c, g, m, v, trainable,
                       transform, span, step, lr_sched, b1, b2, eps, info, ninfo);
    hipLaunchKernelGGL(k_step_record, dim3(1), dim3(64), 0, st, out, klm, loss_hist, kl_hist, step, info, ninfo);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace mfgp
