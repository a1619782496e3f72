// SVGP hot path (value): batched K_uu factor, the K_uf K_uu^{-1} products of the
// whitened conditional, output mixing, Gaussian variational expectations and KL.
//
// Reference: mfgpflow/linear_svgp.py:64-203 (LinearCoregionalization over L
// per-latent LinearMultiFidelityKernels, SharedIndependentInducingVariables,
// whiten=True) and mfgpflow/singlebin_svgp.py:13-97 (SeparateIndependent, W = I),
// both through GPflow 2.9 SVGP.elbo -> posteriors / base_conditional_with_lm /
// gauss_kl / Gaussian.variational_expectations.
//
// Per latent l:  Lm = chol(Kuu_l),  A = Lm^{-1} Kuf_l,  B = tril(q_sqrt_l)^T A,
//   g_mu = A^T q_mu[:, l],  g_var = Kff_l - colsum(A^2) + colsum(B^2).
// B is formed as (Lq^T Lm^{-1}) Kuf so that A and B come out of ONE fused tile
// loop over Kuf (K6 below); they are written to HBM only for the gradient pass
// (mfgp_svgp_grad.hip re-associates its adjoints around them).
#include "mfgp_device.h"
#include "mfgp_internal.h"

namespace mfgp {

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

static thread_local SvgpSide t_side{nullptr, nullptr, nullptr};
void svgp_set_side(const SvgpSide& sd) { t_side = sd; }
const SvgpSide& svgp_side() { return t_side; }
hipStream_t svgp_fork(hipStream_t s) {
    if (!t_side.side || !t_side.fork || !t_side.join) return s;
    (void)hipEventRecord(t_side.fork, s);
    (void)hipStreamWaitEvent(t_side.side, t_side.fork, 0);
    return t_side.side;
}
void svgp_join(hipStream_t s) {
    if (!t_side.side || !t_side.fork || !t_side.join) return;
    (void)hipEventRecord(t_side.join, t_side.side);
    (void)hipStreamWaitEvent(s, t_side.join, 0);
}


struct SvgpLayout {
    int nb, Tm, mpad, Tn, npad, G;
    double *Kuu, *R, *Xo, *Dd, *ldiag, *Lq, *C, *Kuf, *pa, *pb, *pm, *ve_part, *kl_part;
    size_t bytes;
};

static SvgpLayout svgp_layout(int nb, int n, int m, int l, int p, int d, void* ws) {
    SvgpLayout S;
    S.nb = nb;
    S.Tm = cdiv(m, nb);
    S.mpad = S.Tm * nb;
    S.Tn = cdiv(n, nb);
    S.npad = S.Tn * nb;
    S.G = theta_size(d);
    const size_t mm = (size_t)S.mpad * S.mpad;
    size_t off = 0;
    char* base = (char*)ws;
    auto take = [&](size_t count) {
        off = (off + 255) & ~(size_t)255;
        double* ptr = base ? reinterpret_cast<double*>(base + off) : nullptr;
        off += count * sizeof(double);
        return ptr;
    };
    S.Kuu = take(mm * l);
    S.R = take(mm * l);
    S.Xo = take(mm * l);
    S.Dd = take((size_t)S.Tm * nb * nb * l);
    S.ldiag = take((size_t)S.mpad * l);
    S.Lq = take(mm * l);
    S.C = take(mm * l);
    S.Kuf = take((size_t)S.mpad * S.npad * l);
    S.pa = take((size_t)l * S.Tm * S.npad);
    S.pb = take((size_t)l * S.Tm * S.npad);
    S.pm = take((size_t)l * S.Tm * S.npad);
    S.ve_part = take(1024);
    S.kl_part = take((size_t)l * 8 + 8);   // KL_SLICES partials per latent
    S.bytes = off + 256;
    return S;
}

size_t svgp_workspace_bytes(int nb, int n, int m, int l, int p, int d) {
    return svgp_layout(nb, n, m, l, p, d, nullptr).bytes;
}

// forward intermediates for the gradient pass (mfgp_svgp_grad.hip)
void svgp_forward_buffers(int nb, int n, int m, int l, int p, int d, void* ws, double** Xo, double** C, double** Kuf,
                          double** Lq, int* mpad, int* npad) {
    const SvgpLayout S = svgp_layout(nb, n, m, l, p, d, ws);
    *Xo = S.Xo;
    *C = S.C;
    *Kuf = S.Kuf;
    *Lq = S.Lq;
    *mpad = S.mpad;
    *npad = S.npad;
}

// Zeros in the strictly-upper tiles of L^{-1} (the step sequence writes only tiles (i, c <= i)):
// the matvecs and the E = Lq C - Li input read whole rows of it.  One workgroup per 8 rows, 16-B
// stores of each row's part right of its tile (a thread per element with a division by mpad took
// 23 us for 64 latents, beside the K_uu chain on the critical path).
constexpr int ZU_ROWS = 8;
__global__ void k_zero_upper_tiles(double* Xo, int nb, int mpad, long mm) {
    const int l = blockIdx.z;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int rr = w; rr < ZU_ROWS; rr += blockDim.x >> 6) {   // a wave per row
        const int r = blockIdx.x * ZU_ROWS + rr;
        if (r >= mpad) break;
        const int c0 = (r / nb + 1) * nb;                      // first column right of the tile (even)
        double* row = Xo + l * mm + (long)r * mpad;
        for (int c = c0 + 2 * lane; c < mpad; c += 128)
            *reinterpret_cast<f64x2*>(row + c) = f64x2{0.0, 0.0};
    }
}

// tril(q_sqrt_l) into a zero-padded Mpad x Mpad buffer (packed: q_sqrt_l as its lower triangle,
// (r, c <= r) at r (r + 1) / 2 + c).  A wave per row: its packed segment read in order, the row
// written in order (16-B stores; the per-element form with two divisions took 33 us for 64 latents)
__global__ void k_lq_pad(const double* q_sqrt, int m, int mpad, double* Lq, int packed) {
    const int l = blockIdx.z;
    const long tot = (long)mpad * mpad, tri = (long)m * (m + 1) / 2;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int rr = w; rr < ZU_ROWS; rr += blockDim.x >> 6) {
        const int r = blockIdx.x * ZU_ROWS + rr;
        if (r >= mpad) break;
        const double* src = (r < m) ? (packed ? q_sqrt + l * tri + (long)r * (r + 1) / 2 : q_sqrt + (long)l * m * m + (long)r * m)
                                    : nullptr;
        double* row = Lq + l * tot + (long)r * mpad;
        for (int c = 2 * lane; c < mpad; c += 128) {
            f64x2 v = {0.0, 0.0};
            if (src && c <= r) v.x = src[c];
            if (src && c + 1 <= r) v.y = src[c + 1];
            *reinterpret_cast<f64x2*>(row + c) = v;
        }
    }
}

// C_l = Lq_l^T Linv_l  (tile (i, j): sum over m >= max(i, j))
template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_lqt_linv(const double* Lq, const double* Xo, double* C, int Tm) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* As = smem;
    double* Bs = As + E;
    int bx, l;
    xcd_swizzle(bx, l);
    const int i = bx / Tm, j = bx % Tm;
    const long mp = (long)Tm * NB, mm = mp * mp;
    const double* lq = Lq + l * mm;
    const double* xo = Xo + l * mm;
    Acc<NB> acc;
    acc_zero(acc);
    for (int mt = max(i, j); mt < Tm; ++mt) {
        tile_load<NB>(As, lq + (long)mt * NB * mp + (long)i * NB, mp);
        tile_load<NB>(Bs, xo + (long)mt * NB * mp + (long)j * NB, mp);
        __syncthreads();
        tile_mma<NB, true, false>(acc, As, Bs, 1.0);
        __syncthreads();
    }
    acc_store(acc, C + l * mm + (long)i * NB * mp + (long)j * NB, mp);
}

// Fused conditional: task (l, i, tn): A_i = sum_{m<=i} Linv_im Kuf_m ; B_i = sum_m C_im Kuf_m
template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_svgp_cond(const double* Xo, const double* C, const double* Kuf,
                                                        const double* q_mu, int L, int m, int Tm, int npad,
                                                        double* pa, double* pb, double* pm, double* Aout,
                                                        double* Bout) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Ls = smem;
    double* Ks = Ls + E;
    double* As = Ks + E;
    double* red = As + E;   // 3 x 4 x NB
    int bx, l;
    xcd_swizzle(bx, l);
    const int Tn = npad / NB;
    const int i = bx / Tn, tn = bx % Tn;
    const long mp = (long)Tm * NB, mm = mp * mp;
    const double* xo = Xo + l * mm;
    const double* cc = C + l * mm;
    const double* kuf = Kuf + (long)l * mp * npad;
    Acc<NB> accA, accB;
    acc_zero(accA);
    acc_zero(accB);
    for (int mt = 0; mt < Tm; ++mt) {
        tile_load<NB>(Ks, kuf + (long)mt * NB * npad + (long)tn * NB, npad);
        if (mt <= i) tile_load<NB>(Ls, xo + (long)i * NB * mp + (long)mt * NB, mp);
        tile_load<NB>(As, cc + (long)i * NB * mp + (long)mt * NB, mp);
        __syncthreads();
        if (mt <= i) tile_mma<NB, false, false>(accA, Ls, Ks, 1.0);
        tile_mma<NB, false, false>(accB, As, Ks, 1.0);
        __syncthreads();
    }
    if (Aout) {   // gradient pass: keep A and B (L x Mpad x Npad each)
        const long o = (long)l * mp * npad + (long)i * NB * npad + (long)tn * NB;
        acc_store(accA, Aout + o, npad);
        acc_store(accB, Bout + o, npad);
    }
    // column reductions: thread owns (row, col) elements; reduce over rows via LDS
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double qm[TileCfg<NB>::NBLK * 4];
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int gr = i * NB + acc_row<NB>(q, r);
            qm[q * 4 + r] = (gr < m) ? q_mu[(long)gr * L + l] : 0.0;
        }
    // per-thread partial column sums (each thread owns NBLK distinct columns)
    for (int e = threadIdx.x; e < 3 * 4 * NB; e += NTHREADS) red[e] = 0.0;
    __syncthreads();
    // each column is shared by 4 lane-groups x (wave row halves); accumulate with LDS atomics-free passes
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q) {
        double sa = 0.0, sb = 0.0, sm = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double a = accA.v[q][r], b = accB.v[q][r];
            sa += a * a;
            sb += b * b;
            sm += a * qm[q * 4 + r];
        }
        // lanes l, l+16, l+32, l+48 share a column: reduce across lane>>4
        sa += __shfl_xor(sa, 16, 64); sa += __shfl_xor(sa, 32, 64);
        sb += __shfl_xor(sb, 16, 64); sb += __shfl_xor(sb, 32, 64);
        sm += __shfl_xor(sm, 16, 64); sm += __shfl_xor(sm, 32, 64);
        if (lane < 16) {
            // waves w and w^2 share columns (w>>1 selects the row half)
            const int col = acc_col<NB>(q);
            const int slot = (w >> 1);
            red[(0 * 4 + slot) * NB + col] += sa;   // distinct (slot, col) per writer
            red[(1 * 4 + slot) * NB + col] += sb;
            red[(2 * 4 + slot) * NB + col] += sm;
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NB; c += NTHREADS) {
        const long o = ((long)l * Tm + i) * npad + (long)tn * NB + c;
        double sa = 0.0, sb = 0.0, sm = 0.0;
        for (int slot = 0; slot < 4; ++slot) {
            sa += red[(0 * 4 + slot) * NB + c];
            sb += red[(1 * 4 + slot) * NB + c];
            sm += red[(2 * 4 + slot) * NB + c];
        }
        pa[o] = sa;
        pb[o] = sb;
        pm[o] = sm;
    }
    (void)S;
}

// k_svgp_cond on a 64 x 64 block of (A, B) per workgroup (NB = 32 operands): wave w owns tile
// (2 bi + (w >> 1), 2 bj + (w & 1)) of both A and B as 2 x 2 independent 16 x 16 accumulators
// each; every m-step stages the two Kuf tiles, two Li tiles and two C tiles once for the four waves
// (k_svgp_cond: one Kuf, one Li, one C tile per 32 x 32 output), the next m-step's loads issued
// into registers before the current products.  Same per-block MFMA sequence and the same column
// reduction order as k_svgp_cond, so A, B and the partials are bitwise its results.
constexpr int SC2_E = 32 * 34;
size_t svgp_cond2_smem() { return 6 * sizeof(double) * (size_t)SC2_E; }

__global__ __launch_bounds__(NTHREADS) void k_svgp_cond2(const double* Xo, const double* C, const double* Kuf,
                                                        const double* q_mu, int L, int m, int Tm, int npad,
                                                        double* pa, double* pb, double* pm, double* Aout,
                                                        double* Bout) {
    constexpr int S = 34, NB = 32;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    int bx, l;
    xcd_swizzle(bx, l);
    const int Tn = npad / NB, Nb = (Tn + 1) >> 1;
    const int bi = bx / Nb, bj = bx % Nb;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ti = 2 * bi + (w >> 1), tn = 2 * bj + (w & 1);
    const bool live = ti < Tm && tn < Tn;
    const long mp = (long)Tm * NB, mm = mp * mp;
    const double* xo = Xo + l * mm;
    const double* cc = C + l * mm;
    const double* kuf = Kuf + (long)l * mp * npad;
    const int r0 = min(2 * bi, Tm - 1), r1 = min(2 * bi + 1, Tm - 1);
    const int c0 = min(2 * bj, Tn - 1), c1 = min(2 * bj + 1, Tn - 1);
    TileRegs<32> rg[6];
    auto fetch = [&](int mt) {
        tile_fetch<32>(rg[0], kuf + (long)mt * NB * npad + (long)c0 * NB, npad);
        tile_fetch<32>(rg[1], kuf + (long)mt * NB * npad + (long)c1 * NB, npad);
        tile_fetch<32>(rg[2], xo + (long)r0 * NB * mp + (long)mt * NB, mp);
        tile_fetch<32>(rg[3], xo + (long)r1 * NB * mp + (long)mt * NB, mp);
        tile_fetch<32>(rg[4], cc + (long)r0 * NB * mp + (long)mt * NB, mp);
        tile_fetch<32>(rg[5], cc + (long)r1 * NB * mp + (long)mt * NB, mp);
    };
    f64x4 accA[2][2], accB[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            accA[p][q] = f64x4{0.0, 0.0, 0.0, 0.0};
            accB[p][q] = f64x4{0.0, 0.0, 0.0, 0.0};
        }
    const double* Ks = smem + (w & 1) * SC2_E;          // Kuf(mt, tn)
    const double* Ls = smem + (2 + (w >> 1)) * SC2_E;   // Li(ti, mt)
    const double* Cs = smem + (4 + (w >> 1)) * SC2_E;   // C(ti, mt)
    fetch(0);
    for (int mt = 0; mt < Tm; ++mt) {
#pragma unroll
        for (int t = 0; t < 6; ++t) tile_put<32>(smem + t * SC2_E, rg[t]);
        if (mt + 1 < Tm) fetch(mt + 1);
        __syncthreads();
        if (live) {
            const bool doA = mt <= ti;   // Li lower
#pragma unroll 4
            for (int k0 = 0; k0 < NB; k0 += 4) {   // A: the old k_svgp_cond's first chain of the m-step
                if (!doA) break;
                const int k = k0 + lk;
                double av[2], bv[2];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    av[t] = 1.0 * Ls[(16 * t + li) * S + k];
                    bv[t] = Ks[k * S + 16 * t + li];
                }
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        accA[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[p], bv[q], accA[p][q], 0, 0, 0);
            }
#pragma unroll 4
            for (int k0 = 0; k0 < NB; k0 += 4) {
                const int k = k0 + lk;
                double av[2], bv[2];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    av[t] = 1.0 * Cs[(16 * t + li) * S + k];
                    bv[t] = Ks[k * S + 16 * t + li];
                }
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        accB[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[p], bv[q], accB[p][q], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    if (!live) return;
    if (Aout) {   // gradient pass: keep A and B (L x Mpad x Npad each)
        const long o = (long)l * mp * npad + (long)ti * NB * npad + (long)tn * NB;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const long e = o + (long)(16 * p + lk + 4 * r) * npad + 16 * q + li;
                    Aout[e] = accA[p][q][r];
                    Bout[e] = accB[p][q][r];
                }
    }
    // column partials of the tile: rows 0-15 then 16-31 (k_svgp_cond's two row-half slots)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        double ta = 0.0, tb = 0.0, tm = 0.0;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            double sa = 0.0, sb = 0.0, sm = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gr = ti * NB + 16 * p + lk + 4 * r;
                const double qm = (gr < m) ? q_mu[(long)gr * L + l] : 0.0;
                const double a = accA[p][q][r], b = accB[p][q][r];
                sa += a * a;
                sb += b * b;
                sm += a * qm;
            }
            sa += __shfl_xor(sa, 16, 64); sa += __shfl_xor(sa, 32, 64);
            sb += __shfl_xor(sb, 16, 64); sb += __shfl_xor(sb, 32, 64);
            sm += __shfl_xor(sm, 16, 64); sm += __shfl_xor(sm, 32, 64);
            ta += sa;
            tb += sb;
            tm += sm;
        }
        if (lk == 0) {
            const long o = ((long)l * Tm + ti) * npad + (long)tn * NB + 16 * q + li;
            pa[o] = ta;
            pb[o] = tb;
            pm[o] = tm;
        }
    }
}

// g_mu[l][n], g_var[l][n] from the partials (+ Kff = K_diag_l(X))
__global__ void k_svgp_moments(const double* pa, const double* pb, const double* pm, const double* X, long ldx,
                               const double* thetas, int G, int D, int n, int npad, int Tm, double* g_mu,
                               double* g_var) {
    const int l = blockIdx.z;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    double sa = 0.0, sb = 0.0, sm = 0.0;
    for (int i = 0; i < Tm; ++i) {
        const long o = ((long)l * Tm + i) * npad + c;
        sa += pa[o];
        sb += pb[o];
        sm += pm[o];
    }
    const MFTheta th{thetas + (long)l * G, D};
    const double f = X[(long)c * ldx + D];
    const double rho = th.rho();
    const double kff = (f == 0.0) ? th.vL() : ((f == 1.0) ? th.vL() * (rho * rho) + th.vD() : 0.0);
    g_mu[(long)l * n + c] = sm;
    g_var[(long)l * n + c] = kff - sa + sb;
}

// Gaussian variational expectations summed over (n, p); mixing f = g W^T, f_var = g_var (W o W)^T
__global__ __launch_bounds__(NTHREADS) void k_svgp_ve(const double* g_mu, const double* g_var, const double* W,
                                                      const double* Y, long ldy, int n, int p, int L, double noise_h,
                                                      const double* noise_dev, double* ve_part) {
    __shared__ double red[4];
    const double noise = noise_dev ? noise_dev[0] : noise_h;
    const double LOG2PI = 1.8378770664093453;
    const double c0 = -0.5 * LOG2PI - 0.5 * log(noise);
    const double inv = 1.0 / noise;
    double acc = 0.0;
    const long tot = (long)n * p;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / p), c = (int)(e % p);
        double fm, fv;
        if (W) {
            fm = 0.0;
            fv = 0.0;
            for (int l = 0; l < L; ++l) {
                const double w = W[(long)c * L + l];
                fm += g_mu[(long)l * n + r] * w;
                fv += g_var[(long)l * n + r] * (w * w);
            }
        } else {
            fm = g_mu[(long)c * n + r];
            fv = g_var[(long)c * n + r];
        }
        const double dy = Y[(long)r * ldy + c] - fm;
        acc += c0 - 0.5 * (dy * dy + fv) * inv;
    }
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) ve_part[blockIdx.x] = acc;
}

// posteriors mix_latent_gp (full_cov=False): f_mu = g_mu W^T, f_var = g_var (W o W)^T  (W NULL: identity)
__global__ void k_svgp_mix(const double* g_mu, const double* g_var, const double* W, int n, int p, int L,
                           double* f_mu, double* f_var) {
    const long tot = (long)n * p;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / p), c = (int)(e % p);
        double fm = 0.0, fv = 0.0;
        if (W) {
            for (int l = 0; l < L; ++l) {
                const double w = W[(long)c * L + l];
                fm += g_mu[(long)l * n + r] * w;
                fv += g_var[(long)l * n + r] * (w * w);
            }
        } else {
            fm = g_mu[(long)c * n + r];
            fv = g_var[(long)c * n + r];
        }
        f_mu[e] = fm;
        f_var[e] = fv;
    }
}

// gauss_kl(q_mu, q_sqrt, K=None) per latent (whitened prior), KL_SLICES workgroups per latent:
// slice s sums rows [s m / KL_SLICES, (s+1) m / KL_SLICES) with coalesced row-major reads (a thread per
// row walked its row alone: 78 us for 64 latents of M = 300).  Partial 1/2 (maha + tr - logdet)
// per (l, s); the -M L / 2 term is added in k_svgp_final.
constexpr int KL_SLICES = 8;
__global__ __launch_bounds__(NTHREADS) void k_svgp_kl(const double* q_mu, const double* q_sqrt, int m, int L,
                                                      double* kl_part, int packed) {
    __shared__ double red[4];
    const int sl = blockIdx.x, l = blockIdx.y;
    const int r0 = (int)((long)m * sl / KL_SLICES), r1 = (int)((long)m * (sl + 1) / KL_SLICES);
    double maha = 0.0, tr = 0.0, ld = 0.0;
    for (int r = r0 + threadIdx.x; r < r1; r += NTHREADS) {
        const double q = q_mu[(long)r * L + l];
        maha += q * q;
    }
    if (packed) {   // the rows' lower triangles are one contiguous range; the diagonal one per row
        const double* base = q_sqrt + (long)l * m * (m + 1) / 2;
        const long e0 = (long)r0 * (r0 + 1) / 2, e1 = (long)r1 * (r1 + 1) / 2;
        for (long e = e0 + threadIdx.x; e < e1; e += NTHREADS) {
            const double v = base[e];
            tr += v * v;
        }
        for (int r = r0 + threadIdx.x; r < r1; r += NTHREADS) {
            const double v = base[(long)r * (r + 1) / 2 + r];
            ld += log(v * v);
        }
    } else {
        const double* base = q_sqrt + (long)l * m * m + (long)r0 * m;
        const long ne = (long)(r1 - r0) * m;
        for (long e = threadIdx.x; e < ne; e += NTHREADS) {
            const int r = r0 + (int)(e / m), c = (int)(e % m);
            const double v = base[e];
            if (c <= r) tr += v * v;
            if (c == r) ld += log(v * v);
        }
    }
    maha = block_sum(maha, red);
    tr = block_sum(tr, red);
    ld = block_sum(ld, red);
    if (threadIdx.x == 0) kl_part[(long)l * KL_SLICES + sl] = 0.5 * (maha + tr - ld);
}

// ELBO = VE * scale - KL from the partials (one 256-thread workgroup, fixed summation order)
__global__ __launch_bounds__(NTHREADS) void k_svgp_final(const double* ve_part, int nve, const double* kl_part,
                                                         int nkl, int m, int L, double scale, const int* info,
                                                         double* out) {
    __shared__ double red[4];
    double ve = 0.0, kl = 0.0;
    for (int i = threadIdx.x; i < nve; i += NTHREADS) ve += ve_part[i];
    for (int i = threadIdx.x; i < nkl; i += NTHREADS) kl += kl_part[i];
    ve = block_sum(ve, red);
    kl = block_sum(kl, red) - 0.5 * (double)m * (double)L;
    if (threadIdx.x != 0) return;
    double elbo = ve * scale - kl;
    if (info[0] != 0) elbo = NAN;
    out[0] = elbo;
    out[1] = kl;
    out[2] = ve;
}

template <int NB>
static int svgp_run(hipStream_t s, int n, int m, int L, int p, int d, const double* X, int ldx, const double* Y,
                    int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                    const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                    size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info, double* f_mu = nullptr,
                    double* f_var = nullptr, const double* noise_dev = nullptr, double* Aout = nullptr,
                    double* Bout = nullptr) {
    const SvgpLayout S = svgp_layout(NB, n, m, L, p, d, ws);
    if (ws_bytes < S.bytes) return -2;
    const long mm = (long)S.mpad * S.mpad;
    // The gradient pass keeps A and B (Aout / Bout) anyway, so there they come from two batched
    // GEMMs, A = Li Kuf (Li lower) and B = Lq^T A (Lq^T upper): 2 x 8.5 GF at Goku (L = 64)
    // against the fused conditional's 8.5 + 17 (B = C Kuf with the full C = Lq^T Li, which it
    // needs to form A and B in one tile loop without keeping A), and no C.  The column moments
    // come out of the GEMMs' epilogues in the fused kernel's partial layout and order.
    const bool two_gemm = NB == 32 && Aout != nullptr;
    // K_uu (+ jitter, RHS = I) by one Gram launch and the first diagonal factor of every latent
    // (the first writer of info) on the caller's stream, alone; then the rest of the K_uu pipeline
    // (latency-bound: ~20 launches of small grids, the forward's critical path) on the side stream,
    // and the K_uf Gram, tril(q_sqrt), the zeros above Li's tiles (the step sequence never writes
    // there) and the KL on the caller's beside it.  (Forked before the first factor, the K_uf
    // Gram's 24k workgroups held the CUs: the 64 one-workgroup factors took 64 us instead of ~5.)
    hipStream_t sk;
    {
        GramArgs g{};
        g.X1 = Z; g.ldx1 = ldz; g.sx1 = 0; g.n1 = m;
        g.X2 = Z; g.ldx2 = ldz; g.sx2 = 0; g.n2 = m;
        g.theta = thetas; g.stheta = S.G; g.D = d; g.rbf_only = 0;
        g.out = S.Kuu; g.ldo = S.mpad; g.so = mm;
        g.padded = 1; g.npad = S.mpad; g.tiles_c = S.Tm; g.add_noise = 0; g.diag_add = jitter;
        // NB = 32: R = I stays implicit in the batched steps (CholArgs::r_implicit); the Gram
        // wrote 52 MB of identity at Goku on the chain's critical path
        g.R = NB == 32 ? nullptr : S.R; g.ldr = S.mpad; g.sR = mm;
        // the dense-layout Gram (64 x 64 entries a workgroup, both triangles): the lean tile
        // launch took 56-66 us for 64 latents of 300 x 300 on the chain's critical path
        launch_gram_dense(g, L, S.mpad, S.mpad, s);
        launch_first_factor<NB>(S.Kuu, S.mpad, mm, S.Dd, (long)S.Tm * NB * NB, S.ldiag, S.mpad, info, L, s);
        sk = svgp_fork(s);
        CholArgs c{};
        c.A = S.Kuu; c.lda = S.mpad; c.sA = mm;
        c.R = S.R; c.ldr = S.mpad; c.sR = mm;
        c.Xo = S.Xo; c.ldx = S.mpad; c.sX = mm;
        c.Dd = S.Dd; c.sD = (long)S.Tm * NB * NB; c.ldiag = S.ldiag; c.sL = S.mpad; c.info = info;
        c.T = S.Tm; c.Tp = 0; c.k = 0;
        c.r_implicit = NB == 32 ? 1 : 0;   // k_chol_fused (NB = 32) forms R's identity and zeros itself
        launch_chol_steps<NB>(c, L, sk);
    }
    hipLaunchKernelGGL(k_zero_upper_tiles, dim3(cdiv(S.mpad, ZU_ROWS), 1, L), dim3(256), 0, s, S.Xo, NB, S.mpad, mm);
    // Kuf_l = K_l(Z, X), zero padded to Mpad x Npad
    {
        GramArgs g{};
        g.X1 = Z; g.ldx1 = ldz; g.sx1 = 0; g.n1 = m;
        g.X2 = X; g.ldx2 = ldx; g.sx2 = 0; g.n2 = n;
        g.theta = thetas; g.stheta = S.G; g.D = d; g.rbf_only = 0;
        g.out = S.Kuf; g.ldo = S.npad; g.so = (long)S.mpad * S.npad;
        g.padded = 0; g.tiles_c = S.Tn; g.diag_add = 0.0;
        launch_gram_dense(g, L, S.mpad, S.npad, s);   // zero padding written by the kernel
    }
    const int qp = t_side.qs_packed;
    hipLaunchKernelGGL(k_lq_pad, dim3(cdiv(S.mpad, ZU_ROWS), 1, L), dim3(256), 0, s, q_sqrt, m, S.mpad, S.Lq, qp);
    if (!f_mu) hipLaunchKernelGGL(k_svgp_kl, dim3(KL_SLICES, L), dim3(NTHREADS), 0, s, q_mu, q_sqrt, m, L, S.kl_part, qp);
    svgp_join(s);
    if (!two_gemm)   // C = Lq^T Li (the fused conditional's B = C Kuf), after Lq and Li
        hipLaunchKernelGGL(k_lqt_linv<NB>, dim3(S.Tm * S.Tm, 1, L), dim3(NTHREADS), 2 * sizeof(double) * NB * (NB + 2),
                           s, S.Lq, S.Xo, S.C, S.Tm);
    if (two_gemm) {
        const long mn = (long)S.mpad * S.npad;
        BgemmArgs ga{};
        ga.amask = 1;   // Li lower
        ga.A = S.Xo; ga.lda = S.mpad; ga.sA = mm;
        ga.B = S.Kuf; ga.ldb = S.npad; ga.sB = mn;
        ga.D = Aout; ga.ldd = S.npad; ga.sD = mn;
        ga.alpha = 1.0;
        ga.Mt = S.Tm; ga.Nt = S.Tn; ga.Kt = S.Tm;
        ga.csq = S.pa; ga.csq2 = S.pm; ga.ldcs = S.npad; ga.qv = q_mu; ga.qs = L; ga.qn = m;
        launch_bgemm(NB, s, 0, 0, ga, L);
        BgemmArgs gb{};
        gb.amask = 2;   // Lq^T upper
        gb.A = S.Lq; gb.lda = S.mpad; gb.sA = mm;
        gb.B = Aout; gb.ldb = S.npad; gb.sB = mn;
        gb.D = Bout; gb.ldd = S.npad; gb.sD = mn;
        gb.alpha = 1.0;
        gb.Mt = S.Tm; gb.Nt = S.Tn; gb.Kt = S.Tm;
        gb.csq = S.pb; gb.ldcs = S.npad;
        launch_bgemm(NB, s, 1, 0, gb, L);
    } else if (NB == 32) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_svgp_cond2),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)svgp_cond2_smem());
            attr = true;
        }
        hipLaunchKernelGGL(k_svgp_cond2, dim3(((S.Tm + 1) >> 1) * ((S.Tn + 1) >> 1), 1, L), dim3(NTHREADS),
                           svgp_cond2_smem(), s, S.Xo, S.C, S.Kuf, q_mu, L, m, S.Tm, S.npad, S.pa, S.pb, S.pm, Aout,
                           Bout);
    } else {
        hipLaunchKernelGGL(k_svgp_cond<NB>, dim3(S.Tm * S.Tn, 1, L), dim3(NTHREADS),
                           sizeof(double) * (3 * NB * (NB + 2) + 12 * NB), s, S.Xo, S.C, S.Kuf, q_mu, L, m, S.Tm,
                           S.npad, S.pa, S.pb, S.pm, Aout, Bout);
    }
    hipLaunchKernelGGL(k_svgp_moments, dim3(cdiv(n, 256), 1, L), dim3(256), 0, s, S.pa, S.pb, S.pm, X, (long)ldx,
                       thetas, S.G, d, n, S.npad, S.Tm, g_mu, g_var);
    if (f_mu) {   // predict: mixed moments only
        hipLaunchKernelGGL(k_svgp_mix, dim3(std::min(cdiv(n * p, 256), 2048)), dim3(256), 0, s, g_mu, g_var, W, n, p, L,
                           f_mu, f_var);
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    const int nve = 512;
    hipLaunchKernelGGL(k_svgp_ve, dim3(nve), dim3(NTHREADS), 0, s, g_mu, g_var, W, Y, (long)ldy, n, p, L, noise,
                       noise_dev, S.ve_part);
    hipLaunchKernelGGL(k_svgp_final, dim3(1), dim3(NTHREADS), 0, s, S.ve_part, nve, S.kl_part, L * KL_SLICES, m, L,
                       scale, info, out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int svgp_elbo_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx,
                   const double* Y, int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                   const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                   size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info, const double* noise_dev) {
    if (nb == 64)
        return svgp_run<64>(s, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise, scale, jitter,
                            ws, ws_bytes, out, g_mu, g_var, info, nullptr, nullptr, noise_dev);
    return svgp_run<32>(s, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise, scale, jitter, ws,
                        ws_bytes, out, g_mu, g_var, info, nullptr, nullptr, noise_dev);
}

// the ELBO forward that also writes A = Li Kuf and B = C Kuf ([L][Mpad][Npad] each) for the gradient pass
int svgp_elbo_keep_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx,
                        const double* Y, int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                        const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                        size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info, const double* noise_dev,
                        double* Aout, double* Bout) {
    if (nb == 64)
        return svgp_run<64>(s, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise, scale, jitter,
                            ws, ws_bytes, out, g_mu, g_var, info, nullptr, nullptr, noise_dev, Aout, Bout);
    return svgp_run<32>(s, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise, scale, jitter, ws,
                        ws_bytes, out, g_mu, g_var, info, nullptr, nullptr, noise_dev, Aout, Bout);
}

int svgp_predict_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* Xs, int ldx,
                      const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                      const double* W, double jitter, void* ws, size_t ws_bytes, double* g_mu, double* g_var,
                      double* f_mu, double* f_var, int* info) {
    if (nb == 64)
        return svgp_run<64>(s, n, m, l, p, d, Xs, ldx, Xs, 0, Z, ldz, thetas, q_mu, q_sqrt, W, 1.0, 1.0, jitter, ws,
                            ws_bytes, nullptr, g_mu, g_var, info, f_mu, f_var);
    return svgp_run<32>(s, n, m, l, p, d, Xs, ldx, Xs, 0, Z, ldz, thetas, q_mu, q_sqrt, W, 1.0, 1.0, jitter, ws,
                        ws_bytes, nullptr, g_mu, g_var, info, f_mu, f_var);
}

}  // namespace mfgp
