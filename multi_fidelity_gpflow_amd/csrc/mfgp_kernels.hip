// MI355X-native kernels for the multi-fidelity GPR hot path (fp64).
//
//   K1  k_gram            per-fidelity RBF distance + rho-scaled block assembly
//                         (mfgpflow/linear.py:55-104, GPflow SquaredExponential.K)
//   K2  k_chol_step       right-looking tile Cholesky fused with the inverse
//                         factor L^{-1}, the forward solve Z = L^{-1} Y and, as rows
//                         become final, alpha = L^{-T} Z and the sum Z^2 partials
//   K5  k_grad            W = alpha alpha^T - P K^{-1} contracted with dK/dtheta,
//                         K^{-1} = L^{-T} L^{-1} formed tile-by-tile, never stored
//   K4  k_reduce_items    LML / gradient reductions; the last workgroup finalizes (+Adam)
//   K6  k_pred_a / k_pred_out   posterior mean / variance (GPflow base_conditional)
//
// Every kernel runs 256-thread workgroups on NB x NB fp64 tiles; tile products
// go through v_mfma_f64_16x16x4_f64 (mfgp_device.h).
#include "../../include/mfgp.h"
#include "mfgp_device.h"
#include "mfgp_internal.h"
#include "mfgp_flow.h"

namespace mfgp {

constexpr int MAXD = 32;
constexpr int XS = MAXD + 1;   // LDS row stride of staged inputs: odd, so a wave reading one
                                // dimension of 16-32 different rows hits distinct banks

// ============================================================ K1: gram

__device__ void build_grad_order(int T, int chunk, int Tp, int* order, int* hist);

// one Gram entry from staged rows (GPflow: dist = -2 a.b + (|a|^2 + |b|^2); k = v exp(-dist/2))
// kernel scalars held in registers (one load each per workgroup, issued with the row loads)
struct MFScal {
    double vL_, vD_, rho_;
    __device__ double vL() const { return vL_; }
    __device__ double vD() const { return vD_; }
    __device__ double rho() const { return rho_; }
};

// Both row blocks of a tile in ONE memory round trip: every X element, fidelity flag and
// lengthscale a thread needs is loaded before any is used (the two-pass stage_rows took ~4
// dependent global-load latencies).  Split in two so a workgroup that loops over several tiles
// issues the next tile's loads before it computes the current one (the per-tile round trip was
// ~3 us of the ~5.5 us a tile took): stage_pair_load fills registers, stage_pair_commit turns
// them into aL = X / lL (GPflow divides; here X * rcp(lL), within an ulp), squared norms and
// flags in LDS.
__host__ __device__ __forceinline__ int pad4(int D) { return (D + 3) & ~3; }

// sum_d a[d] b[d] over d < D4 (a multiple of 4; slots past D hold 0.0): the same sequential
// accumulation as a d < D loop, bit for bit, with the 8 LDS reads of a step issued together (a
// runtime-D loop waited on each read: ~2/3 of a tile's time in k_gram)
__device__ __forceinline__ double dot4(const double* a, const double* b, int D4) {
    double dot = 0.0;
    for (int d = 0; d < D4; d += 4) {
        const double a0 = a[d], a1 = a[d + 1], a2 = a[d + 2], a3 = a[d + 3];
        const double b0 = b[d], b1 = b[d + 1], b2 = b[d + 2], b3 = b[d + 3];
        dot += a0 * b0;
        dot += a1 * b1;
        dot += a2 * b2;
        dot += a3 * b3;
    }
    return dot;
}

template <int NB>
struct StageRegs {
    static constexpr int PER = (NB * MAXD + NTHREADS - 1) / NTHREADS;
    double x1[PER], x2[PER];
    double fv;
};

template <int NB>
__device__ __forceinline__ void stage_pair_load(StageRegs<NB>& g, const double* X1, long ldx1, int n1, int r01,
                                                const double* X2, long ldx2, int n2, int r02,
                                                int D, int rbf_only) {
    constexpr int PER = StageRegs<NB>::PER;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + q * NTHREADS;
        if (e < NB * D) {
            const int r = e / D, d = e % D;
            g.x1[q] = (r01 + r < n1) ? X1[(long)(r01 + r) * ldx1 + d] : 0.0;
            g.x2[q] = (r02 + r < n2) ? X2[(long)(r02 + r) * ldx2 + d] : 0.0;
        }
    }
    const int t = threadIdx.x;
    g.fv = -1.0;
    if (t < NB) g.fv = (r01 + t < n1) ? (rbf_only ? 0.0 : X1[(long)(r01 + t) * ldx1 + D]) : -1.0;
    else if (t < 2 * NB) g.fv = (r02 + t - NB < n2) ? (rbf_only ? 0.0 : X2[(long)(r02 + t - NB) * ldx2 + D]) : -1.0;
}

// il: LDS [1/lL(0..MAXD) | 1/lD(0..MAXD)], staged once per workgroup (stage_inv_lengthscales)
template <int NB>
__device__ __forceinline__ void stage_pair_commit(StageRegs<NB>& g, const double* il, double* aL1, double* aD1,
                                                  double* nL1, double* nD1, double* f1, double* aL2, double* aD2,
                                                  double* nL2, double* nD2, double* f2, int D, int rbf_only) {
    constexpr int PER = StageRegs<NB>::PER;
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + q * NTHREADS;
        if (e < NB * D) {
            const int r = e / D, d = e % D;
            const double lL = il[d];
            aL1[r * XS + d] = g.x1[q] * lL;
            aL2[r * XS + d] = g.x2[q] * lL;
            if (!rbf_only) {
                const double lD = il[MAXD + d];
                aD1[r * XS + d] = g.x1[q] * lD;
                aD2[r * XS + d] = g.x2[q] * lD;
            }
        }
    }
    if (t < NB) f1[t] = g.fv;
    else if (t < 2 * NB) f2[t - NB] = g.fv;
    const int D4 = pad4(D), np4 = D4 - D;
    if (np4 && t < NB * np4) {   // zero slots D..D4-1: the dots run 4 dimensions per step
        const int r = t / np4, d = D + t % np4;
        aL1[r * XS + d] = 0.0;
        aL2[r * XS + d] = 0.0;
        if (!rbf_only) { aD1[r * XS + d] = 0.0; aD2[r * XS + d] = 0.0; }
    }
    __syncthreads();
    if (t < 2 * NB) {
        const int r = t & (NB - 1);
        const double* aL = (t < NB ? aL1 : aL2) + r * XS;
        const double* aD = (t < NB ? aD1 : aD2) + r * XS;
        const double sL = dot4(aL, aL, D4);
        const double sD = rbf_only ? 0.0 : dot4(aD, aD, D4);
        if (t < NB) { nL1[r] = sL; nD1[r] = sD; }
        else { nL2[r] = sL; nD2[r] = sD; }
    }
}

template <class TH>
__device__ __forceinline__ double gram_entry(const double* aL1, const double* aD1, double nL1, double nD1, double f1,
                                             const double* aL2, const double* aD2, double nL2, double nD2, double f2,
                                             int D, const TH& th, int rbf_only) {
    const int D4 = pad4(D);
    if (rbf_only) {
        if (f1 < 0.0 || f2 < 0.0) return 0.0;
        const double dot = dot4(aL1, aL2, D4);
        const double r2 = -2.0 * dot + (nL1 + nL2);
        return th.vL() * exp_lib(-0.5 * r2);
    }
    const bool L1 = (f1 == 0.0), H1 = (f1 == 1.0), L2 = (f2 == 0.0), H2 = (f2 == 1.0);
    if (!(L1 || H1) || !(L2 || H2)) return 0.0;        // linear.py:67-70 exact masks
    const double dot = dot4(aL1, aL2, D4);
    const double kL = th.vL() * exp_lib(-0.5 * (-2.0 * dot + (nL1 + nL2)));
    const double rho = th.rho();
    if (L1 && L2) return kL;                           // K_LL
    if (!(H1 && H2)) return kL * rho;                  // K_LH, K_HL
    const double dotD = dot4(aD1, aD2, D4);
    const double kD = th.vD() * exp_lib(-0.5 * (-2.0 * dotD + (nD1 + nD2)));
    return kL * (rho * rho) + kD;                      // K_HH (linear.py:96)
}

// k_reduce_items' item slots to FLOW_SENTINEL (sc1, as the publication area: no XCD's L2 may keep
// a clean sentinel copy for the finalizer's sc1 polls), for its sentinel protocol (FinArgs::flag)
__device__ __forceinline__ void gram_fill_items(const GramArgs& a) {
    for (int e = threadIdx.x; e < a.nisent; e += NTHREADS)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.isent) + e, FLOW_SENTINEL, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Sentinel fill of the k_chol_flow publication area (grid-stride over ALL workgroups of the
// launch).  sc1 (write-through, line dropped from this XCD's L2): a plain store would leave a
// clean copy of the sentinel in this XCD's L2 that the flow's sc1 polls could be served from.
// 16-B buffer stores (buffer_store_dwordx4 ... sc1): an 8-B sc1 store costs ~2.7x the bytes of
// a 16-B one (MI355X_MICROARCH.md, store flavours).  Run LAST in a workgroup: the stores share
// the vmcnt queue with later loads, and a load's data waits for every older store.
typedef unsigned int fill_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void gram_fill_pub(const GramArgs& a) {
    if (a.fpub && blockIdx.z == 0) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.fpub, (short)0, (int)(a.npub * 8), 0x00020000);
        const unsigned lo = (unsigned)(FLOW_SENTINEL & 0xffffffffull), hi = (unsigned)(FLOW_SENTINEL >> 32);
        const fill_u32x4 v = {lo, hi, lo, hi};
        const long npair = a.npub / 2;
        for (long e = blockIdx.x * (long)NTHREADS + threadIdx.x; e < npair; e += (long)gridDim.x * NTHREADS)
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(e * 16), 0, 16);
        if ((a.npub & 1) && blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.fpub) + a.npub - 1, FLOW_SENTINEL,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Y block of R (rows < n1, columns < p; zero padding), a grid-stride slice per tile workgroup
// of the padded launch (the extra workgroups after the T(T+1)/2 tiles do not take part)
template <int NB>
__device__ __forceinline__ void gram_copy_y(const GramArgs& a) {
    if (a.R == nullptr) return;
    const int T = a.npad / NB;
    const long nt = a.tile_wgs > 1 ? a.tile_wgs : (long)T * (T + 1) / 2;   // tile workgroups
    const long ne = (long)a.npad * a.ppad;
    const int b = blockIdx.z;
    const double* Yb = a.Y + b * a.sY;
    double* Rb = a.R + b * a.sR;
    for (long e = blockIdx.x * (long)NTHREADS + threadIdx.x; e < ne; e += nt * NTHREADS) {
        const int r = (int)(e / a.ppad), c = (int)(e % a.ppad);
        Rb[(long)r * a.ldr + a.npad + c] = (r < a.n1 && c < a.p) ? Yb[(long)r * a.ldy + c] : 0.0;
    }
}

// Fused factor of the first diagonal tile (step "-1" of the tile Cholesky), run by one workgroup
// of k_gram.  Not inlined: inlined, its register demand set the whole kernel's allocation (222
// SGPR spills to VGPR lanes that every tile loop reloaded).
template <int NB>
__device__ __attribute__((noinline)) void gram_first_factor(double* tile, double* rtile, double* dg, int* bad,
                                                            double* Dd, double* ldiag, int* info) {
    __syncthreads();
    tile_potrf_inv<NB>(tile, rtile, dg, bad);
    tile_store<NB>(Dd, NB, rtile);
    for (int r = threadIdx.x; r < NB; r += NTHREADS) ldiag[r] = dg[r];
    if (threadIdx.x == 0) *info = *bad;   // first writer of info in the sequence: initialises it
}

// LEAN: no fused first factor and no set-up workgroups (a.Dd, a.gorder, a.fown unused): the
// factor call's register demand (noinline, but it still sets the kernel's allocation) is left out,
// which lifts the occupancy of the many small tile workgroups of the batched SVGP K_uu launch.
template <int NB, bool LEAN>
__global__ __launch_bounds__(NTHREADS) void k_gram(GramArgs a) {
    constexpr int S = TileCfg<NB>::S;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* aL1 = smem;
    double* aD1 = aL1 + NB * XS;
    double* aL2 = aD1 + NB * XS;
    double* aD2 = aL2 + NB * XS;
    double* nL1 = aD2 + NB * XS;
    double* nD1 = nL1 + NB;
    double* f1 = nD1 + NB;
    double* nL2 = f1 + NB;
    double* nD2 = nL2 + NB;
    double* f2 = nD2 + NB;
    double* tile = f2 + NB;                    // NB x S
    double* rtile = tile + TileCfg<NB>::ELEMS; // NB x S (factor scratch)
    double* dg = rtile + TileCfg<NB>::ELEMS;   // NB
    int& bad = *reinterpret_cast<int*>(dg + NB);   // keep ALL LDS dynamic: a static __shared__
                                                   // would shift the dynamic base off 16 B (G17)
    double* il = dg + NB + 2;                  // 2 x MAXD inverse lengthscales

    const int b = blockIdx.z;
    const long long dbg_t0 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    if (!LEAN && a.gorder && blockIdx.x == gridDim.x - 1) {   // extra workgroup: k_grad task order
        if (b == 0) build_grad_order(a.gT, a.gchunk, a.gTp, a.gorder, reinterpret_cast<int*>(smem));
        if (a.dbg && threadIdx.x == 0) a.dbg[3 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime() - dbg_t0;
        gram_fill_pub(a);
        return;
    }
    if (!LEAN && a.fown && blockIdx.x == gridDim.x - 1 - (a.gorder ? 1 : 0)) {   // extra: flow owner table
        if (b == 0) build_flow_owner(a.npad / NB, a.ppad / NB, a.fW, a.fown, a.fflags, a.nfflags,
                                     reinterpret_cast<int*>(smem));
        if (a.dbg && threadIdx.x == 0) a.dbg[3 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime() - dbg_t0;
        gram_fill_pub(a);
        return;
    }
    if (a.cnt && blockIdx.x == 0 && b == 0)
        for (int e = threadIdx.x; e < a.ncnt; e += NTHREADS) a.cnt[e] = 0;
    if (a.isent && blockIdx.x == 0 && b == 0) gram_fill_items(a);
    const MFTheta th{a.theta + b * a.stheta, a.D};
    MFScal sc{0.0, 0.0, 0.0};
    double noise = 0.0;
    if (!a.nlf) {   // scalars first: their loads overlap the row loads of stage_pair
        const double* tp = a.theta + b * a.stheta;
        sc.vL_ = tp[0];
        if (!a.rbf_only) { sc.vD_ = tp[1 + a.D]; sc.rho_ = tp[2 + 2 * a.D]; }
        if (a.add_noise) noise = tp[kernel_theta_size(0, a.D) - 1];
    } else if (a.add_noise) {
        noise = a.theta[b * a.stheta + kernel_theta_size(a.nlf, a.D) - 1];
    }
    (void)th;
    const GraphTheta gth{a.theta + b * a.stheta, a.D, a.nlf};
    const double* X1 = a.X1 + b * a.sx1;
    const double* X2 = a.X2 + b * a.sx2;
    // tiles of this workgroup: one (tile_wgs == 0, or the dense layout); with tile_wgs > 0
    // workgroup 0 takes tile (0,0) alone -- the first diagonal factor runs on a CU of its own
    // instead of beside two other tile workgroups -- and workgroups 1.. stride over the rest
    const int Tl = a.npad / NB;
    const int ntl = a.padded ? Tl * (Tl + 1) / 2 : 0;
    int t0 = blockIdx.x, tstep = 1 << 30;
    if (a.padded && a.tile_wgs > 1) {
        if (blockIdx.x == 0) tstep = 1 << 30;
        else tstep = a.tile_wgs - 1;
    }
    auto decode = [&](int t, int& ti, int& tj) {
        if (a.padded) {   // lower tiles: t -> (ti, tj), ti >= tj
            ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
            while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
            while (ti * (ti + 1) / 2 > t) --ti;
            tj = t - ti * (ti + 1) / 2;
        } else {
            ti = blockIdx.x / a.tiles_c;
            tj = blockIdx.x % a.tiles_c;
        }
    };
    const int tend = a.padded ? ntl : t0 + 1;
    StageRegs<NB> sr;   // the row loads of the tile this workgroup computes next
    if (!a.nlf && t0 < tend) {
        int ti, tj;
        decode(t0, ti, tj);
        stage_pair_load<NB>(sr, X1, a.ldx1, a.n1, ti * NB, X2, a.ldx2, a.n2, tj * NB, a.D, a.rbf_only);
        // 1/l once per workgroup (was: every thread, every tile: 2 loads + 2 Newton reciprocals per
        // staged element); rcp_nr is 1/l to <= 1 ulp, x * (1/l) for the IEEE division's ~30 ops
        const double* tp = a.theta + b * a.stheta;
        if (threadIdx.x < a.D) {
            il[threadIdx.x] = rcp_nr(tp[1 + threadIdx.x]);
            il[MAXD + threadIdx.x] = a.rbf_only ? 1.0 : rcp_nr(tp[2 + a.D + threadIdx.x]);
        }
        __syncthreads();
    }
    for (int t = t0; t < tend; t += tstep) {
    int ti, tj;
    decode(t, ti, tj);
    if (t != t0) __syncthreads();   // the previous tile's LDS is consumed
    if (a.nlf) {   // graph kernel: raw rows + source index (f1/f2 hold the source as a double)
        for (int e = threadIdx.x; e < NB * (a.D + 1); e += NTHREADS) {
            const int r = e / (a.D + 1), d = e % (a.D + 1);
            const int g1 = ti * NB + r, g2 = tj * NB + r;
            const double v1 = (g1 < a.n1) ? X1[(long)g1 * a.ldx1 + d] : 0.0;
            const double v2 = (g2 < a.n2) ? X2[(long)g2 * a.ldx2 + d] : 0.0;
            if (d < a.D) { aL1[r * XS + d] = v1; aL2[r * XS + d] = v2; }
            else {
                f1[r] = (g1 < a.n1) ? (double)graph_source(v1, a.nlf) : -1.0;
                f2[r] = (g2 < a.n2) ? (double)graph_source(v2, a.nlf) : -1.0;
            }
        }
    } else {
        stage_pair_commit<NB>(sr, il, aL1, aD1, nL1, nD1, f1, aL2, aD2, nL2, nD2, f2, a.D, a.rbf_only);
    }
    __syncthreads();
    if (!a.nlf && t + tstep < tend) {   // next tile's rows: in flight while this one is computed
        int ni, nj;
        decode(t + tstep, ni, nj);
        stage_pair_load<NB>(sr, X1, a.ldx1, a.n1, ni * NB, X2, a.ldx2, a.n2, nj * NB, a.D, a.rbf_only);
    }
    if (a.dbg && threadIdx.x == 0) a.dbg[3 * blockIdx.x] = __builtin_amdgcn_s_memrealtime() - dbg_t0;   // stage time (ticks)

    double* out = a.out + b * a.so;
    if (a.padded && !a.nlf) {
        // the NB*NB/256 entries of a thread side by side (one wave per SIMD: a lone entry's LDS
        // reads -> dot -> exp chain was latency-bound); same arithmetic as gram_entry, bit for bit
        constexpr int PT = NB * NB / NTHREADS;
        static_assert(NB * NB % NTHREADS == 0, "entries per thread");
        const int D4 = pad4(a.D);
        double kl[PT];
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const int e = threadIdx.x + k * NTHREADS;
            const int r = e / NB, c = e % NB;
            const double dot = dot4(aL1 + r * XS, aL2 + c * XS, D4);
            kl[k] = sc.vL() * exp_lib(-0.5 * (-2.0 * dot + (nL1[r] + nL2[c])));
        }
#pragma unroll
        for (int k = 0; k < PT; ++k) {
            const int e = threadIdx.x + k * NTHREADS;
            const int r = e / NB, c = e % NB;
            const int gi = ti * NB + r, gj = tj * NB + c;
            const double fa = f1[r], fb = f2[c];
            double v;
            if (a.rbf_only) {
                v = (fa < 0.0 || fb < 0.0) ? 0.0 : kl[k];
            } else {
                const bool L1 = (fa == 0.0), H1 = (fa == 1.0), L2 = (fb == 0.0), H2 = (fb == 1.0);
                const double rho = sc.rho();
                double kD = 0.0;
                if (H1 && H2) {   // K_HH (linear.py:96): rare, a branch of its own
                    const double dotD = dot4(aD1 + r * XS, aD2 + c * XS, D4);
                    kD = sc.vD() * exp_lib(-0.5 * (-2.0 * dotD + (nD1[r] + nD2[c])));
                }
                const double vhh = kl[k] * (rho * rho) + kD;
                v = (L1 && L2) ? kl[k] : (!(H1 && H2) ? kl[k] * rho : vhh);
                if (!(L1 || H1) || !(L2 || H2)) v = 0.0;    // linear.py:67-70 exact masks
            }
            if (gi == gj) v = (gi < a.n1) ? v + noise + a.diag_add : 1.0;   // identity padding
            tile[r * S + c] = v;
        }
    } else
    for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
        const int r = e / NB, c = e % NB;
        const int gi = ti * NB + r, gj = tj * NB + c;
        double v = a.nlf ? graph_entry(aL1 + r * XS, aL2 + c * XS, (int)f1[r], (int)f2[c], gth)
                         : gram_entry(aL1 + r * XS, aD1 + r * XS, nL1[r], nD1[r], f1[r],
                                      aL2 + c * XS, aD2 + c * XS, nL2[c], nD2[c], f2[c], a.D, sc, a.rbf_only);
        if (a.padded) {
            if (gi == gj) v = (gi < a.n1) ? v + noise + a.diag_add : 1.0;   // identity padding
            tile[r * S + c] = v;
        } else {
            if (gi == gj) v += a.diag_add;
            if (gi < a.n1 && gj < a.n2) out[(long)gi * a.ldo + gj] = v;
        }
    }
    if (!a.padded) { gram_fill_pub(a); return; }
    if (a.R != nullptr && a.fown == nullptr) {
        // fused RHS init: R tile (ti, tj) of the identity part, and row block ti of Y (the
        // persistent k_chol_flow never reads R's identity block: it starts those tiles from zero)
        double* Rb = a.R + b * a.sR;
        for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
            const int r = e / NB, c = e % NB;
            Rb[(long)(ti * NB + r) * a.ldr + tj * NB + c] = (ti == tj && r == c) ? 1.0 : 0.0;
        }
        // the Y block of R is copied by every tile workgroup at its end (gram_copy_y), not by the
        // column-0 ones: that copy kept the workgroup of the first diagonal factor the longest
    }
    __syncthreads();
    if (a.dbg && threadIdx.x == 0) a.dbg[3 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - dbg_t0;
    tile_store<NB>(out + (long)ti * NB * a.ldo + tj * NB, a.ldo, tile);
    if constexpr (!LEAN)
        if (a.Dd != nullptr && ti == 0 && tj == 0)
            gram_first_factor<NB>(tile, rtile, dg, &bad, a.Dd + b * a.sD, a.ldiag + b * a.sL, a.info + b);
    }   // tiles of this workgroup
    gram_copy_y<NB>(a);
    gram_fill_pub(a);
    if (a.dbg && threadIdx.x == 0) a.dbg[3 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime() - dbg_t0;
}

size_t gram_smem_bytes(int nb) {
    const size_t tile = (size_t)nb * (nb + 2);
    return sizeof(double) * (4 * (size_t)nb * XS + 6 * (size_t)nb + 2 * tile + nb + 2 + 2 * MAXD);
}

// ------------------------------------------------------------ K1 dense (rectangular) layout
// K(X1, X2) written row-major (Kuf, K(X, X*), K(X*, X*), the mfgp_*_gram entry points).  A lean
// kernel of its own: k_gram carries the fused diagonal factor and the flow set-up, whose register
// demand (256 VGPRs, one wave per SIMD) starved these launches of thousands of small tiles (the
// Goku SingleBinSVGP Kuf: 64 latents x 300 x 1164).  64 x 64 entries per 256-thread workgroup:
// lane = column (coalesced 512-B row stores), wave w = rows w, w+4, .., w+60; the column's scaled
// row lives in registers (D4 = dimensions padded to 4, a template parameter), the row side is
// read from LDS as a wave-wide broadcast.  Same arithmetic as gram_entry, bit for bit (same
// scaling x * rcp_nr(l), same dot4 accumulation order, same expressions).
// Entries with gi < wr1, gj < wr2 outside n1 x n2 are written 0.0 (the padded Kuf / Kmn buffers
// need no memset), or 1.0 on the diagonal with GramArgs::padded (called directly, not through
// launch_gram: the SVGP K_uu, whose padded rows factor as identity; with GramArgs::R it also
// writes that factorization's right-hand side R = I over the same extent).
constexpr int GD_T = 64;

template <int D4>
__device__ __forceinline__ double dot_rl(const double* a, const double (&b)[D4]) {
    double dot = 0.0;
#pragma unroll
    for (int d = 0; d < D4; d += 4) {
        const double a0 = a[d], a1 = a[d + 1], a2 = a[d + 2], a3 = a[d + 3];
        dot += a0 * b[d];
        dot += a1 * b[d + 1];
        dot += a2 * b[d + 2];
        dot += a3 * b[d + 3];
    }
    return dot;
}

template <int D4>
__global__ __launch_bounds__(NTHREADS) void k_gram_dense(GramArgs a, int wr1, int wr2, int tc) {
    __shared__ __attribute__((aligned(16))) double sL1[GD_T * D4];
    __shared__ __attribute__((aligned(16))) double sD1[GD_T * D4];
    __shared__ __attribute__((aligned(16))) double sD2[GD_T * D4];
    __shared__ double nL1[GD_T], nD1[GD_T], f1[GD_T];
    __shared__ double il[2 * MAXD];
    const int b = blockIdx.z, t = threadIdx.x;
    const int ti = blockIdx.x / tc, tj = blockIdx.x % tc;
    const int r0 = ti * GD_T, c0 = tj * GD_T;
    const int D = a.D;
    const double* tp = a.theta + b * a.stheta;
    const double* X1 = a.X1 + b * a.sx1;
    const double* X2 = a.X2 + b * a.sx2;
    if (t < D) {
        il[t] = rcp_nr(tp[1 + t]);
        il[MAXD + t] = a.rbf_only ? 1.0 : rcp_nr(tp[2 + D + t]);
    }
    const double vL = tp[0];
    const double vD = a.rbf_only ? 0.0 : tp[1 + D];
    const double rho = a.rbf_only ? 0.0 : tp[2 + 2 * D];
    __syncthreads();
    // stage the row side (X1) and the column side's delta rows (X2, for K_HH pairs)
    for (int e = t; e < GD_T * D4; e += NTHREADS) {
        const int r = e / D4, d = e % D4;
        const bool in = d < D;
        const double x1 = (in && r0 + r < a.n1) ? X1[(long)(r0 + r) * a.ldx1 + d] : 0.0;
        sL1[e] = in ? x1 * il[d] : 0.0;
        if (!a.rbf_only) {
            const double x2 = (in && c0 + r < a.n2) ? X2[(long)(c0 + r) * a.ldx2 + d] : 0.0;
            sD1[e] = in ? x1 * il[MAXD + d] : 0.0;
            sD2[e] = in ? x2 * il[MAXD + d] : 0.0;
        }
    }
    if (t < GD_T) f1[t] = (r0 + t < a.n1) ? (a.rbf_only ? 0.0 : X1[(long)(r0 + t) * a.ldx1 + D]) : -1.0;
    // the column's LF-scaled row in registers
    const int c = t & 63, gj = c0 + c;
    double bl[D4];
#pragma unroll
    for (int d = 0; d < D4; ++d)
        bl[d] = (d < D && gj < a.n2) ? X2[(long)gj * a.ldx2 + d] * il[d] : 0.0;
    const double f2 = (gj < a.n2) ? (a.rbf_only ? 0.0 : X2[(long)gj * a.ldx2 + D]) : -1.0;
    __syncthreads();
    if (t < GD_T) {
        nL1[t] = dot4(sL1 + t * D4, sL1 + t * D4, D4);
        nD1[t] = a.rbf_only ? 0.0 : dot4(sD1 + t * D4, sD1 + t * D4, D4);
    }
    const double nL2 = dot_rl<D4>(bl, bl);
    const double nD2 = a.rbf_only ? 0.0 : dot4(sD2 + c * D4, sD2 + c * D4, D4);
    __syncthreads();
    double* out = a.out + b * a.so;
    double* Rb = (a.padded && a.R) ? a.R + b * a.sR : nullptr;   // fused RHS = I of the factorization
    const bool L2 = (f2 == 0.0), H2 = (f2 == 1.0);
    for (int rr = t >> 6; rr < GD_T; rr += NTHREADS / 64) {
        const int gi = r0 + rr;
        if (gi >= wr1) break;
        if (gj >= wr2) continue;
        double v = 0.0;
        if (gi < a.n1 && gj < a.n2) {
            const double fa = f1[rr];
            const double dot = dot_rl<D4>(sL1 + rr * D4, bl);
            const double kl = vL * exp_lib(-0.5 * (-2.0 * dot + (nL1[rr] + nL2)));
            if (a.rbf_only) {
                v = (fa < 0.0 || f2 < 0.0) ? 0.0 : kl;
            } else {
                const bool L1 = (fa == 0.0), H1 = (fa == 1.0);
                double kD = 0.0;
                if (H1 && H2) {   // K_HH (linear.py:96)
                    const double dotD = dot4(sD1 + rr * D4, sD2 + c * D4, D4);
                    kD = vD * exp_lib(-0.5 * (-2.0 * dotD + (nD1[rr] + nD2)));
                }
                const double vhh = kl * (rho * rho) + kD;
                v = (L1 && L2) ? kl : (!(H1 && H2) ? kl * rho : vhh);
                if (!(L1 || H1) || !(L2 || H2)) v = 0.0;   // linear.py:67-70 exact masks
            }
            if (gi == gj) v += a.diag_add;
        } else if (a.padded && gi == gj) {
            v = 1.0;   // identity padding (a batched K_uu for the step factorization)
        }
        out[(long)gi * a.ldo + gj] = v;
        if (Rb) Rb[(long)gi * a.ldr + gj] = (gi == gj) ? 1.0 : 0.0;
    }
}

// dense-layout Gram of a (batch of) rectangular blocks; write extents wr1 >= n1, wr2 >= n2
void launch_gram_dense(const GramArgs& g, int batch, int wr1, int wr2, hipStream_t s) {
    wr1 = wr1 > g.n1 ? wr1 : g.n1;
    wr2 = wr2 > g.n2 ? wr2 : g.n2;
    const int tr = (wr1 + GD_T - 1) / GD_T, tc = (wr2 + GD_T - 1) / GD_T;
    const dim3 grid(tr * tc, 1, batch);
    switch (pad4(g.D)) {
        case 4: hipLaunchKernelGGL(k_gram_dense<4>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        case 8: hipLaunchKernelGGL(k_gram_dense<8>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        case 12: hipLaunchKernelGGL(k_gram_dense<12>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        case 16: hipLaunchKernelGGL(k_gram_dense<16>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        case 20: hipLaunchKernelGGL(k_gram_dense<20>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        case 24: hipLaunchKernelGGL(k_gram_dense<24>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        case 28: hipLaunchKernelGGL(k_gram_dense<28>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
        default: hipLaunchKernelGGL(k_gram_dense<32>, grid, dim3(NTHREADS), 0, s, g, wr1, wr2, tc); break;
    }
}

// ------------------------------------------------------------ K1 flow set-up (LML layout, NB = 32)
// The launch in front of k_chol_flow when the workspace is not known to be set up (eager calls,
// value-only calls; mfgp_set_resident): every workgroup sentinel-fills its share of the
// publication area; the last two build (or verify, when intact from an earlier call) the flow
// owner table -- zeroing the abort word -- and the k_grad task order; workgroup 0 sentinel-fills
// k_reduce_items' item slots and initialises info.  The Gram itself is formed inside the flow
// (flow_gram_tile, mfgp_flow.hip), and the flow reads Y directly.
__global__ __launch_bounds__(NTHREADS) void k_flow_prep(GramArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    int* sh = reinterpret_cast<int*>(smem);
    const int bx = blockIdx.x, last = (int)gridDim.x - 1;
    if (a.gorder && bx == last) build_grad_order(a.gT, a.gchunk, a.gTp, a.gorder, sh);
    else if (a.fown && bx == last - (a.gorder ? 1 : 0))
        build_flow_owner(a.npad / 32, a.ppad / 32, a.fW, a.fown, a.fflags, a.nfflags, sh);
    if (bx == 0) {
        if (a.isent) gram_fill_items(a);
        if (a.cnt)
            for (int e = threadIdx.x; e < a.ncnt; e += NTHREADS) a.cnt[e] = 0;
        if (threadIdx.x == 0 && a.info) *a.info = 0;
    }
    gram_fill_pub(a);
}

constexpr size_t FLOW_PREP_LDS = 16384;   // the set-up workgroups' tables (gorder: < 2048 ints + hash)

void launch_flow_prep(const GramArgs& g, int nwg, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_flow_prep),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)FLOW_PREP_LDS);
        attr = true;
    }
    hipLaunchKernelGGL(k_flow_prep, dim3(nwg), dim3(NTHREADS), FLOW_PREP_LDS, s, g);
}

// ============================================================ K2: tile Cholesky step

__device__ __forceinline__ void tri_decode(int t, int& i, int& j) {
    int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    i = r;
    j = t - r * (r + 1) / 2;
}

// zpart[k*Tp + cy] = sum of Z_k^2 over the valid (n x p) region of Y tile cy; Xs holds
// Z_k tile cy in LDS, visible to the whole workgroup.  red: >= 4 doubles of LDS.
template <int NB>
__device__ void chol_zpart(const CholArgs& a, int k, int cy, const double* Xs, double* red) {
    constexpr int S = TileCfg<NB>::S;
    double z2 = 0.0;
    for (int e = threadIdx.x; e < NB * NB; e += NTHREADS) {
        const int r = e / NB, col = e % NB;
        if (k * NB + r < a.n && cy * NB + col < a.p) {
            const double z = Xs[r * S + col];
            z2 += z * z;
        }
    }
    z2 = block_sum(z2, red);
    if (threadIdx.x == 0) a.zpart[k * a.Tp + cy] = z2;
}

template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_chol_step(CholArgs a) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Ds = smem;           // D_k
    double* T0 = Ds + E;         // scratch / A tile / X tile
    double* Pi = T0 + E;         // L_ik = A_ik D_k^T
    double* Pj = Pi + E;         // L_jk
    double* dg = Pj + E;         // NB
    int& bad = *reinterpret_cast<int*>(dg + NB);

    int t, b;   // task t of system b (XCD-aware order: a run of systems per XCD, mfgp_device.h)
    xcd_swizzle(t, b);
    const int k = a.k, T = a.T, Tp = a.Tp;
    double* A = a.A + b * a.sA;
    double* R = a.R + b * a.sR;
    double* Xo = a.Xo + b * a.sX;
    const long lda = a.lda, ldr = a.ldr, ldx = a.ldx;
    auto At = [&](int i, int j) { return A + (long)i * NB * lda + (long)j * NB; };
    auto Rt = [&](int i, int c) { return R + (long)i * NB * ldr + (long)c * NB; };
    auto Xt = [&](int i, int c) { return Xo + (long)i * NB * ldx + (long)c * NB; };

    const int rem = T - k - 1;
    const int nA = rem * (rem + 1) / 2;
    const int ncol = k + 1 + Tp;               // active RHS column tiles
    const int nR = rem * ncol;

    tile_load<NB>(Ds, a.Dd + b * a.sD + (long)k * NB * NB, NB);

    if (t < nA) {
        // ---- trailing update A_ij -= L_ik L_jk^T, i >= j > k
        int ii, jj;
        tri_decode(t, ii, jj);
        const int i = k + 1 + ii, j = k + 1 + jj;
        tile_load<NB>(T0, At(i, k), lda);
        Acc<NB> cij;                                     // A_ij in flight with the panel loads
        acc_load(cij, At(i, j), lda);
        __syncthreads();
        Acc<NB> acc;
        acc_zero(acc);
        tile_mma<NB, false, true>(acc, T0, Ds, 1.0);     // P_i = A_ik D_k^T
        acc_to_lds(acc, Pi);
        const double* PJ = Pi;
        if (j != i) {
            __syncthreads();
            tile_load<NB>(T0, At(j, k), lda);
            __syncthreads();
            acc_zero(acc);
            tile_mma<NB, false, true>(acc, T0, Ds, 1.0);
            acc_to_lds(acc, Pj);
            PJ = Pj;
        }
        __syncthreads();
        acc = cij;
        tile_mma<NB, false, true>(acc, Pi, PJ, -1.0);    // A_ij -= P_i P_j^T
        if (i == j && i == k + 1) {
            // next diagonal tile is final: factor it and publish D_{k+1}
            if constexpr (NB == 32) {
                tile_potrf_inv_w1_acc(acc.v[0], T0, Pj, dg, &bad);   // straight from registers
            } else {
                acc_to_lds(acc, T0);
                __syncthreads();
                tile_potrf_inv<NB>(T0, Pj, dg, &bad);
            }
            tile_store<NB>(a.Dd + b * a.sD + (long)(k + 1) * NB * NB, NB, Pj);
            for (int r = threadIdx.x; r < NB; r += NTHREADS) a.ldiag[b * a.sL + (k + 1) * NB + r] = dg[r];
            if (threadIdx.x == 0 && bad && a.info[b] == 0) a.info[b] = (k + 1) * NB + bad;
        } else {
            acc_store(acc, At(i, j), lda);
        }
        return;
    }
    t -= nA;
    if (t < nR) {
        // ---- RHS update R_ic -= L_ik X_kc, X_kc = D_k R_kc (row k of [L^{-1} | Z])
        const int i = k + 1 + t / ncol;
        const int cc = t % ncol;
        const int c = (cc <= k) ? cc : T + (cc - k - 1);
        tile_load<NB>(T0, Rt(k, c), ldr);
        tile_load<NB>(Pi, At(i, k), lda);                // A_ik staged in Pi's buffer
        Acc<NB> ric;
        acc_load(ric, Rt(i, c), ldr);
        __syncthreads();
        Acc<NB> acc;
        acc_zero(acc);
        tile_mma<NB, false, false>(acc, Ds, T0, 1.0);    // X_kc
        acc_to_lds(acc, Pj);
        if (i == k + 1) acc_store(acc, Xt(k, c), ldx);
        acc_zero(acc);
        tile_mma<NB, false, true>(acc, Pi, Ds, 1.0);     // P_i = A_ik D_k^T
        __syncthreads();                                 // everyone done reading Pi / Pj(X) writes
        acc_to_lds(acc, Pi);
        __syncthreads();
        acc = ric;
        tile_mma<NB, false, false>(acc, Pi, Pj, -1.0);
        acc_store(acc, Rt(i, c), ldr);
        if (a.alpha && i == k + 1 && c >= T) chol_zpart<NB>(a, k, c - T, Pj, dg);
        return;
    }
    t -= nR;
    if (a.alpha) {
        // ---- alpha_c (+)= X_kc^T Z_k for c <= k: row k of [L^{-1} | Z] is final in this
        // launch (X = D_k R_k).  alpha_c is first written at k == c, then accumulated in
        // launch order -- replaces a separate alpha = L^{-T} Z pass.
        const int nAl = (k + 1) * Tp;
        if (t < nAl) {
            const int c = t / Tp, cy = t % Tp;
            double* al = a.alpha + (long)c * NB * a.ldal + (long)cy * NB;
            tile_load<NB>(T0, Rt(k, c), ldr);
            tile_load<NB>(Pi, Rt(k, T + cy), ldr);
            Acc<NB> acc;
            if (c == k) acc_zero(acc);
            else acc_load(acc, al, a.ldal);
            __syncthreads();
            Acc<NB> x, z;
            acc_zero(x);
            tile_mma<NB, false, false>(x, Ds, T0, 1.0);   // X_kc
            acc_zero(z);
            tile_mma<NB, false, false>(z, Ds, Pi, 1.0);   // Z_k (tile cy)
            __syncthreads();
            acc_to_lds(x, Pj);
            acc_to_lds(z, T0);
            __syncthreads();
            tile_mma<NB, true, false>(acc, Pj, T0, 1.0);
            acc_store(acc, al, a.ldal);
            if (k == T - 1) {
                // alpha_c is final: also store alpha^T under [L^{-1} | Z] for k_grad, whose
                // items are then all TN products: row block T + cy holds -alpha^T / P (A side),
                // row block T + Tp + cy holds alpha^T (B side).
                const double sA = -1.0 / (double)a.p;
                double* xa = Xo + (long)(T + cy) * NB * ldx + (long)c * NB;
                double* xb = Xo + (long)(T + Tp + cy) * NB * ldx + (long)c * NB;
#pragma unroll
                for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const long o = (long)acc_col<NB>(q) * ldx + acc_row<NB>(q, r);
                        xa[o] = sA * acc.v[q][r];
                        xb[o] = acc.v[q][r];
                    }
            }
            return;
        }
        t -= nAl;
    }
    // ---- last step writers: X_{T-1,c} = D_{T-1} R_{T-1,c}
    {
        const int c = t;   // 0..T-1 identity tiles, T..T+Tp-1 Y tiles
        tile_load<NB>(T0, Rt(k, c), ldr);
        __syncthreads();
        Acc<NB> acc;
        acc_zero(acc);
        tile_mma<NB, false, false>(acc, Ds, T0, 1.0);
        acc_store(acc, Xt(k, c), ldx);
        if (a.alpha && c >= T) {
            acc_to_lds(acc, Pj);
            __syncthreads();
            chol_zpart<NB>(a, k, c - T, Pj, dg);
        }
    }
}

// Batched systems (the SVGP K_uu of every latent, batch > 1): each step of k_chol_step as two
// launches.  k_chol_step's tasks recompute L_ik = A_ik D_k^T (twice per trailing tile) and
// X_kc = D_k R_kc per task -- three tile products for one update; here the panel launch forms
// each L_ik (stored over A_ik, which no later step reads) and each X_kc (row k of [L^{-1} | Z],
// stored to Xo) once, and the update launch does one product per tile (the trailing task of
// tile (k+1, k+1) then factors it).  The same products in the same order: bitwise k_chol_step's
// results.  (Goku SVGP, 64 latents x 10 tiles: 9 x 20.5 us of steps.)
// LDS tile <- the NB x NB identity (CholArgs::r_implicit: the RHS's R_kk)
template <int NB>
__device__ __forceinline__ void tile_identity(double* __restrict__ s) {
    constexpr int S = TileCfg<NB>::S;
    for (int p = threadIdx.x; p < NB * NB; p += NTHREADS) {
        const int r = p / NB, c = p % NB;
        s[r * S + c] = (r == c) ? 1.0 : 0.0;
    }
}

template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_chol_panel(CholArgs a) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Ds = smem;
    double* T0 = Ds + E;
    int t, b;
    xcd_swizzle(t, b);
    const int k = a.k, T = a.T, rem = T - k - 1;
    tile_load<NB>(Ds, a.Dd + b * a.sD + (long)k * NB * NB, NB);
    Acc<NB> acc;
    acc_zero(acc);
    if (t < rem) {   // L_ik = A_ik D_k^T
        double* Aik = a.A + b * a.sA + (long)(k + 1 + t) * NB * a.lda + (long)k * NB;
        tile_load<NB>(T0, Aik, a.lda);
        __syncthreads();
        tile_mma<NB, false, true>(acc, T0, Ds, 1.0);
        acc_store(acc, Aik, a.lda);
        return;
    }
    t -= rem;        // X_kc = D_k R_kc, c = 0..k, then the Y tiles
    const int c = (t <= k) ? t : T + (t - k - 1);
    if (a.r_implicit && c == k) tile_identity<NB>(T0);
    else tile_load<NB>(T0, a.R + b * a.sR + (long)k * NB * a.ldr + (long)c * NB, a.ldr);
    __syncthreads();
    tile_mma<NB, false, false>(acc, Ds, T0, 1.0);
    acc_store(acc, a.Xo + b * a.sX + (long)k * NB * a.ldx + (long)c * NB, a.ldx);
}

// Dispatch order of k_chol_update: task 0 of every batch entry (the trailing tile (k+1, k+1), which
// also factors it: the longest task and the next step's critical path) in the first slots, then
// the other tasks; both parts in XCD-aware chunks (xcd_swizzle's remap).  Placement only.
__device__ __forceinline__ void chol_update_order(int per, int& t, int& b) {
    const int nb = gridDim.z, g = blockIdx.x + gridDim.x * blockIdx.z;
    if (g < nb) {
        t = 0;
        b = (nb % 8 == 0) ? (g & 7) * (nb >> 3) + (g >> 3) : g;
        return;
    }
    const int r = g - nb, rest = per - 1, cpx = (nb * rest) >> 3;
    const int s = r < 8 * cpx ? (r & 7) * cpx + (r >> 3) : r;
    b = s / rest;
    t = 1 + s % rest;
}

template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_chol_update(CholArgs a) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* T0 = smem + E;       // (the k_chol_step carve: Ds | T0 | Pi | Pj | dg | bad)
    double* Pi = T0 + E;
    double* Pj = Pi + E;
    double* dg = Pj + E;
    int& bad = *reinterpret_cast<int*>(dg + NB);
    const int k = a.k, T = a.T, Tp = a.Tp;
    const int rem = T - k - 1, nA = rem * (rem + 1) / 2, ncol = k + 1 + Tp;
    int t, b;
    chol_update_order(gridDim.x, t, b);
    double* A = a.A + b * a.sA;
    auto At = [&](int i, int j) { return A + (long)i * NB * a.lda + (long)j * NB; };
    Acc<NB> acc;
    if (t < nA) {    // A_ij -= L_ik L_jk^T
        int ii, jj;
        tri_decode(t, ii, jj);
        const int i = k + 1 + ii, j = k + 1 + jj;
        tile_load<NB>(Pi, At(i, k), a.lda);
        if (j != i) tile_load<NB>(Pj, At(j, k), a.lda);
        acc_load(acc, At(i, j), a.lda);
        __syncthreads();
        tile_mma<NB, false, true>(acc, Pi, j != i ? Pj : Pi, -1.0);
        if (i == j && i == k + 1) {
            if constexpr (NB == 32) {
                tile_potrf_inv_w1_acc(acc.v[0], T0, Pj, dg, &bad);
            } else {
                acc_to_lds(acc, T0);
                __syncthreads();
                tile_potrf_inv<NB>(T0, Pj, dg, &bad);
            }
            tile_store<NB>(a.Dd + b * a.sD + (long)(k + 1) * NB * NB, NB, Pj);
            for (int r = threadIdx.x; r < NB; r += NTHREADS) a.ldiag[b * a.sL + (k + 1) * NB + r] = dg[r];
            if (threadIdx.x == 0 && bad && a.info[b] == 0) a.info[b] = (k + 1) * NB + bad;
        } else {
            acc_store(acc, At(i, j), a.lda);
        }
        return;
    }
    t -= nA;         // R_ic -= L_ik X_kc
    const int i = k + 1 + t / ncol, cc = t % ncol;
    const int c = (cc <= k) ? cc : T + (cc - k - 1);
    double* Ric = a.R + b * a.sR + (long)i * NB * a.ldr + (long)c * NB;
    tile_load<NB>(Pi, At(i, k), a.lda);
    tile_load<NB>(Pj, a.Xo + b * a.sX + (long)k * NB * a.ldx + (long)c * NB, a.ldx);
    acc_load(acc, Ric, a.ldr);
    __syncthreads();
    tile_mma<NB, false, false>(acc, Pi, Pj, -1.0);
    acc_store(acc, Ric, a.ldr);
}

// Batched step k with the panel folded in (NB = 32, batch > 1, k < T - 1): each task forms the
// panel tiles it needs itself -- L_ik = A_ik D_k^T (and L_jk, or X_kc = D_k R_kc) -- from the
// unscaled tiles, then does its update, with the same tile products in the same order as the
// k_chol_panel + k_chol_update pair (bitwise the same results).  The tasks of row k + 1 store
// X_kc (row k of L^{-1}) for the step after; L_ik itself is not stored (nothing reads the factor's
// off-diagonal tiles after step k).  Saves the panel launch and its hand-off through memory on
// the K_uu chain of the SVGP forward (10 steps at Goku).
template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_chol_fused(CholArgs a) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Ds = smem;           // D_k
    double* T0 = Ds + E;         // A_ik, later factor scratch
    double* T1 = T0 + E;         // A_jk or R_kc
    double* Pi = T1 + E;         // L_ik
    double* Pj = Pi + E;         // L_jk or X_kc, later D_{k+1}
    double* dg = Pj + E;
    int& bad = *reinterpret_cast<int*>(dg + NB);
    const int k = a.k, T = a.T, Tp = a.Tp;
    const int rem = T - k - 1, nA = rem * (rem + 1) / 2, ncol = k + 1 + Tp;
    int t, b;
    chol_update_order(gridDim.x, t, b);
    double* A = a.A + b * a.sA;
    auto At = [&](int i, int j) { return A + (long)i * NB * a.lda + (long)j * NB; };
    tile_load<NB>(Ds, a.Dd + b * a.sD + (long)k * NB * NB, NB);
    Acc<NB> acc, lp;
    if (t < nA) {    // A_ij -= L_ik L_jk^T
        int ii, jj;
        tri_decode(t, ii, jj);
        const int i = k + 1 + ii, j = k + 1 + jj;
        tile_load<NB>(T0, At(i, k), a.lda);
        if (j != i) tile_load<NB>(T1, At(j, k), a.lda);
        acc_load(acc, At(i, j), a.lda);
        __syncthreads();
        acc_zero(lp);
        tile_mma<NB, false, true>(lp, T0, Ds, 1.0);
        acc_to_lds(lp, Pi);
        if (j != i) {
            acc_zero(lp);
            tile_mma<NB, false, true>(lp, T1, Ds, 1.0);
            acc_to_lds(lp, Pj);
        }
        __syncthreads();
        tile_mma<NB, false, true>(acc, Pi, j != i ? Pj : Pi, -1.0);
        if (i == j && i == k + 1) {
            __syncthreads();   // T0 / Pj are reused below
            if constexpr (NB == 32) {
                tile_potrf_inv_w1_acc(acc.v[0], T0, Pj, dg, &bad);
            } else {
                acc_to_lds(acc, T0);
                __syncthreads();
                tile_potrf_inv<NB>(T0, Pj, dg, &bad);
            }
            tile_store<NB>(a.Dd + b * a.sD + (long)(k + 1) * NB * NB, NB, Pj);
            for (int r = threadIdx.x; r < NB; r += NTHREADS) a.ldiag[b * a.sL + (k + 1) * NB + r] = dg[r];
            if (threadIdx.x == 0 && bad && a.info[b] == 0) a.info[b] = (k + 1) * NB + bad;
        } else {
            acc_store(acc, At(i, j), a.lda);
        }
        return;
    }
    t -= nA;         // R_ic -= L_ik X_kc
    const int i = k + 1 + t / ncol, cc = t % ncol;
    const int c = (cc <= k) ? cc : T + (cc - k - 1);
    double* Ric = a.R + b * a.sR + (long)i * NB * a.ldr + (long)c * NB;
    tile_load<NB>(T0, At(i, k), a.lda);
    const bool first = a.r_implicit && c == k;   // R_kk = I; R_ic (i > k) untouched until now: 0
    if (first) {
        tile_identity<NB>(T1);
        acc_zero(acc);
    } else {
        tile_load<NB>(T1, a.R + b * a.sR + (long)k * NB * a.ldr + (long)c * NB, a.ldr);
        acc_load(acc, Ric, a.ldr);
    }
    __syncthreads();
    acc_zero(lp);
    tile_mma<NB, false, true>(lp, T0, Ds, 1.0);
    acc_to_lds(lp, Pi);
    acc_zero(lp);
    tile_mma<NB, false, false>(lp, Ds, T1, 1.0);
    acc_to_lds(lp, Pj);
    if (i == k + 1) acc_store(lp, a.Xo + b * a.sX + (long)k * NB * a.ldx + (long)c * NB, a.ldx);
    __syncthreads();
    tile_mma<NB, false, false>(acc, Pi, Pj, -1.0);
    acc_store(acc, Ric, a.ldr);
}

int chol_step_blocks(int T, int Tp, int k, bool alpha) {
    const int rem = T - k - 1;
    return rem * (rem + 1) / 2 + rem * (k + 1 + Tp) + (alpha ? (k + 1) * Tp : 0) + ((k == T - 1) ? (T + Tp) : 0);
}

size_t chol_smem_bytes(int nb) { return sizeof(double) * (4 * (size_t)nb * (nb + 2) + nb + 2); }

// RHS init: identity tiles on the diagonal, zeros strictly below, Y (zero padded)
__global__ void k_rhs_init(double* R, long ldr, long sR, int npad, int ppad, const double* Y, long ldy, long sY,
                           int n, int p) {
    const int b = blockIdx.z;
    const long total = (long)npad * (npad + ppad);
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / (npad + ppad)), c = (int)(e % (npad + ppad));
        double v;
        if (c < npad) v = (r == c) ? 1.0 : 0.0;
        else {
            const int pc = c - npad;
            v = (Y != nullptr && r < n && pc < p) ? Y[b * sY + (long)r * ldy + pc] : 0.0;
        }
        R[b * sR + (long)r * ldr + c] = v;
    }
}

// ============================================================ K5: gradient
// k_grad LDS: NBUF operand buffers (2: double-buffered m-loop, one barrier per item;
// NB = 64 tiles are 33 KB each, so one).
// After the loop the region is reused: raw rows xi, xj, flags fi, fj, then the
// per-quad gradient partials R [G][GRAD_RLD] and the inverse squared lengthscales.
template <int NB>
constexpr int GRAD_NBUF = (NB == 32) ? 2 : 1;
constexpr int GRAD_RLD = 65;   // 64 quad partials per gradient entry, +1 against bank conflicts
template <int NB>
constexpr int GRAD_RED_OFF = (2 * NB * XS + 2 * NB + 1) & ~1;

__host__ __device__ inline int grad_row_chunks(int T, int i, int ch) { return (T - i + ch - 1) / ch; }
__host__ __device__ inline int grad_m0(int T, int i, int ch, int c) { (void)T; return i + c * ch; }
__host__ __device__ inline int grad_m1(int T, int m0, int ch) { return min(T, m0 + ch); }

__host__ __device__ int grad_tasks(int T, int ch) {
    int s = 0;
    for (int i = 0; i < T; ++i) s += (i + 1) * grad_row_chunks(T, i, ch);
    return s;
}

// k_grad task -> (row i, column j, chunk ch) in the natural order (rows, then columns,
// then m-chunks); returns the task's item count (m tiles + the alpha items of chunk 0).
__device__ __forceinline__ int grad_decode(int t, int T, int chunk, int Tp, int& i, int& j, int& ch) {
    for (i = 0;; ++i) {
        const int cnt = (i + 1) * grad_row_chunks(T, i, chunk);
        if (t < cnt) break;
        t -= cnt;
    }
    const int nch = grad_row_chunks(T, i, chunk);
    j = t / nch;
    ch = t % nch;
    const int m0 = grad_m0(T, i, chunk, ch);
    return grad_m1(T, m0, chunk) - m0 + (ch == 0 ? Tp : 0);
}

// Flow path (GradArgs::fpub): the next evaluation's set-up, run by every k_grad workgroup after
// its own work -- the flow has ended, so its publication area is dead: 16-B sc1 sentinel stores
// (as gram_fill_pub) over a grid-stride share; workgroup 0 also refills k_reduce_items' item slots
// (this evaluation's reduction polls them; k_reduce_items zeroes the abort word).  With it the next value+grad
// evaluation of the same problem on the same workspace can start with the flow itself
// (mfgp_set_resident): these stores land after the chain, where they slow no hand-off.
__device__ __forceinline__ void grad_next_setup(const GradArgs& a) {
    if (!a.fpub) return;
    if (blockIdx.x == 0) {
        for (int e = threadIdx.x; e < a.nisent; e += NTHREADS)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.isent) + e, FLOW_SENTINEL, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.fpub, (short)0, (int)(a.npub * 8), 0x00020000);
    const unsigned lo = (unsigned)(FLOW_SENTINEL & 0xffffffffull), hi = (unsigned)(FLOW_SENTINEL >> 32);
    const fill_u32x4 v = {lo, hi, lo, hi};
    const long npair = a.npub / 2;
    for (long e = blockIdx.x * (long)NTHREADS + threadIdx.x; e < npair; e += (long)gridDim.x * NTHREADS)
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(e * 16), 0, 16);
    if ((a.npub & 1) && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.fpub) + a.npub - 1, FLOW_SENTINEL,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup -> task table for k_grad.  All k_grad workgroups are resident at once and
// are dealt to CUs in launch order (about blockIdx mod 256), so the natural order piles
// the long early-row chains onto the same CUs.  Tasks are counting-sorted by item count
// (longest first) and dealt in a snake over 256 slots, which evens out the MFMA work per
// CU.  Placement only sets speed: any permutation gives the same result, because k_grad
// indexes its partial sums by task, not by workgroup.  One workgroup; hist: LDS ints.
// order holds ntask + SCHED_KEY ints; a table intact from an earlier call is kept.
constexpr int GRAD_ORDER_MAGIC = 0x4F524431;
__device__ void build_grad_order(int T, int chunk, int Tp, int* order, int* hist) {
    const int ntask = grad_tasks(T, chunk);
    const int lmax = chunk + Tp;
    unsigned* hs = reinterpret_cast<unsigned*>(hist + lmax + 1);
    if (sched_cached(order, ntask, GRAD_ORDER_MAGIC, T, chunk, Tp, hs)) return;
    for (int l = threadIdx.x; l <= lmax; l += NTHREADS) hist[l] = 0;
    __syncthreads();
    int i, j, ch;
    for (int t = threadIdx.x; t < ntask; t += NTHREADS) atomicAdd(&hist[grad_decode(t, T, chunk, Tp, i, j, ch)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive offsets, longest first
        int o = 0;
        for (int l = lmax; l >= 0; --l) {
            const int c = hist[l];
            hist[l] = o;
            o += c;
        }
    }
    __syncthreads();
    constexpr int SLOTS = 256;
    for (int t = threadIdx.x; t < ntask; t += NTHREADS) {
        const int p = atomicAdd(&hist[grad_decode(t, T, chunk, Tp, i, j, ch)], 1);
        const int r = p / SLOTS, k = p % SLOTS;
        const int width = min(SLOTS, ntask - r * SLOTS);
        order[r * SLOTS + ((r & 1) ? width - 1 - k : k)] = t;
    }
    sched_seal(order, ntask, GRAD_ORDER_MAGIC, T, chunk, Tp, hs);
}


template <int NB, bool GRAPH>
__global__ __launch_bounds__(NTHREADS) void k_grad(GradArgs a) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int E = TileCfg<NB>::ELEMS;
    constexpr int NE = TileCfg<NB>::NBLK * 4;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    // LDS: the m-loop operand buffers; after the loop the same region holds the raw
    // input rows and source flags of the two row tiles, and red follows them.
    constexpr int NBUF = GRAD_NBUF<NB>;
    double* As = smem;                // NBUF x E (m-loop operands)
    double* Bs = As + NBUF * E;       // NBUF x E
    double* xi = smem;                // NB x XS raw rows of tile i   (epilogue)
    double* xj = xi + NB * XS;        // NB x XS raw rows of tile j   (epilogue)
    double* fi = xj + NB * XS;        // NB                           (epilogue)
    double* fj = fi + NB;             // NB                           (epilogue)
    static_assert(2 * NB * XS + 2 * NB <= 2 * NBUF * E, "raw rows must fit in the operand region");
    const int G = kernel_theta_size(a.nlf, a.D);
    double* R = smem + GRAD_RED_OFF<NB>;     // G x GRAD_RLD quad partials   (epilogue)
    double* il2 = R + G * GRAD_RLD;          // nsrc x D  1 / l^2            (epilogue)
    const int nsrc = a.nlf ? a.nlf + 1 : 2;
    const MFTheta th{a.theta, a.D};

    // decode task -> (i, j, m0, m1)
    const int task = a.order ? a.order[blockIdx.x] : (int)blockIdx.x;
    int i, j, ch;
    grad_decode(task, a.T, a.chunk, a.Tp, i, j, ch);
    const int m0 = grad_m0(a.T, i, a.chunk, ch);
    const int m1 = grad_m1(a.T, m0, a.chunk);
    auto Xt = [&](int r, int c) { return a.Xo + (long)r * NB * a.ldx + (long)c * NB; };

    // The epilogue's inputs (raw rows of tiles i and j, 1 / l^2) are loaded now, into registers,
    // and land in LDS after the operand stream: their round trip hides under it instead of
    // following it.  (NB (D + 1) <= 2 x 256 entries each; larger D loads the rest afterwards.)
    constexpr int GPRE = 2;
    const int nraw = NB * (a.D + 1);
    double pvi[GPRE], pvj[GPRE];
#pragma unroll
    for (int s = 0; s < GPRE; ++s) {
        const int e = threadIdx.x + s * NTHREADS;
        const int r = e / (a.D + 1), d = e % (a.D + 1);
        const int gi = i * NB + r, gj = j * NB + r;
        pvi[s] = (e < nraw && gi < a.n) ? a.X[(long)gi * a.ldxx + d] : 0.0;
        pvj[s] = (e < nraw && gj < a.n) ? a.X[(long)gj * a.ldxx + d] : 0.0;
    }
    double pl = 1.0;
    if (threadIdx.x < nsrc * a.D) {
        const int src = threadIdx.x / a.D, d = threadIdx.x % a.D;
        pl = a.nlf ? a.theta[src * (1 + a.D) + 1 + d] : (src == 0 ? th.lL(d) : th.lD(d));
    }

    // W_ij (tile) = [alpha_i alpha_j^T] - P * sum_m Linv_mi^T Linv_mj  (= -P * acc below)
    Acc<NB> acc;
    acc_zero(acc);
    const double negP = -(double)a.P;
    {   // Software-pipelined operand stream of TN items acc += A^T B (all unscaled):
        //   q < nm : A = Linv_{m,i}, B = Linv_{m,j}, m = m0 + q
        //   q >= nm (chunk 0): A = -alpha^T_{cy,i} / P, B = alpha^T_{cy,j}  (rows T + cy, T+Tp+cy)
        // so acc = S = sum_m Linv_mi^T Linv_mj - alpha_i alpha_j^T / P and W = -P S (the -P is
        // folded into the epilogue weight).
        const int nm = m1 - m0;
        const int nq = nm + ((ch == 0) ? a.Tp : 0);
        const long rs = (long)NB * a.ldx;
        const double* const XA = a.Xo + (long)i * NB;
        const double* const XB = a.Xo + (long)j * NB;
#define MFGP_GRAD_FETCH(ra, rb, q)                                                          \
    do {                                                                                    \
        const int ra_ = (q) < nm ? m0 + (q) : a.T + (q) - nm;                               \
        const int rb_ = (q) < nm ? ra_ : ra_ + a.Tp;                                        \
        tile_fetch<NB>(ra, XA + ra_ * rs, a.ldx);                                           \
        tile_fetch<NB>(rb, XB + rb_ * rs, a.ldx);                                           \
    } while (0)
        if constexpr (NBUF == 2) {
            // Two LDS buffers + two register sets: item q is fetched two items before it is
            // put into LDS (three before its product); unrolled by two so the register set
            // of each item is a compile-time choice.  Invariant at even q: buffer 0 holds
            // item q, set 1 item q+1, set 0 item q+2.
            TileRegs<NB> ra0, rb0, ra1, rb1;
            double* A0 = As;
            double* B0 = Bs;
            double* A1 = As + E;
            double* B1 = Bs + E;
            MFGP_GRAD_FETCH(ra0, rb0, 0);
            tile_put<NB>(A0, ra0);
            tile_put<NB>(B0, rb0);
            if (nq > 1) MFGP_GRAD_FETCH(ra1, rb1, 1);
            if (nq > 2) MFGP_GRAD_FETCH(ra0, rb0, 2);
            __syncthreads();
            for (int q = 0; q < nq; q += 2) {
                tile_mma<NB, true, false>(acc, A0, B0, 1.0);
                if (q + 1 < nq) {
                    tile_put<NB>(A1, ra1);
                    tile_put<NB>(B1, rb1);
                    if (q + 3 < nq) MFGP_GRAD_FETCH(ra1, rb1, q + 3);
                }
                __syncthreads();
                if (q + 1 < nq) {
                    tile_mma<NB, true, false>(acc, A1, B1, 1.0);
                    if (q + 2 < nq) {
                        tile_put<NB>(A0, ra0);
                        tile_put<NB>(B0, rb0);
                        if (q + 4 < nq) MFGP_GRAD_FETCH(ra0, rb0, q + 4);
                    }
                    __syncthreads();
                }
            }
        } else {                              // single LDS buffer (NB = 64), register prefetch
            TileRegs<NB> ra, rb;
            MFGP_GRAD_FETCH(ra, rb, 0);
            for (int q = 0; q < nq; ++q) {
                tile_put<NB>(As, ra);
                tile_put<NB>(Bs, rb);
                if (q + 1 < nq) MFGP_GRAD_FETCH(ra, rb, q + 1);
                __syncthreads();
                tile_mma<NB, true, false>(acc, As, Bs, 1.0);
                __syncthreads();
            }
        }
#undef MFGP_GRAD_FETCH
    }

    // stage the raw inputs of the two row tiles (operand buffers are free now)
    auto stage = [&](int e, double vi, double vj) {
        const int r = e / (a.D + 1), d = e % (a.D + 1);
        const int gi = i * NB + r, gj = j * NB + r;
        if (d < a.D) { xi[r * XS + d] = vi; xj[r * XS + d] = vj; }
        else if (a.nlf) {   // graph kernel: source index
            fi[r] = (gi < a.n) ? (double)graph_source(vi, a.nlf) : -1.0;
            fj[r] = (gj < a.n) ? (double)graph_source(vj, a.nlf) : -1.0;
        } else { fi[r] = (gi < a.n) ? vi : -1.0; fj[r] = (gj < a.n) ? vj : -1.0; }
    };
#pragma unroll
    for (int s = 0; s < GPRE; ++s) {
        const int e = threadIdx.x + s * NTHREADS;
        if (e < nraw) stage(e, pvi[s], pvj[s]);
    }
    for (int e = threadIdx.x + GPRE * NTHREADS; e < nraw; e += NTHREADS) {
        const int r = e / (a.D + 1), d = e % (a.D + 1);
        const int gi = i * NB + r, gj = j * NB + r;
        stage(e, (gi < a.n) ? a.X[(long)gi * a.ldxx + d] : 0.0, (gj < a.n) ? a.X[(long)gj * a.ldxx + d] : 0.0);
    }
    if (threadIdx.x < nsrc * a.D) il2[threadIdx.x] = 1.0 / (pl * pl);
    for (int e = threadIdx.x + NTHREADS; e < nsrc * a.D; e += NTHREADS) {
        const int src = e / a.D, d = e % a.D;
        const double l = a.nlf ? a.theta[src * (1 + a.D) + 1 + d] : (src == 0 ? th.lL(d) : th.lD(d));
        il2[e] = 1.0 / (l * l);
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // gradient entry qidx: quad-sum in registers, one LDS slot per quad (64 per entry)
    auto put = [&](int qidx, double v) {
        v = quad_sum(v);
        if ((lane & 3) == 0) R[qidx * GRAD_RLD + wv * 16 + (lane >> 2)] = v;
    };
    // after a barrier: entry qidx = sum of its 64 partials, 8 lanes per entry
    auto reduce_entries = [&](auto&& finish) {
        for (int g0 = 0; g0 < G; g0 += NTHREADS / 8) {
            const int qx = g0 + (threadIdx.x >> 3), sub = threadIdx.x & 7;
            double v = 0.0;
            if (qx < G) {
#pragma unroll
                for (int u = 0; u < 8; ++u) v += R[qx * GRAD_RLD + sub * 8 + u];
            }
            v = quad_sum(v);
            v += __shfl_xor(v, 4, 64);
            if (sub == 0 && qx < G) a.gpart[(long)qx * gridDim.x + task] = finish(qx, v);
        }
    };
    if constexpr (GRAPH) {
        // graph kernel (graph.py:55-97): 1/2 W_ab dK_ab/dtheta over all (a, b); a lower tile
        // (i > j) also carries the mirrored entry K_ba, which differs in the LF-LF block.
        const GraphTheta gt{a.theta, a.D, a.nlf};
        const int m = a.nlf;
        double co[MFGP_MAX_LF + 1][NE];       // per element: 1/2 W * dK/dk_s * k_s
        double grho[MFGP_MAX_LF], grl[MFGP_MAX_LF * MFGP_MAX_LF];
        double gn = 0.0;
#pragma unroll
        for (int s2 = 0; s2 < MFGP_MAX_LF; ++s2) grho[s2] = 0.0;
#pragma unroll
        for (int s2 = 0; s2 < MFGP_MAX_LF * MFGP_MAX_LF; ++s2) grl[s2] = 0.0;
#pragma unroll
        for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = q * 4 + r;
                const int ri = acc_row<NB>(q, r), cj = acc_col<NB>(q);
                const int sa = (int)fi[ri], sb = (int)fj[cj];
                const double w = (0.5 * negP) * acc.v[q][r];
#pragma unroll
                for (int s2 = 0; s2 <= MFGP_MAX_LF; ++s2) co[s2][e] = 0.0;
                if (sa >= 0 && sb >= 0) {
                    double ks[MFGP_MAX_LF + 1];
                    for (int s2 = 0; s2 <= m; ++s2)
                        ks[s2] = graph_k_il2(xi + ri * XS, xj + cj * XS, s2, gt, il2 + s2 * a.D);
                    auto accum = [&](int s1, int t1) {   // entry with row source s1, column source t1
                        if (s1 < m && t1 < m) {
                            if (s1 == t1) co[s1][e] += w * ks[s1];
                            else {
                                co[s1][e] += w * gt.rhoLF(s1, t1) * ks[s1];
                                grl[s1 * m + t1] += w * ks[s1];
                            }
                        } else if (s1 < m || t1 < m) {
                            const int u = (s1 < m) ? s1 : t1;
                            co[u][e] += w * gt.rho(u) * ks[u];
                            grho[u] += w * ks[u];
                        } else {
                            for (int k2 = 0; k2 < m; ++k2) {
                                const double rr = gt.rho(k2);
                                co[k2][e] += w * rr * rr * ks[k2];
                                grho[k2] += w * 2.0 * rr * ks[k2];
                            }
                            co[m][e] += w * ks[m];
                        }
                    };
                    accum(sa, sb);
                    if (i != j) accum(sb, sa);
                }
                if (i == j && ri == cj && i * NB + ri < a.n) gn += w;
            }
        for (int s2 = 0; s2 <= m; ++s2) {
            double vs = 0.0;
#pragma unroll
            for (int e = 0; e < NE; ++e) vs += co[s2][e];
            put(s2 * (1 + a.D), vs);
            for (int d = 0; d < a.D; ++d) {
                double tl = 0.0;
#pragma unroll
                for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double df = xi[acc_row<NB>(q, r) * XS + d] - xj[acc_col<NB>(q) * XS + d];
                        tl += co[s2][q * 4 + r] * df * df;
                    }
                put(s2 * (1 + a.D) + 1 + d, tl);
            }
        }
        const int ro = (m + 1) * (1 + a.D);
        for (int k2 = 0; k2 < m; ++k2) put(ro + k2, grho[k2]);
        for (int k2 = 0; k2 < m * m; ++k2) put(ro + m + k2, grl[k2]);
        put(G - 1, gn);
        __syncthreads();
        reduce_entries([&](int qx, double v) {
            if (qx < ro) {
                const int s2 = qx / (1 + a.D), d = qx % (1 + a.D);
                if (d == 0) v /= gt.v(s2);
                else { const double l = gt.l(s2, d - 1); v /= l * l * l; }
            }
            return v;
        });
        return;
    }
    // epilogue: contract with dK/dtheta recomputed from the inputs.  Loops run over d
    // outermost so the lane's elements share each LDS read of their column inputs.
    const double wscale = ((i == j) ? 0.5 : 1.0) * negP;   // -P (W = -P acc), 1/2, x2 mirrored
    const double rho = th.rho();
    int ri[NE], cj[NE];
    bool L1[NE], H1[NE], L2[NE], H2[NE];
    double s2[NE], s2d[NE];
    bool anyHH = false;
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = q * 4 + r;
            ri[e] = acc_row<NB>(q, r);
            cj[e] = acc_col<NB>(q);
            const double f1 = fi[ri[e]], f2 = fj[cj[e]];
            L1[e] = f1 == 0.0; H1[e] = f1 == 1.0; L2[e] = f2 == 0.0; H2[e] = f2 == 1.0;
            anyHH |= H1[e] && H2[e];
            s2[e] = 0.0;
            s2d[e] = 0.0;
        }
    for (int d = 0; d < a.D; ++d) {
        const double il = il2[d], ild = il2[a.D + d];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const double df = xi[ri[e] * XS + d] - xj[cj[e] * XS + d];
            const double d2 = df * df;
            s2[e] += d2 * il;
            s2d[e] += d2 * ild;
        }
    }
    double cL[NE], cD[NE];
    double gvL = 0.0, gvD = 0.0, grho = 0.0, gnoise = 0.0;
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = q * 4 + r;
            const double w = acc.v[q][r] * wscale;
            const bool live = (L1[e] || H1[e]) && (L2[e] || H2[e]);
            // dK/dv = exp(-r2/2), TF's autodiff of v * exp(-r2/2): finite where v underflows to 0
            // (the division form K / v gave 0/0 at L-BFGS line-search points)
            const double eL = live ? exp_lib(-0.5 * s2[e]) : 0.0;
            const double kL = th.vL() * eL;
            double eD = 0.0;
            if (anyHH && H1[e] && H2[e]) eD = exp_lib(-0.5 * s2d[e]);
            const double kD = th.vD() * eD;
            const double si = L1[e] ? 1.0 : (H1[e] ? rho : 0.0), sj = L2[e] ? 1.0 : (H2[e] ? rho : 0.0);
            const double hi = H1[e] ? 1.0 : 0.0, hj = H2[e] ? 1.0 : 0.0;
            cL[e] = w * si * sj * kL;
            cD[e] = w * hi * hj * kD;
            gvL += w * si * sj * eL;
            gvD += w * hi * hj * eD;
            grho += w * (hi * sj + si * hj) * kL;
            if (i == j && ri[e] == cj[e] && i * NB + ri[e] < a.n) gnoise += w;
        }
    put(0, gvL);
    put(1 + a.D, gvD);
    put(2 + 2 * a.D, grho);
    put(3 + 2 * a.D, gnoise);
    for (int d = 0; d < a.D; ++d) {
        double tl = 0.0, td = 0.0;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const double df = xi[ri[e] * XS + d] - xj[cj[e] * XS + d];
            tl += cL[e] * df * df;
            td += cD[e] * df * df;
        }
        put(1 + d, tl);
        put(2 + a.D + d, td);
    }
    __syncthreads();
    reduce_entries([&](int qx, double v) {   // gpart [quantity][task]: coalesced reduction
        if (qx >= 1 && qx <= a.D) { const double l = th.lL(qx - 1); v /= l * l * l; }
        else if (qx >= 2 + a.D && qx <= 1 + 2 * a.D) { const double l = th.lD(qx - 2 - a.D); v /= l * l * l; }
        return v;
    });
    grad_next_setup(a);
}

size_t grad_smem_bytes(int nb, int G, int nil2) {
    const size_t region = 2 * (size_t)(nb == 32 ? GRAD_NBUF<32> : GRAD_NBUF<64>) * nb * (nb + 2);
    const size_t epi = (size_t)(nb == 32 ? GRAD_RED_OFF<32> : GRAD_RED_OFF<64>) + (size_t)G * GRAD_RLD + nil2;
    return sizeof(double) * std::max(region, epi);
}

// ============================================================ K4: finalize (+Adam)


// Stage 2: LML, gradient output and the optional Keras-Adam step; run by the last
// item workgroup of k_reduce_items to arrive.
// Adam inputs of theta entry threadIdx.x, loaded at kernel start by the sentinel protocol
struct FinPre {
    double u, m, v;
    int tr;
};
__device__ void adam_body(const FinArgs& a, int G, int s, const double* gsh, const int* tsh, const FinPre* pre);
static_assert(FIN_MAXG >= kernel_theta_size(MFGP_MAX_LF, MAXD) && FIN_MAXG >= kernel_theta_size(0, MAXD),
              "finalize_body stages every theta entry in LDS");
static_assert(FIN_MAXG <= NTHREADS, "one theta entry per finalize thread");
// gsh = [sum Z^2, sum log L_ii, grad_0 .. grad_{G-1}] in LDS (read after a barrier)
__device__ void finalize_from(const FinArgs& a, int G, const double* gsh, const int* tsh, int info0, int s,
                              const FinPre* pre) {
    const double LOG2PI = 1.8378770664093453;
    double lml = -0.5 * gsh[0] - (double)a.P * gsh[1] - 0.5 * (double)a.n * (double)a.P * LOG2PI;
    if (info0 != 0) lml = NAN;
    if (a.adam && info0 == 0) adam_body(a, G, s, gsh + 2, a.tie ? tsh : nullptr, pre);
    if (threadIdx.x == 0) a.out[0] = lml;
    if (a.want_grad)
        for (int q = threadIdx.x; q < G; q += NTHREADS) a.out[1 + q] = gsh[2 + q];
    if (!a.adam) return;
    if (threadIdx.x == 0) a.loss_hist[s] = -lml;
    __syncthreads();   // every wave has read *a.step
    if (threadIdx.x == 0 && info0 == 0) *a.step = s + 1;
}
__device__ void finalize_body(const FinArgs& a) {
    const int G = a.G ? a.G : theta_size(a.D);
    // every input in ONE round trip into LDS, before the first store (the outputs may alias them
    // as far as the compiler knows; a dependent sc1 load per tied entry cost ~8 us per step)
    __shared__ double gsh[FIN_MAXG + 2];   // [sum Z^2, sum log L_ii, grad_0 .. grad_{G-1}]
    __shared__ int tsh[FIN_MAXG];
    for (int q = threadIdx.x; q < G + 2 && q < FIN_MAXG + 2; q += NTHREADS) gsh[q] = ld_coherent(a.items + q);
    if (a.adam && a.tie)
        for (int q = threadIdx.x; q < G && q < FIN_MAXG; q += NTHREADS) tsh[q] = a.tie[q];
    const int info0 = a.info[0];
    const int s = a.adam ? *a.step : 0;
    __syncthreads();
    finalize_from(a, G, gsh, tsh, info0, s, nullptr);
}

__device__ void adam_body(const FinArgs& a, int G, int s, const double* gsh, const int* tsh, const FinPre* pre) {
    const double t = (double)(s + 1);
    const double alpha = a.lr * sqrt(1.0 - pow(a.b2, t)) / (1.0 - pow(a.b1, t));
    for (int q = threadIdx.x; q < G; q += NTHREADS) {
        if (pre ? pre->tr : a.trainable[q]) {
            const double uq = pre ? pre->u : a.u[q];
            double gc = gsh[q];
            if (tsh) {   // a variable shared by several theta entries gets the summed gradient
                gc = 0.0;
                for (int r = 0; r < G; ++r)
                    if (tsh[r] == tsh[q]) gc += gsh[r];
            }
            const double g = (-gc) / (exp(-uq) + 1.0);   // loss = -lml; TF SoftplusGrad form
            double mq = pre ? pre->m : a.m[q], vq = pre ? pre->v : a.v[q];
            mq += (g - mq) * (1.0 - a.b1);
            vq += (g * g - vq) * (1.0 - a.b2);
            const double un = uq - (mq * alpha) / (sqrt(vq) + a.eps);
            a.m[q] = mq;
            a.v[q] = vq;
            a.u[q] = un;
            a.theta[q] = tf_softplus(un) + (q == a.noise_index ? 1e-6 : 0.0);
        }
    }
}

// Sentinel protocol, workgroup 0 (FinArgs::flag): the finalize inputs (info, step, Adam state,
// ties) are loaded before its own item is summed, then thread q < gridDim.x polls item q (sc1)
// until it is no longer FLOW_SENTINEL.  Against store -> drain -> atomic arrival -> sc1 reload
// by the last workgroup, two memory round trips fewer, and the Adam loads off the tail.  A poll
// that exceeds REDUCE_TIMEOUT_TICKS (100 MHz) marks the evaluation failed: NaN LML, no Adam step.
constexpr long long REDUCE_TIMEOUT_TICKS = 5000000;   // 50 ms
__device__ void reduce_items_wg0(const FinArgs& a) {
    __shared__ double gsh[FIN_MAXG + 2];
    __shared__ int tsh[FIN_MAXG];
    __shared__ double red[4];
    __shared__ int tmo;
    const int t = threadIdx.x;
    const int G = a.G ? a.G : theta_size(a.D);
    FinPre pre{0.0, 0.0, 0.0, 0};
    if (a.adam && t < G) {
        pre.tr = a.trainable[t];
        pre.u = a.u[t];
        pre.m = a.m[t];
        pre.v = a.v[t];
        if (a.tie) tsh[t] = a.tie[t];
    }
    int info0 = a.info[0];
    const int s = a.adam ? *a.step : 0;
    if (t == 0) tmo = 0;
    double z = 0.0;
    for (int e = t; e < a.nz; e += NTHREADS) z += a.zpart[e];
    z = block_sum(z, red);   // (its barriers also order tmo = 0 before the polls)
    if (t >= 1 && t < (int)gridDim.x) {
        const long long t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const double v = ld_coherent(a.items + t);
            if ((unsigned long long)__double_as_longlong(v) != FLOW_SENTINEL) { gsh[t] = v; break; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > REDUCE_TIMEOUT_TICKS) { gsh[t] = NAN; tmo = 1; break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (t == 0) gsh[0] = z;
    // the flow's abort word (a hand-off that gave up): the evaluation timed out, whatever info says
    // (the flow initialises info in its first workgroup, which can land after an early give-up)
    const int aborted = a.abortw ? __hip_atomic_load(a.abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    __syncthreads();
    if ((tmo && info0 == 0) || aborted) {   // (eager callers see it as a timed-out evaluation)
        info0 = MFGP_FLOW_TIMEOUT;
        if (t == 0) const_cast<int*>(a.info)[0] = MFGP_FLOW_TIMEOUT;
    }
    if (a.abortw && t == 0 && aborted) __hip_atomic_store(a.abortw, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    finalize_from(a, G, gsh, tsh, info0, s, &pre);
}

// Stage 1 of the step reduction: workgroup `it` sums item `it` of
// [sum Z^2, sum log L_ii, grad_0 .. grad_{G-1}] (partials stored [item][task]) with
// all 256 threads in flight at once; deterministic order.
__global__ __launch_bounds__(NTHREADS) void k_reduce_items(FinArgs a) {
    __shared__ double red[4];
    const int it = blockIdx.x;
    if (a.flag && it == 0) { reduce_items_wg0(a); return; }
    double s = 0.0;
    if (it == 0) {
        for (int e = threadIdx.x; e < a.nz; e += NTHREADS) s += a.zpart[e];
    } else if (it == 1) {   // 8 loads in flight per thread before the logs
        for (int e0 = threadIdx.x; e0 < a.n; e0 += 8 * NTHREADS) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = (e0 + u * NTHREADS < a.n) ? a.ldiag[e0 + u * NTHREADS] : 1.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) s += log(v[u]);
        }
    } else {
        const double* src = a.gpart + (long)(it - 2) * a.ng;
        double s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int e = threadIdx.x;
        for (; e + 3 * NTHREADS < a.ng; e += 4 * NTHREADS) {
            s += src[e];
            s1 += src[e + NTHREADS];
            s2 += src[e + 2 * NTHREADS];
            s3 += src[e + 3 * NTHREADS];
        }
        for (; e < a.ng; e += NTHREADS) s += src[e];
        s = (s + s1) + (s2 + s3);
    }
    s = block_sum(s, red);
    if (a.flag) {   // sentinel protocol: workgroup 0 polls this item
        if (threadIdx.x == 0) st_coherent(a.items + it, s);
        return;
    }
    __shared__ int last;
    if (threadIdx.x == 0) {
        st_coherent(a.items + it, s);
        drain_stores();
        last = arrive(a.cnt) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    finalize_body(a);
}


__global__ void k_theta_from_u(const double* u, double* theta, int G, int noise_index) {
    const int q = threadIdx.x;
    if (q < G) theta[q] = tf_softplus(u[q]) + (q == noise_index ? 1e-6 : 0.0);
}

// ============================================================ K6: predict

template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_pred_a(PredAArgs a) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Ls = smem;
    double* Ks = Ls + E;
    const int i = blockIdx.x / a.Ts, cs = blockIdx.x % a.Ts;
    Acc<NB> acc;
    acc_zero(acc);
    for (int m = 0; m <= i; ++m) {
        tile_load<NB>(Ls, a.Xo + (long)i * NB * a.ldx + (long)m * NB, a.ldx);
        tile_load<NB>(Ks, a.Kmn + (long)m * NB * a.ldk + (long)cs * NB, a.ldk);
        __syncthreads();
        tile_mma<NB, false, false>(acc, Ls, Ks, 1.0);
        __syncthreads();
    }
    acc_store(acc, a.Am + (long)i * NB * a.ldam + (long)cs * NB, a.ldam);
}


template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_pred_out(PredOutArgs a) {
    constexpr int S = TileCfg<NB>::S;
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* As = smem;
    double* Zs = As + E;
    double* vs = Zs + E;              // NB
    const int cs = blockIdx.x / a.Tp, cy = blockIdx.x % a.Tp;
    Acc<NB> acc;
    acc_zero(acc);
    double vpart = 0.0;               // thread c < NB accumulates column c
    for (int i = 0; i < a.T; ++i) {
        tile_load<NB>(As, a.Am + (long)i * NB * a.ldam + (long)cs * NB, a.ldam);
        tile_load<NB>(Zs, a.Xo + (long)i * NB * a.ldx + (long)(a.T + cy) * NB, a.ldx);
        __syncthreads();
        if (cy == 0 && threadIdx.x < NB)
            for (int r = 0; r < NB; ++r) { const double v = As[r * S + threadIdx.x]; vpart += v * v; }
        tile_mma<NB, true, false>(acc, As, Zs, 1.0);   // mean tile = sum_i A_i^T Z_i
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < TileCfg<NB>::NBLK; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int s = cs * NB + acc_row<NB>(q, r), c = cy * NB + acc_col<NB>(q);
            if (s < a.nstar && c < a.p) a.mean[(long)s * a.ldm + c] = acc.v[q][r];
        }
    if (cy == 0 && threadIdx.x < NB) {
        const int s = cs * NB + threadIdx.x;
        if (s < a.nstar) a.var[s] = a.kdiag[s] - vpart;
    }
    (void)vs;
}

// K_diag (linear.py:106-136)
__global__ void k_kdiag(const double* X, long ldx, int n, int D, const double* theta, double* out, int nlf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double f = X[(long)i * ldx + D];
    if (nlf) {   // graph.py:101-115 (no jitter on the diagonal here)
        const GraphTheta th{theta, D, nlf};
        const int s = graph_source(f, nlf);
        double v = 0.0;
        if (s >= 0 && s < nlf) v = th.v(s);
        else if (s == nlf) {
            for (int k = 0; k < nlf; ++k) v += th.v(k) * (th.rho(k) * th.rho(k));
            v += th.v(nlf);
        }
        out[i] = v;
        return;
    }
    const MFTheta th{theta, D};
    const double rho = th.rho();
    out[i] = (f == 0.0) ? th.vL() : ((f == 1.0) ? th.vL() * (rho * rho) + th.vD() : 0.0);
}

// ============================================================ MFMA self-test
// C = A B for one 16x16x4 f64 MFMA with A[i][k] = i*4+k+1, B[k][j] = 100*k + j (asymmetric).
__global__ void k_selftest_mfma(double* out /* 16x16 */) {
    const int l = threadIdx.x;
    const double a = (double)((l & 15) * 4 + (l >> 4) + 1);
    const double b = (double)(100 * (l >> 4) + (l & 15));
    f64x4 c = {0.0, 0.0, 0.0, 0.0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[((l >> 4) + 4 * r) * 16 + (l & 15)] = c[r];
}

// ============================================================ launch helpers
template <int NB>
void launch_gram(const GramArgs& g, int nblocks, int batch, hipStream_t s) {
    if (!g.padded && !g.nlf) { launch_gram_dense(g, batch, 0, 0, s); return; }
    if (g.Dd == nullptr && g.gorder == nullptr && g.fown == nullptr)
        hipLaunchKernelGGL((k_gram<NB, true>), dim3(nblocks, 1, batch), dim3(NTHREADS), gram_smem_bytes(NB), s, g);
    else
        hipLaunchKernelGGL((k_gram<NB, false>), dim3(nblocks, 1, batch), dim3(NTHREADS), gram_smem_bytes(NB), s, g);
}
// The first diagonal factor of a batch of padded matrices (step "-1" of the tile Cholesky; the
// lean Gram launch leaves it out): A_b(0,0) -> D_0, diag(L) 0..NB-1, info_b.
template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_first_factor(const double* A, long lda, long sA, double* Dd, long sD,
                                                           double* ldiag, long sL, int* info) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int E = TileCfg<NB>::ELEMS;
    double* tile = smem;
    double* rtile = tile + E;
    double* dg = rtile + E;
    int* bad = reinterpret_cast<int*>(dg + NB);
    const int b = blockIdx.z;
    tile_load<NB>(tile, A + b * sA, lda);
    gram_first_factor<NB>(tile, rtile, dg, bad, Dd + b * sD, ldiag + b * sL, info + b);
}
template <int NB>
void launch_first_factor(const double* A, long lda, long sA, double* Dd, long sD, double* ldiag, long sL, int* info,
                         int batch, hipStream_t s) {
    hipLaunchKernelGGL(k_first_factor<NB>, dim3(1, 1, batch), dim3(NTHREADS),
                       sizeof(double) * (2 * TileCfg<NB>::ELEMS + NB + 2), s, A, lda, sA, Dd, sD, ldiag, sL, info);
}
template <int NB>
void launch_chol_steps(CholArgs c, int batch, hipStream_t s) {
    if constexpr (NB == 32) if (batch != 1) {   // one fused launch a step (k_chol_fused), the last row by a panel
        c.alpha = nullptr;
        static bool attr = false;
        const size_t lds = sizeof(double) * (5 * (size_t)TileCfg<NB>::ELEMS + NB + 2);
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_chol_fused<NB>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr = true;
        }
        for (int k = 0; k < c.T; ++k) {
            c.k = k;
            const int rem = c.T - k - 1, ncol = k + 1 + c.Tp;
            if (rem > 0)
                hipLaunchKernelGGL(k_chol_fused<NB>, dim3(rem * (rem + 1) / 2 + rem * ncol, 1, batch), dim3(NTHREADS),
                                   lds, s, c);
            else   // the last step: X_{T-1, c} only
                hipLaunchKernelGGL(k_chol_panel<NB>, dim3(ncol, 1, batch), dim3(NTHREADS),
                                   2 * sizeof(double) * TileCfg<NB>::ELEMS, s, c);
        }
        return;
    }
    if (batch != 1) {   // panel + update launches a step (k_chol_panel); no fused alpha
        c.alpha = nullptr;
        for (int k = 0; k < c.T; ++k) {
            c.k = k;
            const int rem = c.T - k - 1, ncol = k + 1 + c.Tp;
            hipLaunchKernelGGL(k_chol_panel<NB>, dim3(rem + ncol, 1, batch), dim3(NTHREADS),
                               2 * sizeof(double) * TileCfg<NB>::ELEMS, s, c);
            const int nu = rem * (rem + 1) / 2 + rem * ncol;
            if (nu > 0)
                hipLaunchKernelGGL(k_chol_update<NB>, dim3(nu, 1, batch), dim3(NTHREADS), chol_smem_bytes(NB), s, c);
        }
        return;
    }
    for (int k = 0; k < c.T; ++k) {
        c.k = k;
        const int nb = chol_step_blocks(c.T, c.Tp, k, c.alpha != nullptr);
        if (nb > 0)
            hipLaunchKernelGGL(k_chol_step<NB>, dim3(nb, 1, batch), dim3(NTHREADS), chol_smem_bytes(NB), s, c);
    }
}
template <int NB>
void launch_grad(const GradArgs& g, hipStream_t s) {
    const size_t lds = grad_smem_bytes(NB, kernel_theta_size(g.nlf, g.D), (g.nlf ? g.nlf + 1 : 2) * g.D);
    if (g.nlf)
        hipLaunchKernelGGL((k_grad<NB, true>), dim3(grad_tasks(g.T, g.chunk)), dim3(NTHREADS), lds, s, g);
    else
        hipLaunchKernelGGL((k_grad<NB, false>), dim3(grad_tasks(g.T, g.chunk)), dim3(NTHREADS), lds, s, g);
}
template <int NB>
void launch_pred(const PredAArgs& pa, const PredOutArgs& po, int T, hipStream_t s) {
    hipLaunchKernelGGL(k_pred_a<NB>, dim3(T * pa.Ts), dim3(NTHREADS), 2 * sizeof(double) * NB * (NB + 2), s, pa);
    hipLaunchKernelGGL(k_pred_out<NB>, dim3(pa.Ts * po.Tp), dim3(NTHREADS),
                       sizeof(double) * (2 * NB * (NB + 2) + NB), s, po);
}

// ============================================================ small problems: one launch
// The whole value + gradient (+ Keras Adam) evaluation of the AR1 kernel's GPR LML for n <= 64,
// p <= 64, D <= TINY_MAXD in ONE workgroup (mfgpflow/linear.py:200-214 at the HBS size, N = 53,
// P = 49, D = 5, where the step sequence k_gram -> k_chol_step -> k_grad -> k_reduce_items is four
// dependent launches of a few microseconds of work each).  Everything stays in LDS, in NB = 32
// tiles of stride S (the T <= 2 tile grid of the step schedule):
//   K (the same entries as k_gram, bit for bit) -> D_0 = L_00^{-1} (tile_potrf_inv_w1_wave),
//   L_10 = K_10 D_0^T, K_11 -= L_10 L_10^T -> D_1, L^{-1}_10 = -D_1 (L_10 D_0);
//   Z = L^{-1} Y, alpha = L^{-T} Z, S_ij = sum_m L^{-1}_mi^T L^{-1}_mj - alpha_i alpha_j^T / P, and
//   k_grad's epilogue (W = -P S against dK/dtheta recomputed from the inputs) on the three lower
//   tiles; then finalize_body's LML / gradient output and adam_body's step.
// LDS hazards: every workgroup barrier of the kernel is TINY_BARRIER(k), k = 1 .. 19 in source
// order; tests/test_tiny_schedule.py restates which LDS doubles each wave reads and writes between
// them (every shape the kernel takes) and checks on the CPU that no two waves touch a double in one
// interval unless both only read, and that each of the 19 barriers orders some such pair.
#define TINY_BARRIER(k) __syncthreads()
constexpr int TINY_MAXD = 16, TINY_XS = TINY_MAXD + 1, TINY_N = 64, TINY_P = 64;

struct TinyArgs {
    const double* X; long ldx;
    const double* Y; long ldy;
    const double* theta;
    int n, p, D, want_grad;
    int* info;
    FinArgs f;
    // PRED (predict_f): X* rows (ns <= TINY_N), the mean [ns, p] and the variance [ns]
    const double* Xs; long ldxs; int ns;
    double* mean; long ldm;
    double* var;
};

// PRED: the same factorization and Z = L^{-1} Y, then predict_f's A = L^{-1} K(X, X*), mean = A^T Z
// and var = K_diag(X*) - colsum(A^2) (linear.py:237-286; predict_impl's k_pred_a / k_pred_out in
// the same summation order) instead of the gradient
template <bool PRED>
__global__ __launch_bounds__(NTHREADS) void k_gpr_tiny(TinyArgs a) {
    constexpr int S = TileCfg<32>::S, E = TileCfg<32>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int D = a.D, n = a.n, p = a.p;
    const int T = (n + 31) / 32, Tp = (p + 31) / 32;
    const int G = theta_size(D);
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    auto slot = [&](int i) { return smem + (long)i * E; };
    double* K00 = slot(0); double* K10 = slot(1); double* K11 = slot(2);
    double* D0 = slot(3); double* D1 = slot(4); double* L10 = slot(5);
    auto Yt = [&](int r, int c) { return slot(6 + 2 * r + c); };
    double* xr = slot(11);                         // raw rows 64 x TINY_XS (gradient epilogue)
    double* misc = slot(12);
    auto ELt = [&](int tl) { return slot(13 + tl); };   // exp(-r^2 / 2) of the Gram's K_L, tiles (0,0) (1,0) (1,1)
    double* dg = misc;                             // 64
    int* bad = reinterpret_cast<int*>(misc + 64);  // 2
    double* il = misc + 66;                        // 2 x TINY_MAXD   1/l    (Gram)
    double* il2 = il + 2 * TINY_MAXD;              // 2 x TINY_MAXD   1/l^2  (gradient)
    double* red = il2 + 2 * TINY_MAXD;             // (G + 2) x 4     wave partials
    double* gsh = red + 4 * (2 * TINY_MAXD + 6);   // G + 2
    int* tsh = reinterpret_cast<int*>(gsh + 2 * TINY_MAXD + 6);
    double* lv = gsh + 2 * (2 * TINY_MAXD + 6);    // 2 x TINY_MAXD   the lengthscales
    // Gram staging in the Y / alpha slots (free until Y is loaded)
    double* aL = slot(6);
    double* aD = aL + TINY_N * TINY_XS;
    double* nL = aD + TINY_N * TINY_XS;
    double* nD = nL + TINY_N;
    double* fl = nD + TINY_N;
    const MFTheta th{a.theta, D};
    MFScal sc{a.theta[0], a.theta[1 + D], a.theta[2 + 2 * D]};
    const double noise = a.theta[3 + 2 * D];
    // Y (zero padded), loaded now and put into its LDS tiles once the Gram staging is consumed
    constexpr int YPER = TINY_N * TINY_P / NTHREADS;
    double yv[YPER];
#pragma unroll
    for (int q = 0; q < YPER; ++q) {
        const int e = t + q * NTHREADS, tl = e >> 10, r = (e >> 5) & 31, c = e & 31;
        const int ti = tl / Tp, tc = tl % Tp;
        const int gi = 32 * ti + r, gc = 32 * tc + c;
        yv[q] = (e < T * Tp * 1024 && gi < n && gc < p) ? a.Y[(long)gi * a.ldy + gc] : 0.0;
    }
    // the Adam state, loaded now: its latency hides under the whole evaluation (adam_body would
    // issue these loads, dependent on *step, at the very end)
    // (theta entry q = t - 64: wave 1 owns the Adam step, so its step-size and softplus-gradient
    // factors are formed while wave 0 factors D_0)
    const FinArgs& f = a.f;
    const int aq = t - 64;
    const bool aown = aq >= 0 && aq < G;
    double pu = 0.0, pm = 0.0, pv = 0.0;
    int ptr = 0, ptie = 0, pst = 0;
    if (f.adam) {
        if (aown) {
            pu = f.u[aq]; pm = f.m[aq]; pv = f.v[aq]; ptr = f.trainable[aq];
            ptie = f.tie ? f.tie[aq] : aq;
        }
        pst = *f.step;
    }
    double a_alpha = 0.0, a_eu = 0.0;
    // ---- stage: raw rows, scaled rows (x * rcp_nr(l), as k_gram), norms, fidelity flags.  The row
    //      loads are issued before the lengthscale reciprocals wait on theta (one round trip)
    constexpr int XPER = (TINY_N * TINY_XS + NTHREADS - 1) / NTHREADS;
    double xv0[XPER];
#pragma unroll
    for (int q = 0; q < XPER; ++q) {
        const int e = t + q * NTHREADS, r = e / TINY_XS, d = e % TINY_XS;
        xv0[q] = (e < TINY_N * TINY_XS && r < n && d <= D) ? a.X[(long)r * a.ldx + d] : 0.0;
    }
    if (t < D) {
        il[t] = rcp_nr(a.theta[1 + t]);
        il[TINY_MAXD + t] = rcp_nr(a.theta[2 + D + t]);
        il2[t] = 1.0 / (th.lL(t) * th.lL(t));
        il2[TINY_MAXD + t] = 1.0 / (th.lD(t) * th.lD(t));
        lv[t] = th.lL(t);
        lv[TINY_MAXD + t] = th.lD(t);
    }
    const int D4 = pad4(D);
#pragma unroll
    for (int q = 0; q < XPER; ++q)
        if (t + q * NTHREADS < TINY_N * TINY_XS) xr[t + q * NTHREADS] = xv0[q];
    TINY_BARRIER(1);
    for (int e = t; e < TINY_N * TINY_XS; e += NTHREADS) {
        const int r = e / TINY_XS, d = e % TINY_XS;
        const double x = (d < D) ? xr[e] : 0.0;
        aL[e] = (d < D4 && d < D) ? x * il[d] : 0.0;
        aD[e] = (d < D4 && d < D) ? x * il[TINY_MAXD + d] : 0.0;
    }
    if (t < TINY_N) fl[t] = (t < n) ? xr[t * TINY_XS + D] : -1.0;
    TINY_BARRIER(2);
    if (t < TINY_N) { nL[t] = dot4(aL + t * TINY_XS, aL + t * TINY_XS, D4); nD[t] = dot4(aD + t * TINY_XS, aD + t * TINY_XS, D4); }
    TINY_BARRIER(3);
    // ---- K tiles (0,0), (1,0), (1,1): k_gram's padded-entry arithmetic, the dot products a_i . a_j
    //      of the expanded r^2 on the matrix core (16 x 16 blocks, three per wave, D4 / 4
    //      v_mfma_f64_16x16x4 each) instead of a dot4 chain of 2 D4 LDS reads an entry
    {
        const int lc = lane & 15, kk = lane >> 4;
        const double rho = sc.rho();
        for (int bq = 0; bq < 3; ++bq) {
            const int blk = w * 3 + bq, tl = blk >> 2, sub = blk & 3;
            const int ti = tl == 0 ? 0 : 1, tj = tl == 2 ? 1 : 0;
            if (ti >= T) continue;
            const int rb = 2 * ti + (sub >> 1), cb = 2 * tj + (sub & 1);
            f64x4 dl = {0.0, 0.0, 0.0, 0.0}, dd = {0.0, 0.0, 0.0, 0.0};
            for (int s4 = 0; s4 < D4; s4 += 4) {
                dl = __builtin_amdgcn_mfma_f64_16x16x4f64(aL[(16 * rb + lc) * TINY_XS + s4 + kk],
                                                          aL[(16 * cb + lc) * TINY_XS + s4 + kk], dl, 0, 0, 0);
                dd = __builtin_amdgcn_mfma_f64_16x16x4f64(aD[(16 * rb + lc) * TINY_XS + s4 + kk],
                                                          aD[(16 * cb + lc) * TINY_XS + s4 + kk], dd, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int gi = 16 * rb + kk + 4 * q, gj = 16 * cb + lc;
                const double el = exp(-0.5 * (-2.0 * dl[q] + (nL[gi] + nL[gj])));
                const double kl = sc.vL() * el;
                ELt(tl)[(gi - 32 * ti) * S + gj - 32 * tj] = el;   // dK/dvL for the gradient epilogue
                const double fa = fl[gi], fb = fl[gj];
                const bool L1 = (fa == 0.0), H1 = (fa == 1.0), L2 = (fb == 0.0), H2 = (fb == 1.0);
                const double kD = (H1 && H2) ? sc.vD() * exp(-0.5 * (-2.0 * dd[q] + (nD[gi] + nD[gj]))) : 0.0;
                const double vhh = kl * (rho * rho) + kD;
                double v = (L1 && L2) ? kl : (!(H1 && H2) ? kl * rho : vhh);
                if (!(L1 || H1) || !(L2 || H2)) v = 0.0;
                if (gi == gj) v = (gi < n) ? v + noise : 1.0;
                slot(tl)[(gi - 32 * ti) * S + gj - 32 * tj] = v;
            }
        }
    }
    TINY_BARRIER(4);
    // reuse: the Gram staging (slots 6-8) is dead after the barrier above; slots 6-9 become Y tiles
    // ---- factor: D_0; L_10, K_11 update, D_1, L^{-1}_10
    if (w == 0) tile_potrf_inv_w1_wave(K00, S, K00, D0, dg, &bad[0]);
    else if (w == 1 && f.adam && aown) {   // adam_body's step-size and SoftplusGrad factors
        const double tt = (double)(pst + 1);
        a_alpha = f.lr * sqrt(1.0 - pow(f.b2, tt)) / (1.0 - pow(f.b1, tt));
        a_eu = exp(-pu) + 1.0;
    }
    TINY_BARRIER(5);
    // reuse: K00 (slot 0, the factor's in-place scratch) is dead after the barrier above (Ki00 later)
    if (T > 1) {
        Acc<32> acc;
        acc_zero(acc);
        tile_mma<32, false, true>(acc, K10, D0, 1.0);      // L_10 = K_10 D_0^T
        acc_to_lds(acc, L10);
        TINY_BARRIER(6);
        // reuse: K10 (slot 1) was last read by the product above, before this barrier; T goes there
        acc_load<32>(acc, K11, S);
        tile_mma<32, false, true>(acc, L10, L10, -1.0);    // K_11 - L_10 L_10^T
        acc_to_lds(acc, K11);   // each wave rewrites the block it read: no barrier in between
        acc_zero(acc);
        tile_mma<32, false, false>(acc, L10, D0, 1.0);     // T = L_10 D_0 (into K10's slot)
        acc_to_lds(acc, K10);
        TINY_BARRIER(7);
        if (w == 0) tile_potrf_inv_w1_wave(K11, S, K11, D1, dg + 32, &bad[1]);
        TINY_BARRIER(8);
        // reuse: K11 (slot 2, the factor's scratch) and L_10 (slot 5, last read by T = L_10 D_0
        // before the barrier ahead of the factor) are dead; L^{-1}_10 is written over L_10 below
        acc_zero(acc);
        tile_mma<32, false, false>(acc, D1, K10, -1.0);    // L^{-1}_10 = -D_1 T (over L10)
        acc_to_lds(acc, L10);   // (read, and T's slot 1 rewritten as Ki10, only after the barrier below)
    }
    // ---- Y tiles (zero padded; loaded at the start)
#pragma unroll
    for (int q = 0; q < YPER; ++q) {
        const int e = t + q * NTHREADS, tl = e >> 10, r = (e >> 5) & 31, c = e & 31;
        if (e < T * Tp * 1024) Yt(tl / Tp, tl % Tp)[r * S + c] = yv[q];
    }
    // ---- one stage of independent products: Z = L^{-1} Y for every column tile (registers; sum Z^2
    //      is the LML's quadratic term in the step path's form) and K^{-1} = L^{-T} L^{-1} (lower
    //      tiles, over the consumed K00 / T / K11 slots); then alpha = L^{-T} Z, each column tile's
    //      results replacing its Y tiles (all read first)
    TINY_BARRIER(9);   // the Y tiles and every wave's block of L^{-1}_10 are in; every read of T is done
    // reuse: T (slot 1) is dead after the barrier above; Ki10 (or, in PRED, K(X, X*)) goes there
    double* Ki00 = slot(0); double* Ki10 = slot(1); double* Ki11 = slot(2);
    double z2 = 0.0;
    Acc<32> zc[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (c >= Tp) break;
        acc_zero(zc[c][0]);
        tile_mma<32, false, false>(zc[c][0], D0, Yt(0, c), 1.0);
#pragma unroll
        for (int r = 0; r < 4; ++r) z2 += zc[c][0].v[0][r] * zc[c][0].v[0][r];
        if (T > 1) {
            acc_zero(zc[c][1]);
            tile_mma<32, false, false>(zc[c][1], L10, Yt(0, c), 1.0);
            tile_mma<32, false, false>(zc[c][1], D1, Yt(1, c), 1.0);
#pragma unroll
            for (int r = 0; r < 4; ++r) z2 += zc[c][1].v[0][r] * zc[c][1].v[0][r];
        }
    }
    if (!PRED) {
        Acc<32> acc;
        acc_zero(acc);
        tile_mma<32, true, false>(acc, D0, D0, 1.0);
        if (T > 1) tile_mma<32, true, false>(acc, L10, L10, 1.0);
        acc_to_lds(acc, Ki00);
        if (T > 1) {
            acc_zero(acc);
            tile_mma<32, true, false>(acc, D1, L10, 1.0);
            acc_to_lds(acc, Ki10);
            acc_zero(acc);
            tile_mma<32, true, false>(acc, D1, D1, 1.0);
            acc_to_lds(acc, Ki11);
        }
    }
    TINY_BARRIER(10);
    // reuse: the Y tiles (slots 6-9) were last read by the Z products, before the barrier above
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (c >= Tp) break;
        acc_to_lds(zc[c][0], Yt(0, c));
        if (T > 1) acc_to_lds(zc[c][1], Yt(1, c));
    }
    TINY_BARRIER(11);
    if constexpr (PRED) {
        const int ns = a.ns, Ts = (ns + 31) / 32;
        const double rho = sc.rho();
        double* xs = slot(13);   // raw X* rows (the Gram's exp tiles are not needed here)
        auto Km = [&](int i, int c) { return slot(i == 0 ? c : (c == 0 ? 2 : 10)); };   // K(X, X*), then A
        for (int e = t; e < TINY_N * TINY_XS; e += NTHREADS) {
            const int r = e / TINY_XS, d = e % TINY_XS;
            xs[e] = (r < ns && d <= D) ? a.Xs[(long)r * a.ldxs + d] : 0.0;
        }
        TINY_BARRIER(12);
        // reuse: slots 0, 1, 2 (K00 / T / K11, consumed) and 10 become K(X, X*)
        for (int e = t; e < T * Ts * 1024; e += NTHREADS) {   // K(X, X*): the AR1 kernel, exact masks
            const int tl = e >> 10, r = (e >> 5) & 31, c = e & 31;
            const int ti = tl / Ts, tc = tl % Ts;
            const int gi = 32 * ti + r, gs = 32 * tc + c;
            double v = 0.0;
            if (gi < n && gs < ns) {
                const double fa = xr[gi * TINY_XS + D], fb = xs[gs * TINY_XS + D];
                const bool L1 = fa == 0.0, H1 = fa == 1.0, L2 = fb == 0.0, H2 = fb == 1.0;
                double s2 = 0.0, s2d = 0.0;
                for (int d = 0; d < D; ++d) {
                    const double df = xr[gi * TINY_XS + d] - xs[gs * TINY_XS + d];
                    s2 += (df * df) * il2[d];
                    s2d += (df * df) * il2[TINY_MAXD + d];
                }
                const double kl = sc.vL() * exp(-0.5 * s2);
                const double kD = (H1 && H2) ? sc.vD() * exp(-0.5 * s2d) : 0.0;
                v = (L1 && L2) ? kl : (!(H1 && H2) ? kl * rho : kl * (rho * rho) + kD);
                if (!(L1 || H1) || !(L2 || H2)) v = 0.0;
            }
            Km(ti, tc)[r * S + c] = v;
        }
        TINY_BARRIER(13);
        Acc<32> A0[2], A1[2];   // A = L^{-1} Kmn, column tile c
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c >= Ts) break;
            acc_zero(A0[c]);
            tile_mma<32, false, false>(A0[c], D0, Km(0, c), 1.0);
            if (T > 1) {
                acc_zero(A1[c]);
                tile_mma<32, false, false>(A1[c], L10, Km(0, c), 1.0);
                tile_mma<32, false, false>(A1[c], D1, Km(1, c), 1.0);
            }
        }
        TINY_BARRIER(14);
        // reuse: K(X, X*) (slots 0, 1, 2, 10) was last read by the A products, before the barrier above
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c >= Ts) break;
            acc_to_lds(A0[c], Km(0, c));
            if (T > 1) acc_to_lds(A1[c], Km(1, c));
        }
        TINY_BARRIER(15);
        for (int cs = 0; cs < Ts; ++cs)   // mean tile (cs, cy) = sum_i A(i, cs)^T Z(i, cy)
            for (int cy = 0; cy < Tp; ++cy) {
                Acc<32> m;
                acc_zero(m);
                tile_mma<32, true, false>(m, Km(0, cs), Yt(0, cy), 1.0);
                if (T > 1) tile_mma<32, true, false>(m, Km(1, cs), Yt(1, cy), 1.0);
#pragma unroll
                for (int q = 0; q < TileCfg<32>::NBLK; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int gs = 32 * cs + acc_row<32>(q, r), gc = 32 * cy + acc_col<32>(q);
                        if (gs < ns && gc < p) a.mean[(long)gs * a.ldm + gc] = m.v[q][r];
                    }
            }
        if (t < ns) {   // var = K_diag(X*) - sum_i sum_r A(i, cs)[r][s]^2 (k_pred_out's order)
            const int cs = t >> 5, cc = t & 31;
            double sq = 0.0;
            for (int i = 0; i < T; ++i)
                for (int r = 0; r < 32; ++r) {
                    const double v = Km(i, cs)[r * S + cc];
                    sq += v * v;
                }
            const double fb = xs[t * TINY_XS + D];
            const double kd = (fb == 0.0) ? sc.vL() : ((fb == 1.0) ? sc.vL() * (rho * rho) + sc.vD() : 0.0);
            a.var[t] = kd - sq;
        }
        if (t == 0) {
            const int b0 = bad[0], b1 = (T > 1) ? bad[1] : 0;
            a.info[0] = b0 ? b0 : (b1 ? 32 + b1 : 0);
        }
        return;
    }
    Acc<32> ac[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (c >= Tp) break;
        acc_zero(ac[c][0]);
        tile_mma<32, true, false>(ac[c][0], D0, Yt(0, c), 1.0);
        if (T > 1) {
            tile_mma<32, true, false>(ac[c][0], L10, Yt(1, c), 1.0);
            acc_zero(ac[c][1]);
            tile_mma<32, true, false>(ac[c][1], D1, Yt(1, c), 1.0);
        }
    }
    TINY_BARRIER(16);
    // reuse: the Z tiles (slots 6-9) were last read by the alpha products, before the barrier above
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (c >= Tp) break;
        acc_to_lds(ac[c][0], Yt(0, c));
        if (T > 1) acc_to_lds(ac[c][1], Yt(1, c));
    }
    auto At = [&](int r, int c) { return Yt(r, c); };
    double ld = 0.0;
    if (t < n) ld = log(dg[t]);
    TINY_BARRIER(17);
    // ---- gradient: S tiles and k_grad's epilogue (per element: its weights; per dimension: the
    //      lengthscale sums, reduced at once, so no per-thread array is indexed at run time)
    double cLe[12], cDe[12];
    int gie[12], gje[12];
    double gvL = 0.0, gvD = 0.0, grho = 0.0, gnoise = 0.0;
#pragma unroll
    for (int e = 0; e < 12; ++e) { cLe[e] = 0.0; cDe[e] = 0.0; gie[e] = 0; gje[e] = 0; }
    if (a.want_grad) {
        const double invP = 1.0 / (double)p;
        const double rho = sc.rho();
#pragma unroll
        for (int tl = 0; tl < 3; ++tl) {
            if (tl > 0 && T < 2) continue;
            const int ti = tl == 0 ? 0 : 1, tj = tl == 2 ? 1 : 0;
            Acc<32> acc;
            acc_load<32>(acc, tl == 0 ? Ki00 : (tl == 1 ? Ki10 : Ki11), S);
            for (int c = 0; c < Tp; ++c) tile_mma<32, false, true>(acc, At(ti, c), At(tj, c), -invP);
            const double wscale = ((ti == tj) ? 0.5 : 1.0) * (-(double)p);
            // dK/dvL = exp(-r^2 / 2) as the Gram formed it (the expanded r^2 of GPflow's K, whose
            // TF gradient this is); the HF x HF part's squared distance (four entries side by side,
            // one LDS round trip a dimension, each sum in dimension order) and exponential only in
            // a wave that holds such a pair (HBS: 3 HF points)
            const int gj = 32 * tj + acc_col<32>(0);
            const bool H2c = gj < n && xr[gj * TINY_XS + D] == 1.0;
            bool hhw = false;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = 32 * ti + acc_row<32>(0, r);
                hhw |= H2c && gi < n && xr[gi * TINY_XS + D] == 1.0;
            }
            double s2dv[4] = {0.0, 0.0, 0.0, 0.0};
            if (__ballot(hhw) != 0) {   // wave-uniform
                for (int d = 0; d < D; ++d) {
                    const double xj = xr[gj * TINY_XS + d], i2 = il2[TINY_MAXD + d];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double df = xr[(32 * ti + acc_row<32>(0, r)) * TINY_XS + d] - xj;
                        s2dv[r] += (df * df) * i2;
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = 4 * tl + r;
                const int gi = 32 * ti + acc_row<32>(0, r);
                gie[e] = gi;
                gje[e] = gj;
                const double f1 = (gi < n) ? xr[gi * TINY_XS + D] : -1.0, f2 = (gj < n) ? xr[gj * TINY_XS + D] : -1.0;
                const bool L1 = f1 == 0.0, H1 = f1 == 1.0, L2 = f2 == 0.0, H2 = f2 == 1.0;
                const bool live = (L1 || H1) && (L2 || H2);
                const double s2d = s2dv[r];
                const double wv = acc.v[0][r] * wscale;
                const double eL = live ? ELt(tl)[acc_row<32>(0, r) * S + acc_col<32>(0)] : 0.0;
                const double kL = sc.vL() * eL;
                double eD = 0.0;
                if (H1 && H2) eD = exp(-0.5 * s2d);
                const double kD = sc.vD() * eD;
                const double si = L1 ? 1.0 : (H1 ? rho : 0.0), sj = L2 ? 1.0 : (H2 ? rho : 0.0);
                const double hi = H1 ? 1.0 : 0.0, hj = H2 ? 1.0 : 0.0;
                cLe[e] = wv * si * sj * kL;
                cDe[e] = wv * hi * hj * kD;
                gvL += wv * si * sj * eL;
                gvD += wv * hi * hj * eD;
                grho += wv * (hi * sj + si * hj) * kL;
                if (ti == tj && gi == gj && gi < n) gnoise += wv;
            }
        }
    }
    // ---- reductions (L^{-1} is consumed: its slots hold 64 quad partials per quantity): quantity
    //      q < G the gradient entry q, G the quadratic term, G + 1 sum log L_ii
    // reuse: D_0, D_1, L^{-1}_10 (slots 3-5) were last read by the K^{-1} / Z / alpha products, before
    // TINY_BARRIER(16); the reduction buffer RB spans them (the gradient above reads none of them)
    double* RB = slot(3);
    auto put = [&](int q, double v) {
        v = quad_sum(v);
        if ((lane & 3) == 0) RB[q * 64 + w * 16 + (lane >> 2)] = v;
    };
    put(G, z2);
    put(G + 1, ld);
    if (a.want_grad) {
        put(0, gvL);
        put(1 + D, gvD);
        put(2 + 2 * D, grho);
        put(3 + 2 * D, gnoise);
        for (int d = 0; d < D; ++d) {
            double tl = 0.0, td = 0.0;
#pragma unroll
            for (int e = 0; e < 12; ++e) {
                const double df = xr[gie[e] * TINY_XS + d] - xr[gje[e] * TINY_XS + d];
                tl += cLe[e] * df * df;
                td += cDe[e] * df * df;
            }
            put(1 + d, tl);
            put(2 + D + d, td);
        }
    }
    TINY_BARRIER(18);
    for (int g0 = 0; g0 < G + 2; g0 += NTHREADS / 8) {
        const int qx = g0 + (t >> 3), sub = t & 7;
        double v = 0.0;
        if (qx < G + 2 && (a.want_grad || qx >= G)) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v += RB[qx * 64 + sub * 8 + u];
        }
        v = quad_sum(v);
        v += __shfl_xor(v, 4, 64);
        if (sub == 0 && qx < G + 2) {
            if (qx >= 1 && qx <= D) { const double l = lv[qx - 1]; v /= l * l * l; }
            else if (qx >= 2 + D && qx <= 1 + 2 * D) { const double l = lv[TINY_MAXD + qx - 2 - D]; v /= l * l * l; }
            if (qx < G) gsh[2 + qx] = v;
            else gsh[qx - G] = v;
        }
    }
    if (f.adam && aown) tsh[aq] = ptie;
    if (t == 0) {
        const int b0 = bad[0], b1 = (T > 1) ? bad[1] : 0;
        a.info[0] = b0 ? b0 : (b1 ? 32 + b1 : 0);
    }
    TINY_BARRIER(19);
    // ---- finalize_body / adam_body (LDS staging instead of the item round trip)
    const double LOG2PI = 1.8378770664093453;
    const int info0 = (bad[0] != 0 || (T > 1 && bad[1] != 0)) ? 1 : 0;
    const int st = pst;
    double lml = -0.5 * gsh[0] - (double)p * gsh[1] - 0.5 * (double)n * (double)p * LOG2PI;
    if (info0 != 0) lml = NAN;
    if (f.adam && info0 == 0 && aown && ptr) {   // adam_body's step on the prefetched state
        const double alpha = a_alpha;
        double gc = gsh[2 + aq];
        if (f.tie) {
            gc = 0.0;
            for (int r = 0; r < G; ++r)
                if (tsh[r] == tsh[aq]) gc += gsh[2 + r];
        }
        const double g = (-gc) / a_eu;
        double mq = pm, vq = pv;
        mq += (g - mq) * (1.0 - f.b1);
        vq += (g * g - vq) * (1.0 - f.b2);
        const double un = pu - (mq * alpha) / (sqrt(vq) + f.eps);
        f.m[aq] = mq;
        f.v[aq] = vq;
        f.u[aq] = un;
        f.theta[aq] = tf_softplus(un) + (aq == f.noise_index ? 1e-6 : 0.0);
    }
    if (t == 0) f.out[0] = lml;
    if (a.want_grad)
        for (int q = t; q < G; q += NTHREADS) f.out[1 + q] = gsh[2 + q];
    if (!f.adam) return;
    if (t == 0) {
        f.loss_hist[st] = -lml;
        if (info0 == 0) *f.step = st + 1;
    }
}

size_t gpr_tiny_smem_bytes() {
    return sizeof(double) * (16 * (size_t)TileCfg<32>::ELEMS);
}

bool gpr_tiny_fits(int n, int p, int d, int nlf) {
    return nlf == 0 && n >= 1 && n <= TINY_N && p >= 1 && p <= TINY_P && d >= 1 && d <= TINY_MAXD;
}

void launch_gpr_tiny(const double* X, long ldx, const double* Y, long ldy, const double* theta, int n, int p, int d,
                     int want_grad, int* info, const FinArgs& f, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gpr_tiny<false>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)gpr_tiny_smem_bytes());
        attr = true;
    }
    TinyArgs a{X, ldx, Y, ldy, theta, n, p, d, want_grad, info, f};
    hipLaunchKernelGGL(k_gpr_tiny<false>, dim3(1), dim3(NTHREADS), gpr_tiny_smem_bytes(), s, a);
}

bool gpr_tiny_pred_fits(int n, int p, int d, int nstar) { return gpr_tiny_fits(n, p, d, 0) && nstar >= 1 && nstar <= TINY_N; }

void launch_gpr_tiny_pred(const double* X, long ldx, const double* Y, long ldy, const double* Xs, long ldxs, int nstar,
                          const double* theta, int n, int p, int d, double* mean, long ldm, double* var, int* info,
                          hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gpr_tiny<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)gpr_tiny_smem_bytes());
        attr = true;
    }
    TinyArgs a{};
    a.X = X; a.ldx = ldx; a.Y = Y; a.ldy = ldy; a.theta = theta; a.n = n; a.p = p; a.D = d; a.want_grad = 0;
    a.info = info;
    a.Xs = Xs; a.ldxs = ldxs; a.ns = nstar; a.mean = mean; a.ldm = ldm; a.var = var;
    hipLaunchKernelGGL(k_gpr_tiny<true>, dim3(1), dim3(NTHREADS), gpr_tiny_smem_bytes(), s, a);
}

template void launch_gram<32>(const GramArgs&, int, int, hipStream_t);
template void launch_first_factor<32>(const double*, long, long, double*, long, double*, long, int*, int, hipStream_t);
template void launch_first_factor<64>(const double*, long, long, double*, long, double*, long, int*, int, hipStream_t);
template void launch_gram<64>(const GramArgs&, int, int, hipStream_t);
template void launch_chol_steps<32>(CholArgs, int, hipStream_t);
template void launch_chol_steps<64>(CholArgs, int, hipStream_t);
template void launch_grad<32>(const GradArgs&, hipStream_t);
template void launch_grad<64>(const GradArgs&, hipStream_t);
template void launch_pred<32>(const PredAArgs&, const PredOutArgs&, int, hipStream_t);
template void launch_pred<64>(const PredAArgs&, const PredOutArgs&, int, hipStream_t);

}  // namespace mfgp
