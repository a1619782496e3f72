// Tile catalogue and owner table of the persistent dataflow Cholesky (k_chol_flow,
// mfgp_flow.hip).  Header-only: k_gram's extra workgroup builds the owner table.
#pragma once
#include "mfgp_device.h"
#include "mfgp_internal.h"

namespace mfgp {

// k_gram timeline of a trace-mode call (diagnostic): [3 G] per-workgroup stamps, then [2 G] staging
// stamps at 3 gridDim.x; G bounds the grid of both set-up Grams (k_gram_flow: nb(nb+1)/2 blocks
// of 64 + factor + two set-up workgroups; the looping k_gram: at most T(T+1)/2 tiles + two).
__host__ __device__ inline int flow_gram_dbg_wgs(int T) { return T * (T + 1) / 2 + 4; }
__host__ __device__ inline int flow_gram_dbg_count(int T) { return 5 * flow_gram_dbg_wgs(T); }

// ---------------------------------------------------------------- tile catalogue
// code = type << 20 | i << 10 | j ; R tiles use j = column tile c in [0, T + Tp)
// FT_G: the initial value (K + s2 I) of a band tile (3,1), (3,2), (3,3), formed at the launch's
// start by an otherwise idle worker wave and published to the diag workgroup (FlowArgs::gram).
// (Type 3 was the coupling H_k = D_k L(k,k-1) of the earlier R finalize, retired in round 5.)
enum : int { FT_A = 0, FT_R = 1, FT_AL = 2, FT_G = 4 };
__host__ __device__ inline int flow_code(int type, int i, int j) { return (type << 20) | (i << 10) | j; }

__host__ __device__ inline void flow_tri(int t, int& i, int& j) {   // row-major lower triangle
    int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    i = r;
    j = t - r * (r + 1) / 2;
}

// Owned A tiles: every lower tile except (0,0) (k_gram) and the band tiles (k,k-2), (k,k-1),
// (k,k) of rows k <= 3, which the diag workgroup takes from their initial values.
__host__ __device__ inline int flow_nA(int T) { return T >= 4 ? T * (T + 1) / 2 - 9 : 0; }
// the band tiles of row 3: (3,1) (3,2) (3,3) (rows 0-2: the diag workgroup's own Gram phase)
__host__ __device__ inline int flow_nG(int T) { return T > 3 ? 3 : 0; }
__host__ __device__ inline void flow_gtile(int g, int& i, int& j) {
    i = 3;
    j = 1 + g;
}
__host__ __device__ inline int flow_ntiles(int T, int Tp) {
    return flow_nA(T) + T * (T - 1) / 2 + 2 * T * Tp + flow_nG(T);
}

__device__ inline int flow_decode(int g, int T, int Tp) {
    const int nA = flow_nA(T);
    int i, j;
    if (g < nA) { flow_tri(g == 0 ? 6 : g + 9, i, j); return flow_code(FT_A, i, j); }   // (3,0), then rows >= 4
    g -= nA;
    const int nR = T * (T - 1) / 2;
    if (g < nR) { flow_tri(g, i, j); return flow_code(FT_R, i + 1, j); }
    g -= nR;
    if (g < T * Tp) return flow_code(FT_R, g / Tp, T + g % Tp);
    g -= T * Tp;
    if (g < T * Tp) return flow_code(FT_AL, g / Tp, g % Tp);
    g -= T * Tp;
    flow_gtile(g, i, j);
    return flow_code(FT_G, i, j);
}

// items of a tile: updates at levels [lo, hi] (hi < lo: none), finalize at level fin (-1: none),
// pub: the last update hands the tile to the diag workgroup
struct FlowTile {
    int type, i, j, lo, hi, fin, pub;
};
__host__ __device__ inline FlowTile flow_tile(int code, int T) {
    FlowTile t;
    t.type = (code >> 20) & 15;
    t.i = (code >> 10) & 1023;
    t.j = code & 1023;
    t.pub = 0;
    if (t.type == FT_A) {
        t.lo = 0;
        // band tiles (k,k), (k,k-1), (k,k-2): panels < k-3 here, the rest and L(k,k-2) in diag
        if (t.i <= t.j + 2) {
            t.hi = t.i - 4;
            t.fin = -1;
            t.pub = 1;
        }
        else { t.hi = t.j - 1; t.fin = t.j; }
    } else if (t.type == FT_R) {
        // every panel j .. i-1 as an update (the last one, panel i-1, needs only L(i,i-1), out a
        // step before D_i), the finalize X(i,c) = D_i R''' merged into it: ONE product after D_i.
        // (The coupling form D_i R'' - H_i X(i-1,c), H_i = D_i L(i,i-1) a worker item, put three
        // after it: its column pipelines ran ~10 us behind the chain, the launch's tail 14 us
        // past D_{T-1}.)
        t.lo = (t.j < T) ? t.j : 0;
        t.hi = t.i - 1;
        t.fin = t.i;
    } else if (t.type == FT_AL) {
        t.lo = t.i;
        t.hi = T - 1;
        t.fin = -1;
    } else {   // FT_G: no items (formed in the Gram phase at the start)
        t.lo = 0;
        t.hi = -1;
        t.fin = -1;
    }
    return t;
}
__host__ __device__ inline int flow_items(int code, int T) {
    const FlowTile t = flow_tile(code, T);
    return (t.hi >= t.lo ? t.hi - t.lo + 1 : 0) + (t.fin >= 0 ? 1 : 0);
}

// Owner table: tiles by descending item count, dealt in snake order over the W worker waves
// (slot r of wave w).  Run by ONE workgroup (k_gram's extra workgroup) before the flow launch;
// it also zeroes the flags.  sh: >= 512 + 64 ints of LDS.
// own holds W * FLOW_MAXOWN + SCHED_KEY ints: a table found intact from an earlier call with the
// same (T, Tp, W) is kept (sched_cached); the flags are zeroed every call.
constexpr int FLOW_OWN_MAGIC = 0x464C4F57;
// Key: the item count (< 256: the flow's T is bounded by the owner table, ~90).
__host__ __device__ inline int flow_owner_key(int code, int T) { return flow_items(code, T); }
__device__ inline void build_flow_owner(int T, int Tp, int W, int* own, int* flags, int nflags, int* sh) {
    int* hist = sh;          // [256] count per key, then the start of its rank range
    int* cur = sh + 256;     // [256]
    unsigned* hs = reinterpret_cast<unsigned*>(sh + 512);
    for (int e = threadIdx.x; e < nflags; e += NTHREADS) flags[e * FLOW_FSTRIDE] = 0;
    if (sched_cached(own, W * FLOW_MAXOWN, FLOW_OWN_MAGIC, T, Tp, W, hs)) return;
    for (int e = threadIdx.x; e < 256; e += NTHREADS) { hist[e] = 0; cur[e] = 0; }
    for (int e = threadIdx.x; e < W * FLOW_MAXOWN; e += NTHREADS) own[e] = -1;
    __syncthreads();
    const int n = flow_ntiles(T, Tp);
    for (int g = threadIdx.x; g < n; g += blockDim.x) atomicAdd(&hist[flow_owner_key(flow_decode(g, T, Tp), T)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int L = 255; L >= 0; --L) { const int c = hist[L]; hist[L] = s; s += c; }
    }
    __syncthreads();
    for (int g = threadIdx.x; g < n; g += blockDim.x) {
        const int code = flow_decode(g, T, Tp);
        const int L = flow_owner_key(code, T);
        const int p = hist[L] + atomicAdd(&cur[L], 1);
        const int r = p / W, q = p % W;
        const int sn = (r & 1) ? W - 1 - q : q;
        // snake position -> wave: first wave 0 of every workgroup, then wave 1, ...: the longest
        // tiles get a SIMD of their own (waves w and w + 4 share one), spread over all CUs / XCDs
        const int nwg = W / FLOW_WAVES;
        const int w = (sn % nwg) * FLOW_WAVES + sn / nwg;
        if (r < FLOW_MAXOWN) own[w * FLOW_MAXOWN + r] = code;
    }
    sched_seal(own, W * FLOW_MAXOWN, FLOW_OWN_MAGIC, T, Tp, W, hs);
}

}  // namespace mfgp
