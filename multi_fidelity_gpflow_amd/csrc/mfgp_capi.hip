// C-ABI entry points of libmfgp.so (declared in include/mfgp.h).
//
// Host-side orchestration only: workspace carving, argument blocks, kernel
// launch sequences on the handle's stream.  No allocation, no synchronisation
// (every sequence is hipGraph-capturable).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "../../include/mfgp.h"
#include "mfgp_device.h"
#include "mfgp_internal.h"
#include "mfgp_flow.h"

struct mfgp_handle_s {
    int device;
    hipStream_t stream;
    int nb;
    int grad_chunk;
    int flow_wgs;   // k_chol_flow grid (one workgroup per CU); 0: launch-per-step Cholesky
    int flow_min_t; // fewest 32-tiles a factorization needs to take the flow (below: the step launches)
    int ncu;        // compute units of the device
    int gram_wgs;   // k_gram tile workgroups, LML layout (0: one per CU; < 0: one per tile; MFGP_GRAM_WGS)
    int flow_trace; // k_chol_flow writes its diagnostic timeline into the workspace
    long long flow_timeout;   // k_chol_flow hand-off wait bound (100 MHz ticks)
    int f32_panel;  // fp32 path: 128-wide tile columns per outer panel (trailing-update K = 128 * f32_panel)
    int f32_lookahead;          // fp32 sweep: factor the next panel beside the trailing update
    int f32_reserve;            // CUs the capped trailing update leaves to the side stream
    int f32_refine;             // fp32 value-only LML (one step) / predict mean (this many steps): fp64 refinement (mfgp_set_f32_refine)
    int tiny;                   // small problems (n, p <= 64, D <= 16, AR1 kernel): one-launch LML step (default on; MFGP_TINY=0 / mfgp_set_tiny(h, 0) disables)
    hipStream_t side;           // its high-priority side stream + fork / join events (created with the handle)
    hipEvent_t ev_fork, ev_join;
    int svgp_qs_packed;         // mfgp_set_svgp_qs_packed: mfgp_svgp_elbo_grad's q_sqrt / gq_sqrt as packed triangles
    int resident;               // mfgp_set_resident: fp64 value+grad flow calls may skip the set-up launch
    struct {                    // the last fp64 LML call on this handle, when it left its workspace set
        const void* ws;         // up for the next one (k_grad's grad_next_setup); ws == nullptr: none
        int n, p, d, flow_wgs;
    } res;
};

namespace mfgp {

// Diagnostic: with MFGP_SEGV_TRACE=1 in the environment when the library loads, a host SIGSEGV prints
// the native call stack (symbol names from the dynamic tables) to stderr before the default action.
static void segv_trace(int sig) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    static const char msg[] = "\nlibmfgp: SIGSEGV, native stack:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
__attribute__((constructor)) static void segv_trace_install() {
    const char* e = getenv("MFGP_SEGV_TRACE");
    if (e && atoi(e) != 0) signal(SIGSEGV, segv_trace);
}

static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

constexpr double GRAPH_JITTER = 1e-6;   // graph.py:96: K_full += 1e-6 I

struct Carve {
    char* base;
    size_t off = 0;
    explicit Carve(void* b) : base((char*)b) {}
    template <class T>
    T* take(size_t count) {
        off = (off + 255) & ~(size_t)255;
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += count * sizeof(T);
        return p;
    }
};

struct GprLayout {
    int nb, npad, T, ppad, Tp, G, gstride, ng;
    double *A, *R, *Xo, *Dd, *ldiag, *alpha, *zpart, *gpart, *items;
    int* gorder;   // k_grad workgroup -> task table (+ key), built or verified by k_gram each call
    int* cnt;   // reduce-arrival counter, zeroed by k_gram each call
    int ncnt;
    // k_chol_flow (flow_wgs > 0): flags (zeroed) + owner table (built or verified) by k_gram each call
    int flow_wgs, nflags;
    int *flags, *own;
    double* pub;        // publication area (sentinel-filled by k_gram)
    long npub;
    long long* trace;   // k_chol_flow timeline (diagnostic; written only when enabled)
    int ntrace;
    int gchunk;         // k_grad's task chunk (m-tiles per task)
    size_t bytes;
};

// The persistent Cholesky needs every workgroup resident (one per CU) and the owner table
// to hold every tile; otherwise the launch-per-step sequence runs.
static int flow_grid(int nb, int T, int Tp, int flow_wgs, int min_t) {
    if (nb != 32 || flow_wgs < 2 || T > 255 || T < min_t) return 0;
    if (flow_ntiles(T, Tp) > FLOW_WAVES * (flow_wgs - 1) * FLOW_MAXOWN) return 0;
    return flow_wgs;
}

static GprLayout gpr_layout(int nb, int n, int p, int d, void* ws, int grad_chunk, int nlf = 0, int flow_wgs = 0,
                            int flow_min_t = 0) {
    GprLayout L;
    L.nb = nb;
    L.T = ceil_div(n, nb);
    L.npad = L.T * nb;
    L.Tp = ceil_div(p > 0 ? p : 1, nb);
    L.ppad = L.Tp * nb;
    L.G = kernel_theta_size(nlf, d);
    L.gstride = (L.G + 3) & ~3;
    L.flow_wgs = flow_grid(nb, L.T, L.Tp, flow_wgs, flow_min_t);
    L.gchunk = grad_chunk;
    L.ng = grad_tasks(L.T, L.gchunk);
    Carve c(ws);
    const size_t ldr = (size_t)L.npad + L.ppad;
    L.A = c.take<double>((size_t)L.npad * L.npad);
    L.R = c.take<double>((size_t)L.npad * ldr);
    L.Xo = c.take<double>((size_t)(L.npad + 2 * L.ppad) * ldr);   // + alpha^T rows (k_grad)
    L.Dd = c.take<double>((size_t)L.T * nb * nb);
    L.ldiag = c.take<double>(L.npad);
    L.alpha = c.take<double>((size_t)L.npad * L.ppad);
    L.zpart = c.take<double>((size_t)L.T * L.Tp);
    L.gpart = c.take<double>((size_t)L.ng * L.gstride);
    L.items = c.take<double>((size_t)L.G + 8);
    L.ncnt = 1;
    L.cnt = c.take<int>((size_t)L.ncnt);
    L.gorder = c.take<int>((size_t)L.ng + SCHED_KEY);
    L.nflags = L.flow_wgs ? flow_nflags(L.T, L.Tp) : 0;
    L.flags = c.take<int>((size_t)L.nflags * FLOW_FSTRIDE);
    L.npub = L.flow_wgs ? flow_npub(L.T, L.Tp) : 0;
    L.pub = c.take<double>((size_t)L.npub);
    L.own = c.take<int>(L.flow_wgs ? (size_t)FLOW_WAVES * (L.flow_wgs - 1) * FLOW_MAXOWN + SCHED_KEY : 0);
    L.ntrace = L.flow_wgs ? flow_trace_count(L.T, L.flow_wgs) : 0;
    L.trace = c.take<long long>((size_t)L.ntrace);
    L.bytes = c.off + 256;
    return L;
}

static inline hipError_t last() { return hipGetLastError(); }

// Below this many 32-tiles the launch-per-step Cholesky is faster than the persistent flow (one
// 256-workgroup launch costs more than a few short step launches): fp64 value+grad evaluation,
// flow vs steps (tools/flow_threshold.py): T = 2: 67.5 vs 56.8 us, T = 5: 83.2 vs 79.7, T = 7:
// 95.3 vs 96.2, T = 9: 106.2 vs 110.6, T = 24: 195.9 vs 247.1.
constexpr int FLOW_MIN_TILES = 8;

// ---------------------------------------------------------------- device-wide flow fence
// k_chol_flow needs every CU: two flows whose workgroups interleave (launched on two streams
// at once) each wait for workgroups the other keeps off the CUs, and stall to the hand-off bound.
// One fence per device for the whole process (every handle, every stream, every host thread):
// each flow launch waits for the previous one and becomes the new last one.  Stream-ordered
// (hipStreamWaitEvent), never a host synchronisation.  Inside a stream capture the wait / record
// are skipped (an event recorded outside a capture cannot be waited on inside it): the caller
// orders the replay of such a graph with mfgp_flow_fence (the Python sessions do).
// mfgp_flow_fence(WAIT) .. (RECORD) brackets such a replay and HOLDS the fence in between: a flow
// launch from another host thread blocks on the host (a condition variable, no device
// synchronisation) until the holder records, so it cannot be enqueued beside the replay's
// unfenced flows.  The holding thread itself passes (its eager calls inside the bracket are
// ordered by their streams as usual).
// Holds nest per thread (Engine.ordered blocks inside one another): only the outermost RECORD
// releases.  A thread that finds the fence held by another waits at most fence_bound() on the
// host (10 s; env MFGP_FENCE_BOUND_MS) and then fails with MFGP_ERR_FENCE (a client that issued
// WAIT and never RECORD cannot block every other thread's flow launches for ever).
static std::chrono::milliseconds fence_bound() {
    const char* e = getenv("MFGP_FENCE_BOUND_MS");
    const long ms = e ? atol(e) : 10000;
    return std::chrono::milliseconds(ms > 0 ? ms : 10000);
}
struct FlowFence {
    std::mutex mu;
    std::condition_variable cv;
    hipEvent_t ev = nullptr;
    bool armed = false;
    bool held = false;
    int depth = 0;   // WAITs of the holder not yet matched by a RECORD
    std::thread::id holder;
};
constexpr int FENCE_MAX_DEVICES = 64;
static FlowFence g_fence[FENCE_MAX_DEVICES];

static bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

// with f.mu locked: wait (bounded) until no other thread holds the fence
static bool fence_enter(FlowFence& f, std::unique_lock<std::mutex>& lk) {
    const std::thread::id me = std::this_thread::get_id();
    return f.cv.wait_for(lk, fence_bound(), [&] { return !f.held || f.holder == me; });
}

static int fence_wait(int dev, hipStream_t s, bool hold = false) {
    if (dev < 0 || dev >= FENCE_MAX_DEVICES || stream_capturing(s)) return MFGP_OK;
    FlowFence& f = g_fence[dev];
    std::unique_lock<std::mutex> lk(f.mu);
    if (!fence_enter(f, lk)) return MFGP_ERR_FENCE;
    if (f.armed) (void)hipStreamWaitEvent(s, f.ev, 0);
    if (hold) {
        if (f.held) {
            ++f.depth;   // nested hold of the same thread
        } else {
            f.held = true;
            f.depth = 1;
            f.holder = std::this_thread::get_id();
        }
    }
    return MFGP_OK;
}

// with f.mu locked: record the fence event on s (created on first use)
static void fence_arm(FlowFence& f, int dev, hipStream_t s) {
    if (!f.ev) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        if (hipEventCreateWithFlags(&f.ev, hipEventDisableTiming) != hipSuccess) f.ev = nullptr;
        if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
    }
    if (f.ev && hipEventRecord(f.ev, s) == hipSuccess) f.armed = true;
}

static int fence_record(int dev, hipStream_t s, bool release = false) {
    if (dev < 0 || dev >= FENCE_MAX_DEVICES || stream_capturing(s)) return MFGP_OK;
    FlowFence& f = g_fence[dev];
    std::unique_lock<std::mutex> lk(f.mu);
    if (!fence_enter(f, lk)) return MFGP_ERR_FENCE;
    fence_arm(f, dev, s);
    if (release && f.held && --f.depth <= 0) {   // the outermost RECORD of the holder
        f.held = false;
        f.depth = 0;
        lk.unlock();
        f.cv.notify_all();
    }
    return MFGP_OK;
}

// An eager flow launch's turn at the fence.  Taken before the first launch of the
// sequence: the bounded host wait happens here, so a fence held past its bound by another thread
// fails the call with NOTHING enqueued.  The fence's mutex is then kept until commit(), which
// follows the flow launch and records the event unconditionally: no other thread's flow, WAIT or
// hold can be ordered between this launch's wait and its record, and a launch that was enqueued
// always becomes the fence's last flow.
struct FenceTurn {
    FlowFence* f = nullptr;
    std::unique_lock<std::mutex> lk;
    int dev = -1;
    int rc = MFGP_OK;
    FenceTurn(int device, hipStream_t s) {
        if (device < 0 || device >= FENCE_MAX_DEVICES || stream_capturing(s)) return;
        FlowFence& ff = g_fence[device];
        lk = std::unique_lock<std::mutex>(ff.mu);
        if (!fence_enter(ff, lk)) {
            rc = MFGP_ERR_FENCE;
            lk.unlock();
            return;
        }
        if (ff.armed) (void)hipStreamWaitEvent(s, ff.ev, 0);
        f = &ff;
        dev = device;
    }
    void commit(hipStream_t s) {
        if (!f) return;
        fence_arm(*f, dev, s);
        f = nullptr;
        lk.unlock();
    }
};

// k_gram (LML layout) with more lower tiles than CUs: one workgroup per CU, tile (0,0) and its
// fused factor alone on workgroup 0 (beside two other tile workgroups it took ~2x as long, and
// it is the launch's tail), the rest looping over the other tiles.  0: one tile per workgroup.
static int gram_tile_wgs(mfgp_handle_t h, int T, int extra) {
    const int nt = T * (T + 1) / 2;
    if (h->gram_wgs < 0) return 0;
    const int wgs = (h->gram_wgs > 0 ? h->gram_wgs : h->ncu) - extra;
    return (wgs > 1 && nt > wgs) ? wgs : 0;
}

template <int NB>
static void gram_lml_and_factor(hipStream_t s, const GprLayout& L, int n, int p, int d, const double* X, int ldx,
                                const double* Y, int ldy, const double* theta, int* info, int nlf = 0) {
    const long ldr = L.npad + L.ppad;
    GramArgs g{};
    g.R = L.R; g.ldr = ldr; g.sR = 0; g.Y = Y; g.ldy = ldy; g.sY = 0; g.p = p; g.ppad = L.ppad;
    g.X1 = X; g.ldx1 = ldx; g.sx1 = 0; g.n1 = n;
    g.X2 = X; g.ldx2 = ldx; g.sx2 = 0; g.n2 = n;
    g.theta = theta; g.stheta = 0; g.D = d; g.rbf_only = 0;
    g.out = L.A; g.ldo = L.npad; g.so = 0;
    g.padded = 1; g.npad = L.npad; g.tiles_c = L.T; g.add_noise = 1; g.diag_add = nlf ? GRAPH_JITTER : 0.0;
    g.Dd = L.Dd; g.sD = 0; g.ldiag = L.ldiag; g.sL = 0; g.info = info; g.nlf = nlf;
    launch_gram<NB>(g, L.T * (L.T + 1) / 2, 1, s);
    CholArgs c{};
    c.A = L.A; c.lda = L.npad; c.sA = 0;
    c.R = L.R; c.ldr = ldr; c.sR = 0;
    c.Xo = L.Xo; c.ldx = ldr; c.sX = 0;
    c.Dd = L.Dd; c.sD = 0; c.ldiag = L.ldiag; c.sL = 0; c.info = info;
    c.T = L.T; c.Tp = L.Tp; c.k = 0;
    launch_chol_steps<NB>(c, 1, s);
}

// Optional per-phase event marks (diagnostic timing; never used on the hot path).
struct PhaseMarks {
    hipEvent_t ev[8];
    int count = 0;
    void mark(hipStream_t s) { (void)hipEventRecord(ev[count++], s); }
};

template <int NB>
static int gpr_value_grad(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y, int ldy,
                          double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info,
                          const FinArgs* adam, PhaseMarks* pm = nullptr, int nlf = 0) {
    const GprLayout L = gpr_layout(NB, n, p, d, ws, h->grad_chunk, nlf, h->flow_wgs, h->flow_min_t);
    if (ws_bytes < L.bytes) return MFGP_ERR_WORKSPACE;
    if (L.G > FIN_MAXG) return MFGP_ERR_ARG;   // finalize_body stages theta in LDS
    hipStream_t s = h->stream;
    const long ldr = L.npad + L.ppad;
    if (pm) pm->mark(s);
    if (NB == 32 && h->tiny && gpr_tiny_fits(n, p, d, nlf)) {   // the whole step in one workgroup
        FinArgs f{};
        if (adam) f = *adam;
        f.info = info; f.P = p; f.D = d; f.want_grad = want_grad; f.out = out; f.n = n;
        f.adam = adam != nullptr;
        f.G = L.G;
        if (pm) pm->mark(s);
        launch_gpr_tiny(X, ldx, Y, ldy, theta, n, p, d, want_grad, info, f, s);
        if (pm) { pm->mark(s); pm->mark(s); pm->mark(s); }
        return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
    }
    if (pm) pm->mark(s);
    // the flow fence before any launch of the sequence: a fence held past its bound by another
    // host thread fails the call with nothing enqueued; once past it, the flow is always recorded
    FenceTurn fence(L.flow_wgs ? h->device : -1, s);
    if (fence.rc != MFGP_OK) return fence.rc;
    // The AR1 flow path (NB = 32, nlf = 0): the Gram is formed inside k_chol_flow, so the launch
    // in front of it only sets up the workspace (sentinel fill, schedule tables, item slots) --
    // and a value+grad call leaves exactly that set-up behind (k_grad's tail).  In resident mode
    // a value+grad call whose workspace the previous fp64 LML call on this handle left set up for
    // the same problem starts with the flow itself.
    const bool flow_gram = NB == 32 && L.flow_wgs && !nlf;
    const bool leaves_setup = flow_gram && want_grad;
    const bool skip_prep = leaves_setup && h->resident && h->res.ws == ws && h->res.n == n && h->res.p == p &&
                           h->res.d == d && h->res.flow_wgs == L.flow_wgs;
    h->res.ws = nullptr;
    if (!skip_prep) {
        GramArgs g{};
        g.R = L.R; g.ldr = ldr; g.sR = 0; g.Y = Y; g.ldy = ldy; g.sY = 0; g.p = p; g.ppad = L.ppad;
        g.X1 = X; g.ldx1 = ldx; g.sx1 = 0; g.n1 = n;
        g.X2 = X; g.ldx2 = ldx; g.sx2 = 0; g.n2 = n;
        g.theta = theta; g.stheta = 0; g.D = d; g.rbf_only = 0;
        g.out = L.A; g.ldo = L.npad; g.so = 0;
        g.padded = 1; g.npad = L.npad; g.tiles_c = L.T; g.add_noise = 1; g.diag_add = nlf ? GRAPH_JITTER : 0.0;
        g.Dd = L.Dd; g.sD = 0; g.ldiag = L.ldiag; g.sL = 0; g.info = info; g.nlf = nlf;
        g.cnt = L.cnt; g.ncnt = L.ncnt;
        if (MFGP_REDUCE_FLAG) { g.isent = L.items; g.nisent = L.G + 2; }
        const bool order = want_grad && L.gchunk + L.T + L.Tp < 2048;   // gram LDS holds the histogram
        if (order) { g.gorder = L.gorder; g.gT = L.T; g.gchunk = L.gchunk; g.gTp = L.Tp; }
        if (L.flow_wgs) { g.fown = L.own; g.fW = FLOW_WAVES * (L.flow_wgs - 1); g.fflags = L.flags; g.nfflags = L.nflags; g.fpub = L.pub; g.npub = L.npub; }
        const int extra = (order ? 1 : 0) + (L.flow_wgs ? 1 : 0);
        if (flow_gram) {
            launch_flow_prep(g, std::max(h->ncu, 2) + extra, s);
        } else {
            if (L.flow_wgs) g.Dd = nullptr;   // the flow factors D_0 itself
            g.tile_wgs = gram_tile_wgs(h, L.T, extra);
            launch_gram<NB>(g, (g.tile_wgs ? g.tile_wgs : L.T * (L.T + 1) / 2) + extra, 1, s);
        }
    }
    if (pm) pm->mark(s);
    if (L.flow_wgs) {
        FlowArgs fa{};
        fa.A = L.A; fa.lda = L.npad;
        fa.R = L.R; fa.ldr = ldr;
        fa.Xo = L.Xo; fa.ldx = ldr;
        fa.Dd = L.Dd; fa.ldiag = L.ldiag; fa.info = info;
        fa.alpha = L.alpha; fa.ldal = L.ppad; fa.zpart = L.zpart;
        fa.flags = L.flags; fa.own = L.own; fa.pub = L.pub;
        fa.T = L.T; fa.Tp = L.Tp; fa.n = n; fa.p = p;
        fa.trace = h->flow_trace ? L.trace : nullptr;
        fa.nwaves = FLOW_WAVES * (L.flow_wgs - 1);
        fa.timeout = h->flow_timeout;
        fa.X = X; fa.ldxi = ldx; fa.Y = Y; fa.ldy = ldy; fa.theta = theta; fa.D = d;
        fa.gram = flow_gram ? 1 : 0;
        launch_chol_flow(fa, L.flow_wgs, s);
        fence.commit(s);
    } else {
        CholArgs c{};
        c.A = L.A; c.lda = L.npad; c.sA = 0;
        c.R = L.R; c.ldr = ldr; c.sR = 0;
        c.Xo = L.Xo; c.ldx = ldr; c.sX = 0;
        c.Dd = L.Dd; c.sD = 0; c.ldiag = L.ldiag; c.sL = 0; c.info = info;
        c.T = L.T; c.Tp = L.Tp; c.k = 0;
        c.alpha = L.alpha; c.ldal = L.ppad; c.zpart = L.zpart; c.n = n; c.p = p;
        launch_chol_steps<NB>(c, 1, s);
    }
    if (pm) pm->mark(s);
    if (want_grad) {
        GradArgs ga{L.Xo, ldr, X, (long)ldx, theta, L.gpart, L.gstride, L.T, L.Tp, n, p, d,
                    L.gchunk, nlf, L.gchunk + L.T + L.Tp < 2048 ? L.gorder : nullptr};
        if (leaves_setup) {   // the next evaluation's set-up, after the flow
            ga.fpub = L.pub; ga.npub = L.npub;
            ga.isent = L.items; ga.nisent = L.G + 2;
        }
        launch_grad<NB>(ga, s);
    }
    if (pm) pm->mark(s);
    FinArgs f{};
    if (adam) f = *adam;
    f.zpart = L.zpart; f.nz = L.T * L.Tp;
    f.ldiag = L.ldiag; f.n = n;
    f.gpart = L.gpart; f.ng = L.ng; f.gstride = L.gstride;
    f.info = info; f.P = p; f.D = d; f.want_grad = want_grad;
    f.out = out;
    f.adam = adam != nullptr;
    f.items = L.items;
    f.G = L.G;
    f.cnt = L.cnt;
    f.flag = MFGP_REDUCE_FLAG;   // the Gram / set-up launch (or the previous k_grad) filled items[] with the sentinel
    f.abortw = L.flow_wgs ? L.flags : nullptr;
    hipLaunchKernelGGL(k_reduce_items, dim3(2 + (want_grad ? L.G : 0)), dim3(NTHREADS), 0, s, f);
    if (pm) pm->mark(s);
    if (last() != hipSuccess) return MFGP_ERR_LAUNCH;
    if (leaves_setup) {
        h->res.ws = ws; h->res.n = n; h->res.p = p; h->res.d = d; h->res.flow_wgs = L.flow_wgs;
    }
    return MFGP_OK;
}

// ---------------------------------------------------------------- potrf_inv
template <int NB>
__global__ void k_pad_copy(const double* A, long lda, long sA, double* Ap, int n, int npad) {
    const int b = blockIdx.z;
    const long total = (long)npad * npad;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / npad), c = (int)(e % npad);
        double v = (r == c) ? 1.0 : 0.0;
        if (r < n && c < n) v = A[b * sA + (long)r * lda + c];
        Ap[b * total + e] = v;
    }
}

template <int NB>
__global__ __launch_bounds__(NTHREADS) void k_factor_first(double* Ap, int npad, double* Dd, long sD, double* ldiag,
                                                           int* info) {
    constexpr int E = TileCfg<NB>::ELEMS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* T0 = smem;
    double* R0 = T0 + E;
    double* dg = R0 + E;
    int& bad = *reinterpret_cast<int*>(dg + NB);
    const int b = blockIdx.z;
    tile_load<NB>(T0, Ap + (long)b * npad * npad, npad);
    __syncthreads();
    tile_potrf_inv<NB>(T0, R0, dg, &bad);
    tile_store<NB>(Dd + b * sD, NB, R0);
    for (int r = threadIdx.x; r < NB; r += NTHREADS) ldiag[(long)b * npad + r] = dg[r];
    if (threadIdx.x == 0 && bad && info[b] == 0) info[b] = bad;
}

__global__ void k_copy_lower_out(const double* Xo, long ldx, long sX, double* Linv, long ldl, long sL, int n) {
    const int b = blockIdx.z;
    const long total = (long)n * n;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / n), c = (int)(e % n);
        Linv[b * sL + (long)r * ldl + c] = (c <= r) ? Xo[b * sX + (long)r * ldx + c] : 0.0;
    }
}

__global__ void k_copy_vec(const double* src, long ss, double* dst, long sd, int n) {
    const int b = blockIdx.z;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        dst[b * sd + i] = src[b * ss + i];
}

struct PotrfLayout {
    int npad, T;
    double *A, *R, *Xo, *Dd, *ldiag;
    size_t bytes;
};

static PotrfLayout potrf_layout(int nb, int n, int batch, void* ws) {
    PotrfLayout L;
    L.T = ceil_div(n, nb);
    L.npad = L.T * nb;
    const size_t mat = (size_t)L.npad * L.npad;
    Carve c(ws);
    L.A = c.take<double>(mat * batch);
    L.R = c.take<double>(mat * batch);
    L.Xo = c.take<double>(mat * batch);
    L.Dd = c.take<double>((size_t)L.T * nb * nb * batch);
    L.ldiag = c.take<double>((size_t)L.npad * batch);
    L.bytes = c.off + 256;
    return L;
}

template <int NB>
static int potrf_inv_impl(mfgp_handle_t h, int n, int batch, const double* A, int lda, long sA, void* ws,
                          size_t ws_bytes, double* Linv, int ldl, long sLo, double* ldiag, int* info) {
    const PotrfLayout L = potrf_layout(NB, n, batch, ws);
    if (ws_bytes < L.bytes) return MFGP_ERR_WORKSPACE;
    hipStream_t s = h->stream;
    const long mat = (long)L.npad * L.npad;
    const int blocks = (int)std::min<long>((mat + 255) / 256, 2048);
    (void)hipMemsetAsync(info, 0, sizeof(int) * batch, s);
    hipLaunchKernelGGL(k_pad_copy<NB>, dim3(blocks, 1, batch), dim3(256), 0, s, A, (long)lda, sA, L.A, n, L.npad);
    hipLaunchKernelGGL(k_rhs_init, dim3(blocks, 1, batch), dim3(256), 0, s, L.R, (long)L.npad, mat, L.npad, 0,
                       (const double*)nullptr, 0L, 0L, n, 0);
    hipLaunchKernelGGL(k_factor_first<NB>, dim3(1, 1, batch), dim3(NTHREADS),
                       sizeof(double) * (2 * NB * (NB + 2) + NB + 2), s, L.A, L.npad, L.Dd, (long)L.T * NB * NB,
                       L.ldiag, info);
    CholArgs c{};
    c.A = L.A; c.lda = L.npad; c.sA = mat;
    c.R = L.R; c.ldr = L.npad; c.sR = mat;
    c.Xo = L.Xo; c.ldx = L.npad; c.sX = mat;
    c.Dd = L.Dd; c.sD = (long)L.T * NB * NB; c.ldiag = L.ldiag; c.sL = L.npad; c.info = info;
    c.T = L.T; c.Tp = 0; c.k = 0;
    launch_chol_steps<NB>(c, batch, s);
    const long tot = (long)n * n;
    const int b2 = (int)std::min<long>((tot + 255) / 256, 2048);
    hipLaunchKernelGGL(k_copy_lower_out, dim3(b2, 1, batch), dim3(256), 0, s, L.Xo, (long)L.npad, mat, Linv,
                       (long)ldl, sLo, n);
    if (ldiag)
        hipLaunchKernelGGL(k_copy_vec, dim3(ceil_div(n, 256), 1, batch), dim3(256), 0, s, L.ldiag, (long)L.npad,
                           ldiag, (long)n, n);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

// ---------------------------------------------------------------- predict
struct PredLayout {
    GprLayout g;
    int nspad, Ts;
    double *Kmn, *Am, *kdiag;
    double *Kss, *Cov;   // full_cov only: K(X*, X*) and Kss - A^T A (nspad x nspad)
    size_t bytes;
};

static PredLayout pred_layout(int nb, int n, int p, int d, int nstar, void* ws, int grad_chunk, int nlf = 0,
                              int full_cov = 0) {
    PredLayout P;
    P.g = gpr_layout(nb, n, p, d, ws, grad_chunk, nlf);
    P.Ts = ceil_div(nstar > 0 ? nstar : 1, nb);
    P.nspad = P.Ts * nb;
    Carve c(ws);
    c.off = P.g.bytes;
    P.Kmn = c.take<double>((size_t)P.g.npad * P.nspad);
    P.Am = c.take<double>((size_t)P.g.npad * P.nspad);
    P.kdiag = c.take<double>(P.nspad);
    const size_t sq = full_cov ? (size_t)P.nspad * P.nspad : 0;
    P.Kss = c.take<double>(sq);
    P.Cov = c.take<double>(sq);
    P.bytes = c.off + 256;
    return P;
}

__global__ void k_copy_block(const double* src, long lds, double* dst, long ldd, int rows, int cols) {
    const long total = (long)rows * cols;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / cols), c = (int)(e % cols);
        dst[(long)r * ldd + c] = src[(long)r * lds + c];
    }
}

template <int NB>
static int predict_impl(mfgp_handle_t h, int n, int p, int d, int nstar, const double* X, int ldx, const double* Y,
                        int ldy, const double* Xs, int ldxs, const double* theta, void* ws, size_t ws_bytes,
                        double* mean, int ldm, double* var, int* info, int nlf = 0, double* cov = nullptr,
                        int ldc = 0) {
    const PredLayout P = pred_layout(NB, n, p, d, nstar, ws, h->grad_chunk, nlf, cov != nullptr);
    if (ws_bytes < P.bytes) return MFGP_ERR_WORKSPACE;
    hipStream_t s = h->stream;
    if (NB == 32 && h->tiny && !nlf && !cov && gpr_tiny_pred_fits(n, p, d, nstar)) {   // small problems: one launch
        launch_gpr_tiny_pred(X, ldx, Y, ldy, Xs, ldxs, nstar, theta, n, p, d, mean, ldm, var, info, s);
        return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
    }
    const GprLayout& L = P.g;
    gram_lml_and_factor<NB>(s, L, n, p, d, X, ldx, Y, ldy, theta, info, nlf);
    if (nlf) (void)hipMemsetAsync(P.Kmn, 0, sizeof(double) * (size_t)L.npad * P.nspad, s);
    GramArgs g{};
    g.X1 = X; g.ldx1 = ldx; g.n1 = n;
    g.X2 = Xs; g.ldx2 = ldxs; g.n2 = nstar;
    g.theta = theta; g.D = d; g.rbf_only = 0;
    g.out = P.Kmn; g.ldo = P.nspad; g.padded = 0; g.tiles_c = P.Ts; g.diag_add = 0.0; g.nlf = nlf;
    if (nlf) launch_gram<NB>(g, L.T * P.Ts, 1, s);
    else launch_gram_dense(g, 1, L.npad, P.nspad, s);   // zero padding written by the kernel
    hipLaunchKernelGGL(k_kdiag, dim3(ceil_div(nstar, 256)), dim3(256), 0, s, Xs, (long)ldxs, nstar, d, theta,
                       P.kdiag, nlf);
    const long ldr = L.npad + L.ppad;
    PredAArgs pa{L.Xo, ldr, P.Kmn, (long)P.nspad, P.Am, (long)P.nspad, P.Ts};
    PredOutArgs po{P.Am, (long)P.nspad, L.Xo, ldr, P.kdiag, mean, (long)ldm, var, L.T, L.Tp, nstar, p};
    launch_pred<NB>(pa, po, L.T, s);
    if (cov) {
        // base_conditional(full_cov=True): Kss - A^T A with A = L^{-1} Kmn (padded rows of A are 0)
        if (nlf) (void)hipMemsetAsync(P.Kss, 0, sizeof(double) * (size_t)P.nspad * P.nspad, s);
        GramArgs gs{};
        gs.X1 = Xs; gs.ldx1 = ldxs; gs.n1 = nstar;
        gs.X2 = Xs; gs.ldx2 = ldxs; gs.n2 = nstar;
        gs.theta = theta; gs.D = d; gs.rbf_only = 0;
        gs.out = P.Kss; gs.ldo = P.nspad; gs.padded = 0; gs.tiles_c = P.Ts; gs.nlf = nlf;
        gs.diag_add = nlf ? GRAPH_JITTER : 0.0;   // graph.py:96 adds the jitter inside K(X*, X*) too
        if (nlf) launch_gram<NB>(gs, P.Ts * P.Ts, 1, s);
        else launch_gram_dense(gs, 1, P.nspad, P.nspad, s);
        BgemmArgs b{};
        b.A = P.Am; b.lda = P.nspad;
        b.B = P.Am; b.ldb = P.nspad;
        b.Cin = P.Kss; b.ldc = P.nspad; b.beta = 1.0;
        b.D = P.Cov; b.ldd = P.nspad;
        b.alpha = -1.0;
        b.Mt = P.Ts; b.Nt = P.Ts; b.Kt = L.T;
        launch_bgemm(NB, s, 1, 0, b, 1);
        const long tot = (long)nstar * nstar;
        hipLaunchKernelGGL(k_copy_block, dim3((int)std::min<long>((tot + 255) / 256, 2048)), dim3(256), 0, s, P.Cov,
                           (long)P.nspad, cov, (long)ldc, nstar, nstar);
    }
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

size_t svgp_workspace_bytes(int nb, int n, int m, int l, int p, int d);
int svgp_elbo_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx,
                   const double* Y, int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                   const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                   size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info, const double* noise_dev);
size_t svgp_grad_workspace_bytes(int nb, int n, int m, int l, int p, int d);
int svgp_grad_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* X, int ldx, const double* Y,
                   int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                   const double* W, const double* noise_dev, double noise_host, double scale, double kl_mult,
                   double jitter, void* ws, size_t ws_bytes, double* out, double* g_mu, double* g_var, double* gZ,
                   double* gtheta, double* gq_mu, double* gq_sqrt, double* gW, double* gnoise, int* info);
int adam_packed_impl(hipStream_t st, int n, double* u, double* c, const double* g, double* m, double* v,
                     const unsigned char* trainable, const unsigned char* transform, const unsigned char* span,
                     int* step, const double* lr_sched, double b1, double b2, double eps, const double* out,
                     double klm, double* loss_hist, double* kl_hist, const int* info, int ninfo);

size_t svgp_predict_cov_workspace_bytes(int nb, int ns, int m, int l, int p, int d);
int svgp_predict_cov_impl(hipStream_t s, int nb, int mode, int ns, int m, int l, int p, int d, const double* Xs,
                          int ldx, const double* Z, int ldz, const double* thetas, const double* q_mu,
                          const double* q_sqrt, const double* W, double jitter, void* ws, size_t ws_bytes,
                          double* g_mu, double* g_var, double* f_mu, double* f_var, double* f_cov, int* info);
int svgp_predict_impl(hipStream_t s, int nb, int n, int m, int l, int p, int d, const double* Xs, int ldx,
                      const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                      const double* W, double jitter, void* ws, size_t ws_bytes, double* g_mu, double* g_var,
                      double* f_mu, double* f_var, int* info);

// ---------------------------------------------------------------- fp32 path (mfgp_f32.hip)
struct F32Layout {
    F32Args a;
    F32Refine r;
    double* items;
    int ntask, G;
    size_t bytes;
};

// ns > 0: predict rows; want_grad: identity rows + alpha + gradient partials; refine (value-only /
// predict): L^T tiles, fp32 work rows, fp64 alpha and residual (mfgp_set_f32_refine)
static F32Layout f32_layout(int n, int p, int d, int ns, int want_grad, int panel, void* ws, int refine = 0) {
    F32Layout L{};
    F32Args& a = L.a;
    const int TB = F32_TILE;
    a.T = ceil_div(n, TB);
    a.Tp = ceil_div(p, TB);
    a.Ts = ns > 0 ? ceil_div(ns, TB) : 0;
    a.Ti = want_grad ? a.T : 0;
    a.W = panel;
    a.ld = (long)a.T * TB;
    a.n = n; a.p = p; a.ns = ns; a.D = d;
    Carve c(ws);
    a.M = c.take<float>((size_t)(a.T + a.Tp + a.Ts + a.Ti) * TB * a.ld);
    a.Dd = c.take<float>((size_t)a.T * TB * TB);
    a.ldiag = c.take<double>((size_t)a.T * TB);
    a.ldal = (long)a.Tp * TB;
    a.alpha = c.take<float>(want_grad ? (size_t)a.ld * a.ldal : 0);
    a.nz = 256;
    a.zpart = c.take<double>((size_t)a.nz);
    L.ntask = a.T * (a.T + 1) / 2;
    L.G = theta_size(d);
    a.gpart = c.take<double>(want_grad ? (size_t)L.G * L.ntask : 0);
    L.items = c.take<double>((size_t)L.G + 8);
    a.cnt = c.take<int>(1);
    if (refine && !want_grad) {
        a.LT = c.take<float>((size_t)a.T * TB * a.ld);
        L.r.XB = c.take<float>((size_t)a.Tp * TB * a.ld);
        L.r.ld64 = (long)ceil_div(a.Tp * TB, 256) * 256;   // k64_kmat reads 256-column blocks
        L.r.A64 = c.take<double>((size_t)a.ld * L.r.ld64);
        L.r.R64 = c.take<double>((size_t)a.ld * L.r.ld64);
    }
    L.bytes = c.off + 256;
    return L;
}

static int f32_value_grad(mfgp_handle_t h, int n, int p, int d, const float* X, int ldx, const float* Y, int ldy,
                          double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info,
                          const FinArgs* adam, F32Marks* mk = nullptr) {
    const int refine = h->f32_refine && !want_grad && !adam && !mk;
    F32Layout L = f32_layout(n, p, d, 0, want_grad, h->f32_panel, ws, refine);
    if (ws_bytes < L.bytes) return MFGP_ERR_WORKSPACE;
    hipStream_t s = h->stream;
    F32Args& a = L.a;
    a.info = info; a.X = X; a.ldx = ldx; a.Y = Y; a.ldy = ldy; a.theta = theta;
    a.upd_slots = (h->f32_reserve > 0 && h->ncu > h->f32_reserve) ? 2 * (h->ncu - h->f32_reserve) : 0;
    if (h->f32_lookahead) launch_f32_sweep(a, s, mk, h->side, h->ev_fork, h->ev_join);
    else launch_f32_sweep(a, s, mk);
    if (want_grad) launch_f32_grad(a, s, mk);
    if (mk) mk->begin(s, F32_FIN);
    if (refine) launch_f32_refine_lml(a, L.r, s);   // q = Y.a0 + a0.R + |L~^-1 R|^2 partials into zpart
    else launch_f32_zsum(a, s);
    FinArgs f{};
    if (adam) f = *adam;
    f.zpart = a.zpart; f.nz = a.nz;
    f.ldiag = a.ldiag; f.n = n;
    f.gpart = a.gpart; f.ng = L.ntask; f.gstride = 0;
    f.info = info; f.P = p; f.D = d; f.want_grad = want_grad;
    f.out = out;
    f.adam = adam != nullptr;
    f.items = L.items;
    f.G = L.G;
    f.cnt = a.cnt;
    hipLaunchKernelGGL(k_reduce_items, dim3(2 + (want_grad ? L.G : 0)), dim3(NTHREADS), 0, s, f);
    if (mk) mk->end(s, 0.0);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

static int f32_predict(mfgp_handle_t h, int n, int p, int d, int ns, const float* X, int ldx, const float* Y, int ldy,
                       const float* Xs, int ldxs, const double* theta, void* ws, size_t ws_bytes, float* mean, int ldm,
                       float* var, int* info, float* cov = nullptr, int ldc = 0) {
    F32Layout L = f32_layout(n, p, d, ns, 0, h->f32_panel, ws, h->f32_refine);
    if (ws_bytes < L.bytes) return MFGP_ERR_WORKSPACE;
    F32Args& a = L.a;
    a.info = info; a.X = X; a.ldx = ldx; a.Y = Y; a.ldy = ldy; a.Xs = Xs; a.ldxs = ldxs; a.theta = theta;
    a.upd_slots = (h->f32_reserve > 0 && h->ncu > h->f32_reserve) ? 2 * (h->ncu - h->f32_reserve) : 0;
    if (h->f32_lookahead) launch_f32_sweep(a, h->stream, nullptr, h->side, h->ev_fork, h->ev_join);
    else launch_f32_sweep(a, h->stream);
    launch_f32_predict(a, mean, ldm, var, h->stream);   // variance (and the unrefined mean)
    if (h->f32_refine) launch_f32_refine_mean(a, L.r, mean, ldm, h->f32_refine, h->stream);
    if (cov) launch_f32_predict_cov(a, cov, ldc, h->stream);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

}  // namespace mfgp

using namespace mfgp;

#define CHECK_H(h) \
    if ((h) == nullptr) return MFGP_ERR_ARG
#define CHECK_D(d) \
    if ((d) < 1 || (d) > MFGP_MAX_D) return MFGP_ERR_DIM

extern "C" {

int mfgp_version(void) { return 100; }

// Build provenance: build.py passes the hash of the sources the library is compiled from (every
// file of csrc/ and include/mfgp.h, build.source_hash()); the marker string also lets the builder
// read the id from the file without loading it.
#ifndef MFGP_BUILD_ID
#define MFGP_BUILD_ID "unknown"
#endif
__attribute__((used)) static const char k_build_marker[] = "mfgp-build-id:" MFGP_BUILD_ID;
const char* mfgp_build_id(void) { return k_build_marker + 14; }

const char* mfgp_error_string(int code) {
    switch (code) {
        case MFGP_OK: return "ok";
        case MFGP_ERR_ARG: return "invalid argument";
        case MFGP_ERR_WORKSPACE: return "workspace too small";
        case MFGP_ERR_LAUNCH: return "kernel launch failed";
        case MFGP_ERR_DIM: return "unsupported input dimension (1 <= d <= 32)";
        case MFGP_ERR_FENCE: return "flow fence held by another host thread past the bound (WAIT without RECORD?)";
        default: return "unknown error";
    }
}

int mfgp_create(int device, mfgp_handle_t* out) {
    if (!out) return MFGP_ERR_ARG;
    mfgp_handle_s* h = (mfgp_handle_s*)calloc(1, sizeof(mfgp_handle_s));
    if (!h) return MFGP_ERR_ARG;
    h->device = device;
    h->stream = nullptr;
    h->nb = 32;
    h->grad_chunk = 24;   // k_grad m-tiles per task (sweep at Goku T = 37: 16 -> 33.8 us, 24 -> 31.9, 40 -> 36.7)
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 0;
    h->ncu = ncu;
    h->flow_wgs = ncu;
    h->flow_min_t = FLOW_MIN_TILES;
    h->flow_timeout = FLOW_TIMEOUT_TICKS;
    h->f32_panel = 6;
    h->f32_lookahead = 1;
    h->f32_reserve = 32;
    h->gram_wgs = 0;
    if (const char* gv = getenv("MFGP_GRAM_WGS")) h->gram_wgs = atoi(gv);
    h->tiny = 1;   // small problems (n, p <= 64, D <= 16) in one launch: 37.0 us against 43.5 us of kernel
                   // time for the step sequence at HBS, 3.93 vs 4.31 ms for 100 captured Adam steps
                   // (MFGP_TINY=0 / mfgp_set_tiny(h, 0): the step sequence)
    if (const char* tv = getenv("MFGP_TINY")) h->tiny = atoi(tv) != 0;
    if (const char* rv = getenv("MFGP_F32_RESERVE")) h->f32_reserve = std::max(0, atoi(rv));
    if (const char* la = getenv("MFGP_F32_LOOKAHEAD")) h->f32_lookahead = atoi(la) != 0;
    h->f32_refine = 2;
    if (const char* rf = getenv("MFGP_F32_REFINE")) h->f32_refine = std::min(2, std::max(0, atoi(rf)));
    {
        int lo = 0, hi = 0;
        int cur = -1;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
        if (hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, hi) != hipSuccess) h->side = nullptr;
        if (hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess) h->ev_fork = nullptr;
        if (hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess) h->ev_join = nullptr;
        if (cur >= 0) (void)hipSetDevice(cur);
    }
    if (const char* fp = getenv("MFGP_F32_PANEL")) h->f32_panel = std::max(1, atoi(fp));
    if (const char* fl = getenv("MFGP_FLOW")) if (atoi(fl) == 0) h->flow_wgs = 0;
    if (const char* gc = getenv("MFGP_GRAD_CHUNK")) h->grad_chunk = std::max(1, atoi(gc));
    const char* env = getenv("MFGP_TILE");
    if (env && atoi(env) == 64) h->nb = 64;
    *out = h;
    return MFGP_OK;
}

int mfgp_destroy(mfgp_handle_t h) {
    if (h) {
        if (h->side) (void)hipStreamDestroy(h->side);
        if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
        if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    }
    free(h);
    return MFGP_OK;
}

int mfgp_set_stream(mfgp_handle_t h, void* stream) {
    CHECK_H(h);
    h->stream = (hipStream_t)stream;
    return MFGP_OK;
}

int mfgp_set_tile(mfgp_handle_t h, int nb) {
    CHECK_H(h);
    if (nb != 32 && nb != 64) return MFGP_ERR_ARG;
    h->nb = nb;
    return MFGP_OK;
}

int mfgp_get_tile(mfgp_handle_t h) { return h ? h->nb : MFGP_ERR_ARG; }

int mfgp_set_f32_refine(mfgp_handle_t h, int enable) {
    CHECK_H(h);
    if (enable < 0 || enable > 2) return MFGP_ERR_ARG;
    h->f32_refine = enable;
    return MFGP_OK;
}

int mfgp_set_flow(mfgp_handle_t h, int enable) {
    CHECK_H(h);
    if (enable < 0 || enable > 3) return MFGP_ERR_ARG;
    h->flow_wgs = enable ? h->ncu : 0;
    h->flow_trace = enable == 2;
    h->flow_min_t = enable == 3 ? 0 : FLOW_MIN_TILES;
    return MFGP_OK;
}

int mfgp_gpr_flow_trace(mfgp_handle_t h, int n, int p, int d, size_t* offset, int* count) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || !offset || !count) return MFGP_ERR_ARG;
    char* const base = reinterpret_cast<char*>((uintptr_t)1 << 20);   // any 256-B aligned stand-in
    const GprLayout L = gpr_layout(h->nb, n, p, d, base, h->grad_chunk, 0, h->flow_wgs, h->flow_min_t);
    *offset = (size_t)(reinterpret_cast<char*>(L.trace) - base);
    *count = L.ntrace;
    return MFGP_OK;
}

int mfgp_set_flow_timeout_us(mfgp_handle_t h, long long us) {
    CHECK_H(h);
    if (us < 0) return MFGP_ERR_ARG;
    h->flow_timeout = us * 100;   // s_memrealtime: 100 MHz
    return MFGP_OK;
}

int mfgp_set_tiny(mfgp_handle_t h, int enable) {
    if (!h) return MFGP_ERR_ARG;
    h->tiny = enable != 0;
    return MFGP_OK;
}

int mfgp_get_tiny(mfgp_handle_t h) { return h ? h->tiny : MFGP_ERR_ARG; }

int mfgp_set_resident(mfgp_handle_t h, int enable) {
    if (!h) return MFGP_ERR_ARG;
    h->resident = enable != 0;
    return MFGP_OK;
}

int mfgp_get_grad_chunk(mfgp_handle_t h) { return h ? h->grad_chunk : MFGP_ERR_ARG; }

int mfgp_get_flow(mfgp_handle_t h) { return h ? (h->flow_wgs > 0 ? (h->flow_min_t ? 1 : 3) : 0) : MFGP_ERR_ARG; }

int mfgp_flow_fence(mfgp_handle_t h, int op) {
    CHECK_H(h);
    // only the fence's own outcome: it enqueues an event wait / record, no kernel (hipGetLastError
    // would report whatever an earlier call left behind)
    if (op == MFGP_FENCE_WAIT) return fence_wait(h->device, h->stream, true);
    if (op == MFGP_FENCE_RECORD) return fence_record(h->device, h->stream, true);
    return MFGP_ERR_ARG;
}

static int gram_common(mfgp_handle_t h, int n1, int n2, int d, const double* X1, int ldx1, const double* X2,
                       int ldx2, const double* params, double diag_add, double* K, int ldk, int rbf, int nlf = 0) {
    CHECK_H(h);
    CHECK_D(d);
    if (n1 < 0 || n2 < 0 || !X1 || !X2 || !params || !K) return MFGP_ERR_ARG;
    if (n1 == 0 || n2 == 0) return MFGP_OK;
    GramArgs g{};
    g.X1 = X1; g.ldx1 = ldx1; g.n1 = n1;
    g.X2 = X2; g.ldx2 = ldx2; g.n2 = n2;
    g.theta = params; g.D = d; g.rbf_only = rbf;
    g.out = K; g.ldo = ldk; g.padded = 0; g.diag_add = diag_add; g.nlf = nlf;
    const int nb = h->nb;
    g.tiles_c = ceil_div(n2, nb);
    const int blocks = ceil_div(n1, nb) * g.tiles_c;
    if (nb == 64) launch_gram<64>(g, blocks, 1, h->stream);
    else launch_gram<32>(g, blocks, 1, h->stream);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

int mfgp_rbf_gram(mfgp_handle_t h, int n1, int n2, int d, const double* X1, int ldx1, const double* X2, int ldx2,
                  const double* params, double* K, int ldk) {
    return gram_common(h, n1, n2, d, X1, ldx1, X2, ldx2, params, 0.0, K, ldk, 1);
}

int mfgp_mf_gram(mfgp_handle_t h, int n1, int n2, int d, const double* X1, int ldx1, const double* X2, int ldx2,
                 const double* theta, double diag_add, double* K, int ldk) {
    return gram_common(h, n1, n2, d, X1, ldx1, X2, ldx2, theta, diag_add, K, ldk, 0);
}

int mfgp_mf_kdiag(mfgp_handle_t h, int n, int d, const double* X, int ldx, const double* theta, double* out) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 0 || !X || !theta || !out) return MFGP_ERR_ARG;
    if (n == 0) return MFGP_OK;
    hipLaunchKernelGGL(k_kdiag, dim3(ceil_div(n, 256)), dim3(256), 0, h->stream, X, (long)ldx, n, d, theta, out, 0);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

// ---------------------------------------------------------------- graph kernel (graph.py)
#define CHECK_LF(m) \
    if ((m) < 1 || (m) > MFGP_MAX_LF) return MFGP_ERR_ARG

int mfgp_gmf_gram(mfgp_handle_t h, int nlf, int n1, int n2, int d, const double* X1, int ldx1, const double* X2,
                  int ldx2, const double* theta, double diag_add, double* K, int ldk) {
    CHECK_LF(nlf);
    return gram_common(h, n1, n2, d, X1, ldx1, X2, ldx2, theta, diag_add, K, ldk, 0, nlf);
}

int mfgp_gmf_kdiag(mfgp_handle_t h, int nlf, int n, int d, const double* X, int ldx, const double* theta,
                   double* out) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_LF(nlf);
    if (n < 0 || !X || !theta || !out) return MFGP_ERR_ARG;
    if (n == 0) return MFGP_OK;
    hipLaunchKernelGGL(k_kdiag, dim3(ceil_div(n, 256)), dim3(256), 0, h->stream, X, (long)ldx, n, d, theta, out,
                       nlf);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

int mfgp_gmf_gpr_workspace_size(mfgp_handle_t h, int nlf, int n, int p, int d, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_LF(nlf);
    if (n < 1 || p < 1 || !bytes) return MFGP_ERR_ARG;
    *bytes = gpr_layout(h->nb, n, p, d, nullptr, h->grad_chunk, nlf, h->flow_wgs, h->flow_min_t).bytes;
    return MFGP_OK;
}

int mfgp_gmf_gpr_lml(mfgp_handle_t h, int nlf, int n, int p, int d, const double* X, int ldx, const double* Y,
                     int ldy, const double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_LF(nlf);
    if (n < 1 || p < 1 || !X || !Y || !theta || !ws || !out || !info) return MFGP_ERR_ARG;
    if (h->nb == 64)
        return gpr_value_grad<64>(h, n, p, d, X, ldx, Y, ldy, (double*)theta, want_grad, ws, ws_bytes, out, info,
                                  nullptr, nullptr, nlf);
    return gpr_value_grad<32>(h, n, p, d, X, ldx, Y, ldy, (double*)theta, want_grad, ws, ws_bytes, out, info,
                              nullptr, nullptr, nlf);
}

int mfgp_gmf_gpr_predict_workspace_size(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_LF(nlf);
    if (n < 1 || p < 1 || nstar < 0 || !bytes) return MFGP_ERR_ARG;
    *bytes = pred_layout(h->nb, n, p, d, nstar, nullptr, h->grad_chunk, nlf).bytes;
    return MFGP_OK;
}

int mfgp_gmf_gpr_predict(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, const double* X, int ldx,
                         const double* Y, int ldy, const double* Xs, int ldxs, const double* theta, void* ws,
                         size_t ws_bytes, double* mean, int ldm, double* var, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_LF(nlf);
    if (n < 1 || p < 1 || nstar < 0 || !X || !Y || !theta || !ws || !info) return MFGP_ERR_ARG;
    if (nstar == 0) return MFGP_OK;
    if (!Xs || !mean || !var) return MFGP_ERR_ARG;
    if (h->nb == 64)
        return predict_impl<64>(h, n, p, d, nstar, X, ldx, Y, ldy, Xs, ldxs, theta, ws, ws_bytes, mean, ldm, var,
                                info, nlf);
    return predict_impl<32>(h, n, p, d, nstar, X, ldx, Y, ldy, Xs, ldxs, theta, ws, ws_bytes, mean, ldm, var, info,
                            nlf);
}

int mfgp_gpr_workspace_size(mfgp_handle_t h, int n, int p, int d, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || !bytes) return MFGP_ERR_ARG;
    *bytes = gpr_layout(h->nb, n, p, d, nullptr, h->grad_chunk, 0, h->flow_wgs, h->flow_min_t).bytes;
    return MFGP_OK;
}

int mfgp_gpr_lml(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y, int ldy,
                 const double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || !X || !Y || !theta || !ws || !out || !info) return MFGP_ERR_ARG;
    if (h->nb == 64)
        return gpr_value_grad<64>(h, n, p, d, X, ldx, Y, ldy, (double*)theta, want_grad, ws, ws_bytes, out, info,
                                  nullptr);
    return gpr_value_grad<32>(h, n, p, d, X, ldx, Y, ldy, (double*)theta, want_grad, ws, ws_bytes, out, info,
                              nullptr);
}

int mfgp_gpr_adam_step(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y, int ldy,
                       double* theta, double* u, double* m, double* v, const unsigned char* trainable,
                       const int* tie, int* step, double lr, double beta1, double beta2, double eps,
                       double* loss_hist, void* ws, size_t ws_bytes, double* out, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || !X || !Y || !theta || !u || !m || !v || !trainable || !step || !loss_hist || !ws ||
        !out || !info)
        return MFGP_ERR_ARG;
    FinArgs f{};
    f.theta = theta; f.u = u; f.m = m; f.v = v; f.trainable = trainable; f.tie = tie; f.step = step;
    f.lr = lr; f.b1 = beta1; f.b2 = beta2; f.eps = eps; f.loss_hist = loss_hist;
    f.noise_index = theta_size(d) - 1;
    if (h->nb == 64) return gpr_value_grad<64>(h, n, p, d, X, ldx, Y, ldy, theta, 1, ws, ws_bytes, out, info, &f);
    return gpr_value_grad<32>(h, n, p, d, X, ldx, Y, ldy, theta, 1, ws, ws_bytes, out, info, &f);
}

int mfgp_gpr_lml_phase_times(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y,
                             int ldy, const double* theta, void* ws, size_t ws_bytes, double* out, int* info,
                             float* ms) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || !X || !Y || !theta || !ws || !out || !info || !ms) return MFGP_ERR_ARG;
    PhaseMarks pm;
    for (int i = 0; i < 6; ++i) (void)hipEventCreate(&pm.ev[i]);
    int rc = (h->nb == 64)
                 ? gpr_value_grad<64>(h, n, p, d, X, ldx, Y, ldy, (double*)theta, 1, ws, ws_bytes, out, info,
                                      nullptr, &pm)
                 : gpr_value_grad<32>(h, n, p, d, X, ldx, Y, ldy, (double*)theta, 1, ws, ws_bytes, out, info,
                                      nullptr, &pm);
    if (rc == MFGP_OK) {
        (void)hipEventSynchronize(pm.ev[pm.count - 1]);
        for (int i = 0; i + 1 < pm.count; ++i) (void)hipEventElapsedTime(&ms[i], pm.ev[i], pm.ev[i + 1]);
    }
    for (int i = 0; i < 6; ++i) (void)hipEventDestroy(pm.ev[i]);
    return rc;
}

int mfgp_theta_from_u(mfgp_handle_t h, const double* u, double* theta, int g, int noise_index) {
    CHECK_H(h);
    if (!u || !theta || g < 1 || g > 256) return MFGP_ERR_ARG;
    hipLaunchKernelGGL(k_theta_from_u, dim3(1), dim3(256), 0, h->stream, u, theta, g, noise_index);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

int mfgp_gpr_predict_workspace_size(mfgp_handle_t h, int n, int p, int d, int nstar, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || nstar < 0 || !bytes) return MFGP_ERR_ARG;
    *bytes = pred_layout(h->nb, n, p, d, nstar, nullptr, h->grad_chunk).bytes;
    return MFGP_OK;
}

int mfgp_gpr_predict(mfgp_handle_t h, int n, int p, int d, int nstar, const double* X, int ldx, const double* Y,
                     int ldy, const double* Xs, int ldxs, const double* theta, void* ws, size_t ws_bytes,
                     double* mean, int ldm, double* var, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || p < 1 || nstar < 0 || !X || !Y || !theta || !ws || !info) return MFGP_ERR_ARG;
    if (nstar == 0) return MFGP_OK;
    if (!Xs || !mean || !var) return MFGP_ERR_ARG;
    if (h->nb == 64)
        return predict_impl<64>(h, n, p, d, nstar, X, ldx, Y, ldy, Xs, ldxs, theta, ws, ws_bytes, mean, ldm, var,
                                info);
    return predict_impl<32>(h, n, p, d, nstar, X, ldx, Y, ldy, Xs, ldxs, theta, ws, ws_bytes, mean, ldm, var, info);
}

int mfgp_gpr_predict_cov_workspace_size(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    if (nlf < 0 || nlf > MFGP_MAX_LF || n < 1 || p < 1 || nstar < 0 || !bytes) return MFGP_ERR_ARG;
    *bytes = pred_layout(h->nb, n, p, d, nstar, nullptr, h->grad_chunk, nlf, 1).bytes;
    return MFGP_OK;
}

int mfgp_gpr_predict_cov(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, const double* X, int ldx,
                         const double* Y, int ldy, const double* Xs, int ldxs, const double* theta, void* ws,
                         size_t ws_bytes, double* mean, int ldm, double* var, double* cov, int ldc, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (nlf < 0 || nlf > MFGP_MAX_LF) return MFGP_ERR_ARG;
    if (n < 1 || p < 1 || nstar < 0 || !X || !Y || !theta || !ws || !info) return MFGP_ERR_ARG;
    if (nstar == 0) return MFGP_OK;
    if (!Xs || !mean || !var || !cov || ldc < nstar) return MFGP_ERR_ARG;
    if (h->nb == 64)
        return predict_impl<64>(h, n, p, d, nstar, X, ldx, Y, ldy, Xs, ldxs, theta, ws, ws_bytes, mean, ldm, var,
                                info, nlf, cov, ldc);
    return predict_impl<32>(h, n, p, d, nstar, X, ldx, Y, ldy, Xs, ldxs, theta, ws, ws_bytes, mean, ldm, var, info,
                            nlf, cov, ldc);
}

int mfgp_potrf_inv_workspace_size(mfgp_handle_t h, int n, int batch, size_t* bytes) {
    CHECK_H(h);
    if (n < 1 || batch < 1 || !bytes) return MFGP_ERR_ARG;
    *bytes = potrf_layout(h->nb, n, batch, nullptr).bytes;
    return MFGP_OK;
}

int mfgp_potrf_inv(mfgp_handle_t h, int n, int batch, const double* A, int lda, long sA, void* ws, size_t ws_bytes,
                   double* Linv, int ldl, long sL, double* ldiag, int* info) {
    CHECK_H(h);
    if (n < 1 || batch < 1 || !A || !ws || !Linv || !info) return MFGP_ERR_ARG;
    if (h->nb == 64) return potrf_inv_impl<64>(h, n, batch, A, lda, sA, ws, ws_bytes, Linv, ldl, sL, ldiag, info);
    return potrf_inv_impl<32>(h, n, batch, A, lda, sA, ws, ws_bytes, Linv, ldl, sL, ldiag, info);
}

int mfgp_svgp_workspace_size(mfgp_handle_t h, int n, int m, int l, int p, int d, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || m < 1 || l < 1 || p < 1 || !bytes) return MFGP_ERR_ARG;
    *bytes = (size_t)svgp_workspace_bytes(h->nb, n, m, l, p, d);
    return MFGP_OK;
}

int mfgp_svgp_elbo(mfgp_handle_t h, int n, int m, int l, int p, int d, const double* X, int ldx, const double* Y,
                   int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                   const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                   size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || m < 1 || l < 1 || p < 1 || !X || !Y || !Z || !thetas || !q_mu || !q_sqrt || !ws || !out || !info)
        return MFGP_ERR_ARG;
    if (!W && l != p) return MFGP_ERR_ARG;
    svgp_set_side(SvgpSide{h->side, h->ev_fork, h->ev_join});
    return svgp_elbo_impl(h->stream, h->nb, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise,
                          scale, jitter, ws, ws_bytes, out, g_mu, g_var, info, nullptr);
}

int mfgp_svgp_grad_workspace_size(mfgp_handle_t h, int n, int m, int l, int p, int d, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    if (bytes == nullptr || n < 1 || m < 1 || l < 1 || p < 1) return MFGP_ERR_ARG;
    *bytes = svgp_grad_workspace_bytes(h->nb, n, m, l, p, d);
    return MFGP_OK;
}

int mfgp_svgp_elbo_grad(mfgp_handle_t h, int n, int m, int l, int p, int d, const double* X, int ldx,
                        const double* Y, int ldy, const double* Z, int ldz, const double* thetas,
                        const double* q_mu, const double* q_sqrt, const double* W, const double* noise,
                        double scale, double kl_mult, double jitter, void* ws, size_t ws_bytes, double* out, double* g_mu,
                        double* g_var, double* gZ, double* gtheta, double* gq_mu, double* gq_sqrt, double* gW,
                        double* gnoise, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (n < 1 || m < 1 || l < 1 || p < 1 || !X || !Y || !Z || !thetas || !q_mu || !q_sqrt || !noise || !ws ||
        !out || !g_mu || !g_var || !gZ || !gtheta || !gq_mu || !gq_sqrt || !gnoise || !info)
        return MFGP_ERR_ARG;
    if (W == nullptr && l != p) return MFGP_ERR_ARG;
    if (W != nullptr && gW == nullptr) return MFGP_ERR_ARG;
    if (ldx < d + 1 || ldz < d + 1 || ldy < p) return MFGP_ERR_ARG;
    svgp_set_side(SvgpSide{h->side, h->ev_fork, h->ev_join, h->svgp_qs_packed});
    return svgp_grad_impl(h->stream, h->nb, n, m, l, p, d, X, ldx, Y, ldy, Z, ldz, thetas, q_mu, q_sqrt, W, noise, 0.0,
                          scale, kl_mult, jitter, ws, ws_bytes, out, g_mu, g_var, gZ, gtheta, gq_mu, gq_sqrt, gW,
                          gnoise, info);
}

int mfgp_set_svgp_qs_packed(mfgp_handle_t h, int packed) {
    CHECK_H(h);
    if (packed != 0 && packed != 1) return MFGP_ERR_ARG;
    h->svgp_qs_packed = packed;
    return MFGP_OK;
}

int mfgp_adam_packed(mfgp_handle_t h, int n, double* u, double* c, const double* g, double* m, double* v,
                     const unsigned char* trainable, const unsigned char* transform, const unsigned char* span,
                     int* step, const double* lr_sched, double beta1, double beta2, double eps, const double* out,
                     double kl_mult, double* loss_hist, double* kl_hist) {
    CHECK_H(h);
    if (n < 1 || !u || !c || !g || !m || !v || !trainable || !transform || !step || !lr_sched || !out)
        return MFGP_ERR_ARG;
    return adam_packed_impl(h->stream, n, u, c, g, m, v, trainable, transform, span, step, lr_sched, beta1, beta2, eps,
                            out, kl_mult, loss_hist, kl_hist, nullptr, 0);
}

int mfgp_adam_packed_ex(mfgp_handle_t h, int n, double* u, double* c, const double* g, double* m, double* v,
                        const unsigned char* trainable, const unsigned char* transform, const unsigned char* span,
                        int* step, const double* lr_sched, double beta1, double beta2, double eps,
                        const double* out, double kl_mult, double* loss_hist, double* kl_hist, const int* info,
                        int ninfo) {
    CHECK_H(h);
    if (n < 1 || !u || !c || !g || !m || !v || !trainable || !transform || !step || !lr_sched || !out || ninfo < 0 ||
        (ninfo > 0 && !info))
        return MFGP_ERR_ARG;
    return adam_packed_impl(h->stream, n, u, c, g, m, v, trainable, transform, span, step, lr_sched, beta1, beta2, eps,
                            out, kl_mult, loss_hist, kl_hist, info, ninfo);
}

int mfgp_svgp_predict(mfgp_handle_t h, int nstar, int m, int l, int p, int d, const double* Xs, int ldxs,
                      const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                      const double* W, double jitter, void* ws, size_t ws_bytes, double* g_mu, double* g_var,
                      double* f_mu, double* f_var, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (nstar < 1 || m < 1 || l < 1 || p < 1 || !Xs || !Z || !thetas || !q_mu || !q_sqrt || !ws || !g_mu ||
        !g_var || !f_mu || !f_var || !info)
        return MFGP_ERR_ARG;
    if (!W && l != p) return MFGP_ERR_ARG;
    svgp_set_side(SvgpSide{h->side, h->ev_fork, h->ev_join});
    return svgp_predict_impl(h->stream, h->nb, nstar, m, l, p, d, Xs, ldxs, Z, ldz, thetas, q_mu, q_sqrt, W, jitter,
                             ws, ws_bytes, g_mu, g_var, f_mu, f_var, info);
}

int mfgp_svgp_predict_cov_workspace_size(mfgp_handle_t h, int nstar, int m, int l, int p, int d, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    if (nstar < 1 || m < 1 || l < 1 || p < 1 || !bytes) return MFGP_ERR_ARG;
    *bytes = svgp_predict_cov_workspace_bytes(h->nb, nstar, m, l, p, d);
    return MFGP_OK;
}

int mfgp_svgp_predict_cov(mfgp_handle_t h, int mode, int nstar, int m, int l, int p, int d, const double* Xs,
                          int ldxs, const double* Z, int ldz, const double* thetas, const double* q_mu,
                          const double* q_sqrt, const double* W, double jitter, void* ws, size_t ws_bytes,
                          double* g_mu, double* g_var, double* f_mu, double* f_var, double* f_cov, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    if (mode < 1 || mode > 3 || nstar < 1 || m < 1 || l < 1 || p < 1 || !Xs || !Z || !thetas || !q_mu || !q_sqrt ||
        !ws || !g_mu || !g_var || !f_mu || !f_var || !f_cov || !info)
        return MFGP_ERR_ARG;
    if (!W && l != p) return MFGP_ERR_ARG;
    svgp_set_side(SvgpSide{h->side, h->ev_fork, h->ev_join});
    const int rc = svgp_predict_cov_impl(h->stream, h->nb, mode, nstar, m, l, p, d, Xs, ldxs, Z, ldz, thetas, q_mu,
                                         q_sqrt, W, jitter, ws, ws_bytes, g_mu, g_var, f_mu, f_var, f_cov, info);
    return rc == -2 ? MFGP_ERR_WORKSPACE : (rc ? MFGP_ERR_LAUNCH : MFGP_OK);
}

int mfgp_selftest_mfma(mfgp_handle_t h, double* out) {
    CHECK_H(h);
    if (!out) return MFGP_ERR_ARG;
    hipLaunchKernelGGL(k_selftest_mfma, dim3(1), dim3(64), 0, h->stream, out);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

// ---------------------------------------------------------------- dtype-generic forms
#define CHECK_DT(dt) \
    if ((dt) != MFGP_F64 && (dt) != MFGP_F32) return MFGP_ERR_ARG

int mfgp_set_f32_panel(mfgp_handle_t h, int tiles) {
    CHECK_H(h);
    if (tiles < 1 || tiles > 64) return MFGP_ERR_ARG;
    h->f32_panel = tiles;
    return MFGP_OK;
}

int mfgp_set_f32_lookahead(mfgp_handle_t h, int enable) {
    CHECK_H(h);
    h->f32_lookahead = enable != 0;
    return MFGP_OK;
}

int mfgp_set_f32_reserve(mfgp_handle_t h, int cus) {
    CHECK_H(h);
    if (cus < 0) return MFGP_ERR_ARG;
    h->f32_reserve = cus;
    return MFGP_OK;
}

int mfgp_mf_gram_ex(mfgp_handle_t h, int dtype, int n1, int n2, int d, const void* X1, int ldx1, const void* X2,
                    int ldx2, const double* theta, double diag_add, void* K, int ldk) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64)
        return mfgp_mf_gram(h, n1, n2, d, (const double*)X1, ldx1, (const double*)X2, ldx2, theta, diag_add,
                            (double*)K, ldk);
    if (n1 < 1 || n2 < 1 || !X1 || !X2 || !theta || !K || ldx1 < d + 1 || ldx2 < d + 1 || ldk < n2)
        return MFGP_ERR_ARG;
    launch_f32_gram_dense((const float*)X1, ldx1, n1, (const float*)X2, ldx2, n2, d, theta, (float)diag_add,
                          (float*)K, ldk, h->stream);
    return last() == hipSuccess ? MFGP_OK : MFGP_ERR_LAUNCH;
}

int mfgp_gpr_workspace_size_ex(mfgp_handle_t h, int dtype, int n, int p, int d, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64) return mfgp_gpr_workspace_size(h, n, p, d, bytes);
    if (n < 1 || p < 1 || !bytes) return MFGP_ERR_ARG;
    *bytes = f32_layout(n, p, d, 0, 1, h->f32_panel, nullptr).bytes;
    if (h->f32_refine) *bytes = std::max(*bytes, f32_layout(n, p, d, 0, 0, h->f32_panel, nullptr, 1).bytes);
    return MFGP_OK;
}

int mfgp_gpr_lml_ex(mfgp_handle_t h, int dtype, int n, int p, int d, const void* X, int ldx, const void* Y, int ldy,
                    const double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64)
        return mfgp_gpr_lml(h, n, p, d, (const double*)X, ldx, (const double*)Y, ldy, theta, want_grad, ws, ws_bytes,
                            out, info);
    if (n < 1 || p < 1 || !X || !Y || !theta || !ws || !out || !info || ldx < d + 1 || ldy < p) return MFGP_ERR_ARG;
    return f32_value_grad(h, n, p, d, (const float*)X, ldx, (const float*)Y, ldy, (double*)theta, want_grad, ws,
                          ws_bytes, out, info, nullptr);
}

int mfgp_gpr_adam_step_ex(mfgp_handle_t h, int dtype, int n, int p, int d, const void* X, int ldx, const void* Y,
                          int ldy, double* theta, double* u, double* m, double* v, const unsigned char* trainable,
                          const int* tie, int* step, double lr, double beta1, double beta2, double eps,
                          double* loss_hist, void* ws, size_t ws_bytes, double* out, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64)
        return mfgp_gpr_adam_step(h, n, p, d, (const double*)X, ldx, (const double*)Y, ldy, theta, u, m, v, trainable,
                                  tie, step, lr, beta1, beta2, eps, loss_hist, ws, ws_bytes, out, info);
    if (n < 1 || p < 1 || !X || !Y || !theta || !u || !m || !v || !trainable || !step || !loss_hist || !ws ||
        !out || !info || ldx < d + 1 || ldy < p)
        return MFGP_ERR_ARG;
    FinArgs f{};
    f.theta = theta; f.u = u; f.m = m; f.v = v; f.trainable = trainable; f.tie = tie; f.step = step;
    f.lr = lr; f.b1 = beta1; f.b2 = beta2; f.eps = eps; f.loss_hist = loss_hist;
    f.noise_index = theta_size(d) - 1;
    return f32_value_grad(h, n, p, d, (const float*)X, ldx, (const float*)Y, ldy, theta, 1, ws, ws_bytes, out, info,
                          &f);
}

int mfgp_gpr_phase_times_ex(mfgp_handle_t h, int dtype, int n, int p, int d, const void* X, int ldx, const void* Y,
                            int ldy, const double* theta, void* ws, size_t ws_bytes, double* out, int* info,
                            float* ms, double* flops, int* launches, int nphase) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (!ms || nphase < 1) return MFGP_ERR_ARG;
    if (dtype == MFGP_F64) {
        float m5[5] = {};
        const int rc = mfgp_gpr_lml_phase_times(h, n, p, d, (const double*)X, ldx, (const double*)Y, ldy, theta, ws,
                                                ws_bytes, out, info, m5);
        for (int i = 0; i < nphase; ++i) {
            ms[i] = i < 5 ? m5[i] : 0.0f;
            if (flops) flops[i] = 0.0;
            if (launches) launches[i] = 0;
        }
        return rc;
    }
    if (n < 1 || p < 1 || !X || !Y || !theta || !ws || !out || !info) return MFGP_ERR_ARG;
    F32Marks* mk = new F32Marks();
    const int rc = f32_value_grad(h, n, p, d, (const float*)X, ldx, (const float*)Y, ldy, (double*)theta, 1, ws,
                                  ws_bytes, out, info, nullptr, mk);
    float all[F32_NPHASE];
    mk->collect(all);
    for (int i = 0; i < nphase; ++i) {
        ms[i] = i < F32_NPHASE ? all[i] : 0.0f;
        if (flops) flops[i] = i < F32_NPHASE ? mk->flops[i] : 0.0;
        if (launches) launches[i] = i < F32_NPHASE ? mk->launches[i] : 0;
    }
    delete mk;
    return rc;
}

int mfgp_gpr_predict_workspace_size_ex(mfgp_handle_t h, int dtype, int n, int p, int d, int nstar, size_t* bytes) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64) return mfgp_gpr_predict_workspace_size(h, n, p, d, nstar, bytes);
    if (n < 1 || p < 1 || nstar < 0 || !bytes) return MFGP_ERR_ARG;
    *bytes = f32_layout(n, p, d, nstar > 0 ? nstar : 1, 0, h->f32_panel, nullptr, h->f32_refine).bytes;
    return MFGP_OK;
}

int mfgp_gpr_predict_ex(mfgp_handle_t h, int dtype, int n, int p, int d, int nstar, const void* X, int ldx,
                        const void* Y, int ldy, const void* Xs, int ldxs, const double* theta, void* ws,
                        size_t ws_bytes, void* mean, int ldm, void* var, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64)
        return mfgp_gpr_predict(h, n, p, d, nstar, (const double*)X, ldx, (const double*)Y, ldy, (const double*)Xs,
                                ldxs, theta, ws, ws_bytes, (double*)mean, ldm, (double*)var, info);
    if (n < 1 || p < 1 || nstar < 0 || !X || !Y || !theta || !ws || !info) return MFGP_ERR_ARG;
    if (nstar == 0) return MFGP_OK;
    if (!Xs || !mean || !var || ldx < d + 1 || ldy < p || ldxs < d + 1 || ldm < p) return MFGP_ERR_ARG;
    return f32_predict(h, n, p, d, nstar, (const float*)X, ldx, (const float*)Y, ldy, (const float*)Xs, ldxs, theta,
                       ws, ws_bytes, (float*)mean, ldm, (float*)var, info);
}

int mfgp_gpr_predict_cov_workspace_size_ex(mfgp_handle_t h, int dtype, int nlf, int n, int p, int d, int nstar,
                                           size_t* bytes) {
    CHECK_H(h);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64) return mfgp_gpr_predict_cov_workspace_size(h, nlf, n, p, d, nstar, bytes);
    if (nlf != 0) return MFGP_ERR_ARG;   // the fp32 path runs the linear multi-fidelity kernel
    return mfgp_gpr_predict_workspace_size_ex(h, dtype, n, p, d, nstar, bytes);
}

int mfgp_gpr_predict_cov_ex(mfgp_handle_t h, int dtype, int nlf, int n, int p, int d, int nstar, const void* X,
                            int ldx, const void* Y, int ldy, const void* Xs, int ldxs, const double* theta, void* ws,
                            size_t ws_bytes, void* mean, int ldm, void* var, void* cov, int ldc, int* info) {
    CHECK_H(h);
    CHECK_D(d);
    CHECK_DT(dtype);
    if (dtype == MFGP_F64)
        return mfgp_gpr_predict_cov(h, nlf, n, p, d, nstar, (const double*)X, ldx, (const double*)Y, ldy,
                                    (const double*)Xs, ldxs, theta, ws, ws_bytes, (double*)mean, ldm, (double*)var,
                                    (double*)cov, ldc, info);
    if (nlf != 0 || n < 1 || p < 1 || nstar < 0 || !X || !Y || !theta || !ws || !info) return MFGP_ERR_ARG;
    if (nstar == 0) return MFGP_OK;
    if (!Xs || !mean || !var || !cov || ldx < d + 1 || ldy < p || ldxs < d + 1 || ldm < p || ldc < nstar)
        return MFGP_ERR_ARG;
    return f32_predict(h, n, p, d, nstar, (const float*)X, ldx, (const float*)Y, ldy, (const float*)Xs, ldxs, theta,
                       ws, ws_bytes, (float*)mean, ldm, (float*)var, info, (float*)cov, ldc);
}

}  // extern "C"
