// Internal (host<->device) argument blocks and launchers of the MI355X GP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace mfgp {

struct GramArgs {
    const double* X1; long ldx1; long sx1; int n1;
    const double* X2; long ldx2; long sx2; int n2;
    const double* theta; long stheta;         // per-batch theta stride (doubles)
    int D;
    int rbf_only;                             // 1: plain SquaredExponential on all D columns
    double* out; long ldo; long so;
    int padded;                               // 1: LML layout (square, lower tiles, identity pad)
    int npad;                                 // padded size (LML layout)
    int tiles_c;                              // number of column tiles (dense layout)
    int add_noise;                            // add theta noise on i==j<n (LML layout)
    double diag_add;                          // extra constant on i==j<n (jitter)
    // fused factor of tile (0,0) (LML layout only)
    double* Dd; long sD; double* ldiag; long sL; int* info;
    // fused RHS init (LML layout only; R == nullptr: skip): R = [I | Y]
    double* R; long ldr; long sR; const double* Y; long ldy; long sY; int p, ppad;
    int nlf;                                  // 0: LinearMultiFidelityKernel; m >= 1: graph kernel, m LF sources
    int* cnt; int ncnt;                       // arrival counters zeroed by workgroup 0 (reduce merge)
    double* isent; int nisent;                // k_reduce_items' items, FLOW_SENTINEL-filled by workgroup 0 (FinArgs::flag)
    // k_grad task order (nullptr: none): one extra LAST workgroup builds it (grad_order)
    int* gorder; int gT, gchunk, gTp;
    // k_chol_flow owner table (nullptr: none): one more extra workgroup builds it and zeroes
    // the flow flags (build_flow_owner); every workgroup fills its share of the publication
    // area with the sentinel
    int* fown; int fW; int* fflags; int nfflags;
    double* fpub; long npub;
    long long* dbg;               // diagnostic per-workgroup timeline (nullptr: off)
    // LML layout: > 0 -> that many tile workgroups, workgroup 0 takes tile (0,0) (and its fused
    // factor) alone on its CU, the others loop over the remaining tiles; 0 -> one tile each
    int tile_wgs;
};

// k_chol_flow (mfgp_flow.hip): persistent dataflow Cholesky + L^{-1} + Z + alpha, NB = 32, batch 1
constexpr int FLOW_MAXOWN = 4;                      // tiles per worker wave
constexpr int FLOW_WAVES = 8;                       // waves per workgroup (two per SIMD)
constexpr int FLOW_THREADS = 64 * FLOW_WAVES;
constexpr int FLOW_FSTRIDE = 32;                    // ints per flag: one 128-B line each (polled lines
                                                    // are not shared, no hot line under 2k pollers)
constexpr size_t FLOW_LDS_BYTES = 128 * 1024;       // > 80 KB: one workgroup per CU
constexpr unsigned long long FLOW_SENTINEL = 0x7FF4DEAD7FF4DEADull;   // signalling NaN: "not yet published"
struct FlowArgs {
    double* A; long lda;          // K + s2 I lower tiles -> L tiles (in place)
    double* R; long ldr;          // [I | Y] accumulators -> X^T tiles (in place)
    double* Xo; long ldx;         // [L^{-1} | Z] (+ alpha^T rows for k_grad)
    double* Dd;                   // T diagonal inverses D_k (NB x NB)
    double* ldiag;
    int* info;
    double* alpha; long ldal;
    double* zpart;
    int* flags;                   // abort word (zeroed by build_flow_owner)
    double* pub;                  // publication area, flow_npub(T, Tp) doubles of FLOW_SENTINEL
    const int* own;               // [W * FLOW_MAXOWN] tile codes (-1: none)
    int T, Tp, n, p;
    long long* trace;             // diagnostic timeline (nullptr: off), flow_trace_count entries
    int nwaves;                   // worker waves (trace layout)
    long long timeout;            // bound of every hand-off wait, 100 MHz ticks (FLOW_TIMEOUT_TICKS)
    // the K + s2 I tiles are formed inside the launch (flow_gram_tile): each A tile by its owner
    // wave before its first item, tile (0,0) and the band tiles of rows 1-2 by the diag
    // workgroup's waves, row 3's by idle worker waves (FT_G); the Y column tiles of R are read
    // from Y on first touch
    const double* X; long ldxi;   // inputs [n, D+1] (fidelity flag in column D)
    const double* Y; long ldy;    // outputs [n, p]
    const double* theta;          // [vL, lL(D), vD, lD(D), rho0, noise]
    int D;
    int gram;                     // 1: the AR1 Gram formed in the launch; 0: A holds K + s2 I already
                                  // (the graph kernel's k_gram ran first)
};
constexpr long long FLOW_TIMEOUT_TICKS = 5000000;   // 50 ms (s_memrealtime is 100 MHz)
int flow_trace_count(int T, int nwg);

struct CholArgs {
    double* A; long lda; long sA;        // SPD matrix, lower tiles, updated in place
    double* R; long ldr; long sR;        // RHS [I | Y] (identity tiles 0..T-1, Y tiles T..T+Tp-1)
    double* Xo; long ldx; long sX;       // output [L^{-1} | Z]
    double* Dd; long sD;                 // T inverse diagonal factors (NB x NB each)
    double* ldiag; long sL;              // diag(L)
    int* info;
    int T, Tp, k;
    // Batched steps (k_chol_fused / k_chol_panel): R = [I | ...] is implicit -- the identity tile
    // R_kk and the untouched strictly-lower tiles (zero until the step c == k that first updates
    // R_ic) are formed in the kernels, so R needs no initialisation (the Gram skips writing it)
    int r_implicit;
    // Optional (batch 1, LML path): alpha = L^{-T} Z accumulated row by row as rows of
    // [L^{-1} | Z] become final, and the sum Z^2 partials.  nullptr: skipped.
    double* alpha; long ldal;            // Npad x Ppad
    double* zpart;                       // [T*Tp]
    int n, p;
};


struct GradArgs {
    const double* Xo; long ldx;           // [L^{-1} | Z], then rows [-alpha^T / P ; alpha^T] (Ppad each)
    const double* X; long ldxx;           // inputs [n, D+1]
    const double* theta;
    double* gpart; int gstride;           // per task partial gradient
    int T, Tp, n, P, D;
    int chunk;                            // m-tiles per task
    int nlf;                              // kernel family (GramArgs::nlf)
    const int* order;                     // workgroup -> task (nullptr: identity), see grad_order
    // flow path: the next evaluation's set-up, done here after the flow has ended -- every
    // workgroup sentinel-fills its share of the publication area, workgroup 0 the item slots of
    // k_reduce_items (nullptr: none)
    double* fpub; long npub;
    double* isent; int nisent;
};

constexpr int FIN_MAXG = 254;   // theta entries finalize_body stages in LDS (graph kernel: <= 186)
// k_reduce_items' sentinel protocol (FinArgs::flag) on the fp64 LML path; 0: arrival counter
#ifndef MFGP_REDUCE_FLAG
#define MFGP_REDUCE_FLAG 1
#endif
struct FinArgs {
    const double* zpart; int nz;
    const double* ldiag; int n;
    const double* gpart; int ng; int gstride;
    const int* info;
    int P, D, want_grad;
    double* out;                      // [lml, grad(G)]
    // Adam (optional, unconstrained parameters)
    int adam;
    double* theta;                    // constrained theta, refreshed after the step
    double* u; double* m; double* v;
    const unsigned char* trainable;
    const int* tie;                   // tie[q]: entries sharing one variable (isotropic lengthscales)
    int* step;
    double lr, b1, b2, eps;
    double* loss_hist;                // loss_hist[step] = -lml (pre-step)
    int noise_index;                  // theta entry using Shift(1e-6) o Softplus
    double* items;                    // [2 + G] stage-1 reduction results
    int G;                            // theta entries (kernel_theta_size)
    int* cnt;                         // arrival counter (zero on entry): last item workgroup finalizes
    int flag;                         // 1: items[] hold FLOW_SENTINEL on entry (the Gram launch filled them):
                                      //    workgroup 0 finalizes once every other item is published
    int* abortw;                      // flow path: k_chol_flow's abort word -- set: the evaluation timed
                                      // out (info := MFGP_FLOW_TIMEOUT); workgroup 0 zeroes it for the next
};

struct PredAArgs {
    const double* Xo; long ldx;       // [L^{-1} | Z]
    const double* Kmn; long ldk;      // Npad x Nspad
    double* Am; long ldam;            // Npad x Nspad   A = L^{-1} Kmn
    int Ts;
};

struct PredOutArgs {
    const double* Am; long ldam;
    const double* Xo; long ldx;
    const double* kdiag;              // nstar
    double* mean; long ldm;           // nstar x p
    double* var;                      // nstar
    int T, Tp, nstar, p;
};

// Batched fp64 MFMA GEMM (k_bgemm, mfgp_svgp_grad.hip), NB x NB output tiles:
// D = (alpha * op(A) diag(s) op(B) + beta * Cin) [* diag(colscale)] + x y^T   (tril: zero j > i)
struct BgemmArgs {
    const double* A; long lda; long sA;
    const double* B; long ldb; long sB;
    const double* s; long ss;              // k scaling (nullptr: none)
    const double* colscale; long scs;      // output column scaling (nullptr: none)
    const double* Cin; long ldc; long sC; double beta;
    const double* x; long sx; const double* y; long sy;   // rank-1 term (nullptr: none)
    double* D; long ldd; long sD;
    double alpha;
    int Mt, Nt, Kt, tril;
    // sym (k_bgemm2 only, with tril; a symmetric product formed from its lower tiles): 1 stores
    // Psi(D) = (tril D + tril D^T - diag D) / 2, the lower tiles' values halved and mirrored
    // across the diagonal; 2 stores tril D mirrored (D itself, exactly symmetric)
    int sym;
    // known-zero triangles of the operands, so their k-tiles are skipped (never read):
    // amask 1: op(A) lower (k-tile <= row tile), 2: op(A) upper (k-tile >= row tile);
    // bmask 1: op(B) lower (k-tile >= column tile), 2: op(B) upper (k-tile <= column tile)
    int amask, bmask;
    // column statistics of the output (NB = 32, k_bgemm2 only; nullptr: none), one partial per
    // 32-row output tile: csq[(b Mt + ti) ldcs + j] = sum over the tile's rows of D^2, and with
    // qv, csq2 likewise of D[i][j] qv[i qs + b] over rows i < qn (the SVGP conditional's moments)
    double* csq; double* csq2; long ldcs;
    const double* qv; long qs; int qn;
};
void launch_bgemm(int nb, hipStream_t st, int ta, int tb, const BgemmArgs& a, int batch);

// The handle's side stream and fork / join events for the SVGP calls' independent branches (the
// K_uu factorization beside the K_uf Gram; the reverse pass's dE/dm, dE/dLq and K_diag terms beside
// the gA -> Sigma_bar / K_bar -> kernel-derivative chain).  Set by the C-ABI entry points for the
// calling thread; side == nullptr: everything on the caller's stream.
// per-call SVGP settings of the calling thread (svgp_set_side, from the handle at each entry):
// its side stream and fork / join events; qs_packed: q_sqrt / gq_sqrt of the gradient entry as packed
// lower triangles [L][M(M+1)/2] (mfgp_set_svgp_qs_packed)
struct SvgpSide { hipStream_t side; hipEvent_t fork, join; int qs_packed = 0; };
void svgp_set_side(const SvgpSide& sd);
const SvgpSide& svgp_side();

// fork the side stream off s (nothing without a side stream); returns the stream to launch on
hipStream_t svgp_fork(hipStream_t s);
void svgp_join(hipStream_t s);

constexpr int MAXD_HOST = 32;

// fp32 path (mfgp_f32.hip): one tall row-major matrix M, 128 x 128 tiles, ld = Npad; row tiles
// [A = K + s2 I: T][Y^T: Tp][K(X*, X): Ts][I: Ti] (see the file header).
constexpr int F32_TILE = 128;
struct F32Args {
    float* M; long ld;                    // tall matrix, ld = Npad
    int T, Tp, Ts, Ti;                    // row-tile counts of the four regions
    int W;                                // tile columns per outer panel
    float* Dd;                            // T diagonal inverses D_k = L_kk^-1 (128 x 128, upper zero)
    double* ldiag;                        // diag(L), Npad
    int* info;                            // LAPACK-style, zeroed by k32_gram
    const float* X; long ldx; int n;      // inputs [n, D+1]
    const float* Y; long ldy; int p;      // targets [n, p]
    const float* Xs; long ldxs; int ns;   // predict inputs [ns, D+1] (Ts > 0)
    const double* theta; int D;           // constrained theta (fp64, include/mfgp.h layout)
    float* alpha; long ldal;              // K^-1 Y, Npad x Ppad (gradient)
    double* zpart; int nz;                // sum Z^2 partials (nz workgroups)
    double* gpart;                        // [G][T(T+1)/2] gradient partials
    int* cnt;                             // k_reduce_items arrival counter, zeroed by k32_gram
    int upd_slots;                        // lookahead: cap on resident trailing-update workgroups (0: none)
    float* LT;                            // refinement: L^T tiles (L(r,k)^T at tile (k,r), D_k^T at (k,k)), or nullptr
};
// fp64 refinement of the fp32 solve (value-only LML and predict mean, mfgp_set_f32_refine)
struct F32Refine {
    double* A64;                          // alpha (Npad x Ppad, fp64)
    double* R64;                          // R = Y - K alpha (Npad x Ppad, fp64)
    long ld64;                            // = Ppad
    float* XB;                            // work rows (Ppad x Npad, fp32, ld = Npad)
};
size_t f32_gemm_smem();
// Diagnostic timing of the fp32 launches (never on the hot path): events around every launch,
// summed per category after a sync; flops = the tile work each category performed.
enum F32Phase { F32_GRAM = 0, F32_DIAG, F32_PANEL, F32_UPD_IN, F32_UPD_OUT, F32_ALPHA, F32_GRAD, F32_FIN, F32_NPHASE };
struct F32Marks {
    static constexpr int MAXEV = 4096;
    hipEvent_t ev[MAXEV];
    int cat[MAXEV / 2];
    int n = 0;
    double flops[F32_NPHASE] = {};
    int launches[F32_NPHASE] = {};
    void begin(hipStream_t s, int c) {
        if (n + 2 > MAXEV) return;
        (void)hipEventCreate(&ev[n]);
        (void)hipEventCreate(&ev[n + 1]);
        cat[n / 2] = c;
        (void)hipEventRecord(ev[n], s);
    }
    void end(hipStream_t s, double fl) {
        if (n + 2 > MAXEV) return;
        (void)hipEventRecord(ev[n + 1], s);
        flops[cat[n / 2]] += fl;
        launches[cat[n / 2]] += 1;
        n += 2;
    }
    void collect(float* ms) {   // synchronises; ms[F32_NPHASE]
        for (int c = 0; c < F32_NPHASE; ++c) ms[c] = 0.0f;
        if (n) (void)hipEventSynchronize(ev[n - 1]);
        for (int i = 0; i < n; i += 2) {
            float t = 0.0f;
            (void)hipEventElapsedTime(&t, ev[i], ev[i + 1]);
            ms[cat[i / 2]] += t;
        }
        for (int i = 0; i < n; ++i) (void)hipEventDestroy(ev[i]);
        n = 0;
    }
};
void launch_f32_sweep(const F32Args& a, hipStream_t s, F32Marks* mk = nullptr, hipStream_t side = nullptr,
                      hipEvent_t fork = nullptr, hipEvent_t join = nullptr);
void launch_f32_grad(const F32Args& a, hipStream_t s, F32Marks* mk = nullptr);
void launch_f32_zsum(const F32Args& a, hipStream_t s);
void launch_f32_predict(const F32Args& a, float* mean, long ldm, float* var, hipStream_t s);
void launch_f32_predict_cov(const F32Args& a, float* cov, long ldc, hipStream_t s);
void launch_f32_gram_dense(const float* X1, long ldx1, int n1, const float* X2, long ldx2, int n2, int D,
                           const double* theta, float diag_add, float* K, long ldk, hipStream_t s);
void launch_f32_refine_lml(const F32Args& a, const F32Refine& r, hipStream_t s);
void launch_f32_refine_mean(const F32Args& a, const F32Refine& r, float* mean, long ldm, int steps, hipStream_t s);

size_t gram_smem_bytes(int nb);
size_t chol_smem_bytes(int nb);
size_t grad_smem_bytes(int nb, int G, int nil2);
int chol_step_blocks(int T, int Tp, int k, bool alpha = false);
__host__ __device__ int grad_tasks(int T, int chunk);


int flow_nflags(int T, int Tp);
long flow_npub(int T, int Tp);
void launch_chol_flow(const FlowArgs& a, int nwg, hipStream_t s);

// LML layout (padded) or graph kernel: k_gram; dense layout of the linear MF / RBF kernel: k_gram_dense
template <int NB> void launch_gram(const GramArgs& g, int nblocks, int batch, hipStream_t s);
template <int NB> void launch_first_factor(const double* A, long lda, long sA, double* Dd, long sD, double* ldiag,
                                           long sL, int* info, int batch, hipStream_t s);
// dense layout, write extents wr1 x wr2 (>= n1 x n2; the excess is written 0.0)
void launch_gram_dense(const GramArgs& g, int batch, int wr1, int wr2, hipStream_t s);
void launch_flow_prep(const GramArgs& g, int nwg, hipStream_t s);    // set-up launch of k_chol_flow
// one-launch value + gradient (+ Adam) of the AR1 GPR LML for small problems (k_gpr_tiny)
bool gpr_tiny_fits(int n, int p, int d, int nlf);
bool gpr_tiny_pred_fits(int n, int p, int d, int nstar);
void launch_gpr_tiny_pred(const double* X, long ldx, const double* Y, long ldy, const double* Xs, long ldxs, int nstar,
                          const double* theta, int n, int p, int d, double* mean, long ldm, double* var, int* info,
                          hipStream_t s);
void launch_gpr_tiny(const double* X, long ldx, const double* Y, long ldy, const double* theta, int n, int p, int d,
                     int want_grad, int* info, const FinArgs& f, hipStream_t s);
template <int NB> void launch_chol_steps(CholArgs c, int batch, hipStream_t s);
template <int NB> void launch_grad(const GradArgs& g, hipStream_t s);
template <int NB> void launch_pred(const PredAArgs& pa, const PredOutArgs& po, int T, hipStream_t s);

__global__ void k_rhs_init(double* R, long ldr, long sR, int npad, int ppad, const double* Y, long ldy, long sY,
                           int n, int p);
__global__ void k_reduce_items(FinArgs a);
__global__ void k_theta_from_u(const double* u, double* theta, int G, int noise_index);
__global__ void k_kdiag(const double* X, long ldx, int n, int D, const double* theta, double* out, int nlf);
__global__ void k_selftest_mfma(double* out);

}  // namespace mfgp
