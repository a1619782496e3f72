/*
 * mfgp.h — C ABI of the MI355X-native multi-fidelity GP engine (libmfgp.so).
 *
 * This is the drop-in boundary below the Python mirror of the reference's
 * GPflow-facing API.  The reference (qezlou/multi_fidelity_gpflow) is pure
 * Python and has no FFI of its own; each entry point below names the reference
 * interface whose arithmetic it replaces.  The Python side binds it with ctypes
 * (multi_fidelity_gpflow_amd/_lib.py).
 *
 * Conventions
 *   - Every array argument is a caller-owned DEVICE pointer (fp64, row-major,
 *     leading dimensions in elements).  The library never allocates or frees in
 *     a compute call; scratch comes from a caller-provided workspace whose size
 *     is queried with the matching *_workspace_size function.
 *   - theta (device, fp64, constrained values) has the layout
 *         [vL, lL[0..d-1], vD, lD[0..d-1], rho0, noise]      (2d + 4 entries)
 *     i.e. kernel_L (variance, lengthscales), kernel_delta (variance,
 *     lengthscales), rho[0,0] and the Gaussian likelihood variance.
 *   - X rows hold d input columns followed by the fidelity flag (0.0 / 1.0);
 *     rows whose flag is neither exactly 0 nor 1 produce zero kernel rows
 *     (mfgpflow/linear.py:67-70).
 *   - Calls are asynchronous and ordered on the handle's stream (default: the
 *     null stream); none synchronises, so they can be captured in a hipGraph.
 *   - Return value: 0 = ok, < 0 = bad argument / launch error (see
 *     mfgp_error_string).  A Cholesky that meets a non-positive pivot writes a
 *     LAPACK-style info > 0 (1-based row) into the caller's device int; the
 *     Python layer raises the analogue of TF's InvalidArgumentError.
 *   - Threading: a handle must not be used by two host threads at once.
 */
#ifndef MFGP_H_
#define MFGP_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mfgp_handle_s* mfgp_handle_t;

#define MFGP_OK 0
#define MFGP_ERR_ARG (-1)
#define MFGP_ERR_WORKSPACE (-2)
#define MFGP_ERR_LAUNCH (-3)
#define MFGP_ERR_DIM (-4)
/* mfgp_flow_fence / a flow-bearing call found the device's flow fence held by another host thread
 * for longer than the library's bound (10 s): an MFGP_FENCE_WAIT that was never paired with its
 * MFGP_FENCE_RECORD.  Nothing of the failed call was enqueued. */
#define MFGP_ERR_FENCE (-5)
#define MFGP_MAX_D 32
/* info value written when the persistent Cholesky launch gave up waiting (bounded spin) */
#define MFGP_FLOW_TIMEOUT (-100)

int mfgp_version(void);
/* Hash of the sources this library was built from (every file of csrc/ and include/mfgp.h:
 * multi_fidelity_gpflow_amd/build.py source_hash()); "unknown" for a build made without it. */
const char* mfgp_build_id(void);
const char* mfgp_error_string(int code);

/* Handle: device + stream + tile size (32 or 64).  No reference analogue
 * (TensorFlow's implicit device context). */
int mfgp_create(int device, mfgp_handle_t* out);
int mfgp_destroy(mfgp_handle_t h);
int mfgp_set_stream(mfgp_handle_t h, void* hip_stream);
int mfgp_set_tile(mfgp_handle_t h, int nb);
int mfgp_get_tile(mfgp_handle_t h);
/* Cholesky schedule of the LML path (tile 32): 1 = one persistent dataflow launch
 * (k_chol_flow, default when the device reports its CU count) for factorizations of 8 or more
 * 32-tiles (smaller ones are faster as step launches), 3 = the flow at every size, 0 = one launch
 * per tile step.  mfgp_get_flow returns the mode (0, 1 or 3).
 * Results agree to rounding; a workspace must be sized under the setting it is used with. */
int mfgp_set_flow(mfgp_handle_t h, int enable);   /* 2: flow + diagnostic timeline; 3: flow at every size */
/* Small problems (n <= 64, p <= 64, D <= 16, the AR1 kernel, 32-tiles): the LML value + gradient
 * (+ the Adam step of mfgp_gpr_adam_step), and mfgp_gpr_predict for n* <= 64, as ONE launch each
 * instead of the step sequence (default 1: 36 vs 43.5 us at HBS; 0, or MFGP_TINY=0 in the
 * environment: the step sequence).  Same results to rounding. */
int mfgp_set_tiny(mfgp_handle_t h, int enable);
int mfgp_get_tiny(mfgp_handle_t h);
/* Resident workspace (default 0).  On the fp64 flow path (the AR1 kernel, 32-tiles, the persistent
 * Cholesky) the Gram is formed inside the flow launch; the launch in front of it only sets up the
 * workspace (the publication area's sentinel fill, schedule tables, reduction slots), and every
 * value+grad call (mfgp_gpr_lml with want_grad, mfgp_gpr_adam_step) leaves exactly that set-up
 * behind.  With resident = 1 a value+grad call whose workspace the previous fp64 LML call ON THIS
 * HANDLE left set up for the same (n, p, d) skips the set-up launch and starts with the flow.  The
 * caller guarantees that nothing else wrote the workspace in between (a training session's private
 * workspace); graphs captured in this mode replay that way.  Results are identical either way. */
int mfgp_set_resident(mfgp_handle_t h, int enable);
/* k_grad m-tiles per task (fixed at mfgp_create; env MFGP_GRAD_CHUNK).  Workspace sizes depend on it. */
int mfgp_get_grad_chunk(mfgp_handle_t h);
/* fp32 path (dtype MFGP_F32): iterative refinement with an fp64 residual for the value-only LML
 * (want_grad = 0; one step whenever steps >= 1) and the predictive mean (`steps` steps, 0..2;
 * default 2; 0: plain fp32 solve).  The gradient / Adam calls are never refined.  Workspace sizes follow the setting (size after
 * setting it).  Replaces nothing in the reference (it computes in fp64: linear.py:63-64). */
int mfgp_set_f32_refine(mfgp_handle_t h, int steps);
int mfgp_get_flow(mfgp_handle_t h);
/* Bound of every k_chol_flow hand-off wait, in microseconds from the start of that wait
 * (default 50000).  On expiry the launch drains and info = MFGP_FLOW_TIMEOUT: a scheduling
 * failure (not every workgroup resident, e.g. another kernel holding CUs), not a numerical one.
 * 0 makes any wait that polls 8 times give up (diagnostic: exercises the abort path). */
int mfgp_set_flow_timeout_us(mfgp_handle_t h, long long us);
/* Device-wide ordering of the persistent flow (k_chol_flow needs every CU; two flows launched
 * on two streams at once would each stall waiting for workgroups the other keeps off the CUs).
 * The library fences every flow it launches outside a stream capture: the launch waits for the
 * previous flow on the device (any handle, stream or host thread of the process) and becomes the
 * last one.  A captured graph's flows are not fenced at capture: before replaying such a graph
 * call mfgp_flow_fence(h, MFGP_FENCE_WAIT) on the replay stream, and after enqueueing the replay
 * mfgp_flow_fence(h, MFGP_FENCE_RECORD).  Between the two the calling host thread holds the
 * fence: a flow launch or fence call from another host thread blocks on the host until the
 * RECORD (so it cannot land beside the replay's unfenced flows); the holder's own calls pass.
 * Every WAIT MUST be paired with a RECORD from the same host thread (also on error paths).  Holds
 * nest: a thread's nested WAIT / RECORD brackets release the fence only at the outermost RECORD.
 * A thread that finds the fence held by another waits at most 10 s, then the call returns
 * MFGP_ERR_FENCE.  Device ordering is stream-ordered only (no device synchronisation). */
#define MFGP_FENCE_WAIT 0
#define MFGP_FENCE_RECORD 1
int mfgp_flow_fence(mfgp_handle_t h, int op);
/* Where the flow timeline sits inside an mfgp_gpr_* workspace (diagnostic): `count` int64
 * ticks of the 100 MHz device clock from byte `offset`: per step k the diag workgroup's step
 * start [k], A' ready [T+k], factor start [2T+k], D_k published [3T+k], owner hand-offs of
 * A(k,k-2) [4T+k], A(k,k-1) [5T+k], A(k,k) [6T+k] seen, L(k,k-2) formed [7T+k]; then per
 * worker wave w: first item [8T+3w], done [8T+3w+1], ticks spent waiting [8T+3w+2]. */
int mfgp_gpr_flow_trace(mfgp_handle_t h, int n, int p, int d, size_t* offset, int* count);

/* gpflow.kernels.SquaredExponential.K(X1, X2) (GPflow 2.9 stationaries.py via
 * utilities/ops.py:square_distance).  params = [variance, lengthscales[d]]. */
int mfgp_rbf_gram(mfgp_handle_t h, int n1, int n2, int d, const double* X1, int ldx1, const double* X2, int ldx2,
                  const double* params, double* K, int ldk);

/* LinearMultiFidelityKernel.K(X, X2) — mfgpflow/linear.py:55-104.
 * diag_add is added to K[i][i] (use only for X2 == X). */
int mfgp_mf_gram(mfgp_handle_t h, int n1, int n2, int d, const double* X1, int ldx1, const double* X2, int ldx2,
                 const double* theta, double diag_add, double* K, int ldk);

/* LinearMultiFidelityKernel.K_diag(X) — mfgpflow/linear.py:106-136. */
int mfgp_mf_kdiag(mfgp_handle_t h, int n, int d, const double* X, int ldx, const double* theta, double* out);

/* GPR.log_marginal_likelihood() of MultiFidelityGPModel (mfgpflow/linear.py:138-156;
 * GPflow models/gpr.py) and, with want_grad, its gradient w.r.t. theta (the
 * GradientTape of linear.py:205-207).  out[0] = LML, out[1 + q] = dLML/dtheta[q].
 * Y is [n, p]: all p columns share the one Gram / Cholesky (linear.py:90). */
int mfgp_gpr_workspace_size(mfgp_handle_t h, int n, int p, int d, size_t* bytes);
int mfgp_gpr_lml(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y, int ldy,
                 const double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info);

/* One iteration of MultiFidelityGPModel.optimize(use_adam=True) (linear.py:200-214):
 * value+grad at theta, loss_hist[*step] = -LML, Keras-Adam update of the
 * unconstrained vector u for entries with trainable[q] != 0 (entries with equal
 * tie[q] share one variable and its summed gradient; tie may be NULL), theta refreshed
 * (Softplus; Shift(1e-6)+Softplus for the noise entry), ++*step.  lr / beta1 /
 * beta2 are passed already rounded as the caller wants them (TF 2.10 keeps them
 * as float32 hyper variables). */
int mfgp_gpr_adam_step(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y, int ldy,
                       double* theta, double* u, double* m, double* v, const unsigned char* trainable,
                       const int* tie, int* step, double lr, double beta1, double beta2, double eps,
                       double* loss_hist, void* ws, size_t ws_bytes, double* out, int* info);

/* Diagnostic: the mfgp_gpr_lml(want_grad=1) sequence with hipEvents recorded on
 * the handle's stream between its phases; synchronises and writes the elapsed
 * milliseconds of [pre (empty), gram+R init+first factor, tile Cholesky steps (with
 * alpha = L^{-T} Z fused in), gradient, reductions+finalize] into the HOST array ms[5]. */
int mfgp_gpr_lml_phase_times(mfgp_handle_t h, int n, int p, int d, const double* X, int ldx, const double* Y,
                             int ldy, const double* theta, void* ws, size_t ws_bytes, double* out, int* info,
                             float* ms);

/* theta[q] = softplus(u[q]) (+1e-6 for q == noise_index); GPflow positive(). */
int mfgp_theta_from_u(mfgp_handle_t h, const double* u, double* theta, int g, int noise_index);

/* GPR.predict_f(Xnew, full_cov=False) (GPflow models/gpr.py -> base_conditional;
 * mirror at mfgpflow/linear.py:237-286).  mean [nstar, p]; var [nstar] (the
 * reference tiles it over the p outputs). */
int mfgp_gpr_predict_workspace_size(mfgp_handle_t h, int n, int p, int d, int nstar, size_t* bytes);
int mfgp_gpr_predict(mfgp_handle_t h, int n, int p, int d, int nstar, const double* X, int ldx, const double* Y,
                     int ldy, const double* Xs, int ldxs, const double* theta, void* ws, size_t ws_bytes,
                     double* mean, int ldm, double* var, int* info);

/* GPR.predict_f(Xnew, full_cov=True) (GPflow base_conditional full_cov branch: fvar =
 * Knn - A^T A, A = L^{-1} Kmn, the same [nstar, nstar] block for every output; the Python
 * layer tiles it to [p, nstar, nstar]).  nlf = 0: LinearMultiFidelityKernel (theta as
 * mfgp_gpr_*); nlf = m >= 1: GraphMultiFidelityKernel (theta as mfgp_gmf_*, K(X*, X*)
 * carries the kernel's 1e-6 jitter like graph.py:96).  mean / var as mfgp_gpr_predict;
 * cov [nstar][ldc]. */
int mfgp_gpr_predict_cov_workspace_size(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, size_t* bytes);
int mfgp_gpr_predict_cov(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, const double* X, int ldx,
                         const double* Y, int ldy, const double* Xs, int ldxs, const double* theta, void* ws,
                         size_t ws_bytes, double* mean, int ldm, double* var, double* cov, int ldc, int* info);

/* GraphMultiFidelityKernel / GraphMultiFidelityGPModel (mfgpflow/graph.py:7-188) with
 * nlf = m LF sources (fidelity flags 0..m-1 LF, m HF; 1 <= m <= 4).  theta layout
 * (graph_theta_size = (m+1)(d+1) + m + m^2 + 1 entries):
 *   [v_0, l_0(d), .., v_{m-1}, l_{m-1}(d), v_delta, l_delta(d), rho_0..rho_{m-1},
 *    rhoLF[m][m] (row-major; diagonal unused, 1.0), noise]
 * K's LF-LF block (i, j) is rhoLF[i][j] k_i (the ROW source's kernel, graph.py:61-63), so K
 * is not symmetric for rhoLF[i][j] != rhoLF[j][i]; like TF, the factorization reads the
 * lower triangle.  The LML adds the kernel's 1e-6 jitter (graph.py:96) and the noise;
 * mfgp_gmf_gram adds diag_add (pass 1e-6 to mirror K(X)).  The gradient (want_grad) is
 * d LML / d theta over every entry of K, as TF differentiates it. */
int mfgp_gmf_gram(mfgp_handle_t h, int nlf, int n1, int n2, int d, const double* X1, int ldx1, const double* X2,
                  int ldx2, const double* theta, double diag_add, double* K, int ldk);
int mfgp_gmf_kdiag(mfgp_handle_t h, int nlf, int n, int d, const double* X, int ldx, const double* theta,
                   double* out);
int mfgp_gmf_gpr_workspace_size(mfgp_handle_t h, int nlf, int n, int p, int d, size_t* bytes);
int mfgp_gmf_gpr_lml(mfgp_handle_t h, int nlf, int n, int p, int d, const double* X, int ldx, const double* Y,
                     int ldy, const double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info);
int mfgp_gmf_gpr_predict_workspace_size(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, size_t* bytes);
int mfgp_gmf_gpr_predict(mfgp_handle_t h, int nlf, int n, int p, int d, int nstar, const double* X, int ldx,
                         const double* Y, int ldy, const double* Xs, int ldxs, const double* theta, void* ws,
                         size_t ws_bytes, double* mean, int ldm, double* var, int* info);

/* Batched Cholesky factor inverse of SPD matrices (tf.linalg.cholesky +
 * triangular_solve(L, I) as used by GPflow's conditionals): Linv = chol(A)^{-1},
 * ldiag = diag(chol(A)).  A, Linv: [batch][n][n] with strides sA / sL elements. */
int mfgp_potrf_inv_workspace_size(mfgp_handle_t h, int n, int batch, size_t* bytes);
int mfgp_potrf_inv(mfgp_handle_t h, int n, int batch, const double* A, int lda, long sA, void* ws, size_t ws_bytes,
                   double* Linv, int ldl, long sL, double* ldiag, int* info);

/* SVGP ELBO value (GPflow SVGP.elbo, whiten=True, Gaussian likelihood) for the
 * latent LinearCoregionalization model (mfgpflow/linear_svgp.py:64-203) and the
 * SingleBinSVGP (SeparateIndependent, mfgpflow/singlebin_svgp.py:13-97, W = I):
 *   thetas [L][2d+4] per-latent constrained kernel parameters (noise entry unused),
 *   Z [M, d+1], q_mu [M, L], q_sqrt [L, M, M] (lower used), W [P, L] or NULL
 *   (identity mixing; requires L == P).  out = [elbo, KL, VE]; g_mu / g_var
 *   [L][N] receive the latent predictive moments. */
int mfgp_svgp_workspace_size(mfgp_handle_t h, int n, int m, int l, int p, int d, size_t* bytes);
int mfgp_svgp_elbo(mfgp_handle_t h, int n, int m, int l, int p, int d, const double* X, int ldx, const double* Y,
                   int ldy, const double* Z, int ldz, const double* thetas, const double* q_mu,
                   const double* q_sqrt, const double* W, double noise, double scale, double jitter, void* ws,
                   size_t ws_bytes, double* out, double* g_mu, double* g_var, int* info);

/* Gradient of the same objective (the GradientTape of LatentMFCoregionalizationSVGP.optimize,
 * mfgpflow/linear_svgp.py:181-191, and SingleBinSVGP.optimize, singlebin_svgp.py:81-86)
 * E = VE * scale - kl_mult * KL (kl_mult = 1: the ELBO) with respect to the CONSTRAINED
 * parameters: gZ [M][d+1] (fidelity column 0), gtheta [L][2d+4] (noise slot 0),
 * gq_mu [M][L], gq_sqrt [L][M][M] (lower part), gW [P][L] (unused if W == NULL), gnoise [1].
 * noise is a DEVICE pointer (so a training step can be graph-captured).  out / g_mu / g_var
 * as mfgp_svgp_elbo (out[0] is the plain ELBO).  Workspace: mfgp_svgp_grad_workspace_size. */
int mfgp_svgp_grad_workspace_size(mfgp_handle_t h, int n, int m, int l, int p, int d, size_t* bytes);
int mfgp_svgp_elbo_grad(mfgp_handle_t h, int n, int m, int l, int p, int d, const double* X, int ldx,
                        const double* Y, int ldy, const double* Z, int ldz, const double* thetas,
                        const double* q_mu, const double* q_sqrt, const double* W, const double* noise,
                        double scale, double kl_mult, double jitter, void* ws, size_t ws_bytes, double* out, double* g_mu,
                        double* g_var, double* gZ, double* gtheta, double* gq_mu, double* gq_sqrt, double* gW,
                        double* gnoise, int* info);
/* Layout of mfgp_svgp_elbo_grad's q_sqrt (input) and gq_sqrt (output) on this handle: 0 (default)
 * [L][M][M] (lower part used / written, upper zero), 1 packed lower triangles [L][M(M+1)/2], entry
 * (i, j <= i) at i(i+1)/2 + j -- the size of GPflow's unconstrained q_sqrt variable (the
 * FillTriangular bijector's vector; q_sqrt of singlebin_svgp.py:57-62 and GPflow SVGP), so a training
 * state's parameter, gradient and Adam moments hold no upper halves.  Other entry points always
 * take [L][M][M]. */
int mfgp_set_svgp_qs_packed(mfgp_handle_t h, int packed);

/* One Keras-2.10 (legacy) Adam step on a packed parameter vector (the apply_gradients of
 * the SVGP optimize loops, linear_svgp.py:190 / singlebin_svgp.py:86): u unconstrained,
 * c constrained with transform[q] = 0 identity, 1 Softplus, 2 Shift(1e-6) o Softplus, 3 Sigmoid;
 * g = d(+objective)/dc (e.g. the mfgp_svgp_elbo_grad outputs laid out in c's packing);
 * entries with trainable[q] == 0 are left alone; span (may be NULL) ties contiguous entries
 * to one variable (isotropic lengthscales): span[q] = k > 0 for a variable of k entries
 * starting at q (gradient summed, value written to all k), 0 for its followers; learning
 * rate lr_sched[*step] (device array, e.g. the float32 CosineDecay schedule).  Then loss_hist[*step] =
 * -out[0] + (kl_mult - 1) out[1], kl_hist[*step] = out[1] (either may be NULL) and ++*step. */
int mfgp_adam_packed(mfgp_handle_t h, int n, double* u, double* c, const double* g, double* m, double* v,
                     const unsigned char* trainable, const unsigned char* transform, const unsigned char* span,
                     int* step,
                     const double* lr_sched, double beta1, double beta2, double eps, const double* out,
                     double kl_mult, double* loss_hist, double* kl_hist);
/* mfgp_adam_packed gated on the evaluation's info words (info[0..ninfo), e.g. the per-latent
 * Cholesky info of mfgp_svgp_elbo_grad or the info of mfgp_gpr_lml): if any is nonzero the step
 * leaves u / c / m / v and the step counter unchanged (loss_hist[step] still records the loss),
 * like the fused step of mfgp_gpr_adam_step: a session can tell lost steps by the counter. */
int mfgp_adam_packed_ex(mfgp_handle_t h, int n, double* u, double* c, const double* g, double* m, double* v,
                        const unsigned char* trainable, const unsigned char* transform, const unsigned char* span,
                        int* step, const double* lr_sched, double beta1, double beta2, double eps,
                        const double* out, double kl_mult, double* loss_hist, double* kl_hist, const int* info,
                        int ninfo);

/* SVGP.predict_f(Xnew, full_cov, full_output_cov) covariance forms (GPflow base_conditional_with_lm
 * full_cov branch per latent, G_l = Knn_l - A^T A + (Lq^T A)^T Lq^T A, then mix_latent_gp):
 *   mode 1 (full_cov)            f_cov [P][nstar][nstar]     = sum_l W_pl^2 G_l
 *   mode 2 (full_output_cov)     f_cov [nstar][P][P]         = sum_l W_pl W_ql g_var_l
 *   mode 3 (both)                f_cov [nstar][P][nstar][P]  = sum_l W_pl W_ql G_l
 * W == NULL: independent outputs (SeparateIndependent, P == l).  Also writes the diagonal outputs
 * of mfgp_svgp_predict (g_mu, g_var, f_mu, f_var).
 * Workspace: mfgp_svgp_predict_cov_workspace_size(h, nstar, m, l, p, d).
 * Replaces: gpflow SVGP.predict_f(full_cov / full_output_cov) inherited by
 * mfgpflow/linear_svgp.py:64 and singlebin_svgp.py:13. */
int mfgp_svgp_predict_cov_workspace_size(mfgp_handle_t h, int nstar, int m, int l, int p, int d, size_t* bytes);
int mfgp_svgp_predict_cov(mfgp_handle_t h, int mode, int nstar, int m, int l, int p, int d, const double* Xs,
                          int ldxs, const double* Z, int ldz, const double* thetas, const double* q_mu,
                          const double* q_sqrt, const double* W, double jitter, void* ws, size_t ws_bytes,
                          double* g_mu, double* g_var, double* f_mu, double* f_var, double* f_cov, int* info);

/* SVGP.predict_f(Xnew, full_cov=False) of the same models (GPflow posteriors with
 * mix_latent_gp): latent moments g_mu / g_var [L][nstar] and mixed f_mu / f_var
 * [nstar][P].  Workspace: mfgp_svgp_workspace_size(h, nstar, m, l, p, d). */
int mfgp_svgp_predict(mfgp_handle_t h, int nstar, int m, int l, int p, int d, const double* Xs, int ldxs,
                      const double* Z, int ldz, const double* thetas, const double* q_mu, const double* q_sqrt,
                      const double* W, double jitter, void* ws, size_t ws_bytes, double* g_mu, double* g_var,
                      double* f_mu, double* f_var, int* info);

/* Diagnostic: one v_mfma_f64_16x16x4_f64 with A[i][k] = 4i+k+1, B[k][j] = 100k+j;
 * writes C (16x16 row-major, device). */
int mfgp_selftest_mfma(mfgp_handle_t h, double* out);

/* ---- dtype-generic forms (mfgp_mf_gram(h, dtype, ...)).
 * dtype MFGP_F64: X / Y / K / mean / var are double and the call is exactly the fp64 entry point
 * of the same name without "_ex".  dtype MFGP_F32: those arrays are float (device, row-major);
 * theta, out and the Adam state stay double.  The fp32 path is the BASELINE "Synth" config's
 * (N_L = 16384, N_H = 2048, D = 10, P = 512): the reference forces fp64 (linear.py:63-64), so
 * its semantics are the fp64 ones computed in fp32 -- r^2 in direct-difference form (not
 * GPflow's expanded form, which cancels in fp32), every GEMM on v_mfma_f32_32x32x2_f32, the
 * LML / gradient reductions in fp64.  Tolerances against the fp64 oracle: DESIGN.md §8. */
#define MFGP_F64 0
#define MFGP_F32 1
/* fp32 path: 128-wide tile columns per outer Cholesky panel (default 6; env MFGP_F32_PANEL). */
int mfgp_set_f32_panel(mfgp_handle_t h, int tiles);
/* fp32 path: 1 (default; env MFGP_F32_LOOKAHEAD) factors the next panel on a high-priority side
 * stream beside the trailing update (fork / join events, graph-capturable); 0: one stream. */
int mfgp_set_f32_lookahead(mfgp_handle_t h, int enable);
/* fp32 lookahead: CUs the trailing update leaves free for the side stream (default 32; env
 * MFGP_F32_RESERVE; 0: uncapped grid).  Speed only: results do not depend on it. */
int mfgp_set_f32_reserve(mfgp_handle_t h, int cus);
/* LinearMultiFidelityKernel.K (linear.py:55-104), as mfgp_mf_gram. */
int mfgp_mf_gram_ex(mfgp_handle_t h, int dtype, int n1, int n2, int d, const void* X1, int ldx1, const void* X2,
                    int ldx2, const double* theta, double diag_add, void* K, int ldk);
/* GPR.log_marginal_likelihood (+ gradient), as mfgp_gpr_workspace_size / mfgp_gpr_lml. */
int mfgp_gpr_workspace_size_ex(mfgp_handle_t h, int dtype, int n, int p, int d, size_t* bytes);
int mfgp_gpr_lml_ex(mfgp_handle_t h, int dtype, int n, int p, int d, const void* X, int ldx, const void* Y, int ldy,
                    const double* theta, int want_grad, void* ws, size_t ws_bytes, double* out, int* info);
/* One optimize(use_adam=True) iteration (linear.py:200-214), as mfgp_gpr_adam_step. */
int mfgp_gpr_adam_step_ex(mfgp_handle_t h, int dtype, int n, int p, int d, const void* X, int ldx, const void* Y,
                          int ldy, double* theta, double* u, double* m, double* v, const unsigned char* trainable,
                          const int* tie, int* step, double lr, double beta1, double beta2, double eps,
                          double* loss_hist, void* ws, size_t ws_bytes, double* out, int* info);
/* GPR.predict_f(full_cov=False) (linear.py:237-286), as mfgp_gpr_predict; mean / var in dtype. */
int mfgp_gpr_predict_workspace_size_ex(mfgp_handle_t h, int dtype, int n, int p, int d, int nstar, size_t* bytes);
int mfgp_gpr_predict_ex(mfgp_handle_t h, int dtype, int n, int p, int d, int nstar, const void* X, int ldx,
                        const void* Y, int ldy, const void* Xs, int ldxs, const double* theta, void* ws,
                        size_t ws_bytes, void* mean, int ldm, void* var, int* info);
/* predict_f(full_cov=True) in either dtype: mfgp_gpr_predict_cov for MFGP_F64 (any nlf);
 * MFGP_F32 (nlf = 0): cov [nstar x nstar] (ldc) = K(X*, X*) - A^T A computed in fp32 from the
 * same factor sweep as mfgp_gpr_predict_ex.  Workspace: mfgp_gpr_predict_cov_workspace_size_ex. */
int mfgp_gpr_predict_cov_workspace_size_ex(mfgp_handle_t h, int dtype, int nlf, int n, int p, int d, int nstar,
                                           size_t* bytes);
int mfgp_gpr_predict_cov_ex(mfgp_handle_t h, int dtype, int nlf, int n, int p, int d, int nstar, const void* X,
                            int ldx, const void* Y, int ldy, const void* Xs, int ldxs, const double* theta, void* ws,
                            size_t ws_bytes, void* mean, int ldm, void* var, void* cov, int ldc, int* info);
/* Diagnostic: one LML value+grad evaluation with hipEvents around its launches; synchronises.
 * Per phase (HOST arrays of nphase entries): ms, flops performed (fp32 only) and launch count.
 * fp32 phases: [gram, diag factors, panels, in-panel updates, trailing updates, alpha, gradient,
 * reductions]; fp64: mfgp_gpr_lml_phase_times' five phases. */
int mfgp_gpr_phase_times_ex(mfgp_handle_t h, int dtype, int n, int p, int d, const void* X, int ldx, const void* Y,
                            int ldy, const double* theta, void* ws, size_t ws_bytes, double* out, int* info,
                            float* ms, double* flops, int* launches, int nphase);

#ifdef __cplusplus
}
#endif
#endif /* MFGP_H_ */
