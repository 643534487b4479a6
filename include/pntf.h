/* pntf.h — C ABI of libpntf.so, the MI355X (gfx950) hot path of P-NTFields.
 *
 * The reference (yhsong0804/P-NTFields) has no FFI: its hot path is the Python methods of
 * `NN` / `Model` in models/model_res_sigmoid_multi.py and models/model_res_sigmoid.py.
 * Each entry point below replaces one of those methods; the Python drop-in modules under
 * p-ntfields_amd/models/ bind them with ctypes.
 *
 * Conventions (all entry points):
 *   - every array argument is a caller-owned DEVICE pointer (HIP memory on the current
 *     device), fp32 row-major unless stated, int32 for ids/counts;
 *   - calls are stream-ordered and asynchronous on `stream` (NULL = legacy default);
 *   - no internal threads, no allocation: scratch is the caller's `ws` of `ws_bytes`
 *     (query with pntf_workspace_bytes); a smaller ws lowers the grid, never fails
 *     unless it holds less than one workgroup's slots;
 *   - return PNTF_OK (0) or a positive pntf_status; no exceptions cross the ABI;
 *   - thread-compatible, not thread-safe (pntf_last_error is per thread).
 *
 * Shapes: n pairs `xp` (n, 2*dim) = [x_start | x_goal]; `Btab` (n_env, dim, 128) per-env
 * Fourier matrices B (the multi model's B.npy (3,128); the arm model's B^T);
 * `env` (n) int32 env id per pair or NULL (all env 0).  dim is 3 or 6.
 */
#ifndef PNTF_H_
#define PNTF_H_

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNTF_ABI_VERSION 1

typedef enum {
  PNTF_OK = 0,
  PNTF_ERR_ARG = 1,         /* bad shape / null pointer / unsupported dim */
  PNTF_ERR_WORKSPACE = 2,   /* ws too small for a single workgroup */
  PNTF_ERR_HIP = 3          /* HIP launch / runtime error (see pntf_last_error) */
} pntf_status;

/* Gradient flavours for the reverse sweep. */
#define PNTF_GRAD_EXACT 0            /* == Model.gradient(NN.out) autograd (:890-896)     */
#define PNTF_GRAD_BACKGRAD_COMPAT 1  /* == NN.out_backgrad incl. its encoder[0] quirk     */
                                     /*    (model_res_sigmoid_multi.py:402-647, :435-438) */

/* Kernel schedules (pntf_field_ex, pntf_plan_ex, pntf_set_field_schedule):
 *   WAVE_TILE   one wave per 16-pair tile, v_mfma_f32_16x16x4_f32 (pntf_field.h);
 *   SPLIT_TILE  the 4 waves of a workgroup share a 16-pair tile (pntf_split.h; latency);
 *   WIDE_TILE   one wave per 32-pair tile, v_mfma_f32_32x32x2_f32 (pntf_wide.h; throughput,
 *               field entry points only — the planner treats it as WAVE_TILE);
 *   QUAD_TILE   the 4 waves of a workgroup share a 4-pair tile, v_mfma_f32_4x4x1_16b_f32
 *               (pntf_quad.h; lowest latency per planner step, no workspace needed);
 *   AUTO        quad while ceil(n/4) <= the CU count, split while ceil(n/16) <= 2 x the CU
 *               count, wide above.  For the planner AUTO's quad path also runs batches of at
 *               most one query per CU (q <= CUs, the reference's Q = 1 included) one query per
 *               workgroup on VALU layers (SOLO), and larger quad batches hand their last
 *               <= CUs active queries off to a SOLO launch (tail hand-off; needs 8 + 8q bytes
 *               of `ws`).  SOLO and the MFMA layers give bit-identical results.  Environment
 *               PNTF_QSOLO=0 (read once) disables both. */
#define PNTF_SCHED_AUTO 0
#define PNTF_SCHED_WAVE_TILE 1
#define PNTF_SCHED_SPLIT_TILE 2
#define PNTF_SCHED_WIDE_TILE 3
#define PNTF_SCHED_QUAD_TILE 4

int pntf_abi_version(void);
const char* pntf_status_string(int status);
const char* pntf_last_error(void);

/* Number of floats of the packed weight blob. */
size_t pntf_packed_floats(void);

/* Pack the 30 state-dict tensors (device pointers, reference state-dict order:
 * encoder.{0..3}, encoder1.{0..2}, generator.{0..4}, generator1.{0..2}, each .weight then
 * .bias — NN.__init__, model_res_sigmoid_multi.py:155-175) into `packed`
 * (pntf_packed_floats() floats).  encoder1.0 is ignored (never used by NN.out, :227). */
int pntf_pack_weights(const float* const* params, int n_params, float* packed,
                      hipStream_t stream);

/* Handle form of the same: pntf_net_create allocates the packed weights
 * (hipMalloc) and packs `params` as pntf_pack_weights does; every entry point below takes
 * pntf_net_packed(net) as its `packed` argument.  pntf_net_update repacks after a weight
 * change (Model.load / an optimizer step, models/model_res_sigmoid_multi.py:1154-1166);
 * pntf_net_destroy frees the buffer (hipFree: call it once the stream's work that reads it
 * is done).  pntf_net_create returns NULL on error (pntf_last_error). */
typedef struct pntf_net pntf_net;
pntf_net* pntf_net_create(const float* const* params, int n_params, hipStream_t stream);
int pntf_net_update(pntf_net* net, const float* const* params, int n_params,
                    hipStream_t stream);
const float* pntf_net_packed(const pntf_net* net);
void pntf_net_destroy(pntf_net* net);

/* DEFAULT kernel schedule of pntf_tau / _tau_grad / _path_velocity / _speed / _travel_time
 * (PNTF_SCHED_*, see pntf_plan_ex; AUTO unless changed).  Process-wide, so not thread-safe
 * against concurrent calls: callers that need a specific schedule pass it per call through
 * pntf_field_ex instead.  Results agree between schedules to fp32 rounding. */
int pntf_set_field_schedule(int schedule);

/* Build identity: "unit=hash;..." — one sha256 prefix per kernel translation unit (its
 * source, the shared headers, defines and flags; p-ntfields_amd/pntf/build.py:unit_ids).
 * Profiles under profiles/ record the hash of the unit they measured. */
const char* pntf_build_info(void);

/* The kernel family (PNTF_SCHED_QUAD/SPLIT/WIDE/WAVE_TILE) a field entry point runs for n
 * pairs when asked for `schedule`; -1 for a negative n or an unknown schedule.  Host-only
 * (no device work; the CU count comes from the current device, 256 without one).  Batches of
 * more than 2^31 - 32 pairs never run WIDE_TILE (its 32-bit tile index): they fall back to
 * WAVE_TILE. */
int pntf_field_schedule_for(int64_t n, int schedule);

/* Device scratch needed by the gradient/planner entry points for n pairs. */
size_t pntf_workspace_bytes(int64_t n);

/* τ only: NN.out / Model.Tau (model_res_sigmoid_multi.py:215-259, :1188-1193). tau (n). */
int pntf_tau(const float* packed, int dim, const float* xp, int64_t n, const float* Btab,
             const int32_t* env, int32_t n_env, float* tau, hipStream_t stream);

/* τ and ∇τ: NN.out + Model.gradient (mode EXACT), NN.out_grad (same values) or
 * NN.out_backgrad (mode BACKGRAD_COMPAT).  tau (n), dtau (n, 2*dim). */
int pntf_tau_grad(const float* packed, int dim, const float* xp, int64_t n,
                  const float* Btab, const int32_t* env, int32_t n_env, int mode,
                  float* tau, float* dtau, void* ws, size_t ws_bytes, hipStream_t stream);

/* Path velocity: Model.Gradient (model_res_sigmoid_multi.py:1218-1248; per-row norms).
 * vel (n, 2*dim) = [v_start | v_goal]; tau (n) optional (may be NULL). */
int pntf_path_velocity(const float* packed, int dim, const float* xp, int64_t n,
                       const float* Btab, const int32_t* env, int32_t n_env, int mode,
                       float* vel, float* tau, void* ws, size_t ws_bytes,
                       hipStream_t stream);

/* Speed at the goal: Model.Speed (model_res_sigmoid_multi.py:1195-1216). speed (n). */
int pntf_speed(const float* packed, int dim, const float* xp, int64_t n, const float* Btab,
               const int32_t* env, int32_t n_env, float* speed, void* ws, size_t ws_bytes,
               hipStream_t stream);

/* Travel time: Model.TravelTimes (model_res_sigmoid_multi.py:1173-1186). tt (n). */
int pntf_travel_time(const float* packed, int dim, const float* xp, int64_t n,
                     const float* Btab, const int32_t* env, int32_t n_env, float* tt,
                     hipStream_t stream);

/* Field kinds of pntf_field_ex (the entry points above, in this order). */
#define PNTF_FIELD_TAU 0          /* pntf_tau:           out0 = tau (n)                     */
#define PNTF_FIELD_TAU_GRAD 1     /* pntf_tau_grad:      out0 = tau (n), out1 = dtau        */
#define PNTF_FIELD_VELOCITY 2     /* pntf_path_velocity: out0 = vel, out1 = tau (optional)  */
#define PNTF_FIELD_SPEED 3        /* pntf_speed:         out0 = speed (n)                   */
#define PNTF_FIELD_TRAVEL 4       /* pntf_travel_time:   out0 = tt (n)                      */

/* Any of the five field entry points above with an explicit per-call schedule
 * (PNTF_SCHED_*); `mode` is ignored by TAU/SPEED/TRAVEL, `ws` by TAU/TRAVEL. */
int pntf_field_ex(int kind, const float* packed, int dim, const float* xp, int64_t n,
                  const float* Btab, const int32_t* env, int32_t n_env, int mode, float* out0,
                  float* out1, void* ws, size_t ws_bytes, int schedule, hipStream_t stream);

/* Batched bidirectional planner = q independent copies of test/gib_plan.py:74-86
 * (Gibson: step 0.03, tol 0.06, max_iter 500, mode BACKGRAD_COMPAT) or
 * test/arm_plan.py:140-152 (arm: step 0.015, tol 0.03, max_iter 300, mode EXACT).
 * A query freezes once |x_goal - x_start| <= tol; the loop body runs at most
 * max_iter + 1 times.  path (q, max_iter + 2, 2*dim): row 0 = start, frozen rows repeat
 * the final state; steps (q) = number of updates taken (-1 for an invalid env id). */
int pntf_plan(const float* packed, int dim, const float* xp0, int64_t q, const float* Btab,
              const int32_t* env, int32_t n_env, int mode, float step, float tol,
              int32_t max_iter, float* path, int32_t* steps, void* ws, size_t ws_bytes,
              hipStream_t stream);

/* pntf_plan with an explicit schedule (pntf_plan uses PNTF_SCHED_AUTO):
 *   PNTF_SCHED_WAVE_TILE   one wave per 16-query tile (throughput: many queries; WIDE_TILE
 *                          is treated as WAVE_TILE);
 *   PNTF_SCHED_SPLIT_TILE  the 4 waves of a workgroup share a tile, each computing a quarter
 *                          of every layer's outputs;
 *   PNTF_SCHED_QUAD_TILE   the 4 waves of a workgroup share a 4-query tile (no workspace);
 *   PNTF_SCHED_AUTO        quad while ceil(q/4) <= the CU count — q <= CUs on the SOLO VALU
 *                          layers, larger batches with the tail hand-off when ws holds
 *                          8 + 8q bytes — split while ceil(q/16) <= 2 x the CU count, wave above.
 * Results agree between schedules to fp32 rounding (the cross-wave sums are reordered);
 * SOLO and the quad MFMA layers agree bit for bit.  WAVE/SPLIT need `ws`
 * (pntf_workspace_bytes(q)). */
int pntf_plan_ex(const float* packed, int dim, const float* xp0, int64_t q, const float* Btab,
                 const int32_t* env, int32_t n_env, int mode, float step, float tol,
                 int32_t max_iter, float* path, int32_t* steps, void* ws, size_t ws_bytes,
                 int schedule, hipStream_t stream);

/* Eikonal residual: NN.out_laplace + the per-pair residual of Model.Loss
 * (model_res_sigmoid_multi.py:710-848, :897-946), Taylor mode.  Each output may be NULL:
 * tau (n), dtau (n, 2*dim), ltau (n, 2*dim) diagonal second derivatives, diff (n) the
 * residual loss0 + loss1 - 4 for observed speeds yobs (n, 2) (required when diff != NULL)
 * and viscosity weight gamma (0.001 in the reference training, :1015). */
int pntf_eikonal_residual(const float* packed, int dim, const float* xp, const float* yobs,
                          int64_t n, const float* Btab, const int32_t* env, int32_t n_env,
                          float gamma, float* tau, float* dtau, float* ltau, float* diff,
                          void* ws, size_t ws_bytes, hipStream_t stream);

/* Deterministic fp64 sum of x (n) into *out (device pointer to one double). */
int pntf_sum(const float* x, int64_t n, double* out, hipStream_t stream);

/* ---------------------------------------------------------------------------------------
 * Training step: what `loss.backward(); optimizer.step()` computes in
 * Model.train (model_res_sigmoid_multi.py:1040-1052; arm models/model_res_sigmoid.py:
 * 1062-1075).  The host (p-ntfields_amd/pntf/train.py) runs the Taylor-mode graph of
 * NN.out_laplace (:710-848) layer by layer: each Linear is one plain fp32 library GEMM over
 * all Taylor rows, everything in between is one of the fused kernels below.
 *
 * "Planes": a Taylor tensor of m points and width w is (R, m, w) fp32 with R = 1 + ndir + nl
 * planes [value | ndir first-derivative rows | nl summed second-derivative rows]: (ndir, nl) =
 * (dim, 1) in the encoder (m = 2n points: the n starts, then the n goals) and (2*dim, 2) after
 * the start/goal merge ([d/dx_start (dim) | d/dx_goal (dim) | Σ d²/dx_start² | Σ d²/dx_goal²],
 * m = n pairs).  The loss needs each endpoint's Laplacian only (Model.Loss :919-920), and the
 * per-direction second-derivative rows of NN.out_laplace enter every layer linearly, so their
 * per-endpoint sum is carried instead of one row per direction (same loss and gradient).
 * `partial` is caller scratch of pntf_tt_partial_floats() floats (per stream).
 * Errors of these entry points are reported by pntf_tt_last_error.
 * ------------------------------------------------------------------------------------- */
size_t pntf_tt_partial_floats(void);
const char* pntf_tt_last_error(void);

/* input_mapping_laplace (:199-213): phi (2 + dim, 2n, 256) = [sin | cos] rows of 2πxB. */
int pntf_tt_fourier(int dim, const float* xp, int64_t n, const float* Btab, const int32_t* env,
                    int32_t n_env, float* phi, hipStream_t stream);

/* Bias (+ residual) + act_laplace (:663-691, residual :744/:828) on GEMM output y (R, m, w),
 * w = 128|256, (ndir, nl) = (3|6, 1), (6|12, 2) (summed second derivatives), (0, 0) (value
 * plane only), (3|6|12, 0) (first derivatives only) or (3, 3), (6, 6), (12, 12) (one
 * second-derivative row per direction; the general VJP tape below): y's value plane += bias,
 * every plane += res (R, m, w) when res is not NULL (y is kept as the tape); act == 1: h (R, m,
 * w) = softplus10 Taylor rows; act == 2 (nl == 0, ndir 3|6, encoder[0] of NN.out_backgrad):
 * the derivative rows are multiplied by σ(10·softplus(y)) instead of σ(10y), the reference's
 * quirk (:435-438).  act == 0 (Linear without activation, res must be NULL): bias only, h
 * unused. */
int pntf_tt_act_fwd(int ndir, int nl, float* y, float* h, const float* bias, const float* res,
                    int64_t m, int w, int act, hipStream_t stream);

/* Adjoint of pntf_tt_act_fwd, in place: g (R, m, w) holds dL/dh on entry and dL/dy on exit
 * (act == 0: unchanged); gbias (w) (+)= sum over points of dL/dy's value plane
 * (accumulate != 0 adds to gbias). */
int pntf_tt_act_bwd(int ndir, int nl, const float* y, float* g, int64_t m, int w, int act,
                    float* gbias, int accumulate, float* partial, hipStream_t stream);

/* Start/goal merge of the encoder output (:755-811): z (2 + dim, 2n, 128) ->
 * u (3 + 2*dim, n, 256), features [logsumexp max-part | min-part]; and its adjoint
 * gu (3 + 2*dim, n, 256) -> gz (2 + dim, 2n, 128). */
int pntf_tt_merge_fwd(int dim, const float* z, int64_t n, float* u, hipStream_t stream);
int pntf_tt_merge_bwd(int dim, const float* z, const float* gu, int64_t n, float* gz,
                      hipStream_t stream);

/* ---- General VJP tape (round 5): the backward of a loss a user writes on NN.out_laplace's
 * (τ, ∇τ, diagonal ∇²τ) (:710-848), NN.out_grad's / out_backgrad's (τ, ∇τ) (:303-400,
 * :402-647) or Model.gradient's ∇τ with create_graph (:890-896), w.r.t. every weight and the
 * coordinates — what the reference's autograd computes through those plain torch graphs.
 * Encoder planes (ndir, nl) = (0, 0), (dim, 0), (dim, 1) or (dim, dim); nle = the encoder's nl
 * (0, 1 = per-endpoint sums, dim = per direction); after the merge (2·ndir, 2·nle). */
/* input_mapping / _grad / _laplace (:186-213): phi (1 + ndir + nl, 2n, 256). */
int pntf_tt_fourier_ex(int dim, int ndir, int nl, const float* xp, int64_t n, const float* Btab,
                       const int32_t* env, int32_t n_env, float* phi, hipStream_t stream);
/* Its adjoint, the coordinates' gradient: gphi (1 + ndir + nl, 2n, 256) = dL/dphi ->
 * gx (n, 2*dim) = dL/dxp (written). */
int pntf_tt_fourier_bwd(int dim, int ndir, int nl, const float* gphi, const float* xp, int64_t n,
                        const float* Btab, const int32_t* env, int32_t n_env, float* gx,
                        hipStream_t stream);
/* Start/goal merge (:755-811) for nle second-derivative rows per endpoint: z (1 + dim + nle,
 * 2n, 128) -> u (1 + 2 dim + 2 nle, n, 256); and its adjoint gu -> gz. */
int pntf_tt_merge_fwd_ex(int dim, int nle, const float* z, int64_t n, float* u,
                         hipStream_t stream);
int pntf_tt_merge_bwd_ex(int dim, int nle, const float* z, const float* gu, int64_t n, float* gz,
                         hipStream_t stream);
/* generator[4] + actout_laplace (:693-708) with a general upstream gradient: v (1 + 2 dim +
 * 2 nle, n, 128) generator[3] output planes -> (each optional) tau (n), dtau (n, 2 dim), lap
 * (n, 2 nle) (per direction for nle == dim, per-endpoint Laplacian for nle == 1); with the
 * upstream gtau (n), gdtau (n, 2 dim), glap (n, 2 nle) (NULL = zero): gv (same shape as v),
 * gw4 (128), gb4 (1) of Σ gtau·τ + gdtau·∇τ + glap·lap. */
int pntf_tt_head_vjp(int dim, int nle, const float* v, const float* w4, const float* b4,
                     int64_t n, const float* gtau, const float* gdtau, const float* glap,
                     float* tau, float* dtau, float* lap, float* gv, float* gw4, float* gb4,
                     float* partial, hipStream_t stream);

/* ---- First-order (value-plane) tape: the weight gradient of a loss on NN.out's τ
 * (models/model_res_sigmoid_multi.py:215-259, arm models/model_res_sigmoid.py:212-256: plain
 * nn.Linear + autograd in the reference, so `net.out(x, B)[0].sum().backward()` fills every
 * parameter's .grad).  The planes are R = 1 (value only, (ndir, nl) = (0, 0) in
 * pntf_tt_act_fwd / pntf_tt_act_bwd / pntf_tt_linear_act); the GEMMs are pntf_tt_gemm's. */
/* input_mapping (:186-190): phi (1, 2n, 256) = [sin | cos] of 2πxB (value plane of
 * pntf_tt_fourier). */
int pntf_tt_fourier_value(int dim, const float* xp, int64_t n, const float* Btab,
                          const int32_t* env, int32_t n_env, float* phi, hipStream_t stream);
/* Start/goal merge (:236-244) of the value plane: z (2n, 128) -> u (n, 256); adjoint
 * (:620-627) gu (n, 256) -> gz (2n, 128). */
int pntf_tt_merge_value_fwd(const float* z, int64_t n, float* u, hipStream_t stream);
int pntf_tt_merge_value_bwd(const float* z, const float* gu, int64_t n, float* gz,
                            hipStream_t stream);
/* Head (:254-255): tau (n) = σ(0.1 (v·w4 + b4)) from generator[3]'s output v (n, 128) when tau
 * is not NULL; with gtau (n) = dL/dτ (not NULL): gv (n, 128) = dL/dv, gw4 (128), gb4 (1). */
int pntf_tt_head_tau(const float* v, const float* w4, const float* b4, int64_t n,
                     const float* gtau, float* tau, float* gv, float* gw4, float* gb4,
                     float* partial, hipStream_t stream);

/* generator[4] + actout_laplace (:693-708) + Model.Loss (:897-946; arm = 1: the arm model's
 * square-root variant, models/model_res_sigmoid.py:869-935), forward and backward per pair:
 * v (3 + 2*dim, n, 128) generator[3] output planes, w4 (128), b4 (1) -> diff (n); the
 * gradient of scale * sum(diff): gv (3 + 2*dim, n, 128) w.r.t. v, gw4 (128), gb4 (1). */
int pntf_tt_head_loss(int dim, int arm, const float* v, const float* w4, const float* b4,
                      const float* xp, const float* yobs, int64_t n, float gamma, float scale,
                      float* diff, float* gv, float* gw4, float* gb4, float* partial,
                      hipStream_t stream);

/* fp32 GEMM of the training step on hand-written MFMA kernels (pntf_gemm.hip; the Linear
 * layers of the Taylor tape: forward X·Wᵀ, input gradient gY·W, weight gradient gYᵀ·X):
 * C (M x N, row stride ldc) = beta*C + A·B with A(m,k) = ta ? A[k*lda + m] : A[m*lda + k] and
 * B(k,n) = tb ? B[n*ldb + k] : B[k*ldb + n].  N must be a multiple of 128.  Long K is split
 * over workgroups (deterministic partial sums in `work`, pntf_tt_gemm_work_floats(M, N, K)
 * floats; may be NULL when that is 0).  beta == 0 never reads C.  With ta == 0, K and N in
 * {128, 256}, dense rows (lda == K, ldc == N), beta 0 or 1 and 16-byte aligned A, C and work,
 * a panel kernel runs: it packs op(B) into `work` (pntf_tt_gemm_work_floats includes it) and
 * keeps it in LDS; otherwise the LDS-tiled kernel.  Panel kernels (PNTF_GEMM_PANEL in the
 * environment, read once, or pntf_tt_set_panel_mode): 0 = none, 1 = fp32 MFMA with the
 * weight streamed from L2, 2 = fp32 MFMA with the weight in LDS, 3 (default) = the split-bf16
 * kernel (every fp32 operand as three bf16 terms, six bf16 MFMA products per fp32 product:
 * fp32 accuracy at 2.67x the fp32 MFMA rate; 1.5*K*N work floats), 8 = its 16x16x32 variant
 * with two waves per SIMD (diagnostic; 4..7 are diagnostic forms of 3 as well). */
size_t pntf_tt_gemm_work_floats(int64_t M, int64_t N, int64_t K);
int pntf_tt_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                 const float* B, int64_t ldb, float* C, int64_t ldc, float beta, float* work,
                 size_t work_floats, hipStream_t stream);
const char* pntf_tt_gemm_last_error(void);
/* Process-wide panel-kernel choice (see pntf_tt_gemm; not thread-safe against concurrent
 * GEMMs); returns the previous mode, leaves it unchanged for a mode outside 0..8. */
int pntf_tt_set_panel_mode(int mode);
/* The same for the weight-gradient shapes (ta, not tb, beta 0, M and N in {128, 256};
 * PNTF_GEMM_WGRAD in the environment): 0 = the LDS-tiled kernel, 1 = the fp32-MFMA wgrad
 * kernel, 2 (default) = the split-bf16 one; returns the previous mode. */
int pntf_tt_set_wgrad_mode(int mode);
/* The kernel of pntf_tt_linear_bwd (PNTF_GEMM_BWD in the environment): 0 = fp32 MFMA, 1
 * (default) = split bf16 (the x6 GEMM of pntf_tt_gemm with the act adjoint as its epilogue);
 * returns the previous mode, leaves it unchanged for a mode outside 0..1. */
int pntf_tt_set_bwd_mode(int mode);

/* One Linear of the Taylor tape with its bias, residual and act_laplace fused (the forward
 * GEMM of pntf_tt_gemm followed by pntf_tt_act_fwd, in one kernel; :663-691, :744/:828):
 * x (R, m, k) planes, W (n, k) the torch weight (y = x·Wᵀ), bias (n), res (R, m, n) or NULL
 * -> y (R, m, n) pre-activation (value plane + bias, every plane + res; kept as the tape) and,
 * when act != 0, h (R, m, n) the softplus10 Taylor rows.  R = 1 + ndir + nl with (ndir, nl) =
 * (3|6, 1), (6|12, 2) or (0, 0); k, n in {128, 256}; all pointers 16-byte aligned; `work` holds the
 * packed weight (pntf_tt_gemm_work_floats(R*m, n, k) floats).  act == 0 requires res == NULL
 * (h unused).  schedule: 0 = AUTO (the two kernels while the split-bf16 panel GEMM is
 * selected, the default; with the fp32-MFMA panel modes the fused kernel when every wave gets
 * >= 3 rounds of 32-point blocks that balance to >= 90 %),
 * 1 = always the fused kernel (one wave per 32-point block), 2 = always pntf_tt_gemm +
 * pntf_tt_act_fwd, 3 = the fused kernel with the four waves of a workgroup sharing a block;
 * errors of either path are reported by pntf_tt_gemm_last_error / pntf_tt_last_error. */
int pntf_tt_linear_act(int ndir, int nl, const float* x, int64_t m, int k, const float* W,
                       int n, const float* bias, const float* res, float* y, float* h, int act,
                       int schedule, float* work, size_t work_floats, hipStream_t stream);

/* The reverse of the same pair: the input gradient of one Linear with the previous layer's
 * act_laplace adjoint (pntf_tt_act_bwd with act = 1) as its epilogue, in one kernel:
 * gy (R, m, kc) the Linear's output-gradient planes, W (kc, nc) its torch weight, yprev (R, m,
 * nc) the previous layer's pre-activation planes (its tape), res (R, m, nc) the residual
 * branch's gradient or NULL -> out (R, m, nc) = the previous layer's dL/dy planes, i.e.
 * act_bwd(gy·W + res), and gbias (nc) = their value plane summed over points (written, not
 * accumulated).  out may alias res.  kc, nc in {128, 256}; (ndir, nl) as pntf_tt_act_fwd;
 * 16-byte aligned pointers; `work` of pntf_tt_linear_bwd_work_floats(kc, nc) floats.  Errors
 * via pntf_tt_gemm_last_error. */
size_t pntf_tt_linear_bwd_work_floats(int kc, int nc);
int pntf_tt_linear_bwd(int ndir, int nl, const float* gy, int64_t m, int kc, const float* W,
                       int nc, const float* yprev, const float* res, float* out, float* gbias,
                       float* work, size_t work_floats, hipStream_t stream);

/* torch.optim.AdamW update of one parameter tensor (the reference's optimizer, :959-961):
 * p, grad, exp_avg, exp_avg_sq (n); `step` = the step count after this update (>= 1). */
int pntf_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
               float beta2, float eps, float weight_decay, int64_t step, hipStream_t stream);
/* The same update for `count` (<= 64) tensors sharing lr, betas, eps, weight decay and step
 * (torch.optim.AdamW's per-parameter loop over one param group, :959-961) in one launch:
 * p[k], g[k], m[k], v[k] hold n[k] floats each (host arrays of device pointers). */
int pntf_adamw_multi(int count, float* const* p, const float* const* g, float* const* m,
                     float* const* v, const int64_t* n, float lr, float beta1, float beta2,
                     float eps, float weight_decay, int64_t step, hipStream_t stream);

/* ---- Speed-sample generator (pntf_mesh.hip) ---------------------- */

/* Unsigned distance from each of n points `pts` (n, 3) to the triangle mesh `tris` (t, 3, 3)
 * (= v_obs[f_obs], dataprocessing/speed_sampling_gpu.py:386-388) -> `dist` (n).  Replaces
 * point_obstacle_distance (speed_sampling_gpu.py:325-336), i.e. bvh_distance_queries.BVH()
 * (squared closest-point distances) followed by torch.sqrt.  `chunks` splits the triangle
 * range over the grid (0 = auto, pntf_mesh_chunks); any value gives the same bits. */
int pntf_point_mesh_distance(const float* pts, int64_t n, const float* tris, int64_t t,
                             float* dist, int chunks, hipStream_t stream);
int pntf_mesh_chunks(int64_t n, int64_t t);
const char* pntf_mesh_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PNTF_H_ */
