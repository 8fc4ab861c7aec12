/*
 * gpscore.h — C-ABI of libgpscore.so, the MI355X (gfx950) GP-regression hot path.
 *
 * Reference being replaced (polarlightman/Scoring-rules-for-Gaussian-process-
 * regression..., aliases as in SURVEY.md §0: KF = kin40k-FULL-compare.py,
 * K20 = KIN40K-COMPARE-ALL-FITC-20.py, SD = "SIMPLE-DATA FULL-comapre.py").
 * The reference has no FFI; its call surface is module-level torch-CPU helpers.
 * Each entry point below names the reference code it replaces.  The ctypes
 * binding that a maintainer would add is gpscore/_lib.py.
 *
 * Conventions
 *  - All arrays are caller-owned, C-contiguous, row-major float64 HOST arrays
 *    unless the name ends in _dev; the library copies H2D/D2H itself.
 *  - Device buffers are owned by the opaque context and reused across calls.
 *  - Return value: 0 ok; >0 LAPACK-style info (the leading minor of that order
 *    is not positive definite, as torch.potrf raises); <0 argument / HIP / RCCL
 *    error, message via gps_last_error().  NaN/Inf propagate, nothing clamps.
 *  - A context is bound to one device and one HIP stream; it is not thread-safe.
 *  - theta layout everywhere: [log_sf2, log_ell_0 .. log_ell_{n_ell-1}, log_sn2]
 *    (n_ell = 1 or d), the reference's log-parameterisation para_k, para_l,
 *    para_noise (KF:7-12, KF:239).  kind: GPS_ARD (b = log ℓ) or GPS_RBF
 *    (b = log ℓ², SD:8-21).
 */
#ifndef GPSCORE_H
#define GPSCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gps_ctx gps_ctx;

enum { GPS_ARD = 0, GPS_RBF = 1 };
enum { GPS_FULL = 0, GPS_LOWER = 1 };

/* objective vector written by the fit calls */
enum {
  GPS_OBJ_NLML = 0,      /* ½n·log2π + ½log|A| + ½yᵀA⁻¹y            KF:334 / K20:339-340 */
  GPS_OBJ_LOO_CRPS = 1,  /* mean LOO CRPS                             KF:241-245 / K20:222-234 */
  GPS_OBJ_LOO_LOGS = 2,  /* mean LOO log score                        KF:416-424 / K20:434-447 */
  GPS_OBJ_LOGDET = 3,    /* log|A|                                    KF:332 (×2) */
  GPS_OBJ_QUAD = 4,      /* yᵀA⁻¹y                                    KF:334 */
  GPS_N_OBJ = 5
};
/* score vector written by gps_*_predict_score / gps_scores (KF:276-292) */
enum {
  GPS_SC_CRPS = 0, GPS_SC_LOGS = 1, GPS_SC_MSLL = 2, GPS_SC_SMSE = 3,
  GPS_SC_MSE = 4, GPS_SC_COVER = 5, GPS_N_SC = 6
};

/* ---- context ------------------------------------------------------------ */
/* ABI version of this header; gps_version() returns the library's.  Bumped whenever an entry
 * point changes its arguments or an array it writes changes size (500: gps_ctx_stats takes a
 * capacity, gps_comm_info and gps_build_id added; 600: gps_phase_enable / gps_phase_collect /
 * gps_rccl_info added).  The binding refuses a mismatch at load. */
#define GPS_ABI_VERSION 600
int gps_version(void);
/* The SHA-256 (hex) of the sources the library was built from (csrc/, this header; computed by
 * gpscore/buildid.py at build time).  Writes at most cap-1 characters and a NUL; returns the
 * id's length. */
int gps_build_id(char* out, int cap);
int gps_ctx_create(int device, gps_ctx** out);
int gps_ctx_destroy(gps_ctx* ctx);
const char* gps_last_error(gps_ctx* ctx);
/* Use an external hipStream_t (e.g. torch's current stream) instead of the ctx's own. */
int gps_ctx_set_stream(gps_ctx* ctx, void* hip_stream);
void* gps_ctx_stream(gps_ctx* ctx);
int gps_ctx_synchronize(gps_ctx* ctx);

/* ---- options ----------------------------------------------------------------
 * Round 6 removed the switches whose other settings had measured slower (4 / 14 fork bounds of
 * the side-stream product, 16 side-stream priority, 22 unfused chain tasks, 24 GEMM wave-priority
 * levels); their keys are refused like any unknown key.  Only options the defaults use.  Round-1 experiments measured neutral or slower on C3
 * (lookahead split, CU-reserved streams, in-launch split-K combine, CU-masked main stream,
 * split-K fill of the trailing update) were removed from the library. */
enum {
  GPS_OPT_OVERLAP = 0,  /* 1 (default): the factorisation's off-critical-path products (and the
                           energy score's folds) run on extra HIP streams; 0: everything on one
                           stream (clean per-kernel timing) */
  GPS_OPT_GEMM_MAP = 3, /* GEMM tile-order override: 0 automatic (default), 1-5 fixed orders, 6 the
                           row norms in paired column tiles (other launches automatic)
                           (A/B measurements; same values bitwise) */
  GPS_OPT_TINY_GEMM = 7, /* 1 (default): the bottom-of-recursion GEMMs (up to the 1280 level)
                            use the small kernel (16/32-blocks per wave, K split over the waves
                            of a workgroup, no LDS staging, no reduce launch); 0: the 64-tile
                            split-K + reduce path for them.  Process-wide. */
  GPS_OPT_GRAM_REG = 9,  /* 2 (default): as 1, with the d = 8, 16 builds on the matrix cores
                            in the reference's expansion 2·x·x'ᵀ − ‖x‖² − ‖x'‖² (KF:15-22;
                            equal to 1 within its rounding); 1: Gram builds with d in {1, 8, 16}
                            keep the column features in registers (128×128 tiles); 0: the
                            LDS-column kernel (bitwise equal to 1).  Process-wide. */
  GPS_OPT_GRAPH = 10,    /* 1 (default): the recursive factorisation's launch sequence is
                            captured once per (buffers, size, streams, options) into a hipGraph
                            and replayed; 0: eager launches.  Same kernels, same results. */
  GPS_OPT_PRED_PRE = 11, /* 1 (default): gps_fitc_fit forms the row-norm columns
                            q_i = ‖Lm⁻¹k_i‖² that need only the top-level Lm11⁻¹ (a quarter of
                            the pass) on a second stream while the rest of Lm's factorisation
                            runs; 0: the whole pass after it.  Same tiles, same results. */
  GPS_OPT_DAG = 12,      /* 1 (default): diagonal blocks of at most GPS_OPT_DAG_TILES 128-tiles
                            at the bottom of the recursive factorisation are factored and
                            inverted by ONE persistent launch (a device task queue of tile
                            products, per-tile arrival counters); 0: the recursion down to
                            the 128-block leaf.  Same algorithm, other summation order. */
  GPS_OPT_AR_CHUNKS = 15, /* sharded FITC: B's all-reduce in this many row blocks (default 4),
                             each on a comm stream while the next block's SYRK runs; 1: one
                             all-reduce after the SYRK.  Same bits either way. */
  GPS_OPT_DAG_TILES = 13, /* largest block (in 128-tiles, 2..64, default 20) the persistent
                            factorisation takes */
  GPS_OPT_STREAM_K = 18,  /* the stream-K tail of a 128-tile GEMM launch with uniform K ranges (the
                             trailing-update SYRKs) whose last round of workgroup slots would be at
                             most 3/4 full: that round's tiles split into equal K runs over every
                             slot (in-launch fixed-order combine).  2 (default): for a trailing update
                             that runs alone (overlap off, or below the fork level) — beside the side
                             stream's T product the round is filled already; 1: every eligible
                             launch; 0: never.  Process-wide. */
  GPS_OPT_DAG_WGS = 19,   /* workgroups of a persistent factorisation launch; 0 (default):
                             automatic — one per CU for the full GP, half the CUs for the FITC
                             m×m factorisations (the test pre-pass runs beside them) */
  GPS_OPT_DAG_GROUP = 17, /* persistent factorisation: 16-deep operand chunks a strip task has in
                             flight per load group (2, 3 (default) or 4).  Same values bitwise. */
  GPS_OPT_SLAB_XCD = 26,  /* 1: split-K GEMM launches (the FITC SYRK, small trailing updates) deal
                             their (tile, K slice) pairs slice-major, each XCD a contiguous run,
                             so one XCD's resident workgroups share a slice's operand rows in its
                             L2 (default; C4's SYRK 7x -> 2.9x its operand in L2-fabric bytes,
                             time neutral); 0: tile-major.  Same values bitwise.  Process-wide. */
  GPS_OPT_DAG_ORDER = 25, /* queue order of the persistent factorisation's tasks: 1 (default)
                             largest upward rank with the round-4 measured task durations, 2 the
                             same with round 3's, 0 earliest estimated start.  Same values bitwise
                             (the order changes only which workgroup runs a task, and when). */
  GPS_OPT_FITC_DEP = 27,  /* 1 (default): when K̃mm's factorisation is one persistent launch (m_pad ≤
                             20 tiles), the q_i = ‖Lm⁻¹k_i‖² row norms start on a second stream while
                             it runs, each column tile as soon as its row of Lm⁻¹ is final
                             (device-side row signals), and a completion launch after it takes
                             the tiles left; with m_pad > 20 tiles (a recursive factorisation)
                             the same for the q pre-pass over the top-level L11⁻¹ columns when
                             that block is one persistent launch and the pre-pass ≤ 8192 tiles,
                             and for the r pre-pass behind Lb's L11 block at ≤ 4096 tiles;
                             0: the row norms after the factorisation.  Same tiles, same values
                             bitwise. */
};
int gps_ctx_set_option(gps_ctx* ctx, int key, int value);

/* Context statistics: out[GPS_STAT_GRAPHS] factorisation graphs cached (one per distinct
 * (buffers, size, streams, options); each holds its instantiated launch sequence, ~1-3 MB of
 * host memory and a few KB of device memory), out[GPS_STAT_GRAPH_CAP] the cache's capacity
 * (least recently used exec destroyed beyond it), out[GPS_STAT_GRAPH_OVERFLOW] 0 (kept for the
 * layout: no factorisation runs eagerly for want of a slot), out[GPS_STAT_DEVICE_BYTES] device
 * memory held by the context's buffers, out[GPS_STAT_GRAPH_DROPPED] execs destroyed because a
 * buffer they use was freed or grown (a graph never outlives its buffers),
 * out[GPS_STAT_GRAPH_EVICTED] execs destroyed by the capacity limit. */
enum { GPS_STAT_GRAPHS = 0, GPS_STAT_GRAPH_CAP = 1, GPS_STAT_GRAPH_OVERFLOW = 2,
       GPS_STAT_DEVICE_BYTES = 3, GPS_STAT_GRAPH_DROPPED = 4, GPS_STAT_GRAPH_EVICTED = 5,
       GPS_N_STATS = 6 };
/* Writes min(cap, GPS_N_STATS) entries; returns GPS_N_STATS (the count this library knows). */
int gps_ctx_stats(gps_ctx* ctx, int64_t* out, int cap);

/* Diagnostics: the persistent factorisation's task queue for a block of T tiles (2..64), one
 * word per strip task (type | part << 3 | fine << 7 | i << 8 | j << 16 | k << 24; types 0 LEAF,
 * 1 TRSM, 2 UPD, 3 UPDX, 4 FIN; flags bit 0: the chain tasks' fine parts (the library's queue),
 * bits 2-3: the order (GPS_OPT_DAG_ORDER: 0 or 1 the default 1, 2 order 2, 3 order 0), other
 * bits rejected — kernels_potrf.hip).  Returns the queue length (writes at most cap words);
 * needs no device. */
int gps_dag_task_list(int T, int flags, uint32_t* out, int cap);

/* on: 0 off, 1 per-kernel-class tags, 2 GEMM tags also carry layout/shape/tri/split-K/lda */
int gps_prof_enable(gps_ctx* ctx, int on);
/* Synchronises, then writes a JSON object {tag: {count, ms, flop, bytes}} and clears. */
int gps_prof_collect(gps_ctx* ctx, char* json_out, int64_t cap);
/* Phase timing of the FITC forward on its production schedule (the launches, streams and their
 * overlap are unchanged; gps_prof_enable instead serialises them): with on, every FITC forward
 * (gps_fitc_fit, the gradients' and block-LOO's forward) records a timing event on its main
 * stream at each phase boundary, and two around every all-reduce on the stream that issues it.
 * Phases, each the main-stream time since the previous mark (K20:222-234 restated):
 *   "kmm_lm"   K̃mm and Lm's factorisation (replicated on every rank; Knm's Gram beside it),
 *   "knm"      the wait for Knm (sharded),  "q" the q row norms and λ (sharded),
 *   "syrk"     B's split-K SYRK with its packing (sharded; the row-block all-reduces beside it),
 *   "exchange" the main stream's wait for B's last all-reduce (exposed exchange),
 *   "lb"       B's unpack and Lb's factorisation, "c" c = B⁻¹b (replicated),
 *   "r"        the r row norms, g and the LOO terms (sharded), "scal" the scalar all-reduce.
 * gps_phase_collect synchronises and writes {"phases": {name: {"count", "ms"}}, "allreduce":
 * [[bytes, ms], ...]} (one pair per all-reduce, on its own stream) and clears. */
int gps_phase_enable(gps_ctx* ctx, int on);
int gps_phase_collect(gps_ctx* ctx, char* json_out, int64_t cap);
/* The RCCL this process runs: ncclGetVersion and the file holding ncclAllReduce as the dynamic
 * linker resolved it (the library links librccl.so.1 from /opt/rocm/lib; a process that loaded a
 * librccl.so.1 first — torch's bundled copy, when torch is imported before the library — runs
 * that one).  Writes at most cap-1 characters and a NUL to path; needs no device. */
int gps_rccl_info(int* version, char* path, int cap);

/* ---- L1 building blocks ---------------------------------------------------- */
/* ARD(x, xp, a, b) KF:7-23 / rbf SD:8-21: out[n][m] = sf2·exp(−½‖(x−x')/ℓ‖²)
 * (+ diag_add where i == j); uplo GPS_LOWER writes only j <= i. */
int gps_gram(gps_ctx* ctx, int kind, const double* X, int64_t n, const double* Xp,
             int64_t m, int d, double log_sf2, const double* log_ell, int n_ell,
             double diag_add, int uplo, double* out);
/* torch.potrf(A).diag().log().sum() (KF:332): lower Cholesky L written into A
 * (lower triangle, upper zeroed); *logdet = log|A|.  Returns info > 0 if not PD. */
int gps_potrf(gps_ctx* ctx, int64_t n, double* A, int64_t lda, double* logdet);
/* chol_solve(B, A) KF:25-29: X = A⁻¹·B for SPD A (n×n) and B (n×nrhs). */
int gps_potrs(gps_ctx* ctx, int64_t n, int64_t nrhs, const double* A, int64_t lda,
              const double* B, int64_t ldb, double* X, int64_t ldx);
/* diag(chol_solve(I, A)) KF:242: dinv[i] = (A⁻¹)_ii. */
int gps_diag_inv(gps_ctx* ctx, int64_t n, const double* A, int64_t lda, double* dinv);
/* torch.mm in the reference helpers (Q KF:38, cal_mean_and_cov KF:123-125,
 * spgp_cal_mean_and_cov K20:81-82): C = alpha·op(A)·op(B) + beta·C on the FP64
 * MFMA path; op(X) = Xᵀ when trans != 0. */
int gps_gemm(gps_ctx* ctx, int transA, int transB, int64_t M, int64_t N, int64_t K, double alpha,
             const double* A, int64_t lda, const double* B, int64_t ldb, double beta, double* C,
             int64_t ldc);
/* crps/logs/trivial_loss/SMSE/MSE/coverage of a Gaussian predictive (KF:52-68,
 * 110-134, 276-292); var is the VARIANCE.  ytr_mean / ytr_var_unbiased are
 * the train-target statistics trivial_loss and SMSE use. */
int gps_scores(gps_ctx* ctx, const double* mu, const double* var, const double* y,
               int64_t nt, double ytr_mean, double ytr_var_unbiased, double out[GPS_N_SC]);

/* ---- full GP (fused hot path) --------------------------------------------- */
/* Upload training data (kept resident until replaced). */
int gps_full_set_data(gps_ctx* ctx, const double* X, const double* y, int64_t n, int d);
int gps_full_set_test(gps_ctx* ctx, const double* Xt, const double* yt, int64_t nt);
/* One forward evaluation of the per-iteration bodies KF:239-245, 329-334,
 * 416-424 at theta: Gram + potrf + L⁻¹ + α + diag(A⁻¹) → objectives.
 * mu_loo / var_loo (length n) may be NULL (kept on device). */
int gps_full_fit(gps_ctx* ctx, int kind, const double* theta, int n_ell,
                 double obj[GPS_N_OBJ], double* mu_loo, double* var_loo);
/* Forward + analytic gradient of one objective (GPS_OBJ_NLML / _LOO_CRPS / _LOO_LOGS) at
 * theta: what one GD iteration of the reference computes with autograd `.backward()`
 * (KF:252 LOO-CRPS, KF:339 NLML, KF:428 LOO-LogS) before its SGD update (KF:254-260).
 * grad (length 2 + n_ell) = [d/d log sf2, d/d b (n_ell), d/d log sigma2] in the
 * reference's parameterisation (para_k, para_l, para_noise).  Also leaves the factor
 * for gps_full_predict, like gps_full_fit. */
int gps_full_grad(gps_ctx* ctx, int kind, const double* theta, int n_ell, int objective,
                  double obj[GPS_N_OBJ], double* grad);
/* Predictive mean/variance at the test points with the last fit's factor
 * (cal_mean_and_cov KF:121-126, diag of the covariance), plus the score bundle
 * against yt (KF:276-292).  mu / var may be NULL; sc may be NULL. */
int gps_full_predict(gps_ctx* ctx, double* mu, double* var, double sc[GPS_N_SC]);

/* ---- FITC sparse GP (Woodbury restatement of K20:32-39, 76-83, 222-340) ----- */
int gps_fitc_set_data(gps_ctx* ctx, const double* X, const double* y, int64_t n, int d,
                      double ytr_mean, double ytr_var_unbiased, int64_t n_total);
int gps_fitc_set_test(gps_ctx* ctx, const double* Xt, const double* yt, int64_t nt,
                      int64_t nt_total);
int gps_fitc_set_inducing(gps_ctx* ctx, const double* Z, int64_t m);
/* FITC objectives over this rank's rows.  With a communicator (gps_comm_init)
 * the m×m accumulator and scalar partials are all-reduced over RCCL; objectives
 * are then global and mu_loo / var_loo hold this rank's rows.  With a test set resident
 * (gps_fitc_set_test) and GPS_OPT_OVERLAP on, the fit also forms the test-side row norms
 * ‖Lm⁻¹k*‖² and ‖Lb⁻¹k*‖² on a second stream where its own chain leaves the chip idle, so
 * gps_fitc_predict is left with μ* and the finalise; a new test set voids them. */
int gps_fitc_fit(gps_ctx* ctx, const double* theta, int n_ell, double obj[GPS_N_OBJ],
                 double* mu_loo, double* var_loo);
/* Forward + analytic gradient of one FITC objective w.r.t. theta AND the inducing
 * inputs: the reference's `.backward()` through its dense FITC bodies at K20:236
 * (LOO-CRPS), K20:344 (NLML), K20:452 (LOO-LogS) before the SGD step that also moves
 * inducing_x (K20:238-247).  grad (2 + n_ell) as gps_full_grad; grad_z (m×d, row-major,
 * may be NULL) = d obj / d Z.  O(n·m²); with a communicator every rank gets the global
 * gradient. */
int gps_fitc_grad(gps_ctx* ctx, const double* theta, int n_ell, int objective,
                  double obj[GPS_N_OBJ], double* grad, double* grad_z);
int gps_fitc_predict(gps_ctx* ctx, double* mu, double* var, double sc[GPS_N_SC]);
/* Diagnostics: the last FITC forward's device intermediates, unpadded and row-major — Knm (n×m,
 * this shard's rows), λ (n), Lm⁻¹ and Lb⁻¹ (m×m, lower; the factorisations' inverses of K̃mm =
 * K(Z, Z) + 1e-3·I and B = K̃mm + KmnΛ⁻¹Knm) and K̃mm (m×m, lower).  Any pointer may be NULL.
 * (DESIGN §9 feeds them one at a time into the oracle's gradient to find which one carries the
 * GPU's extra rounding.) */
int gps_fitc_intermediates(gps_ctx* ctx, double* Knm, double* lam, double* Lm_inv, double* Lb_inv,
                           double* Kmm);

/* ---- block-LOO objectives -----------------------------
 * nfold-fold (the scripts use 4) block leave-out predictive from the diagonal blocks of
 * A⁻¹: fold f = rows [int(f·n/k), int((f+1)·n/k)) (KF:496-499), m_f = y_f − P_f⁻¹α_f,
 * C_f = P_f⁻¹, P_f = (A⁻¹)_ff.  GPS_BLOCK_DSS: Σ_f dss(m_f, C_f, y_f) (KF:487-543,
 * K20:523-587, dss KF:103-108); GPS_BLOCK_KC: Σ_f crps(m_f, diag C_f, y_f) (K20:655-720);
 * GPS_BLOCK_ES: Σ_f ES(m_f, C_f, y_f) (KF:607-663, ES KF:70-101; gps_full_blockloo_es).
 * value = the sum over folds, fold_values (nfold, may be NULL) the per-fold terms. */
enum { GPS_BLOCK_DSS = 0, GPS_BLOCK_KC = 1, GPS_BLOCK_ES = 2 };
/* Full GP, DSS or KC; grad (2 + n_ell, may be NULL) = the `.backward()` at KF:543 in the
 * reference's parameterisation.  Leaves the factor for gps_full_predict. */
int gps_full_blockloo(gps_ctx* ctx, int kind, const double* theta, int n_ell, int nfold,
                      int objective, double* value, double* grad, double* fold_values);
/* Full GP, energy score with num_sim draws per fold (300 at KF:652-655) and exponent beta
 * (1 at KF:70).  draws (2·num_sim·n doubles) hold, fold after fold, ξ_f then ξ'_f
 * (num_sim × b_f, row-major): the two torch.randn(num_sim, shape1) calls of ES (KF:79-80) in
 * the scripts' order.  C_f^½ (an SVD at KF:74-77) is the coupled Newton–Schulz iteration on
 * the MFMA GEMM.  grad as gps_full_blockloo (the `.backward()` at KF:663). */
int gps_full_blockloo_es(gps_ctx* ctx, int kind, const double* theta, int n_ell, int nfold,
                         int num_sim, double beta, const double* draws, double* value,
                         double* grad, double* fold_values);
/* FITC, DSS or KC; grad (2 + n_ell) and grad_z (m×d, row-major) may be NULL: the
 * `.backward()` at K20:587 / K20:720 w.r.t. theta and the inducing inputs, which the scripts
 * move too (K20:593, 726).  With a communicator the rows may be sharded: the nfold folds are
 * those of the GLOBAL rows ([⌊fN/k⌋, ⌊(f+1)N/k⌋), KF:496-499) and each must lie inside one
 * rank's rows (gpscore.dist.fold_shard_rows), else every rank returns -1; every rank gets the
 * global value, gradients and all nfold fold_values. */
int gps_fitc_blockloo(gps_ctx* ctx, const double* theta, int n_ell, int nfold, int objective,
                      double* value, double* grad, double* grad_z, double* fold_values);
/* ES(m, c, shape1, data_y, num_sim, beta) (KF:70-101) of one Gaussian N(m, C) (b×b,
 * row-major) at y with the draws given (ξ then ξ', num_sim × b each): the compat helper. */
int gps_energy_score(gps_ctx* ctx, const double* m, const double* C, int64_t b, const double* y,
                     int num_sim, double beta, const double* draws, double* out);

/* ---- objective surfaces (contour-plot.R) ---------------
 * The objectives of CP.R:43-85 on a length-scale × noise grid, one small full GP per grid
 * point (CP.R uses n = 20 points and a 50 × 50 grid, CP.R:88-141): kernel
 * sf²·exp(−½‖x − x'‖²/ℓ²) with ℓ = ell[j] (CP.R:15-23, not a log) and noise s.d. s = noise_sd[i]
 * entering as s² (CP.R:45).  out (4 · n_noise · n_ell, row-major [objective][i][j], R's
 * matrix(…, nrow = 50) orientation): GPS_SURF_LOO_CRPS (cal_m_crps CP.R:43-53),
 * GPS_SURF_INSAMPLE_CRPS (wrong_cal_m_crps CP.R:55-64), GPS_SURF_NLML (cal_NLML CP.R:68-73),
 * GPS_SURF_LOO_LOGS (cal_m_logs CP.R:75-85).  flags GPS_SURF_LOGS_ADD_NOISE: the LOO-LogS
 * variance is 1/d + s² as CP.R:81 writes it; without it 1/d (the KF:416-424 form).  A grid
 * point whose matrix is not positive definite gets NaN objectives.  n > 128: each grid point
 * is one resident fit (the gps_full_fit path) and X, y become the context's full-GP data, as
 * after gps_full_set_data (no fit is left in place). */
enum { GPS_SURF_LOO_CRPS = 0, GPS_SURF_INSAMPLE_CRPS = 1, GPS_SURF_NLML = 2, GPS_SURF_LOO_LOGS = 3,
       GPS_N_SURF = 4 };
enum { GPS_SURF_LOGS_ADD_NOISE = 1 };
int gps_full_surface(gps_ctx* ctx, const double* X, const double* y, int64_t n, int d,
                     double log_sf2, const double* ell, int64_t n_ell, const double* noise_sd,
                     int64_t n_noise, int flags, double* out);

/* ---- multi-GPU (RCCL over xGMI) ------------------------------------------- */
int gps_comm_unique_id(char uid[128]);
int gps_comm_init(gps_ctx* ctx, int nranks, int rank, const char uid[128]);
/* In-process stand-in for the communicator: nranks contexts of ONE process (each driven by its
 * own host thread, e.g. several shards on one GPU) that pass the same `group` key meet at every
 * all-reduce of the FITC path, where their partials are summed on the host in rank order.
 * Same call sites and element counts as the RCCL path; used to test the row-sharded FITC
 * bookkeeping without a multi-GPU node.  A rank that waits > 60 s, or a member that leaves,
 * aborts the group: every member's current and later all-reduces then fail (call
 * gps_comm_init_local again, which joins a fresh group under the same key).  Two live
 * contexts may not hold the same rank of one group. */
int gps_comm_init_local(gps_ctx* ctx, int nranks, int rank, long long group);
/* What the context's communicator holds: *nranks and *rank as RCCL reports them
 * (ncclCommCount / ncclCommUserRank) for GPS_COMM_RCCL, the group's size and this context's rank
 * for GPS_COMM_LOCAL, 1 and 0 with GPS_COMM_NONE. */
enum { GPS_COMM_NONE = 0, GPS_COMM_RCCL = 1, GPS_COMM_LOCAL = 2 };
int gps_comm_info(gps_ctx* ctx, int* nranks, int* rank, int* kind);
/* Leaves either communicator. */
int gps_comm_destroy(gps_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* GPSCORE_H */
