// C-ABI, FITC: data, the Woodbury fit with its row-norm passes and the row-sharded exchange,
// the θ / Z gradients, predict + score (K20:76-83, 222-340, 434-452), the intermediates export.
#include "api_internal.h"

extern "C" {

// ---------------------------------------------------------------------- FITC
int gps_fitc_set_data(gps_ctx* ctx, const double* X, const double* y, int64_t n, int d,
                      double ytr_mean, double ytr_var_unbiased, int64_t n_total) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(X && y && n > 0 && d >= 1 && d <= GPS_MAX_D && n_total >= n, "bad FITC training data");
  if (d != ctx->fd) ctx->f_test = ctx->f_z = false;  // test set / inducing points of another d
  ctx->fn = n;
  ctx->fd = d;
  ctx->fn_pad = pad_to(n);
  ctx->fn_total = n_total;
  ctx->f_ytr_mean = ytr_mean;
  ctx->f_ytr_var = ytr_var_unbiased;
  if (int rc = upload(ctx, ctx->fX, X, n, d, ctx->fn_pad)) return rc;
  if (int rc = upload(ctx, ctx->fy, y, n, 1, ctx->fn_pad)) return rc;
  ctx->f_data = true;
  ctx->f_fitted = false;
  ctx->f_pre = ctx->f_pre_b = false;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gps_fitc_set_test(gps_ctx* ctx, const double* Xt, const double* yt, int64_t nt,
                      int64_t nt_total) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(ctx->f_data, "gps_fitc_set_data first");
  ARGCHK(Xt && nt >= 0 && nt_total >= nt, "bad FITC test data");
  ctx->fnt = nt;
  ctx->fnt_pad = pad_to(std::max<int64_t>(nt, 1));
  ctx->fnt_total = nt_total;
  if (int rc = upload(ctx, ctx->fXt, Xt, nt, ctx->fd, ctx->fnt_pad)) return rc;
  std::vector<double> zeros;
  if (!yt) zeros.assign(std::max<int64_t>(nt, 1), 0.0);
  if (int rc = upload(ctx, ctx->fyt, yt ? yt : zeros.data(), nt, 1, ctx->fnt_pad)) return rc;
  ctx->f_test = true;
  ctx->f_pre = ctx->f_pre_b = false;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gps_fitc_set_inducing(gps_ctx* ctx, const double* Z, int64_t m) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(ctx->f_data, "gps_fitc_set_data first");
  ARGCHK(Z && m > 0, "bad inducing points");
  ctx->m = m;
  ctx->m_pad = pad_to(m);
  if (int rc = upload(ctx, ctx->Z, Z, m, ctx->fd, ctx->m_pad)) return rc;
  ctx->f_z = true;
  ctx->f_fitted = false;
  ctx->f_pre = ctx->f_pre_b = false;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// split-K SYRK over this shard's rows: dst (lower tiles, strict-upper zeroed) =
// Kmnᵀ diag(kscale) Knm (+ base).  Every workgroup has the same work, so the grid runs
// in whole rounds of 512 slots (2 per CU): take the smallest split whose last round is
// >= 95 % full (528 tiles at m = 4096: ks 3 -> 77 % of the slots busy on average, ks 12
// -> 95 %), with at least 1024 rows per slice and at most 32 slabs.
// With `packed` the sum goes lower-packed (m(m+1)/2, launch_sym_pack) into dst instead: the
// all-reduce payload of the row-sharded path (base must be NULL then).
int fitc_syrk_ks(const gps_ctx* ctx) {
  const int64_t np = ctx->fn_pad, mp = ctx->m_pad, tm = mp / GPS_TILE;
  const int64_t tiles_lower = tm * (tm + 1) / 2;
  int ks = 1;
  for (int k = 1; k <= 32 && (int64_t)k * 1024 <= np; ++k) {
    const int64_t wg = tiles_lower * k, rounds = (wg + 511) / 512;
    ks = k;
    if (wg >= 1024 && (double)wg / (512.0 * rounds) >= 0.95) break;
  }
  // and slices of at most ~8k rows: at n = 200k (C5) 24 slices ran 1 % faster than the 12 the
  // fill rule gives (more workgroups share each slice's rows through the Infinity Cache), at
  // n = 40k (C4) more slices than the fill rule's 11 were slower (profiles/r2_syrk_ks_ab.txt)
  return (int)std::max<int64_t>(ks, std::min<int64_t>(32, (np + 8191) / 8192));
}

// split-K SYRK slabs of B's rows [R0, R1) (128-aligned): the rectangle left of the diagonal
// block and the diagonal block's lower tiles, K slices as the whole-matrix launch would cut them
// (same ks, same per-tile K ranges), so a row block's slab values are bitwise those of the
// unchunked SYRK
int fitc_syrk_rows(gps_ctx* ctx, const double* kscale, int ks, int64_t R0, int64_t R1) {
  const int64_t np = ctx->fn_pad, mp = ctx->m_pad;
  double* slab = ctx->slabB.d();
  if (R0 > 0) {
    GemmParams p = gp0();
    p.A = ctx->Knm.d() + R0; p.lda = mp; p.B = ctx->Knm.d(); p.ldb = mp;
    p.C = slab + R0 * mp; p.ldc = mp; p.c_kslice_stride = mp * mp;
    p.M = (int)(R1 - R0); p.N = (int)R0; p.K = (int)np; p.kscale = kscale; p.ksplit = ks;
    if (int rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p)) return rc;
  }
  GemmParams p = gp0();
  p.A = ctx->Knm.d() + R0; p.lda = mp; p.B = ctx->Knm.d() + R0; p.ldb = mp;
  p.C = slab + R0 * mp + R0; p.ldc = mp; p.c_kslice_stride = mp * mp;
  p.M = (int)(R1 - R0); p.N = (int)(R1 - R0); p.K = (int)np; p.kscale = kscale;
  p.lower_out = 1; p.ksplit = ks;
  return gemm(ctx, LAY_T, LAY_N, EPI_STORE, p);
}

// B_p = Kmnᵀ diag(kscale) Knm over this rank's rows (K20:222-234's big_Q restated as the
// Woodbury m×m form), split-K slabs summed in fixed order; base (if given) added; dst = the
// padded lower tiles.  With `packed` the sum goes lower-packed (m(m+1)/2, launch_sym_pack) into
// dst instead: the payload of the ranks' all-reduce.
int fitc_syrk(gps_ctx* ctx, const double* kscale, const double* base, double* dst,
              bool packed, const double* A, int64_t lda) {
  const int64_t mp = ctx->m_pad;
  const int ks = fitc_syrk_ks(ctx);
  HIPCHK(ensure(ctx, ctx->slabB, (size_t)ks * mp * mp * 8));
  if (!A) {  // the operand: Knm (default) or another n×m row panel (the whitened gradient's U, V)
    A = ctx->Knm.d();
    lda = mp;
  }
  GemmParams p = gp0();
  p.A = A; p.lda = lda; p.B = A; p.ldb = lda;
  p.C = ctx->slabB.d(); p.ldc = mp; p.c_kslice_stride = mp * mp;
  p.M = (int)mp; p.N = (int)mp; p.K = (int)ctx->fn_pad; p.kscale = kscale;
  p.lower_out = 1; p.ksplit = ks;
  if (int rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p)) return rc;
  Prof pr(ctx, "syrk_slab_sum", 0, 8.0 * (ks + 1 + (base ? 1 : 0)) * mp * mp);
  if (packed)
    HIPCHK(launch_sym_pack(ctx->slabB.d(), mp * mp, ks, 0, (int)ctx->m, (int)mp, dst, ctx->stream));
  else
    HIPCHK(launch_sym_slab_sum(ctx->slabB.d(), mp * mp, ks, (int)mp, base, dst, ctx->stream));
  return 0;
}

// The sharded forward's exchange: B_p lower-packed, then [b | Σlogλ | Σy²/λ],
// summed over the ranks.  With ctx->ar_chunks > 1 B's rows go in blocks of about equal packed
// size: block c's slabs are formed and packed on the main stream, then all-reduced on the comm
// stream (aux[1]) while block c+1's SYRK runs; the last block carries b and the scalars, and
// the main stream waits for the comm stream before unpacking.  Chunked and unchunked give the
// same bits (the slab values do not depend on the row blocks; tests/test_gpu_shards.py).
int fitc_syrk_allreduce(gps_ctx* ctx, double* red, int64_t blen, int64_t tail) {
  const int64_t m = ctx->m, mp = ctx->m_pad, tm = mp / GPS_TILE;
  hipStream_t s = ctx->stream;
  const int nch = (int)std::min<int64_t>(std::max(1, ctx->ar_chunks), tm);
  if (nch <= 1) {
    if (int rc = fitc_syrk(ctx, ctx->ilam.d(), nullptr, red, true)) return rc;
    phase_mark(ctx, "syrk");
    Prof pr(ctx, "allreduce_B", 0, 8.0 * (blen + tail));
    const int rc = allreduce_sum(ctx, red, (size_t)(blen + tail), s);
    phase_mark(ctx, "exchange");
    return rc;
  }
  const int ks = fitc_syrk_ks(ctx);
  HIPCHK(ensure(ctx, ctx->slabB, (size_t)ks * mp * mp * 8));
  hipStream_t cs = ctx->aux[1];
  while ((int)ctx->ar_ev.size() < nch + 1) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->ar_ev.push_back(e);
  }
  int64_t R0 = 0;
  for (int c = 0; c < nch; ++c) {
    // row-block ends at equal packed sizes: R_c = m·sqrt(c/nch), 128-aligned, strictly growing
    int64_t R1 = c + 1 == nch ? mp
                              : (int64_t)std::llround(std::sqrt((double)(c + 1) / nch) * (double)tm) * GPS_TILE;
    R1 = std::min<int64_t>(std::max<int64_t>(R1, R0 + GPS_TILE), mp - (int64_t)(nch - 1 - c) * GPS_TILE);
    if (int rc = fitc_syrk_rows(ctx, ctx->ilam.d(), ks, R0, R1)) return rc;
    const int r0 = (int)std::min<int64_t>(R0, m), r1 = (int)std::min<int64_t>(R1, m);
    {
      Prof pr(ctx, "syrk_slab_sum", 0, 8.0 * (ks + 1) * (R1 - R0) * R1);
      HIPCHK(launch_sym_pack(ctx->slabB.d(), mp * mp, ks, r0, r1, (int)mp, red, s));
    }
    HIPCHK(hipEventRecord(ctx->ar_ev[c], s));
    HIPCHK(hipStreamWaitEvent(cs, ctx->ar_ev[c], 0));
    const int64_t e0 = (int64_t)r0 * (r0 + 1) / 2;
    const int64_t e1 = c + 1 == nch ? blen + tail : (int64_t)r1 * (r1 + 1) / 2;
    Prof pr(ctx, "allreduce_B", 0, 8.0 * (e1 - e0), cs);
    if (e1 > e0)
      if (int rc = allreduce_sum(ctx, red + e0, (size_t)(e1 - e0), cs)) return rc;
    R0 = R1;
  }
  HIPCHK(hipEventRecord(ctx->ar_ev[nch], cs));
  phase_mark(ctx, "syrk");
  HIPCHK(hipStreamWaitEvent(s, ctx->ar_ev[nch], 0));
  phase_mark(ctx, "exchange");
  return 0;
}

// Test-side half of the FITC predict that depends only on θ, Z and Lm: K*m and
// q*_i = ‖Lm⁻¹k*_i‖² (spgp_cal_mean_and_cov K20:76-83).  gps_fitc_fit launches it on aux[0]
// just before B's factorisation, whose latency-bound chain leaves most CUs idle; predict
// waits on the join event instead of recomputing (measured in DESIGN.md §7).
int fitc_test_prepass(gps_ctx* ctx) {
  const Theta& th = ctx->fth;
  const int64_t nt = ctx->fnt, ntp = ctx->fnt_pad, m = ctx->m, mp = ctx->m_pad;
  const int64_t tm = mp / GPS_TILE;
  hipStream_t a = ctx->aux[0];
  HIPCHK(ensure(ctx, ctx->Ksm, (size_t)ntp * mp * 8));
  HIPCHK(ensure(ctx, ctx->qm, ntp * 8));
  HIPCHK(ensure(ctx, ctx->fslab_pre, (size_t)tm * ntp * 8));
  for (hipEvent_t* e : {&ctx->pre_fork, &ctx->pre_join})
    if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ctx->pre_fork, ctx->stream));
  HIPCHK(hipStreamWaitEvent(a, ctx->pre_fork, 0));
  int rc;
  if ((rc = gram(ctx, "gram_ksm", ctx->fXt.d(), (int)nt, ctx->Z.d(), (int)m, ctx->fd, th, 0.0, 0, 0,
                 ctx->Ksm.d(), mp, (int)ntp, (int)mp, a)))
    return rc;
  GemmParams p = gp0();
  p.A = ctx->Ksm.d(); p.lda = mp; p.B = ctx->Lm.d(); p.ldb = mp;
  p.M = (int)ntp; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_LE_J; p.kend = (int)pad_to(m, 16);
  p.out0 = ctx->fslab_pre.d(); p.ld_out = ntp;
  if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_ROWSQ, p, a))) return rc;
  HIPCHK(launch_slab_sum(ctx->fslab_pre.d(), ntp, (int)tm, ntp, nullptr, ctx->qm.d(), a));
  HIPCHK(hipEventRecord(ctx->pre_join, a));
  ctx->f_pre = true;
  return 0;
}

// The other test-side row norms, q*b_i = ‖Lb⁻¹k*_i‖², once Lb⁻¹ is final: on aux[0] (after the
// q* pass there) while the main stream runs the training r pass, whose last round of workgroup
// slots they fill; predict then has only μ* and the finalise left (K20:76-83).
int fitc_test_prepass_b(gps_ctx* ctx) {
  const int64_t ntp = ctx->fnt_pad, mp = ctx->m_pad, tm = mp / GPS_TILE;
  hipStream_t a = ctx->aux[0];
  HIPCHK(ensure(ctx, ctx->qb, ntp * 8));
  if (!ctx->preb_fork) HIPCHK(hipEventCreateWithFlags(&ctx->preb_fork, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ctx->preb_fork, ctx->stream));
  HIPCHK(hipStreamWaitEvent(a, ctx->preb_fork, 0));
  GemmParams p = gp0();
  p.A = ctx->Ksm.d(); p.lda = mp; p.B = ctx->Lb.d(); p.ldb = mp;
  p.M = (int)ntp; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_LE_J;
  p.kend = (int)pad_to(ctx->m, 16);
  p.out0 = ctx->fslab_pre.d(); p.ld_out = ntp;  // (the q* slab sum precedes on aux[0])
  if (int rc = gemm(ctx, LAY_N, LAY_T, EPI_ROWSQ, p, a)) return rc;
  HIPCHK(launch_slab_sum(ctx->fslab_pre.d(), ntp, (int)tm, ntp, nullptr, ctx->qb.d(), a));
  HIPCHK(hipEventRecord(ctx->pre_join, a));
  ctx->f_pre_b = true;
  return 0;
}

// forward FITC objectives; leaves Knm, Lm⁻¹, Lb⁻¹, λ, r, g = Knm c, c on the device.
// pre_test: also form the test-side Lm row norms during B's factorisation (gps_fitc_fit)
int fitc_fit_core(gps_ctx* ctx, const double* theta, int n_ell, double obj[GPS_N_OBJ],
                  bool pre_test) {
  ARGCHK(ctx->f_data && ctx->f_z, "gps_fitc_set_data / gps_fitc_set_inducing first");
  ctx->f_fitted = false;  // set again by the callers once check_info has passed
  ctx->f_pre = ctx->f_pre_b = false;
  if (int rc = set_theta(ctx, ctx->fth, GPS_ARD, theta, n_ell, ctx->fd)) return rc;
  const Theta& th = ctx->fth;
  const int64_t n = ctx->fn, np = ctx->fn_pad, m = ctx->m, mp = ctx->m_pad;
  const int64_t tm = mp / GPS_TILE;
  hipStream_t s = ctx->stream;
  // buffers
  HIPCHK(ensure(ctx, ctx->Kmm, (size_t)mp * mp * 8));
  HIPCHK(ensure(ctx, ctx->Am, (size_t)mp * mp * 8));
  if (ctx->Lm.cap < (size_t)mp * mp * 8 || ctx->Lb.cap < (size_t)mp * mp * 8 ||
      !factor_zeroed(ctx, ctx->Lm.d(), mp) || !factor_zeroed(ctx, ctx->Lb.d(), mp)) {
    HIPCHK(ensure(ctx, ctx->Lm, (size_t)mp * mp * 8));
    HIPCHK(ensure(ctx, ctx->Lb, (size_t)mp * mp * 8));
    HIPCHK(zero_factor(ctx, ctx->Lm.d(), mp, s));
    HIPCHK(zero_factor(ctx, ctx->Lb.d(), mp, s));
  }
  HIPCHK(ensure(ctx, ctx->W, std::max(ctx->W.cap, potrf_ws_doubles(mp) * 8)));
  HIPCHK(ensure(ctx, ctx->ldm, mp * 8));
  HIPCHK(ensure(ctx, ctx->ldb, mp * 8));
  HIPCHK(ensure(ctx, ctx->Knm, (size_t)np * mp * 8));
  HIPCHK(ensure(ctx, ctx->q, np * 8));
  HIPCHK(ensure(ctx, ctx->lam, np * 8));
  HIPCHK(ensure(ctx, ctx->ilam, np * 8));
  HIPCHK(ensure(ctx, ctx->ys, np * 8));
  HIPCHK(ensure(ctx, ctx->r, np * 8));
  HIPCHK(ensure(ctx, ctx->g, np * 8));
  HIPCHK(ensure(ctx, ctx->fmu_loo, np * 8));
  HIPCHK(ensure(ctx, ctx->fvar_loo, np * 8));
  HIPCHK(ensure(ctx, ctx->c, mp * 8));
  HIPCHK(ensure(ctx, ctx->tvec, mp * 8));
  // all-reduce buffer [B | b | scalars]: B lower-packed (m(m+1)/2) when the rows are sharded,
  // the padded lower tiles (m_pad²) on one rank
  const bool shard = sharded(ctx);
  const int64_t blen = shard ? m * (m + 1) / 2 : mp * mp;
  const int64_t red_len = mp * mp + mp + 8;
  HIPCHK(ensure(ctx, ctx->red, (size_t)red_len * 8));
  const int64_t nchunk = (std::max(np, mp) + 255) / 256;
  // (row-norm partials tm·np; column passes' chunk partials: Knm's 256-row chunks, and, after
  //  the r pass's first column tiles (formed during B's factorisation), the m×m pass for c in
  //  32-row chunks)
  const int64_t fslab_len = std::max<int64_t>(std::max<int64_t>(tm * np, nchunk * mp * 2),
                                              tm * np + (mp + 31) / 32 * mp);
  HIPCHK(ensure(ctx, ctx->fslab, (size_t)fslab_len * 8));
  double* red = ctx->red.d();
  double* Bacc = red;
  double* bvec = red + blen;
  double* scal = bvec + mp;  // [Σlogλ, Σy²/λ, Σcrps, Σlogs]
  double* sm = ctx->small.d();        // [logdet_m/2, logdet_b/2, bᵀc]
  int rc;
  if ((rc = reset_info(ctx))) return rc;
  phase_mark(ctx, "start");
  // --- replicated m×m part: K̃mm = K(Z,Z) + 1e-3 I (KF:36), Lm⁻¹
  // (built into Am, the factorisation's input, which it overwrites; the copy kept for B's base
  //  and the gradients is a second build on aux[0] beside the factorisation when that stream is
  //  in use — the same kernel on the same inputs, so the same bits — else a copy here)
  if ((rc = gram(ctx, "gram_kmm", ctx->Z.d(), (int)m, ctx->Z.d(), (int)m, ctx->fd, th, 1e-3, 0, 1,
                 ctx->Am.d(), mp, (int)mp, (int)mp)))
    return rc;
  // (a persistent top level has no recursion step to overlap the pre-pass with)
  const bool preq = ctx->pred_pre && mp > GPS_TILE && !dag_block(ctx, mp / GPS_TILE);
  // this shard's rows of K(X, Z): with a pre-pass, first on the main stream (the q column tiles
  // [0, n1) then run on aux[0] inside Lm's captured factorisation, as soon as the top-level
  // Lm11⁻¹ is final); without one, on aux[0] beside Lm's factorisation, whose persistent blocks
  // leave half the CUs free (it needs only X, Z), joined before the q pass
  const bool kside = !preq && ctx->overlap && !ctx->prof;
  // one persistent launch per m×m factorisation: the q and r row norms behind it (GPS_OPT_FITC_DEP)
  const bool dep = kside && ctx->fitc_dep && dag_block(ctx, tm);
  // a recursive m×m factorisation whose top-level L11 is one persistent launch: the q pre-pass
  // over L11⁻¹'s columns behind that launch (potrf_inv_rec, C5) when the pre-pass is at most 8192
  // tiles — about what the CUs beside the launch finish while it runs; a larger one would run
  // on at the dependent launch's column-by-column rate, below the paired order's.  Measured
  // (DESIGN §6.49): C5's rows per rank at N = 8 / 4 (3136 / 6256 tiles) 28.88 → 28.76 / 49.01 →
  // 48.81 ms, at N = 2 / 1 (12 512 / 25 008) 89.38 → 90.51 / 169.8 → 170.7
  const bool pdep = preq && ctx->fitc_dep && ctx->overlap && !ctx->prof &&
                    dag_block(ctx, tm / 2) && (np / GPS_TILE) * (tm / 2) <= 8192;
  int* sig_m = nullptr;
  int* sig_b = nullptr;
  // ... and the r pre-pass behind Lb's top L11 block the same way when it is at most 4096 tiles
  // (once the dependent take was cheap, §6.46: C5r8, 3136 tiles, 27.18-27.28 → 27.05 ms; C5r4,
  // 6256 tiles, 47.35-47.46 → 47.74-47.85; profiles/r6ae_fitc_rpre_dep_ab.txt)
  const bool pdep_b = pdep && (np / GPS_TILE) * (tm / 2) <= 4096;
  if (dep || pdep) {  // (zeroed, stream-ordered before both launches of the pair)
    HIPCHK(ensure(ctx, ctx->dsig, 2 * kSigInts * sizeof(int)));
    sig_m = static_cast<int*>(ctx->dsig.p);
    sig_b = sig_m + kSigInts;
    HIPCHK(hipMemsetAsync(ctx->dsig.p, 0, 2 * kSigInts * sizeof(int), s));
  }
  if (kside) {  // (dedicated events: the factorisation reuses its pool of sync events)
    for (hipEvent_t* e : {&ctx->kn_fork, &ctx->kn_join})
      if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->kn_fork, s));
    HIPCHK(hipStreamWaitEvent(ctx->aux[0], ctx->kn_fork, 0));
    if ((rc = gram(ctx, "gram_kmm", ctx->Z.d(), (int)m, ctx->Z.d(), (int)m, ctx->fd, th, 1e-3, 0,
                   1, ctx->Kmm.d(), mp, (int)mp, (int)mp, ctx->aux[0])))
      return rc;
  } else {
    HIPCHK(hipMemcpyAsync(ctx->Kmm.p, ctx->Am.p, (size_t)mp * mp * 8, hipMemcpyDeviceToDevice, s));
  }
  if ((rc = gram(ctx, "gram_knm", ctx->fX.d(), (int)n, ctx->Z.d(), (int)m, ctx->fd, th, 0.0, 0, 0,
                 ctx->Knm.d(), mp, (int)np, (int)mp, kside ? ctx->aux[0] : nullptr)))
    return rc;
  // q_i = ‖Lm⁻¹ k_i‖² behind Lm's factorisation, on aux[0] after Knm (the dependent launch)
  if (dep && (rc = fitc_rowsq_dep(ctx, ctx->Lm.d(), sig_m, mp, 1, ctx->aux[0], tm))) {
    (void)hipStreamWaitEvent(s, ctx->kn_join, 0);
    return rc;
  }
  if (kside) HIPCHK(hipEventRecord(ctx->kn_join, ctx->aux[0]));
  const int64_t qn1 = preq ? (mp / GPS_TILE / 2) * GPS_TILE : 0;
  ctx->pre.kind = preq ? PRE_FITC_Q : PRE_NONE;
  ctx->pre.n1 = qn1;
  ctx->pre.L = ctx->Lm.d();
  ctx->pre.sig = pdep ? sig_m : nullptr;
  ctx->dag_half = true;  // (the FITC m×m factorisations: see potrf_inv_rec's width)
  ctx->dag_sig = dep ? sig_m : nullptr;
  rc = potrf_inv(ctx, ctx->Am.d(), mp, ctx->Lm.d(), ctx->W.d(), ctx->ldm.d(), (int)m, nullptr);
  ctx->dag_sig = nullptr;
  ctx->pre.sig = nullptr;
  ctx->dag_half = false;
  ctx->pre.kind = PRE_NONE;
  phase_mark(ctx, "kmm_lm");
  if (kside) HIPCHK(hipStreamWaitEvent(s, ctx->kn_join, 0));  // (before any return: Knm in flight)
  if (rc) return rc;
  phase_mark(ctx, "knm");
  HIPCHK(launch_dot(ctx->ldm.d(), nullptr, (int)mp, sm + 0, s));
  // q_i = ‖Lm⁻¹ k_i‖²: the tiles the dependent launch left, or the remaining column tiles
  if ((rc = dep ? fitc_rowsq_dep(ctx, ctx->Lm.d(), sig_m, mp, 2, s, tm)
                : fitc_rowsq_cols(ctx, ctx->Lm.d(), qn1, mp, s)))
    return rc;
  double* part = row_part(ctx, np, 2);
  ARGCHK(part != nullptr, "out of device memory");
  {  // q = Σ of the row-norm partials, fused with Λ (one thread per row, many workgroups)
    Prof pr(ctx, "fitc_lambda", 0, 0);
    HIPCHK(launch_fitc_lambda(ctx->fslab.d(), np, (int)tm, ctx->fy.d(), (int)n, (int)np, th.sf2,
                              th.sn2, ctx->q.d(), ctx->lam.d(), ctx->ilam.d(), ctx->ys.d(), scal,
                              part, s));
  }
  phase_mark(ctx, "q");
  // b_p = Kmnᵀ Λ⁻¹ y: one rank, an HBM-bound pass on aux[1] beside the SYRK (b is first read
  // by c = B⁻¹b after B's factorisation); sharded, it travels in the all-reduce with B
  const bool bside = !shard && ctx->overlap && !ctx->prof;
  if (bside) {
    for (hipEvent_t* e : {&ctx->b_fork, &ctx->b_join})
      if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->b_fork, s));
    HIPCHK(hipStreamWaitEvent(ctx->aux[1], ctx->b_fork, 0));
  }
  {
    hipStream_t bs = bside ? ctx->aux[1] : s;
    Prof pr(ctx, "colred_b", 0, 8.0 * np * mp, bs);
    HIPCHK(launch_colred(ctx->Knm.d(), mp, (int)np, (int)mp, 0, ctx->ys.d(), nullptr, bvec,
                         nullptr, ctx->fslab.d(), bs));
  }
  if (bside) HIPCHK(hipEventRecord(ctx->b_join, ctx->aux[1]));
  // B_p = Kmnᵀ Λ⁻¹ Knm (lower tiles, split-K slabs); sharded: packed and all-reduced with b,
  // Σlogλ, Σy²/λ, in row blocks overlapped with the SYRK (ctx->ar_chunks); one
  // rank: the slab sum adds K̃mm and writes B = K̃mm + Σ slabs straight into Am (one launch)
  if (shard) {
    if ((rc = fitc_syrk_allreduce(ctx, red, blen, mp + 2))) return rc;
  } else if ((rc = fitc_syrk(ctx, ctx->ilam.d(), ctx->Kmm.d(), ctx->Am.d(), false))) {
    if (bside) (void)hipStreamWaitEvent(s, ctx->b_join, 0);
    return rc;
  } else {
    phase_mark(ctx, "syrk");
  }
  if (bside) HIPCHK(hipStreamWaitEvent(s, ctx->b_join, 0));
  if (pre_test && ctx->f_test && ctx->fnt > 0 && ctx->overlap && !ctx->prof)
    if ((rc = fitc_test_prepass(ctx))) return rc;
  // --- B = K̃mm + Σ_p B_p, factor redundantly on every rank
  if (shard) HIPCHK(launch_sym_unpack(Bacc, (int)m, (int)mp, ctx->Kmm.d(), 0, ctx->Am.d(), s));
  // (the r pass's column tiles [0, qn1), like q's, as soon as the top-level Lb11⁻¹ is final)
  ctx->pre.kind = preq ? PRE_FITC_Q : PRE_NONE;
  ctx->pre.n1 = qn1;
  ctx->pre.L = ctx->Lb.d();
  ctx->pre.sig = pdep_b ? sig_b : nullptr;
  // (the r pass behind Lb's factorisation as well — every column tile on aux[1], g = Knm c by a GEMV
  //  after c — measured no faster: C4 11.84 vs 11.80 ms, profiles/r6b_fitc_dep_ab_c4.txt; the CUs
  //  Lb's factorisation leaves already run the test-side q* norms)
  ctx->dag_half = true;
  rc = potrf_inv(ctx, ctx->Am.d(), mp, ctx->Lb.d(), ctx->W.d(), ctx->ldb.d(), (int)m, nullptr);
  ctx->dag_half = false;
  ctx->pre.kind = PRE_NONE;
  ctx->pre.sig = nullptr;
  if (rc) return rc;
  phase_mark(ctx, "lb");
  HIPCHK(launch_dot(ctx->ldb.d(), nullptr, (int)mp, sm + 1, s));
  {  // c = Lb⁻ᵀ Lb⁻¹ b
    Prof pr(ctx, "fitc_c", 0, 0);
    HIPCHK(launch_gemv_lower(ctx->Lb.d(), mp, bvec, ctx->tvec.d(), (int)mp, s));
    // (32-row chunks: an m×m pass has few 256-row chunks, 32 workgroups at m = 2048; fslab
    //  holds the m/32 chunk partials)
    HIPCHK(launch_colred(ctx->Lb.d(), mp, (int)mp, (int)mp, 1, ctx->tvec.d(), nullptr, ctx->c.d(),
                         nullptr, ctx->fslab.d() + tm * np, s, 32));
    HIPCHK(launch_dot(bvec, ctx->c.d(), (int)mp, sm + 2, s));
  }
  phase_mark(ctx, "c");
  if (ctx->f_pre && (rc = fitc_test_prepass_b(ctx))) return rc;
  {  // r_i = ‖Lb⁻¹ k_i‖² (the column tiles [qn1, mp): the rest came with B's factorisation),
            // and g = Knm c from the same pass over Knm (its last column tile spans the whole K range)
    GemmParams p = gp0();
    p.A = ctx->Knm.d(); p.lda = mp; p.B = ctx->Lb.d() + qn1 * mp; p.ldb = mp;
    p.M = (int)np; p.N = (int)(mp - qn1); p.K = (int)mp; p.tri = TRI_K_LE_J; p.tri_off = (int)qn1;
    p.kend = (int)pad_to(m, 16);
    p.out0 = ctx->fslab.d() + (qn1 / GPS_TILE) * np; p.ld_out = np;
    p.w = ctx->c.d(); p.out1 = ctx->g.d();
    if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_ROWSQ_DOT, p))) return rc;
  }
  {  // r = Σ of the row-norm partials, fused with the LOO terms
    part = row_part(ctx, np, 2);
    ARGCHK(part != nullptr, "out of device memory");
    Prof pr(ctx, "fitc_loo", 0, 0);
    HIPCHK(launch_fitc_loo(ctx->fy.d(), ctx->lam.d(), ctx->fslab.d(), np, (int)tm, ctx->g.d(),
                           (int)n, (int)np, ctx->r.d(), ctx->fmu_loo.d(), ctx->fvar_loo.d(),
                           scal + 2, part, s));
  }
  phase_mark(ctx, "r");
  if ((rc = allreduce_sum(ctx, scal + 2, 2, s))) return rc;
  phase_mark(ctx, "scal");
  // the pre-pass reads the test inputs: it is done before this call returns (it finished long
  // before on the timeline — B's factorisation and the r pass came after its launch)
  if (ctx->f_pre) HIPCHK(hipStreamWaitEvent(s, ctx->pre_join, 0));
  HIPCHK(hipMemcpyAsync(ctx->hsmall, scal, 4 * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(ctx->hsmall + 4, sm, 3 * 8, hipMemcpyDeviceToHost, s));
  if ((rc = check_info(ctx))) return rc;
  const double* h = ctx->hsmall;
  const double N = (double)ctx->fn_total;
  const double logdet = h[0] + 2.0 * h[5] - 2.0 * h[4];
  const double quad = h[1] - h[6];
  if (obj) {
    obj[GPS_OBJ_NLML] = 0.5 * N * 1.83787706640934548356 + 0.5 * logdet + 0.5 * quad;
    obj[GPS_OBJ_LOO_CRPS] = h[2] / N;
    obj[GPS_OBJ_LOO_LOGS] = h[3] / N;
    obj[GPS_OBJ_LOGDET] = logdet;
    obj[GPS_OBJ_QUAD] = quad;
  }
  return 0;
}

int gps_fitc_fit(gps_ctx* ctx, const double* theta, int n_ell, double obj[GPS_N_OBJ],
                 double* mu_loo, double* var_loo) {
  if (int rc = bind(ctx)) return rc;
  if (int rc = fitc_fit_core(ctx, theta, n_ell, obj, true)) return rc;
  const int64_t n = ctx->fn;
  hipStream_t s = ctx->stream;
  if (mu_loo) HIPCHK(hipMemcpyAsync(mu_loo, ctx->fmu_loo.p, n * 8, hipMemcpyDeviceToHost, s));
  if (var_loo) HIPCHK(hipMemcpyAsync(var_loo, ctx->fvar_loo.p, n * 8, hipMemcpyDeviceToHost, s));
  if (mu_loo || var_loo) HIPCHK(hipStreamSynchronize(s));
  ctx->f_fitted = true;
  return 0;
}

// Whitened FITC gradient products (round 4; gps_fitc_grad, gps_fitc_blockloo).  The stored
// factors ctx->Lm / ctx->Lb are the lower triangular inverses Lm⁻¹, Lb⁻¹ (m_pad², strict-upper
// zero).  C (n_pad × m_pad, ldc) = Knm · Xᵀ for such an X: V = K Lm⁻ᵀ, U = K Lb⁻ᵀ.
int fitc_knm_xt(gps_ctx* ctx, int64_t ldc, const double* X, double* C) {
  const int64_t mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = ctx->Knm.d(); p.lda = mp; p.B = X; p.ldb = mp; p.C = C; p.ldc = ldc;
  p.M = (int)ctx->fn_pad; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_LE_J;
  return gemm(ctx, LAY_N, LAY_T, EPI_STORE, p);
}
// y (m_pad) = Xᵀ x for a stored lower X (m_pad²): the column reductions of X weighted by x, in
// 256-row chunks through fslab (one chunk per 256 rows when fslab holds their partials)
int fitc_lt_vec(gps_ctx* ctx, const double* X, const double* x, double* y) {
  const int64_t mp = ctx->m_pad;
  const int64_t cap = (int64_t)(ctx->fslab.cap / 8);
  int crows = 256;
  while ((mp + crows - 1) / crows * mp * 2 > cap) crows *= 2;
  HIPCHK(launch_colred(X, mp, (int)mp, (int)mp, 0, x, nullptr, y, nullptr, ctx->fslab.d(),
                       ctx->stream, crows));
  return 0;
}
// C (rows × m_pad) = A · X, X lower (k >= j)
int fitc_tri_right(gps_ctx* ctx, const double* A, int64_t lda, const double* X, double* C,
                          int64_t ldc, int64_t rows) {
  const int64_t mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = A; p.lda = lda; p.B = X; p.ldb = mp; p.C = C; p.ldc = ldc;
  p.M = (int)rows; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_GE_J;
  return gemm(ctx, LAY_N, LAY_N, EPI_STORE, p);
}
// C (m_pad²) = Xᵀ · B, X lower
int fitc_tri_left_t(gps_ctx* ctx, const double* X, const double* B, double* C) {
  const int64_t mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = X; p.lda = mp; p.B = B; p.ldb = mp; p.C = C; p.ldc = mp;
  p.M = (int)mp; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_GE_I;
  return gemm(ctx, LAY_T, LAY_N, EPI_STORE, p);
}

// Objective value + analytic gradient of the FITC objectives w.r.t. θ and the inducing
// inputs Z — the reference's fwd + `.backward()` at K20:236 (LOO-CRPS), K20:344 (NLML),
// K20:452 (LOO-LogS); Z is a trained parameter there (K20:247).  Formulas: header of
// kernels_fitc_grad.hip / oracle.fast_fitc_grad.  Work beyond the forward: two m×m
// LAUUMs, K·[B⁻¹ | N | Km⁻¹] (6nm² flops; NLML skips N), one or two split-K SYRKs
// (nm² each), 2-4 m³ GEMMs, and the HBM-bound contraction (reads the n×3m product once).
// Row-sharded across ranks like the forward: m-vectors, m×m SYRKs and the contraction
// partials are all-reduced; the m×m (Kmm) contraction is replicated.
int gps_fitc_grad(gps_ctx* ctx, const double* theta, int n_ell, int objective,
                  double obj[GPS_N_OBJ], double* grad, double* grad_z) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(grad != nullptr, "grad is NULL");
  ARGCHK(objective == GPS_OBJ_NLML || objective == GPS_OBJ_LOO_CRPS ||
             objective == GPS_OBJ_LOO_LOGS,
         "objective must be GPS_OBJ_NLML, GPS_OBJ_LOO_CRPS or GPS_OBJ_LOO_LOGS");
  double o[GPS_N_OBJ];
  int rc;
  if ((rc = fitc_fit_core(ctx, theta, n_ell, o))) return rc;
  ctx->f_fitted = true;
  const Theta& th = ctx->fth;
  const int64_t n = ctx->fn, np = ctx->fn_pad, m = ctx->m, mp = ctx->m_pad;
  const int d = ctx->fd;
  hipStream_t s = ctx->stream;
  const bool loo = objective != GPS_OBJ_NLML;
  const double a = loo ? 0.0 : 0.5;
  // scratch
  HIPCHK(ensure(ctx, ctx->fgv, (size_t)11 * np * 8));
  HIPCHK(ensure(ctx, ctx->fgm, (size_t)6 * mp * 8));
  const bool shard = sharded(ctx);
  HIPCHK(ensure(ctx, ctx->fgB, (size_t)(shard ? 6 : 5) * mp * mp * 8));
  HIPCHK(ensure(ctx, ctx->fR, (size_t)np * 3 * mp * 8));
  HIPCHK(ensure(ctx, ctx->fgred, (size_t)(mp * mp + 2 * mp + 64) * 8));
  const int passes = fitc_contract_passes(d);
  const int64_t outlen = (int64_t)passes * 17 + m * d;
  HIPCHK(ensure(ctx, ctx->fgslab, (size_t)std::max(fitc_contract_slab_doubles((int)n, (int)mp, d),
                                               fitc_contract_slab_doubles((int)m, (int)mp, d)) * 8));
  HIPCHK(ensure(ctx, ctx->fgout, (size_t)(2 * outlen + 8) * 8));
  double* vbase = ctx->fgv.d();
  double *alpha = vbase, *dinv = vbase + np, *v = vbase + 2 * np, *ulam = vbase + 3 * np,
         *h = vbase + 4 * np, *hl2 = vbase + 5 * np, *md = vbase + 6 * np, *s1 = vbase + 7 * np,
         *s2 = vbase + 8 * np, *s3 = vbase + 9 * np, *zv = vbase + 10 * np;
  double* mb = ctx->fgm.d();
  double *tku = mb, *what = mb + 2 * mp;
  double* Bb = ctx->fgB.d();
  double *Binv = Bb, *Kminv = Bb + mp * mp, *Nm = Bb + 2 * mp * mp, *T1 = Bb + 3 * mp * mp,
         *KmD = Bb + 4 * mp * mp;
  // all-reduce buffer [P | Σ M_ii | (pad) | Kᵀv (mp)]: P an m×m SYRK, lower-packed (m(m+1)/2)
  // when the rows are sharded, else the padded lower tiles (m_pad²)
  const int64_t plen = shard ? m * (m + 1) / 2 : mp * mp;
  const int64_t off_tw = (plen + 2) / 2 * 2;  // 16-byte aligned
  double* red = ctx->fgred.d();
  double* smd = red + plen;
  double* tw = red + off_tw;
  double* Sfull = shard ? Bb + 5 * mp * mp : red;  // the reduced P, both triangles
  auto sym_full = [&]() -> int {
    if (shard) HIPCHK(launch_sym_unpack(red, (int)m, (int)mp, nullptr, 1, Sfull, s));
    else HIPCHK(launch_sym_mirror(red, mp, (int)mp, s));
    return 0;
  };
  double* out1 = ctx->fgout.d();        // Knm contraction [passes*17 | m*d]
  double* out2 = out1 + outlen;         // Kmm contraction
  double* R = ctx->fR.d();
  const int64_t ldr = 3 * mp;
  HIPCHK(launch_fitc_grad_terms(ctx->fy.d(), ctx->lam.d(), ctx->r.d(), ctx->g.d(), (int)n, (int)np,
                                objective, (double)ctx->fn_total, alpha, dinv, v, ulam, h, hl2, s));
  // Whitened (round 4, oracle.fast_fitc_grad): the operands are V = K Lm⁻ᵀ (R slot 2) and
  // U = K Lb⁻ᵀ (slot 0), whose rows are bounded (‖V_i‖² = q_i ≤ sf², ‖U_i‖² = r_i); the explicit
  // Km⁻¹ and B⁻¹ of round 3 (K·Km⁻¹, K·B⁻¹S2B⁻¹) amplified rounding by cond(B) ~1e7 on
  // near-duplicate inducing points.
  //   G_K  = Y Lb⁻¹ + diag(s3) V Lm⁻¹ − v cᵀ − α ŵᵀ,  Y = diag(s1) U + diag(s2) U P,
  //   G_Km = −a(Km⁻¹ − B⁻¹) + Lb⁻ᵀ P Lb⁻¹ + Lm⁻ᵀ(Vᵀdiag(M_ii)V)Lm⁻¹ + ½(ŵcᵀ + cŵᵀ),
  //   P = Uᵀ diag(h/λ²) U,  ŵ = Lm⁻ᵀ(Vᵀv),  v = u/λ − U(Uᵀ(u/λ))/λ.
  double* U = R;
  double* Yp = R + mp;
  double* V = R + 2 * mp;
  if ((rc = fitc_knm_xt(ctx, ldr, ctx->Lb.d(), U))) return rc;
  if ((rc = fitc_knm_xt(ctx, ldr, ctx->Lm.d(), V))) return rc;
  if (loo) {  // v = C⁻¹u = u/λ − U(Uᵀ(u/λ))/λ;  P = Uᵀ diag(h/λ²) U
    HIPCHK(launch_colred(U, ldr, (int)np, (int)mp, 0, ulam, nullptr, tku, nullptr, ctx->fslab.d(), s));
    if ((rc = allreduce_sum(ctx, tku, (size_t)mp, s))) return rc;
    HIPCHK(launch_gemv_full(U, ldr, tku, zv, (int)np, (int)mp, s));
    HIPCHK(launch_fitc_grad_v(ulam, zv, ctx->lam.d(), (int)n, v, s));
    if ((rc = fitc_syrk(ctx, hl2, nullptr, red, shard, U, ldr))) return rc;
  }
  HIPCHK(launch_colred(V, ldr, (int)np, (int)mp, 0, v, nullptr, tw, nullptr, ctx->fslab.d(), s));
  {  // LOO: [P | (Σ M_ii, not yet formed) | Vᵀv] in one call; NLML: Vᵀv.  Vᵀv is final here.
    double* r0 = loo ? red : tw;
    const size_t cnt = loo ? (size_t)(off_tw + mp) : (size_t)mp;
    if ((rc = allreduce_sum(ctx, r0, cnt, s))) return rc;
  }
  if ((rc = fitc_lt_vec(ctx, ctx->Lm.d(), tw, what))) return rc;  // ŵ = Lm⁻ᵀ Vᵀv
  auto gemm_nn = [&](const double* A, int64_t lda, const double* B, double* C, int64_t ldc,
                     int M) -> int {
    GemmParams p = gp0();
    p.A = A; p.lda = lda; p.B = B; p.ldb = mp; p.C = C; p.ldc = ldc;
    p.M = M; p.N = (int)mp; p.K = (int)mp;
    return gemm(ctx, LAY_N, LAY_N, EPI_STORE, p);
  };
  if (loo) {  // U P (slot 1) and N = Lb⁻ᵀ P Lb⁻¹ while P is in the reduction buffer
    if ((rc = sym_full())) return rc;
    if ((rc = gemm_nn(U, ldr, Sfull, Yp, ldr, (int)np))) return rc;
    if ((rc = fitc_tri_right(ctx, Sfull, mp, ctx->Lb.d(), T1, mp, mp))) return rc;
    if ((rc = fitc_tri_left_t(ctx, ctx->Lb.d(), T1, Nm))) return rc;
  }
  {
    Prof pr(ctx, "fitc_grad_mdiag", 0, (loo ? 16.0 : 0.0) * np * mp);
    HIPCHK(launch_fitc_grad_mdiag(loo ? Yp : nullptr, ldr, U, ldr, (int)mp, ctx->lam.d(), ctx->r.d(),
                                  dinv, alpha, v, loo ? h : nullptr, a, (int)n, (int)np, md, s1, s2,
                                  s3, s));
  }
  // Y = diag(s1) U + diag(s2) U P (in slot 1), then Y Lb⁻¹ into slot 0 (U is done)
  HIPCHK(launch_fitc_grad_y(U, loo ? Yp : nullptr, ldr, s1, s2, (int)np, (int)mp, Yp, s));
  if ((rc = fitc_tri_right(ctx, Yp, ldr, ctx->Lb.d(), U, ldr, np))) return rc;
  // Vᵀ diag(M_ii) V and Σ M_ii (this shard) → all-reduce;  then V Lm⁻¹ into slot 1
  if ((rc = fitc_syrk(ctx, md, nullptr, red, shard, V, ldr))) return rc;
  HIPCHK(launch_dot(md, nullptr, (int)np, smd, s));
  if ((rc = allreduce_sum(ctx, red, (size_t)(plen + 1), s))) return rc;  // [P2 | Σ M_ii], not Vᵀv
  if ((rc = fitc_tri_right(ctx, V, ldr, ctx->Lm.d(), Yp, ldr, np))) return rc;
  if ((rc = sym_full())) return rc;
  if ((rc = fitc_tri_right(ctx, Sfull, mp, ctx->Lm.d(), T1, mp, mp))) return rc;
  if ((rc = fitc_tri_left_t(ctx, ctx->Lm.d(), T1, KmD))) return rc;
  if (a != 0.0) {  // NLML: B⁻¹ = Lb⁻ᵀLb⁻¹, Km⁻¹ = Lm⁻ᵀLm⁻¹ (LAUUM, lower tiles) + mirror
    const double* Ls[2] = {ctx->Lb.d(), ctx->Lm.d()};
    double* Is[2] = {Binv, Kminv};
    for (int w = 0; w < 2; ++w) {
      GemmParams p = gp0();
      p.A = Ls[w]; p.lda = mp; p.B = Ls[w]; p.ldb = mp; p.C = Is[w]; p.ldc = mp;
      p.M = (int)mp; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_GE_I; p.lower_out = 1;
      if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p))) return rc;
      HIPCHK(launch_sym_mirror(Is[w], mp, (int)mp, s));
    }
  }
  // contraction with ∂Knm/∂θ, ∂Knm/∂Z
  FitcContractParams cp;
  memset(&cp, 0, sizeof(cp));
  cp.d = d;
  cp.sf2 = th.sf2;
  for (int k = 0; k < d; ++k) cp.inv_ell[k] = th.inv_ell[k];
  cp.slab = ctx->fgslab.d();
  {
    FitcContractParams p = cp;
    p.xr = ctx->fX.d(); p.xc = ctx->Z.d(); p.nr = (int)n; p.nc = (int)m; p.nc_pad = (int)mp;
    p.R[p.nt] = U; p.ldr[p.nt] = ldr; p.coef[p.nt++] = 1.0;                      // Y Lb⁻¹
    p.R[p.nt] = Yp; p.ldr[p.nt] = ldr; p.coef[p.nt] = 1.0; p.rs[p.nt++] = s3;    // V Lm⁻¹
    p.pc[0] = -1.0; p.pv[0] = v; p.qv[0] = ctx->c.d();
    p.pc[1] = -1.0; p.pv[1] = alpha; p.qv[1] = what;
    Prof pr(ctx, "fitc_grad_contract", 0, 8.0 * 2 * np * mp);
    HIPCHK(launch_fitc_grad_contract(p, out1, out1 + passes * 17, s));
  }
  if ((rc = allreduce_sum(ctx, out1, (size_t)outlen, s))) return rc;
  {  // ∂Km/∂θ, ∂Km/∂Z (replicated on every rank; jitter is a constant)
    FitcContractParams p = cp;
    p.xr = ctx->Z.d(); p.xc = ctx->Z.d(); p.nr = (int)m; p.nc = (int)m; p.nc_pad = (int)mp;
    if (a != 0.0) {
      p.R[p.nt] = Binv; p.ldr[p.nt] = mp; p.coef[p.nt++] = a;
      p.R[p.nt] = Kminv; p.ldr[p.nt] = mp; p.coef[p.nt++] = -a;
    }
    if (loo) { p.R[p.nt] = Nm; p.ldr[p.nt] = mp; p.coef[p.nt++] = 1.0; }
    p.R[p.nt] = KmD; p.ldr[p.nt] = mp; p.coef[p.nt++] = 1.0;
    p.pc[0] = 0.5; p.pv[0] = what; p.qv[0] = ctx->c.d();
    p.pc[1] = 0.5; p.pv[1] = ctx->c.d(); p.qv[1] = what;
    Prof pr(ctx, "fitc_grad_contract_mm", 0, 8.0 * p.nt * mp * mp);
    HIPCHK(launch_fitc_grad_contract(p, out2, out2 + passes * 17, s));
  }
  std::vector<double> hout((size_t)2 * outlen + 1);
  HIPCHK(hipMemcpyAsync(hout.data(), out1, (size_t)2 * outlen * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hout.data() + 2 * outlen, smd, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const double* h1 = hout.data();
  const double* h2 = h1 + outlen;
  const double sum_md = hout[2 * outlen];
  if (obj)
    for (int q = 0; q < GPS_N_OBJ; ++q) obj[q] = o[q];
  grad[0] = h1[0] + h2[0] + th.sf2 * sum_md;
  double tot = 0.0;
  for (int k = 0; k < d; ++k) {
    const size_t at = (size_t)(k / 16) * 17 + 1 + (k % 16);
    const double gk = h1[at] + h2[at];
    if (n_ell == d) grad[1 + k] = gk;
    tot += gk;
  }
  if (n_ell == 1) grad[1] = tot;
  grad[1 + n_ell] = th.sn2 * sum_md;
  if (grad_z) {
    const double* z1 = h1 + passes * 17;
    const double* z2 = h2 + passes * 17;
    for (int64_t j = 0; j < m; ++j)
      for (int k = 0; k < d; ++k)
        grad_z[j * d + k] = (z1[j * d + k] + 2.0 * z2[j * d + k]) * th.inv_ell[k];
  }
  return 0;
}


int gps_fitc_intermediates(gps_ctx* ctx, double* Knm, double* lam, double* Lm_inv, double* Lb_inv,
                           double* Kmm) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(ctx->f_fitted, "gps_fitc_fit first");
  const int64_t n = ctx->fn, m = ctx->m, mp = ctx->m_pad;
  hipStream_t s = ctx->stream;
  HIPCHK(hipStreamSynchronize(s));
  auto rows = [&](const DBuf& b, double* dst, int64_t r) -> hipError_t {
    return hipMemcpy2DAsync(dst, (size_t)m * 8, b.p, (size_t)mp * 8, (size_t)m * 8, (size_t)r,
                            hipMemcpyDeviceToHost, s);
  };
  if (Knm) HIPCHK(rows(ctx->Knm, Knm, n));
  if (lam) HIPCHK(hipMemcpyAsync(lam, ctx->lam.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
  if (Lm_inv) HIPCHK(rows(ctx->Lm, Lm_inv, m));
  if (Lb_inv) HIPCHK(rows(ctx->Lb, Lb_inv, m));
  if (Kmm) HIPCHK(rows(ctx->Kmm, Kmm, m));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

int gps_fitc_predict(gps_ctx* ctx, double* mu, double* var, double sc[GPS_N_SC]) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(ctx->f_fitted, "gps_fitc_fit first");
  ARGCHK(ctx->f_test, "gps_fitc_set_test first");
  const Theta& th = ctx->fth;
  const int64_t nt = ctx->fnt, ntp = ctx->fnt_pad, m = ctx->m, mp = ctx->m_pad;
  const int64_t tm = mp / GPS_TILE;
  hipStream_t s = ctx->stream;
  HIPCHK(ensure(ctx, ctx->Ksm, (size_t)ntp * mp * 8));
  HIPCHK(ensure(ctx, ctx->qm, ntp * 8));
  HIPCHK(ensure(ctx, ctx->qb, ntp * 8));
  HIPCHK(ensure(ctx, ctx->fmu, ntp * 8));
  HIPCHK(ensure(ctx, ctx->fvar, ntp * 8));
  HIPCHK(ensure(ctx, ctx->fslab, std::max(ctx->fslab.cap, (size_t)tm * ntp * 8)));
  double* sums = ctx->small.d() + 8;
  int rc;
  const bool pre = ctx->f_pre;  // K*m and q* came with the fit (fitc_test_prepass)
  const int wend = ctx->f_pre_b ? 1 : 2;  // ... and q*b (fitc_test_prepass_b)
  if (pre) {
    HIPCHK(hipStreamWaitEvent(s, ctx->pre_join, 0));
  } else if ((rc = gram(ctx, "gram_ksm", ctx->fXt.d(), (int)nt, ctx->Z.d(), (int)m, ctx->fd, th,
                        0.0, 0, 0, ctx->Ksm.d(), mp, (int)ntp, (int)mp))) {
    return rc;
  }
  const double* Ls[2] = {ctx->Lm.d(), ctx->Lb.d()};
  double* outs[2] = {ctx->qm.d(), ctx->qb.d()};
  for (int w = pre ? 1 : 0; w < wend; ++w) {
    GemmParams p = gp0();
    p.A = ctx->Ksm.d(); p.lda = mp; p.B = Ls[w]; p.ldb = mp;
    p.M = (int)ntp; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_LE_J;
    p.kend = (int)pad_to(ctx->m, 16);
    p.out0 = ctx->fslab.d(); p.ld_out = ntp;
    if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_ROWSQ, p))) return rc;
    HIPCHK(launch_slab_sum(ctx->fslab.d(), ntp, (int)tm, ntp, nullptr, outs[w], s));
  }
  {
    Prof pr(ctx, "fitc_pred_finalize", 0, 8.0 * ntp * mp);
    HIPCHK(launch_gemv_full(ctx->Ksm.d(), mp, ctx->c.d(), ctx->fmu.d(), (int)ntp, (int)mp, s));
    if (nt > 0)  // a rank may hold no test rows; its zero score partials still join the sum
      HIPCHK(launch_fitc_pred_finalize(ctx->qm.d(), ctx->qb.d(), (int)nt, th.sn2 + th.sf2,
                                       ctx->fvar.d(), s));
  }
  {  // the score phase (KF:276-292): its own profiling tag
    Prof pr(ctx, "score_sums", 0, 24.0 * nt);
    double* part = row_part(ctx, nt, 6);
    ARGCHK(part != nullptr, "out of device memory");
    if (nt > 0)
      HIPCHK(launch_score_sums(ctx->fmu.d(), ctx->fvar.d(), ctx->fyt.d(), (int)nt, ctx->f_ytr_mean,
                               ctx->f_ytr_var, sums, part, s));
    else
      HIPCHK(hipMemsetAsync(sums, 0, 6 * 8, s));
  }
  if (int rc2 = allreduce_sum(ctx, sums, 6, s)) return rc2;
  HIPCHK(hipMemcpyAsync(ctx->hsmall, sums, 6 * 8, hipMemcpyDeviceToHost, s));
  if (mu && nt) HIPCHK(hipMemcpyAsync(mu, ctx->fmu.p, nt * 8, hipMemcpyDeviceToHost, s));
  if (var && nt) HIPCHK(hipMemcpyAsync(var, ctx->fvar.p, nt * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (sc) score_bundle(ctx->hsmall, (double)ctx->fnt_total, sc);
  return 0;
}

}  // extern "C"
