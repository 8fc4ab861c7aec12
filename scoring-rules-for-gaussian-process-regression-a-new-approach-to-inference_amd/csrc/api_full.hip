// C-ABI, full GP: data, fit (NLML / LOO-CRPS / LOO-LogS), analytic gradients, predict +
// score (KF:239-292, 329-339, 416-428), and the contour-plot.R objective surfaces (CP.R:43-141).
#include "api_internal.h"

extern "C" {

// ------------------------------------------------------------------- full GP
int gps_full_set_data(gps_ctx* ctx, const double* X, const double* y, int64_t n, int d) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(X && y && n > 1 && d >= 1 && d <= GPS_MAX_D, "bad training data");
  ARGCHK(n <= (int64_t)1 << 30, "n too large");
  if (d != ctx->d) ctx->have_test = false;  // a test set of another input dimension is void
  ctx->n = n;
  ctx->d = d;
  ctx->n_pad = pad_to(n);
  if (int rc = upload(ctx, ctx->X, X, n, d, ctx->n_pad)) return rc;
  if (int rc = upload(ctx, ctx->y, y, n, 1, ctx->n_pad)) return rc;
  double s = 0, s2 = 0;
  for (int64_t i = 0; i < n; ++i) s += y[i];
  const double mean = s / n;
  for (int64_t i = 0; i < n; ++i) s2 += (y[i] - mean) * (y[i] - mean);
  ctx->ytr_mean = mean;
  ctx->ytr_var = s2 / (n - 1);
  ctx->have_data = true;
  ctx->fitted = false;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gps_full_set_test(gps_ctx* ctx, const double* Xt, const double* yt, int64_t nt) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(ctx->have_data, "gps_full_set_data first");
  ARGCHK(Xt && nt > 0, "bad test data");
  ctx->nt = nt;
  ctx->nt_pad = pad_to(nt);
  if (int rc = upload(ctx, ctx->Xt, Xt, nt, ctx->d, ctx->nt_pad)) return rc;
  std::vector<double> zeros;
  if (!yt) zeros.assign(nt, 0.0);
  if (int rc = upload(ctx, ctx->yt, yt ? yt : zeros.data(), nt, 1, ctx->nt_pad)) return rc;
  ctx->have_test = true;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// Gram + factorisation + β, α, diag(A⁻¹) + LOO sums; objectives land in ctx->small (device)
int full_fit_core(gps_ctx* ctx, int kind, const double* theta, int n_ell) {
  ARGCHK(ctx->have_data, "gps_full_set_data first");
  ctx->fitted = false;  // set again only once the factor is known to be PD (check_info)
  if (int rc = set_theta(ctx, ctx->th, kind, theta, n_ell, ctx->d)) return rc;
  ctx->n_ell = n_ell;
  const int64_t n = ctx->n, np = ctx->n_pad;
  hipStream_t s = ctx->stream;
  HIPCHK(ensure(ctx, ctx->A, (size_t)np * np * 8));
  if (ctx->Linv.cap < (size_t)np * np * 8 || !factor_zeroed(ctx, ctx->Linv.d(), np)) {
    HIPCHK(ensure(ctx, ctx->Linv, (size_t)np * np * 8));
    HIPCHK(zero_factor(ctx, ctx->Linv.d(), np, s));
  }
  HIPCHK(ensure(ctx, ctx->W, potrf_ws_doubles(np) * 8));
  HIPCHK(ensure(ctx, ctx->logdiag, np * 8));
  HIPCHK(ensure(ctx, ctx->beta, np * 8));
  HIPCHK(ensure(ctx, ctx->alpha, np * 8));
  HIPCHK(ensure(ctx, ctx->dinv, np * 8));
  HIPCHK(ensure(ctx, ctx->mu_loo, np * 8));
  HIPCHK(ensure(ctx, ctx->var_loo, np * 8));
  const int64_t nchunk = (np + 255) / 256;
  HIPCHK(ensure(ctx, ctx->slab, (size_t)nchunk * np * 2 * 8));
  int rc;
  if ((rc = reset_info(ctx))) return rc;
  if ((rc = gram(ctx, "gram_kff", ctx->X.d(), (int)n, ctx->X.d(), (int)n, ctx->d, ctx->th,
                 ctx->th.sn2, 1, 1, ctx->A.d(), np, (int)np, (int)np)))
    return rc;
  if ((rc = potrf_inv(ctx, ctx->A.d(), np, ctx->Linv.d(), ctx->W.d(), ctx->logdiag.d(), (int)n,
                      nullptr)))
    return rc;
  {
    Prof pr(ctx, "gemv_beta", 0, 4.0 * (double)np * np);
    HIPCHK(launch_gemv_lower(ctx->Linv.d(), np, ctx->y.d(), ctx->beta.d(), (int)np, s));
  }
  int nchunk_c = 0;
  {  // α = L⁻ᵀβ and diag(A⁻¹) = colsum(L⁻¹∘L⁻¹): one column pass, chunk partials
    Prof pr(ctx, "colred_alpha_dinv", 0, 4.0 * (double)np * np);
    nchunk_c = launch_colred_partials(ctx->Linv.d(), np, (int)np, (int)np, 1, ctx->beta.d(),
                                      ctx->slab.d(), s);
    ARGCHK(nchunk_c > 0, "column pass launch failed");
  }
  {  // chunk sums fused with the LOO rows (one thread per row, many workgroups)
    double* part = row_part(ctx, np, 4);
    ARGCHK(part != nullptr, "out of device memory");
    Prof pr(ctx, "loo_finalize", 0, 0);
    HIPCHK(launch_full_loo(ctx->y.d(), ctx->slab.d(), nchunk_c, np, ctx->beta.d(),
                           ctx->logdiag.d(), (int)n, ctx->alpha.d(), ctx->dinv.d(),
                           ctx->mu_loo.d(), ctx->var_loo.d(), ctx->small.d(), part, s));
  }
  return 0;
}

int gps_full_fit(gps_ctx* ctx, int kind, const double* theta, int n_ell, double obj[GPS_N_OBJ],
                 double* mu_loo, double* var_loo) {
  if (int rc = bind(ctx)) return rc;
  int rc;
  if ((rc = full_fit_core(ctx, kind, theta, n_ell))) return rc;
  const int64_t n = ctx->n;
  hipStream_t s = ctx->stream;
  HIPCHK(hipMemcpyAsync(ctx->hsmall, ctx->small.p, GPS_N_OBJ * 8, hipMemcpyDeviceToHost, s));
  if ((rc = check_info(ctx))) return rc;
  if (obj)
    for (int q = 0; q < GPS_N_OBJ; ++q) obj[q] = ctx->hsmall[q];
  if (mu_loo) HIPCHK(hipMemcpyAsync(mu_loo, ctx->mu_loo.p, n * 8, hipMemcpyDeviceToHost, s));
  if (var_loo) HIPCHK(hipMemcpyAsync(var_loo, ctx->var_loo.p, n * 8, hipMemcpyDeviceToHost, s));
  if (mu_loo || var_loo) HIPCHK(hipStreamSynchronize(s));
  ctx->fitted = true;
  return 0;
}

// Objective value + analytic gradient (the reference's fwd + `.backward()` of one GD
// iteration: KF:239-252 LOO-CRPS, KF:329-339 NLML, KF:416-428 LOO-LogS).
//   grad = [∂/∂log sf², ∂/∂b (n_ell entries), ∂/∂log σ²] = Σ_ij M_ij ∂A_ij/∂θ
//   NLML: M = ½(A⁻¹ − ααᵀ); LOO: M = −½(vαᵀ + αvᵀ) − A⁻¹ diag(c̃) A⁻¹ (kernels_grad.hip)
// A⁻¹ = L⁻ᵀL⁻¹ is one triangular SYRK-shaped GEMM (n³/3 flops); the LOO objectives add
// A⁻¹ diag(c̃) A⁻¹ (n³ flops, lower tiles) and one GEMV.
int gps_full_grad(gps_ctx* ctx, int kind, const double* theta, int n_ell, int objective,
                  double obj[GPS_N_OBJ], double* grad) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(grad != nullptr, "grad is NULL");
  ARGCHK(objective == GPS_OBJ_NLML || objective == GPS_OBJ_LOO_CRPS ||
             objective == GPS_OBJ_LOO_LOGS,
         "objective must be GPS_OBJ_NLML, GPS_OBJ_LOO_CRPS or GPS_OBJ_LOO_LOGS");
  int rc;
  if ((rc = full_fit_core(ctx, kind, theta, n_ell))) return rc;
  const int64_t n = ctx->n, np = ctx->n_pad;
  const int d = ctx->d;
  hipStream_t s = ctx->stream;
  {  // A⁻¹ (lower 128-tiles) = L⁻ᵀL⁻¹ into the factorisation's scratch A
    GemmParams p = gp0();
    p.A = ctx->Linv.d(); p.lda = np; p.B = ctx->Linv.d(); p.ldb = np;
    p.C = ctx->A.d(); p.ldc = np;
    p.M = (int)np; p.N = (int)np; p.K = (int)np; p.tri = TRI_K_GE_I; p.lower_out = 1;
    if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p))) return rc;
  }
  GradParams g;
  memset(&g, 0, sizeof(g));
  g.x = ctx->X.d(); g.n = (int)n; g.d = d; g.sf2 = ctx->th.sf2;
  for (int k = 0; k < d; ++k) g.inv_ell[k] = ctx->th.inv_ell[k];
  g.Ainv = ctx->A.d(); g.ldm = np; g.alpha = ctx->alpha.d();
  if (objective == GPS_OBJ_NLML) {
    g.a0 = 0.5;
    g.a1 = -0.5;
  } else {
    HIPCHK(ensure(ctx, ctx->gu, np * 8));
    HIPCHK(ensure(ctx, ctx->gct, np * 8));
    HIPCHK(ensure(ctx, ctx->gv, np * 8));
    HIPCHK(ensure(ctx, ctx->Mx, (size_t)np * np * 8));
    {
      Prof pr(ctx, "grad_mirror", 0, 16.0 * (double)np * np / 2);
      HIPCHK(launch_sym_mirror(ctx->A.d(), np, (int)np, s));
    }
      HIPCHK(launch_loo_grad_terms(ctx->y.d(), ctx->alpha.d(), ctx->dinv.d(), (int)n, (int)np,
                                 objective, ctx->gu.d(), ctx->gct.d(), s));
    {
      Prof pr(ctx, "grad_gemv_v", 0, 8.0 * (double)np * np);
      HIPCHK(launch_gemv_full(ctx->A.d(), np, ctx->gu.d(), ctx->gv.d(), (int)np, (int)np, s));
    }
    {  // Mx = A⁻¹ diag(c̃) A⁻¹ (lower tiles): NT with the per-k scale on the A operand
      GemmParams p = gp0();
      p.A = ctx->A.d(); p.lda = np; p.B = ctx->A.d(); p.ldb = np;
      p.C = ctx->Mx.d(); p.ldc = np; p.kscale = ctx->gct.d();
      p.M = (int)np; p.N = (int)np; p.K = (int)np; p.lower_out = 1;
      if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_STORE, p))) return rc;
    }
    g.a2 = -1.0;
    g.a3 = -1.0;
    g.v = ctx->gv.d();
    g.Mx = ctx->Mx.d();
  }
  const int passes = grad_contract_passes(d);
  HIPCHK(ensure(ctx, ctx->gslab, (size_t)grad_contract_slab_doubles((int)n, d) * 8));
  HIPCHK(ensure(ctx, ctx->gout, (size_t)passes * 18 * 8));
  g.slab = ctx->gslab.d();
  {
    Prof pr(ctx, "grad_contract", 0, (objective == GPS_OBJ_NLML ? 8.0 : 16.0) * (double)n * n / 2);
    HIPCHK(launch_grad_contract(g, ctx->gout.d(), s));
  }
  std::vector<double> hout((size_t)passes * 18);
  HIPCHK(hipMemcpyAsync(ctx->hsmall, ctx->small.p, GPS_N_OBJ * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hout.data(), ctx->gout.p, hout.size() * 8, hipMemcpyDeviceToHost, s));
  if ((rc = check_info(ctx))) return rc;  // synchronises the stream
  if (obj)
    for (int q = 0; q < GPS_N_OBJ; ++q) obj[q] = ctx->hsmall[q];
  // ∂A/∂b_k = K ∘ Δ_k² (ARD, b = log ℓ) or ½ K ∘ Δ_k² (RBF, b = log ℓ²); scalar b sums over k
  const double bscale = kind == GPS_RBF ? 0.5 : 1.0;
  grad[0] = hout[0];
  double tot = 0.0;
  for (int k = 0; k < d; ++k) {
    const double gk = bscale * hout[(size_t)(k / 16) * 18 + 2 + (k % 16)];
    if (n_ell == d) grad[1 + k] = gk;
    tot += gk;
  }
  if (n_ell == 1) grad[1] = tot;
  grad[1 + n_ell] = ctx->th.sn2 * hout[1];
  ctx->fitted = true;
  return 0;
}

int gps_full_predict(gps_ctx* ctx, double* mu, double* var, double sc[GPS_N_SC]) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(ctx->fitted, "gps_full_fit first");
  ARGCHK(ctx->have_test, "gps_full_set_test first");
  const int64_t n = ctx->n, np = ctx->n_pad, nt = ctx->nt, ntp = ctx->nt_pad;
  hipStream_t s = ctx->stream;
  const int64_t tiles_m = np / GPS_TILE;
  HIPCHK(ensure(ctx, ctx->s1, ntp * 8));
  HIPCHK(ensure(ctx, ctx->s2, ntp * 8));
  HIPCHK(ensure(ctx, ctx->mu, ntp * 8));
  HIPCHK(ensure(ctx, ctx->var, ntp * 8));
  int rc;
  HIPCHK(ensure(ctx, ctx->Ksf, (size_t)ntp * np * 8));
  HIPCHK(ensure(ctx, ctx->pslab, (size_t)tiles_m * ntp * 2 * 8));
  if ((rc = gram(ctx, "gram_ksf", ctx->Xt.d(), (int)nt, ctx->X.d(), (int)n, ctx->d, ctx->th, 0.0, 0,
                 0, ctx->Ksf.d(), np, (int)ntp, (int)np)))
    return rc;
  if ((rc = pred_rows(ctx, 0, np, ctx->beta.d(), s))) return rc;
  {
    Prof pr(ctx, "pred_finalize", 0, 0);
    HIPCHK(launch_slab_sum(ctx->pslab.d(), ntp, (int)tiles_m, ntp, nullptr, ctx->s1.d(), s));
    HIPCHK(launch_slab_sum(ctx->pslab.d() + tiles_m * ntp, ntp, (int)tiles_m, ntp, nullptr,
                           ctx->s2.d(), s));
    HIPCHK(launch_pred_finalize(ctx->s1.d(), ctx->s2.d(), (int)nt, ctx->th.sn2 + ctx->th.sf2,
                                ctx->mu.d(), ctx->var.d(), s));
  }
  {  // the score phase (KF:276-292): its own profiling tag
    Prof pr(ctx, "score_sums", 0, 24.0 * nt);
    double* part = row_part(ctx, nt, 6);
    ARGCHK(part != nullptr, "out of device memory");
    HIPCHK(launch_score_sums(ctx->mu.d(), ctx->var.d(), ctx->yt.d(), (int)nt, ctx->ytr_mean,
                             ctx->ytr_var, ctx->small.d(), part, s));
  }
  HIPCHK(hipMemcpyAsync(ctx->hsmall, ctx->small.p, 6 * 8, hipMemcpyDeviceToHost, s));
  if (mu) HIPCHK(hipMemcpyAsync(mu, ctx->mu.p, nt * 8, hipMemcpyDeviceToHost, s));
  if (var) HIPCHK(hipMemcpyAsync(var, ctx->var.p, nt * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (sc) score_bundle(ctx->hsmall, (double)nt, sc);
  return 0;
}


// ------------------------------------------------------------- CP.R surfaces
int gps_full_surface(gps_ctx* ctx, const double* X, const double* y, int64_t n, int d,
                     double log_sf2, const double* ell, int64_t n_ell, const double* noise_sd,
                     int64_t n_noise, int flags, double* out) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(X && y && ell && noise_sd && out, "NULL argument");
  ARGCHK(n >= 1, "surface: n must be >= 1");
  ARGCHK(d >= 1 && d <= GPS_MAX_D, "bad d");
  ARGCHK(n_ell >= 1 && n_noise >= 1 && n_ell * n_noise <= (1 << 24), "bad grid");
  ARGCHK((flags & ~GPS_SURF_LOGS_ADD_NOISE) == 0, "unknown surface flag");
  hipStream_t s = ctx->stream;
  if (n > GPS_SURFACE_MAX_N) {
    // beyond one wavefront's LDS: one resident fit per grid point (the gps_full_fit path:
    // Gram, factorisation, β, α, diag(A⁻¹), LOO sums), then the in-sample CRPS and the CP.R:81
    // LogS from α and diag(A⁻¹); the data become the context's resident full-GP data
    ARGCHK(n > 1, "surface: n must be > 1");
    if (int rc = gps_full_set_data(ctx, X, y, n, d)) return rc;
    const int64_t st = n_noise * n_ell;
    for (int64_t i = 0; i < n_noise; ++i)
      for (int64_t j = 0; j < n_ell; ++j) {
        const double s2 = noise_sd[i] * noise_sd[i];
        const double theta[3] = {log_sf2, std::log(std::fabs(ell[j])), std::log(s2)};  // ℓ² enters
        const int64_t g = i * n_ell + j;
        int rc = full_fit_core(ctx, GPS_ARD, theta, 1);
        double* part = rc == 0 ? row_part(ctx, n, 2) : nullptr;
        if (rc == 0) {
          ARGCHK(part != nullptr, "out of device memory");
          HIPCHK(launch_surface_point_sums(ctx->y.d(), ctx->alpha.d(), ctx->dinv.d(), (int)n, s2,
                                           (flags & GPS_SURF_LOGS_ADD_NOISE) ? 1 : 0,
                                           ctx->small.d() + 16, part, s));
          HIPCHK(hipMemcpyAsync(ctx->hsmall, ctx->small.p, 18 * 8, hipMemcpyDeviceToHost, s));
          rc = check_info(ctx);
        }
        if (rc > 0) {  // not positive definite at this point: NaN there only (as the kernel)
          for (int q = 0; q < 4; ++q) out[q * st + g] = std::nan("");
          continue;
        }
        if (rc < 0) return rc;
        const double* h = ctx->hsmall;
        out[g] = h[GPS_OBJ_LOO_CRPS];
        out[st + g] = h[16] / (double)n;
        out[2 * st + g] = h[GPS_OBJ_NLML];
        out[3 * st + g] = h[17] / (double)n;
      }
    ctx->fitted = false;  // the last point's factor is not a fit the caller asked for
    return 0;
  }
  if (int rc = upload(ctx, ctx->t0, X, n, d, n)) return rc;
  if (int rc = upload(ctx, ctx->t1, y, n, 1, n)) return rc;
  if (int rc = upload(ctx, ctx->t2, ell, n_ell, 1, n_ell)) return rc;
  if (int rc = upload(ctx, ctx->t3, noise_sd, n_noise, 1, n_noise)) return rc;
  const int64_t cnt = 4 * n_ell * n_noise;
  HIPCHK(ensure(ctx, ctx->t4, (size_t)cnt * 8));
  SurfaceParams p;
  p.x = ctx->t0.d(); p.y = ctx->t1.d(); p.n = (int)n; p.d = d; p.sf2 = std::exp(log_sf2);
  p.ell = ctx->t2.d(); p.nl = (int)n_ell; p.sd = ctx->t3.d(); p.ns = (int)n_noise;
  p.logs_add_noise = (flags & GPS_SURF_LOGS_ADD_NOISE) != 0;
  p.out = ctx->t4.d();
  {
    Prof pr(ctx, "surface", 0, 0);
    HIPCHK(launch_surface(p, s));
  }
  HIPCHK(hipMemcpyAsync(out, ctx->t4.p, (size_t)cnt * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

}  // extern "C"
