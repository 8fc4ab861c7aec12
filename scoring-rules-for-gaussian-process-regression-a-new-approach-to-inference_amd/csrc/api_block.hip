// C-ABI, block-LOO objectives (DSS / KC, KF:487-563, K20:523-609, 655-745) and the energy score
// (KF:70-101, 607-672), full GP and FITC, values and gradients.
#include "api_internal.h"

namespace gpsapi {

// ------------------------------------------------------------------ block-LOO (next-2)
// Folds [a_f, b_f) with a_f = int(f·n/k) (KF:496-499).  getP(f, a, b, P, ldp) writes the
// lower tiles of P_f (b_pad×b_pad, padded as diag(P_f, I)).  Per fold: potrf_inv(P_f) →
// Lp⁻¹, t = Lp⁻¹α_f, r = P_f⁻¹α_f and c = diag(P_f⁻¹) in one colred pass; then
//   DSS_f = ½b log2π − ½log|P_f| + ½α_fᵀr,  KC_f = crps(y_f − r, c, y_f),
//   ES_f  = the energy score of N(y_f − r, P_f⁻¹) at y_f (es_fold).
// With want_grad, gdst(a, b) names the destination of ∂obj/∂P_f (b×b, symmetric), gdone(f,
// a, b) runs once it is written, and ∂obj/∂α_f lands in g[a, a+b) (kernels_block.hip).
std::vector<int64_t> fold_bounds(int64_t n, int nfold) {
  std::vector<int64_t> bnd(nfold + 1);
  for (int f = 0; f <= nfold; ++f) bnd[f] = f == nfold ? n : (int64_t)((double)f * n / nfold);
  return bnd;
}

// padded edge of the largest fold
int64_t bounds_pad(const std::vector<int64_t>& bnd) {
  int64_t bmax = 1;
  for (size_t f = 0; f + 1 < bnd.size(); ++f) bmax = std::max(bmax, bnd[f + 1] - bnd[f]);
  return pad_to(bmax);
}

struct EsArgs {
  int S = 0;                      // draws per fold (num_sim: 300 at KF:652-655)
  double beta = 1.0;              // the score's exponent (KF:70)
  const double* draws = nullptr;  // device; fold f holds ξ_f then ξ'_f (S×b_f each, row-major)
  double lam_lb = 0.0;            // λmin(C_f) >= lam_lb; <= 0: unknown, iterate to ‖T − I‖ ≈ 0
  double diag_ub = 0.0;           // diag(C_f) <= diag_ub, so λmax <= b·diag_ub
  double scale = 0.0;             // > 0: λmax(C_f) <= scale (‖C_f‖∞, full_blockloo), used instead
};

// Scaled Newton–Schulz schedule for a spectrum of C/s inside [x0, 1] (round 4).  The eigenvalue x
// of Z_kY_k follows x ← f(x) = x(3 − x)²/4: ×2.25 per step while small (~20 steps from x0 = 8e-6).
// Scaling the iterates by a scalar keeps the invariant Y_kZ_k⁻¹ = C/s (so the limit is still
// (C/s)^½) and turns the step into x ← f(βx) with Y ← √β·Y T, Z ← √β·T Z, T = (3I − βZY)/2.
// With the spectrum known to lie in [l, u], β equalises the images of the two ends,
// f(βl) = f(βu) (βu < 3: f is increasing to 1 at x = 1 and falls to 0 at 3), which maximises the
// new lower bound min f(β[l, u]); the new upper bound is 1 once βl ≤ 1 ≤ βu.  The lower bound then
// grows ×6.7 per step instead of ×2.25: 12 steps instead of 20 from x0 = 8e-6.  Two unscaled
// steps follow, which let the derivative block of the gradient pass settle.  Returns β per step.
std::vector<double> ns_schedule(double x0) {
  auto f = [](double x) { return x * (3.0 - x) * (3.0 - x) / 4.0; };
  double l = std::min(std::max(x0, 1e-300), 1.0), u = 1.0;
  std::vector<double> beta;
  while (1.0 - l > 4e-16 && beta.size() < 200) {
    double b = 1.0 / u;
    // scaled while the lower bound is small; from l = 0.5 on the unscaled step converges
    // quadratically (scaling there only chases rounding in the bounds)
    if (l < 0.5 && f(b * l) < f(b * u)) {  // bisect f(βl) = f(βu) on [1/u, 2.999/u]
      double lo = 1.0 / u, hi = 2.999 / u;
      for (int it = 0; it < 100; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (f(mid * l) < f(mid * u)) lo = mid;
        else hi = mid;
      }
      b = lo;
    }
    const double nl = std::min(f(b * l), f(b * u));
    u = (b * l <= 1.0 && 1.0 <= b * u) ? 1.0 : std::max(f(b * l), f(b * u));
    l = std::min(nl, u);
    beta.push_back(b);
  }
  beta.push_back(1.0);
  beta.push_back(1.0);
  return beta;
}

// Energy score of one fold, ES(m, c, shape1, y, S, β) (KF:70-101) as the scripts call it on
// the block-LOO predictive (KF:652-655): m − y = −r, C = P_f⁻¹ (PI, full, bp×bp).
//   R = C^½ by the scaled coupled Newton–Schulz iteration on C/s (T = (3I − βZY)/2,
//   Y ← √β·YT, Z ← √β·TZ, β per step from ns_schedule: three b×b MFMA GEMMs per step; the scripts take an SVD, KF:74-77, which has no GEMM form);
//   z = ξR, ẑ = [ξ'R; −r], D_ij = ‖z_i − ẑ_j‖ (es_dist),
//   ES = (1/S)Σ_i D_iS^β − Σ_{i,j<S} D_ij^β / (2S(S−1)) (es_reduce) → *out (device).
// With G (ldg): Ḡ = ∂ES/∂R = ξᵀG_z + ξ'ᵀG_ẑ, G_z = diag(ΣW)z − Wẑ, G_ẑ = diag(ΣWᵀ)ẑ − Wᵀz
// (W = ∂ES/∂D ∘ D⁻¹); X with RX + XR = sym Ḡ is the off-diagonal block of the same iteration
// run on [[C, Ḡ], [0, C]] (whose square root is [[R, X], [0, R]]); with w = C·∂ES/∂r:
//   G = ∂ES/∂P_f = −CXC − ½(wrᵀ + rwᵀ),  g = ∂ES/∂α_f = w.
// Everything runs on stream s with work area eb (conc: one of 4 folds in flight).
int es_fold(gps_ctx* ctx, hipStream_t s, DBuf& eb, bool conc, const EsArgs& es, const double* xi_src,
            int64_t b, int64_t bp, const double* PI, const double* r, double trace_c, double* w,
            double* G, int64_t ldg, double* g, double* out) {
  const int S = es.S;
  const int64_t Sp = pad_to(S + 1);
  const bool grad = G != nullptr;
  const int nmat = grad ? 10 : 5;
  const bool bounded = es.lam_lb > 0.0;
  // the scale s of C/s: ‖C_f‖∞ when the caller measured it (round 4: on C2's folds ~1.1 against
  // the trace bound b(sf² + σ²) ≈ 1262, which left the spectrum of C/s three decades below 1 and
  // cost the scaled schedule ~6 more steps), else the trace bound
  const double sc = bounded ? (es.scale > 0.0 ? es.scale : (double)b * es.diag_ub) : trace_c;
  // β per step (ns_schedule); adaptive mode (no spectral bounds) runs unscaled steps
  const std::vector<double> beta = bounded ? ns_schedule(es.lam_lb / sc) : std::vector<double>(200, 1.0);
  const int iters = (int)beta.size();
  // with a gradient and a known step count the forward iterates Y_k, Z_k, T_k are kept
  // (3·iters + 2 matrices, < 1 GB at b = 1250) so the derivative pass runs only the
  // 6 products of the off-diagonal blocks per step instead of 9
  const size_t nstore = grad && bounded ? (size_t)3 * iters + 2 : 0;
  const bool stored = nstore && nstore * bp * bp * 8 <= ((size_t)16 << 30);
  const size_t need = (size_t)(6 * Sp * bp + Sp * Sp + 2 * Sp + bp + 8) +
                      ((size_t)nmat + (stored ? nstore : 0)) * bp * bp;
  HIPCHK(ensure(ctx, eb, need * 8));
  double* q = eb.d();
  auto take = [&](int64_t cnt) {
    double* t = q;
    q += cnt;
    return t;
  };
  double *xi = take(Sp * bp), *xip = take(Sp * bp), *Zs = take(Sp * bp), *Zh = take(Sp * bp);
  double *Gz = take(Sp * bp), *Gh = take(Sp * bp), *D = take(Sp * Sp), *rsum = take(Sp),
         *csum = take(Sp), *dr = take(bp), *res = take(8);
  double* M[10] = {nullptr};
  for (int i = 0; i < nmat; ++i) M[i] = take(bp * bp);
  std::vector<double*> Ys, Zk, Ts;  // stored iterates: Y_0..Y_iters, Z_0..Z_iters, T_0..T_iters-1
  if (stored) {
    for (int k = 0; k <= iters; ++k) Ys.push_back(take(bp * bp));
    for (int k = 0; k <= iters; ++k) Zk.push_back(take(bp * bp));
    for (int k = 0; k < iters; ++k) Ts.push_back(take(bp * bp));
  }
  int rc;
  // C = alpha·op(A)·B + beta·C with N = bp, ldc = bp (every product here has that shape)
  auto mm = [&](int al, const double* A, int64_t lda, const double* B, double* C, int64_t rows,
                int64_t kdim, double alpha, double beta) {
    GemmParams p = gp0();
    p.A = A; p.lda = lda; p.B = B; p.ldb = bp; p.C = C; p.ldc = bp;
    p.M = (int)rows; p.N = (int)bp; p.K = (int)kdim; p.alpha = alpha; p.beta = beta;
    return gemm(ctx, al, LAY_N, EPI_STORE, p, s);
  };
  auto sq = [&](const double* A, const double* B, double* C, double alpha, double beta) {
    return mm(LAY_N, A, bp, B, C, bp, bp, alpha, beta);
  };
  // Every Newton–Schulz iterate is a polynomial in C (Y_k, Z_k, T_k commute), and the
  // off-diagonal blocks of the gradient pass are Fréchet derivatives of those polynomials
  // in the symmetric direction Ḡ: every product (or pair sum) below is symmetric, so it
  // is formed on the lower tiles only (half the flops) and mirrored.
  // (mirror: the product completes C, whose strictly-lower 32-tiles then go above the diagonal
  //  in the same launch sequence — GemmParams::mirror — instead of a sym_mirror launch after it)
  auto sym = [&](const double* A, const double* B, double* C, double alpha, double beta,
                 bool mirror = false) {
    GemmParams p = gp0();
    p.A = A; p.lda = bp; p.B = B; p.ldb = bp; p.C = C; p.ldc = bp;
    p.M = (int)bp; p.N = (int)bp; p.K = (int)bp; p.alpha = alpha; p.beta = beta; p.lower_out = 1;
    p.mirror = mirror ? 1 : 0;
    if (conc) {  // 4 folds in flight: 2 K slices of 64-tiles (C2 ES: ks 1/2/3/4/auto(8) =
      p.tile = 64;  // 54.8 / 53.9 / 54.4 / 55.3 / 58.5 ms per iteration)
      p.ksplit = 2;
    }
    return gemm(ctx, LAY_N, LAY_N, EPI_STORE, p, s);
  };
  HIPCHK(launch_pad_copy(xi_src, b, xi, bp, S, (int)b, (int)Sp, (int)bp, 0, s));
  HIPCHK(launch_pad_copy(xi_src + (int64_t)S * b, b, xip, bp, S, (int)b, (int)Sp, (int)bp, 0, s));
  double *Y = stored ? Ys[0] : M[0], *Z = stored ? Zk[0] : M[1], *T = M[2], *Yn = M[3],
         *Zn = M[4];
  HIPCHK(launch_ns_init(PI, bp, (int)b, (int)bp, 1.0 / sc, 1.0, Y, s));
  HIPCHK(launch_ns_init(nullptr, 0, (int)b, (int)bp, 1.0, 1.0, Z, s));
  int used = 0, extra = -1;  // adaptive mode: steps still to run once converged
  for (int it = 0; it < iters && extra != 0; ++it) {
    if (stored) {
      T = Ts[it];
      Yn = Ys[it + 1];
      Zn = Zk[it + 1];
    }
    const double bt = beta[it], mu = std::sqrt(bt);
    if ((rc = sym(Z, Y, T, -0.5 * bt, 0.0, true))) return rc;
    HIPCHK(launch_diag_add_const(T, bp, (int)bp, 1.5, s));
    if (!bounded && extra < 0) {  // ‖T − I‖²_F = ‖I − ZY‖²_F / 4
      HIPCHK(launch_ns_resid(T, bp, (int)bp, res, s));
      HIPCHK(hipMemcpyAsync(ctx->hsmall, res, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      if (ctx->hsmall[0] < 1e-24 * (double)bp) extra = 3;
    }
    if ((rc = sym(Y, T, Yn, mu, 0.0, true))) return rc;
    if ((rc = sym(T, Z, Zn, mu, 0.0, true))) return rc;
    std::swap(Y, Yn);
    std::swap(Z, Zn);
    ++used;
    if (extra > 0) --extra;
  }
  ARGCHK(bounded || extra == 0, "energy score: C^1/2 did not converge (is C positive definite?)");
  const double rt = std::sqrt(sc);
  if ((rc = mm(LAY_N, xi, bp, Y, Zs, Sp, bp, rt, 0.0))) return rc;
  if ((rc = mm(LAY_N, xip, bp, Y, Zh, Sp, bp, rt, 0.0))) return rc;
  HIPCHK(launch_scaled_row(r, (int)b, (int)bp, -1.0, Zh + (int64_t)S * bp, s));
  HIPCHK(launch_es_dist(Zs, Zh, bp, S, (int)bp, D, Sp, s));
  HIPCHK(launch_es_reduce(D, Sp, S, (int)Sp, es.beta, grad ? 1 : 0, rsum, csum, out, s));
  if (!grad) return 0;
  // G_z = diag(ΣW) z − W ẑ,  G_ẑ = diag(ΣWᵀ) ẑ − Wᵀ z   (W overwrote D, zero-padded)
  if ((rc = mm(LAY_N, D, Sp, Zh, Gz, Sp, Sp, -1.0, 0.0))) return rc;
  HIPCHK(launch_row_axpy(Gz, bp, Zs, bp, rsum, (int)Sp, (int)bp, s));
  if ((rc = mm(LAY_T, D, Sp, Zs, Gh, Sp, Sp, -1.0, 0.0))) return rc;
  HIPCHK(launch_row_axpy(Gh, bp, Zh, bp, csum, (int)Sp, (int)bp, s));
  // ∂ES/∂r = −G_ẑ[S] (ẑ_S = −r);  w = C ∂ES/∂r
  HIPCHK(launch_scaled_row(Gh + (int64_t)S * bp, (int)b, (int)bp, -1.0, dr, s));
  HIPCHK(launch_gemv_full(PI, bp, dr, w, (int)bp, (int)bp, s));
  // Ḡ = ξᵀG_z + ξ'ᵀG_ẑ (ξ' is zero from row S on), symmetrised
  double* Gb = M[5];
  if ((rc = mm(LAY_T, xi, bp, Gz, Gb, bp, Sp, 1.0, 0.0))) return rc;
  if ((rc = mm(LAY_T, xip, bp, Gh, Gb, bp, Sp, 1.0, 1.0))) return rc;
  HIPCHK(launch_sym_avg(Gb, bp, (int)bp, s));
  // the iteration on [[C, Ḡ], [0, C]]/s: diagonal blocks (Y1, Z1, T1) — the forward
  // iterates, stored or recomputed — and off-diagonal blocks (Y2, Z2, T2)
  double *Y1 = M[0], *Z1 = M[1], *T1 = M[2], *Y1n = M[3], *Z1n = M[4], *Z2n = M[5],
         *Y2 = M[6], *Z2 = M[7], *T2 = M[8], *Y2n = M[9];
  HIPCHK(launch_ns_init(Gb, bp, (int)b, (int)bp, 1.0 / sc, 0.0, Y2, s));  // before Z2n reuses Gb
  if (!stored) {
    HIPCHK(launch_ns_init(PI, bp, (int)b, (int)bp, 1.0 / sc, 1.0, Y1, s));
    HIPCHK(launch_ns_init(nullptr, 0, (int)b, (int)bp, 1.0, 1.0, Z1, s));
  }
  HIPCHK(launch_ns_init(nullptr, 0, (int)b, (int)bp, 0.0, 0.0, Z2, s));
  for (int it = 0; it < used; ++it) {
    const double bt = beta[it], mu = std::sqrt(bt);  // the forward step's scaling
    const double *Yk = Y1, *Zkk = Z1, *Tk = T1;
    if (stored) {
      Yk = Ys[it];
      Zkk = Zk[it];
      Tk = Ts[it];
    } else {
      if ((rc = sym(Z1, Y1, T1, -0.5 * bt, 0.0, true))) return rc;
      HIPCHK(launch_diag_add_const(T1, bp, (int)bp, 1.5, s));
    }
    if ((rc = sym(Zkk, Y2, T2, -0.5 * bt, 0.0))) return rc;  // T2 = −½β(Z1Y2 + Z2Y1)
    if ((rc = sym(Z2, Yk, T2, -0.5 * bt, 1.0, true))) return rc;
    if ((rc = sym(Yk, T2, Y2n, mu, 0.0))) return rc;   // Y2 ← √β(Y1T2 + Y2T1)
    if ((rc = sym(Y2, Tk, Y2n, mu, 1.0, true))) return rc;
    if ((rc = sym(Tk, Z2, Z2n, mu, 0.0))) return rc;   // Z2 ← √β(T1Z2 + T2Z1)
    if ((rc = sym(T2, Zkk, Z2n, mu, 1.0, true))) return rc;
    if (!stored) {
      if ((rc = sym(Y1, T1, Y1n, mu, 0.0, true))) return rc;
      if ((rc = sym(T1, Z1, Z1n, mu, 0.0, true))) return rc;
      std::swap(Y1, Y1n);
      std::swap(Z1, Z1n);
    }
    std::swap(Y2, Y2n);
    std::swap(Z2, Z2n);
  }
  T1 = M[2];
  // X = √s·Y2;  H = C X C (into T1);  G, g by fold_grad
  if ((rc = sq(Y2, PI, T2, rt, 0.0))) return rc;
  if ((rc = sq(PI, T2, T1, 1.0, 0.0))) return rc;
  HIPCHK(launch_fold_grad(PI, bp, T1, bp, r, w, (int)b, 0.0, 0.0, -1.0, -1.0, 0.0, 1.0, G, ldg,
                          g, s));
  return 0;
}

template <class GetP, class GDst, class GDone>
int blockloo_folds(gps_ctx* ctx, const std::vector<int64_t>& bnd, int objective, const double* alpha,
                   const double* y, GetP getP, bool want_grad, GDst gdst, GDone gdone, double* g,
                   const EsArgs* es, double* vals) {
  hipStream_t s = ctx->stream;
  const int nfold = (int)bnd.size() - 1;
  const int64_t bp = bounds_pad(bnd);
  HIPCHK(ensure(ctx, ctx->bP, (size_t)bp * bp * 8));
  if (ctx->bL.cap < (size_t)bp * bp * 8 || !factor_zeroed(ctx, ctx->bL.d(), bp)) {
    HIPCHK(ensure(ctx, ctx->bL, (size_t)bp * bp * 8));
    HIPCHK(zero_factor(ctx, ctx->bL.d(), bp, s));
  }
  HIPCHK(ensure(ctx, ctx->bPI, (size_t)bp * bp * 8));
  HIPCHK(ensure(ctx, ctx->bH, (size_t)bp * bp * 8));
  HIPCHK(ensure(ctx, ctx->W, std::max(ctx->W.cap, potrf_ws_doubles(bp) * 8)));
  HIPCHK(ensure(ctx, ctx->bvec, (size_t)(9 * bp + 3 * nfold + 8) * 8));
  const int64_t nchunk = (bp + 255) / 256;
  HIPCHK(ensure(ctx, ctx->slab, std::max(ctx->slab.cap, (size_t)nchunk * bp * 2 * 8)));
  double* v = ctx->bvec.d();
  double *ld = v, *af = v + bp, *t = v + 2 * bp, *r = v + 3 * bp, *c = v + 4 * bp,
         *gm = v + 5 * bp, *gc = v + 6 * bp, *w = v + 7 * bp, *yf = v + 8 * bp;
  double* fs = v + 9 * bp;  // per fold: [Σ log L_ii, α·r, kc / es]
  const bool kc = objective == GPS_BLOCK_KC, esq = objective == GPS_BLOCK_ES;
  // ES with spectral bounds: ‖C_f‖∞ per fold scales the Newton–Schulz iteration (es_fold)
  const bool es_norm = esq && es->lam_lb > 0.0;
  // ES in two passes — every fold's C_f and r_f first, then the square roots — whenever the folds
  // can run concurrently (the overlap option: fold f on stream f mod 4 with its own work area) or
  // their schedules need ‖C_f‖∞: the bounds of all folds then come back in ONE host read instead
  // of a stream drain per fold.  C_f, r_f, w_f are kept per fold (the fold gradients
  // land in disjoint blocks: full GP).
  const int es_streams = ctx->overlap ? (int)std::min<int64_t>(nfold, 4) : 1;
  const bool es_conc = esq && (es_streams > 1 || es_norm);
  if (es_norm) HIPCHK(ensure(ctx, ctx->escale, (size_t)(nfold + bp) * 8));
  std::vector<double> hscale(nfold, 0.0);
  double *PIs = nullptr, *RW = nullptr;
  if (es_conc) {
    HIPCHK(ensure(ctx, ctx->bPIs, (size_t)nfold * bp * bp * 8));
    HIPCHK(ensure(ctx, ctx->bRW, (size_t)2 * nfold * bp * 8));
    PIs = ctx->bPIs.d();
    RW = ctx->bRW.d();
  }
  int rc;
  // no reset_info here: a non-PD minor of the caller's main factor must still be reported
  HIPCHK(hipMemsetAsync(v, 0, (size_t)9 * bp * 8, s));
  for (int f = 0; f < nfold; ++f) {
    const int64_t a = bnd[f], b = bnd[f + 1] - bnd[f];
    if ((rc = getP(f, a, b, ctx->bP.d(), bp))) return rc;
    if ((rc = potrf_inv(ctx, ctx->bP.d(), bp, ctx->bL.d(), ctx->W.d(), ld, (int)b, nullptr)))
      return rc;
    HIPCHK(launch_pad_copy(alpha + a, 1, af, 1, (int)b, 1, (int)bp, 1, 0, s));
    HIPCHK(launch_pad_copy(y + a, 1, yf, 1, (int)b, 1, (int)bp, 1, 0, s));
    HIPCHK(launch_gemv_lower(ctx->bL.d(), bp, af, t, (int)bp, s));
    HIPCHK(launch_colred(ctx->bL.d(), bp, (int)bp, (int)bp, 1, t, nullptr, r, c, ctx->slab.d(), s));
    HIPCHK(launch_dot(ld, nullptr, (int)b, fs + 3 * f, s));
    HIPCHK(launch_dot(af, r, (int)b, fs + 3 * f + 1, s));
    if (kc)
      HIPCHK(launch_fold_terms(yf, r, c, (int)b, want_grad ? gm : nullptr, gc, fs + 3 * f + 2, s));
    if (!want_grad && !esq) continue;
    double* PI = es_conc ? PIs + (int64_t)f * bp * bp : ctx->bPI.d();
    {  // C_f = P⁻¹ = Lp⁻ᵀLp⁻¹ (full)
      GemmParams p = gp0();
      p.A = ctx->bL.d(); p.lda = bp; p.B = ctx->bL.d(); p.ldb = bp; p.C = PI; p.ldc = bp;
      p.M = (int)bp; p.N = (int)bp; p.K = (int)bp; p.tri = TRI_K_GE_I; p.lower_out = 1;
      p.mirror = 1;
      if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p))) return rc;
    }
    if (es_norm)
      HIPCHK(launch_norm_inf(PI, bp, (int)b, ctx->escale.d() + nfold, ctx->escale.d() + f, s));
    if (es_conc) {  // r_f for the second pass below
      HIPCHK(hipMemcpyAsync(RW + (int64_t)2 * f * bp, r, (size_t)bp * 8, hipMemcpyDeviceToDevice,
                            s));
      continue;
    }
    double* G = nullptr;
    int64_t ldg = 0;
    if (want_grad) {
      const std::pair<double*, int64_t> dst = gdst(a, b);
      G = dst.first;
      ldg = dst.second;
    }
    if (esq) {
      EsArgs ef = *es;
      ef.scale = hscale[f] * (1.0 + 1e-12);
      if ((rc = es_fold(ctx, s, ctx->ebuf, false, ef, es->draws + 2 * (int64_t)es->S * a, b, bp, ctx->bPI.d(), r, 0.0,
                        w, G, ldg, want_grad ? g + a : nullptr, fs + 3 * f + 2)))
        return rc;
    } else if (!kc) {  // DSS: G_f = −½(P⁻¹ + r rᵀ), g_f = r
      HIPCHK(launch_fold_grad(ctx->bPI.d(), bp, nullptr, 0, r, nullptr, (int)b, -0.5, -0.5, 0.0,
                              0.0, 1.0, 0.0, G, ldg, g + a, s));
    } else {  // KC: w = P⁻¹gm, G_f = ½(w rᵀ + r wᵀ) − P⁻¹diag(gc)P⁻¹, g_f = −w
      HIPCHK(launch_gemv_full(ctx->bPI.d(), bp, gm, w, (int)bp, (int)bp, s));
      GemmParams p = gp0();
      p.A = ctx->bPI.d(); p.lda = bp; p.B = ctx->bPI.d(); p.ldb = bp; p.C = ctx->bH.d();
      p.ldc = bp; p.kscale = gc; p.M = (int)bp; p.N = (int)bp; p.K = (int)bp;
      if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_STORE, p))) return rc;
      HIPCHK(launch_fold_grad(ctx->bPI.d(), bp, ctx->bH.d(), bp, r, w, (int)b, 0.0, 0.0, 1.0,
                              -1.0, 0.0, -1.0, G, ldg, g + a, s));
    }
    if (want_grad && (rc = gdone(f, a, b))) return rc;
  }
  if (es_conc) {
    if (es_norm) {  // every fold's ‖C_f‖∞ on the host before the schedules are cut
      HIPCHK(hipMemcpyAsync(hscale.data(), ctx->escale.d(), (size_t)nfold * 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    hipStream_t st[4] = {s, ctx->side, ctx->aux[0], ctx->aux[1]};
    DBuf* eb[4] = {&ctx->ebuf, &ctx->ebuf_aux[0], &ctx->ebuf_aux[1], &ctx->ebuf_aux[2]};
    const int nst = es_streams;
    hipEvent_t fork = sync_event(ctx);
    if (!fork) return fail(ctx, -2, "hipEventCreate failed");
    HIPCHK(hipEventRecord(fork, s));
    for (int k = 1; k < nst; ++k) HIPCHK(hipStreamWaitEvent(st[k], fork, 0));
    for (int f = 0; f < nfold; ++f) {
      const int64_t a = bnd[f], b = bnd[f + 1] - bnd[f];
      double* G = nullptr;
      int64_t ldg = 0;
      if (want_grad) {
        const std::pair<double*, int64_t> dst = gdst(a, b);
        G = dst.first;
        ldg = dst.second;
      }
      double* rf = RW + (int64_t)2 * f * bp;
      EsArgs ef = *es;
      ef.scale = hscale[f] * (1.0 + 1e-12);
      if ((rc = es_fold(ctx, st[f % nst], *eb[f % nst], nst > 1, ef, es->draws + 2 * (int64_t)es->S * a, b,
                        bp, PIs + (int64_t)f * bp * bp, rf, 0.0, rf + bp, G, ldg,
                        want_grad ? g + a : nullptr, fs + 3 * f + 2)))
        return rc;
    }
    for (int k = 1; k < nst; ++k) {
      hipEvent_t join = sync_event(ctx);
      if (!join) return fail(ctx, -2, "hipEventCreate failed");
      HIPCHK(hipEventRecord(join, st[k]));
      HIPCHK(hipStreamWaitEvent(s, join, 0));
    }
    if (want_grad)
      for (int f = 0; f < nfold; ++f)
        if ((rc = gdone(f, bnd[f], bnd[f + 1] - bnd[f]))) return rc;
  }
  std::vector<double> h((size_t)3 * nfold);
  HIPCHK(hipMemcpyAsync(h.data(), fs, h.size() * 8, hipMemcpyDeviceToHost, s));
  if ((rc = check_info(ctx))) return rc;
  for (int f = 0; f < nfold; ++f) {
    const double b = (double)(bnd[f + 1] - bnd[f]);
    vals[f] = (kc || esq) ? h[3 * f + 2]
                          : 0.5 * b * 1.83787706640934548356 - h[3 * f] + 0.5 * h[3 * f + 1];
  }
  return 0;
}


// FITC block-LOO folds in low rank (round 5).  With W = K_f L_{−f}⁻ᵀ (b × m, getW) the fold
// covariance is C_f = Λ_f + WWᵀ and no b×b matrix is formed: r = C_fα_f = λα + W(Wᵀα),
// c = diag C_f = λ + ‖W_i‖², and for the gradient F̃_f = G_fŨ_f with
//   DSS: G_f = −½(C_f + rrᵀ):   F̃ = −½(C_fŨ + r(rᵀŨ)),   diag G = −½(c + r²),   g_f = r
//   KC:  G_f = ½(wrᵀ + rwᵀ) − C_fDC_f (w = C_f gm, D = diag gc):
//        F̃ = ½(w(rᵀŨ) + r(wᵀŨ)) − C_f(D·C_fŨ),  C_fX = λX + W(WᵀX),
//        diag G = w∘r − (λ²gc + 2λ·gc·(c − λ) + rowdot(W(WᵀDW), W)),   g_f = −w
// (oracle.fast_fitc_blockloo forms the same G_f densely).  Per fold O(b·m²) — 2 (DSS) or 5 (KC)
// b×m×m products — instead of the b²m covariance and, for KC, the b³ product C_fDC_f.
template <class GetW>
int fitc_lr_folds(gps_ctx* ctx, const std::vector<int64_t>& bnd, int objective, const double* alpha,
                  GetW getW, const double* U, int64_t ldr, double* F, double* gd, double* g,
                  double* vals) {
  hipStream_t s = ctx->stream;
  const int nfold = (int)bnd.size() - 1;
  const int64_t bp = bounds_pad(bnd), mp = ctx->m_pad;
  const bool kc = objective == GPS_BLOCK_KC, want = F != nullptr;
  const int64_t nch = (bp + 255) / 256;
  HIPCHK(ensure(ctx, ctx->bLRv, (size_t)(10 * bp + 4 * mp + 2 * nch * mp + 3 * nfold + 8) * 8));
  if (want) HIPCHK(ensure(ctx, ctx->bLR, (size_t)(3 * bp * mp + 2 * mp * mp) * 8));
  double* lv = ctx->bLRv.d();
  double *af = lv, *yf = lv + bp, *r = lv + 2 * bp, *c = lv + 3 * bp, *gm = lv + 4 * bp,
         *gc = lv + 5 * bp, *w = lv + 6 * bp, *at = lv + 7 * bp, *ab = lv + 8 * bp, *q = lv + 9 * bp;
  double *ta = lv + 10 * bp, *tg = ta + mp, *ru = tg + mp, *wu = ru + mp;
  double* slab = wu + mp;
  double* fs = slab + 2 * nch * mp;  // per fold: [−½log|C_f|, α·r, kc]
  HIPCHK(hipMemsetAsync(lv, 0, (size_t)10 * bp * 8, s));
  HIPCHK(hipMemsetAsync(fs, 0, (size_t)3 * nfold * 8, s));
  double* Wf = ctx->bW.d();
  double *X1 = nullptr, *X2 = nullptr, *X3 = nullptr, *P1 = nullptr, *P2 = nullptr;
  if (want) {
    X1 = ctx->bLR.d(); X2 = X1 + bp * mp; X3 = X2 + bp * mp; P1 = X3 + bp * mp; P2 = P1 + mp * mp;
  }
  // products with W: Wᵀ X (m × m, K = bp) and W P (bp × m, K = m)
  auto wt_x = [&](const double* X, double* P, const double* kscale, bool sym) -> int {
    GemmParams p = gp0();
    p.A = Wf; p.lda = mp; p.B = X; p.ldb = mp; p.C = P; p.ldc = mp;
    p.M = (int)mp; p.N = (int)mp; p.K = (int)bp; p.kscale = kscale;
    if (sym) { p.lower_out = 1; p.mirror = 1; }
    return gemm(ctx, LAY_T, LAY_N, EPI_STORE, p);
  };
  auto w_p = [&](const double* P, double* X) -> int {
    GemmParams p = gp0();
    p.A = Wf; p.lda = mp; p.B = P; p.ldb = mp; p.C = X; p.ldc = mp;
    p.M = (int)bp; p.N = (int)mp; p.K = (int)mp;
    return gemm(ctx, LAY_N, LAY_N, EPI_STORE, p);
  };
  int rc;
  for (int f = 0; f < nfold; ++f) {
    const int64_t a = bnd[f], b = bnd[f + 1] - bnd[f];
    const double* lam = ctx->lam.d() + a;
    if ((rc = getW(f, a, b, bp, fs + 3 * f))) return rc;
    HIPCHK(launch_pad_copy(alpha + a, 1, af, 1, (int)b, 1, (int)bp, 1, 0, s));
    HIPCHK(launch_pad_copy(ctx->fy.d() + a, 1, yf, 1, (int)b, 1, (int)bp, 1, 0, s));
    HIPCHK(launch_colred(Wf, mp, (int)bp, (int)mp, 0, af, nullptr, ta, nullptr, slab, s));
    HIPCHK(launch_row_dots(Wf, mp, Wf, mp, ta, (int)bp, (int)mp, at, ab, s));
    HIPCHK(launch_lr_fold_vec(0, (int)b, (int)bp, lam, af, at, ab, nullptr, nullptr, nullptr,
                              nullptr, nullptr, r, c, s));
    HIPCHK(launch_dot(af, r, (int)b, fs + 3 * f + 1, s));
    if (kc) HIPCHK(launch_fold_terms(yf, r, c, (int)b, want ? gm : nullptr, gc, fs + 3 * f + 2, s));
    if (!want) continue;
    double* Uf = ctx->bEf.d();
    HIPCHK(launch_pad_copy(U + a * ldr, ldr, Uf, mp, (int)b, (int)mp, (int)bp, (int)mp, 0, s));
    if ((rc = wt_x(Uf, P1, nullptr, false)) || (rc = w_p(P1, X1))) return rc;  // X1 = W(WᵀŨ)
    HIPCHK(launch_colred(Uf, mp, (int)bp, (int)mp, 0, r, nullptr, ru, nullptr, slab, s));
    double* Fd = F + a * mp;
    if (!kc) {
      HIPCHK(launch_lr_combine(X1, mp, Uf, mp, lam, nullptr, -0.5, r, ru, -0.5, nullptr, nullptr,
                               0.0, (int)b, (int)b, (int)mp, Fd, mp, s));
      HIPCHK(launch_lr_fold_vec(3, (int)b, (int)b, lam, nullptr, nullptr, nullptr, r, c, nullptr,
                                nullptr, nullptr, gd + a, g + a, s));
      continue;
    }
    HIPCHK(launch_colred(Wf, mp, (int)bp, (int)mp, 0, gm, nullptr, tg, nullptr, slab, s));
    HIPCHK(launch_row_dots(Wf, mp, nullptr, 0, tg, (int)bp, (int)mp, at, nullptr, s));
    HIPCHK(launch_lr_fold_vec(1, (int)b, (int)bp, lam, gm, at, nullptr, nullptr, nullptr, nullptr,
                              nullptr, nullptr, w, nullptr, s));
    // X2 = D·C_fŨ, X3 = W(WᵀX2): C_f(D·C_fŨ) = λX2 + X3
    HIPCHK(launch_lr_combine(X1, mp, Uf, mp, lam, gc, 1.0, nullptr, nullptr, 0.0, nullptr, nullptr,
                             0.0, (int)b, (int)bp, (int)mp, X2, mp, s));
    if ((rc = wt_x(X2, P2, nullptr, false)) || (rc = w_p(P2, X3))) return rc;
    HIPCHK(launch_colred(Uf, mp, (int)bp, (int)mp, 0, w, nullptr, wu, nullptr, slab, s));
    HIPCHK(launch_lr_combine(X3, mp, X2, mp, lam, nullptr, -1.0, w, ru, 0.5, r, wu, 0.5, (int)b,
                             (int)b, (int)mp, Fd, mp, s));
    // diag(C_fDC_f)'s cross term: rowdot(W(WᵀDW), W)
    if ((rc = wt_x(Wf, P1, gc, true)) || (rc = w_p(P1, X1))) return rc;
    HIPCHK(launch_row_dots(X1, mp, Wf, mp, nullptr, (int)bp, (int)mp, nullptr, q, s));
    HIPCHK(launch_lr_fold_vec(2, (int)b, (int)b, lam, nullptr, nullptr, nullptr, r, c, w, gc, q,
                              gd + a, g + a, s));
  }
  std::vector<double> h((size_t)3 * nfold);
  HIPCHK(hipMemcpyAsync(h.data(), fs, h.size() * 8, hipMemcpyDeviceToHost, s));
  if ((rc = check_info(ctx))) return rc;
  for (int f = 0; f < nfold; ++f) {
    const double b = (double)(bnd[f + 1] - bnd[f]);
    vals[f] = kc ? h[3 * f + 2] : 0.5 * b * 1.83787706640934548356 - h[3 * f] + 0.5 * h[3 * f + 1];
  }
  return 0;
}

}  // namespace gpsapi

extern "C" {

// 4-fold (nfold) block-LOO objective of the full GP at theta (DSS: KF:487-543; KC: the
// K20:655-720 body on A = K + σ²I; ES: KF:607-663) and, with grad != NULL, its analytic
// gradient (`.backward()` at KF:543 / 663): M = −A⁻¹ Gblk A⁻¹ − ½(vαᵀ + αvᵀ), v = A⁻¹g.
static int full_blockloo(gps_ctx* ctx, int kind, const double* theta, int n_ell, int nfold,
                         int objective, const EsArgs* es, double* value, double* grad,
                         double* fold_values) {
  int rc;
  if ((rc = full_fit_core(ctx, kind, theta, n_ell))) return rc;
  const int64_t n = ctx->n, np = ctx->n_pad;
  ARGCHK(n >= nfold, "fewer rows than folds");
  hipStream_t s = ctx->stream;
  {  // A⁻¹ (full) = L⁻ᵀL⁻¹ into A
    GemmParams p = gp0();
    p.A = ctx->Linv.d(); p.lda = np; p.B = ctx->Linv.d(); p.ldb = np;
    p.C = ctx->A.d(); p.ldc = np;
    p.M = (int)np; p.N = (int)np; p.K = (int)np; p.tri = TRI_K_GE_I; p.lower_out = 1;
    if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p))) return rc;
    Prof pr(ctx, "grad_mirror", 0, 16.0 * (double)np * np / 2);
    HIPCHK(launch_sym_mirror(ctx->A.d(), np, (int)np, s));
  }
  double* Ainv = ctx->A.d();
  auto getP = [&](int, int64_t a, int64_t b, double* P, int64_t bp) -> int {
    HIPCHK(launch_pad_copy(Ainv + a * np + a, np, P, bp, (int)b, (int)b, (int)bp, (int)bp, 1, s));
    return 0;
  };
  double* Gblk = nullptr;
  if (grad) {  // zero outside the fold squares (which move with n and nfold): cleared per call
    HIPCHK(ensure(ctx, ctx->bGblk, (size_t)np * np * 8));
    HIPCHK(hipMemsetAsync(ctx->bGblk.p, 0, (size_t)np * np * 8, s));
    HIPCHK(ensure(ctx, ctx->gu, np * 8));
    HIPCHK(hipMemsetAsync(ctx->gu.p, 0, np * 8, s));
    Gblk = ctx->bGblk.d();
  }
  auto gdst = [&](int64_t a, int64_t) { return std::make_pair(Gblk + a * np + a, np); };
  auto gdone = [](int, int64_t, int64_t) { return 0; };
  std::vector<double> fv(nfold);
  if ((rc = blockloo_folds(ctx, fold_bounds(n, nfold), objective, ctx->alpha.d(), ctx->y.d(), getP,
                           grad != nullptr, gdst, gdone, grad ? ctx->gu.d() : nullptr, es,
                           fv.data())))
    return rc;
  ctx->fitted = true;  // blockloo_folds checked the main factor (check_info)
  double tot = 0.0;
  for (int f = 0; f < nfold; ++f) tot += fv[f];
  *value = tot;
  if (fold_values)
    for (int f = 0; f < nfold; ++f) fold_values[f] = fv[f];
  if (!grad) return 0;
  const int d = ctx->d;
  HIPCHK(ensure(ctx, ctx->gv, np * 8));
  HIPCHK(ensure(ctx, ctx->Mx, (size_t)np * np * 8));
  HIPCHK(ensure(ctx, ctx->bT, (size_t)np * np * 8));
  HIPCHK(launch_gemv_full(Ainv, np, ctx->gu.d(), ctx->gv.d(), (int)np, (int)np, s));
  {  // T = A⁻¹ Gblk, K restricted per 16-column group to the folds those columns touch
    const std::vector<int64_t> bnd = fold_bounds(n, nfold);
    const int64_t groups = np / 16;
    std::vector<int> kr((size_t)2 * groups, 0);
    auto fold_of = [&](int64_t col) {
      int f = 0;
      while (f + 1 < nfold && col >= bnd[f + 1]) ++f;
      return f;
    };
    for (int64_t q = 0; q < groups; ++q) {
      const int64_t c0 = q * 16, c1 = std::min<int64_t>(c0 + 15, n - 1);
      if (c0 >= n) {  // padded columns of Gblk are zero: any range is exact; repeating the
        kr[2 * q] = kr[2 * q - 2];  // last real group's keeps kr monotone, which the GEMM's
        kr[2 * q + 1] = kr[2 * q - 1];  // first-group begin / last-group end per tile relies on
        continue;
      }
      kr[2 * q] = (int)(bnd[fold_of(c0)] / 16 * 16);
      kr[2 * q + 1] = (int)std::min<int64_t>(np, (bnd[fold_of(c1) + 1] + 15) / 16 * 16);
    }
    HIPCHK(ensure(ctx, ctx->bkr, kr.size() * sizeof(int)));
    HIPCHK(hipMemcpyAsync(ctx->bkr.p, kr.data(), kr.size() * sizeof(int), hipMemcpyHostToDevice, s));
    GemmParams p = gp0();
    p.A = Ainv; p.lda = np; p.B = Gblk; p.ldb = np; p.C = ctx->bT.d(); p.ldc = np;
    p.M = (int)np; p.N = (int)np; p.K = (int)np; p.tri = TRI_KR_J;
    p.kr = static_cast<const int*>(ctx->bkr.p);
    if ((rc = gemm(ctx, LAY_N, LAY_N, EPI_STORE, p))) return rc;
    HIPCHK(hipStreamSynchronize(s));  // the host kr vector must outlive the async copy
  }
  {  // Mx = T A⁻¹ (lower tiles)
    GemmParams p = gp0();
    p.A = ctx->bT.d(); p.lda = np; p.B = Ainv; p.ldb = np; p.C = ctx->Mx.d(); p.ldc = np;
    p.M = (int)np; p.N = (int)np; p.K = (int)np; p.lower_out = 1;
    if ((rc = gemm(ctx, LAY_N, LAY_N, EPI_STORE, p))) return rc;
  }
  GradParams gpar;
  memset(&gpar, 0, sizeof(gpar));
  gpar.x = ctx->X.d(); gpar.n = (int)n; gpar.d = d; gpar.sf2 = ctx->th.sf2;
  for (int k = 0; k < d; ++k) gpar.inv_ell[k] = ctx->th.inv_ell[k];
  gpar.Ainv = Ainv; gpar.ldm = np; gpar.alpha = ctx->alpha.d();
  gpar.a2 = -1.0; gpar.a3 = -1.0; gpar.v = ctx->gv.d(); gpar.Mx = ctx->Mx.d();
  const int passes = grad_contract_passes(d);
  HIPCHK(ensure(ctx, ctx->gslab, (size_t)grad_contract_slab_doubles((int)n, d) * 8));
  HIPCHK(ensure(ctx, ctx->gout, (size_t)passes * 18 * 8));
  gpar.slab = ctx->gslab.d();
  {
    Prof pr(ctx, "grad_contract", 0, 16.0 * (double)n * n / 2);
    HIPCHK(launch_grad_contract(gpar, ctx->gout.d(), s));
  }
  std::vector<double> hout((size_t)passes * 18);
  HIPCHK(hipMemcpyAsync(hout.data(), ctx->gout.p, hout.size() * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const double bscale = kind == GPS_RBF ? 0.5 : 1.0;
  grad[0] = hout[0];
  double gl = 0.0;
  for (int k = 0; k < d; ++k) {
    const double gk = bscale * hout[(size_t)(k / 16) * 18 + 2 + (k % 16)];
    if (n_ell == d) grad[1 + k] = gk;
    gl += gk;
  }
  if (n_ell == 1) grad[1] = gl;
  grad[1 + n_ell] = ctx->th.sn2 * hout[1];
  return 0;
}

int gps_full_blockloo(gps_ctx* ctx, int kind, const double* theta, int n_ell, int nfold,
                      int objective, double* value, double* grad, double* fold_values) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(nfold >= 1 && nfold <= 64, "nfold must be in 1..64");
  ARGCHK(objective == GPS_BLOCK_DSS || objective == GPS_BLOCK_KC,
         "objective must be GPS_BLOCK_DSS or GPS_BLOCK_KC (the energy score: gps_full_blockloo_es)");
  ARGCHK(value != nullptr, "value is NULL");
  return full_blockloo(ctx, kind, theta, n_ell, nfold, objective, nullptr, value, grad,
                       fold_values);
}

// Energy-score block-LOO objective of the full GP (KF:607-663) with the caller's draws.
// C_f = ((A⁻¹)_ff)⁻¹ is a conditional covariance (Schur complement of A = K + σ²I), so
// σ²I <= C_f and diag C_f <= sf2 + σ²: these fix the Newton–Schulz scale and step count.
int gps_full_blockloo_es(gps_ctx* ctx, int kind, const double* theta, int n_ell, int nfold,
                         int num_sim, double beta, const double* draws, double* value,
                         double* grad, double* fold_values) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(nfold >= 1 && nfold <= 64, "nfold must be in 1..64");
  ARGCHK(num_sim >= 2 && num_sim <= 8192, "num_sim must be in 2..8192");
  ARGCHK(beta > 0.0 && beta <= 2.0, "beta must be in (0, 2]");
  ARGCHK(theta && draws && value, "NULL argument");
  ARGCHK(ctx->have_data, "gps_full_set_data first");
  ARGCHK(n_ell == 1 || n_ell == ctx->d, "n_ell must be 1 or d");
  const int64_t cnt = 2 * (int64_t)num_sim * ctx->n;
  HIPCHK(ensure(ctx, ctx->edraws, (size_t)cnt * 8));
  HIPCHK(hipMemcpyAsync(ctx->edraws.p, draws, (size_t)cnt * 8, hipMemcpyHostToDevice, ctx->stream));
  EsArgs es;
  es.S = num_sim;
  es.beta = beta;
  es.draws = ctx->edraws.d();
  es.lam_lb = std::exp(theta[1 + n_ell]);
  es.diag_ub = std::exp(theta[0]) + es.lam_lb;
  return full_blockloo(ctx, kind, theta, n_ell, nfold, GPS_BLOCK_ES, &es, value, grad,
                       fold_values);
}

// ES(m, c, shape1, data_y, num_sim, beta) (KF:70-101) of one Gaussian N(m, C) at y with the
// draws given (ξ then ξ', num_sim × b each): the compat helper.  No spectral bounds are known
// for a general C, so the Newton–Schulz iteration runs on C/trace(C) until ‖I − ZY‖ ≈ 0.
int gps_energy_score(gps_ctx* ctx, const double* m, const double* C, int64_t b, const double* y,
                     int num_sim, double beta, const double* draws, double* out) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(m && C && y && draws && out && b >= 1 && b <= (1 << 16), "bad argument");
  ARGCHK(num_sim >= 2 && num_sim <= 8192, "num_sim must be in 2..8192");
  ARGCHK(beta > 0.0 && beta <= 2.0, "beta must be in (0, 2]");
  hipStream_t s = ctx->stream;
  const int64_t bp = pad_to(b);
  if (int rc = upload(ctx, ctx->t0, C, b, b, b)) return rc;
  HIPCHK(ensure(ctx, ctx->bPI, (size_t)bp * bp * 8));
  HIPCHK(launch_pad_copy(ctx->t0.d(), b, ctx->bPI.d(), bp, (int)b, (int)b, (int)bp, (int)bp, 1, s));
  std::vector<double> r(b);  // the residual y − m (input marshalling: ẑ_S = m − y = −r)
  double tr = 0.0;
  for (int64_t i = 0; i < b; ++i) {
    r[i] = y[i] - m[i];
    tr += C[i * b + i];
  }
  ARGCHK(tr > 0.0, "C must be positive definite");
  if (int rc = upload(ctx, ctx->t1, r.data(), b, 1, bp)) return rc;
  HIPCHK(ensure(ctx, ctx->t2, (size_t)bp * 8));
  const int64_t cnt = 2 * (int64_t)num_sim * b;
  HIPCHK(ensure(ctx, ctx->edraws, (size_t)cnt * 8));
  HIPCHK(hipMemcpyAsync(ctx->edraws.p, draws, (size_t)cnt * 8, hipMemcpyHostToDevice, s));
  EsArgs es;
  es.S = num_sim;
  es.beta = beta;
  es.draws = ctx->edraws.d();
  double* dev_out = ctx->small.d();
  if (int rc = es_fold(ctx, s, ctx->ebuf, false, es, es.draws, b, bp, ctx->bPI.d(), ctx->t1.d(), tr, ctx->t2.d(),
                       nullptr, 0, nullptr, dev_out))
    return rc;
  HIPCHK(hipMemcpyAsync(ctx->hsmall, dev_out, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *out = ctx->hsmall[0];
  return 0;
}

// The folds of the GLOBAL rows (KF:496-499: [⌊fN/k⌋, ⌊(f+1)N/k⌋)) that lie in this rank's rows,
// as local bounds, and their global indices.  Sharded: the ranks' row counts are all-reduced
// (every rank then sees the same shard layout, so all agree on a refusal); a fold that
// straddles two shards is refused (gpscore.dist.fold_shard_rows shards on fold boundaries).
static int local_folds(gps_ctx* ctx, int nfold, std::vector<int64_t>& bnd, std::vector<int>& fid) {
  const int64_t n = ctx->fn;
  bnd.clear();
  fid.clear();
  if (!sharded(ctx)) {
    ARGCHK(n >= nfold, "fewer rows than folds");
    bnd = fold_bounds(n, nfold);
    for (int f = 0; f < nfold; ++f) fid.push_back(f);
    return 0;
  }
  const int P = ctx->nranks;
  hipStream_t s = ctx->stream;
  HIPCHK(ensure(ctx, ctx->bfv, (size_t)std::max(P, 64) * 8));
  std::vector<double> cnt((size_t)P, 0.0);
  cnt[ctx->rank] = (double)n;
  HIPCHK(hipMemcpyAsync(ctx->bfv.p, cnt.data(), (size_t)P * 8, hipMemcpyHostToDevice, s));
  if (int rc = allreduce_sum(ctx, ctx->bfv.d(), (size_t)P, s)) return rc;
  HIPCHK(hipMemcpyAsync(cnt.data(), ctx->bfv.p, (size_t)P * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  int64_t N = 0, off = 0;
  for (int r = 0; r < P; ++r) {
    if (r < ctx->rank) off += (int64_t)cnt[r];
    N += (int64_t)cnt[r];
  }
  ARGCHK(N >= nfold, "fewer rows than folds");
  const std::vector<int64_t> gb = fold_bounds(N, nfold);
  int64_t e = 0;
  for (int r = 0; r + 1 < P; ++r) {  // every interior shard boundary must be a fold boundary
    e += (int64_t)cnt[r];
    for (int f = 0; f < nfold; ++f)
      ARGCHK(!(gb[f] < e && e < gb[f + 1]),
             "sharded FITC block-LOO: a fold straddles two shards (shard the rows on fold "
             "boundaries: gpscore.dist.fold_shard_rows)");
  }
  for (int f = 0; f < nfold; ++f)
    if (gb[f] >= off && gb[f + 1] <= off + n && gb[f + 1] > gb[f]) {
      if (bnd.empty()) bnd.push_back(gb[f] - off);
      bnd.push_back(gb[f + 1] - off);
      fid.push_back(f);
    }
  ARGCHK(!fid.empty(), "sharded FITC block-LOO: this rank holds no whole fold");
  return 0;
}

// FITC block-LOO objective (K20:523-587 DSS, K20:655-720 KC): P_f = ((Q+Λ)⁻¹)_ff =
// Λ_f⁻¹ − Ũ_fŨ_fᵀ with Ũ = Λ⁻¹K Lb⁻ᵀ (one n×m TRMM), α = (y − Kc)/λ.  With grad / grad_z the
// `.backward()` at K20:587 / 720 w.r.t. θ and the inducing inputs (moved at K20:593 / 726):
// M = −C⁻¹GblkC⁻¹ − ½(vαᵀ + αvᵀ), v = C⁻¹g (C = Q + Λ), whitened (round 4, no explicit B⁻¹ or
// Km⁻¹; oracle.fast_fitc_blockloo): F̃ = Gblk Ũ (one b×b×m GEMM per fold), S̃ = ŨᵀF̃ (n·m²),
//   G_K  = (−2Λ⁻¹F̃ + 2ŨS̃) Lb⁻¹ − 2diag(M_ii) V Lm⁻¹ − vcᵀ − αŵᵀ,  V = K Lm⁻ᵀ, ŵ = Lm⁻ᵀVᵀv,
//   G_Km = Lb⁻ᵀS̃Lb⁻¹ + Lm⁻ᵀ(Vᵀdiag(M_ii)V)Lm⁻¹ + ½(ŵcᵀ + cŵᵀ),
//   M_ii = −G_ii/λ_i² + 2F̃_i·Ũ_i/λ_i − (ŨS̃)_i·Ũ_i − v_iα_i   (blk_mdiag, kernels_block.hip),
// contracted with ∂K/∂θ, ∂K/∂Z like gps_fitc_grad (9·n·m² GEMM flops; round 3's explicit-inverse
// form took 14).  Row-sharded like gps_fitc_grad when every fold lies in one rank's rows
// (local_folds): the folds are local, the fold values and the n-sums Ũᵀg, S̃, Vᵀv,
// [Vᵀdiag(M_ii)V | ΣM_ii] and the contraction are all-reduced.
int gps_fitc_blockloo(gps_ctx* ctx, const double* theta, int n_ell, int nfold, int objective,
                      double* value, double* grad, double* grad_z, double* fold_values) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(nfold >= 1 && nfold <= 64, "nfold must be in 1..64");
  ARGCHK(objective == GPS_BLOCK_DSS || objective == GPS_BLOCK_KC,
         "objective must be GPS_BLOCK_DSS or GPS_BLOCK_KC");
  ARGCHK(value != nullptr, "value is NULL");
  double o[GPS_N_OBJ];
  int rc;
  if ((rc = fitc_fit_core(ctx, theta, n_ell, o))) return rc;
  ctx->f_fitted = true;
  const Theta& th = ctx->fth;
  const int64_t n = ctx->fn, np = ctx->fn_pad, m = ctx->m, mp = ctx->m_pad;
  const int d = ctx->fd;
  const bool shard = sharded(ctx);
  std::vector<int64_t> bnd;
  std::vector<int> fid;
  if ((rc = local_folds(ctx, nfold, bnd, fid))) return rc;
  hipStream_t s = ctx->stream;
  const bool want = grad != nullptr || grad_z != nullptr;
  const int64_t ldr = want ? 3 * mp : mp;  // [Ũ → Y Lb⁻¹ | ŨS̃ → Y → V Lm⁻¹ | V]
  const int64_t bp = bounds_pad(bnd);
  HIPCHK(ensure(ctx, ctx->fR, (size_t)np * ldr * 8));
  HIPCHK(ensure(ctx, ctx->fgv, (size_t)13 * np * 8));
  double* U = ctx->fR.d();
  double* vb = ctx->fgv.d();
  double *alpha = vb, *dinv = vb + np, *v = vb + 2 * np, *ulam = vb + 3 * np, *hh = vb + 4 * np,
         *hl2 = vb + 5 * np, *gg = vb + 6 * np, *gd = vb + 7 * np, *md = vb + 8 * np,
         *scl = vb + 11 * np, *zv = vb + 12 * np;
  HIPCHK(launch_fitc_grad_terms(ctx->fy.d(), ctx->lam.d(), ctx->r.d(), ctx->g.d(), (int)n, (int)np,
                                GPS_OBJ_NLML, (double)n, alpha, dinv, v, ulam, hh, hl2, s));
  // Ũ = Λ⁻¹ K Lb⁻ᵀ
  if ((rc = fitc_knm_xt(ctx, ldr, ctx->Lb.d(), U))) return rc;
  HIPCHK(launch_row_scale(U, ldr, (int)np, (int)mp, ctx->ilam.d(), s));
  // gradient buffers (whitened, round 4; oracle.fast_fitc_blockloo): R slots [Ũ | ŨS̃ → Y | V]
  double *Sm = nullptr, *T1 = nullptr, *Sfin = nullptr, *KmD = nullptr, *F = nullptr;
  double* US = U + mp;
  double* V = U + 2 * mp;
  if (want) {
    HIPCHK(ensure(ctx, ctx->fgB, (size_t)(shard ? 5 : 4) * mp * mp * 8));
    double* Bb = ctx->fgB.d();
    Sm = Bb; T1 = Bb + mp * mp; Sfin = Bb + 2 * mp * mp; KmD = Bb + 3 * mp * mp;
    HIPCHK(ensure(ctx, ctx->bF, (size_t)np * mp * 8));
    HIPCHK(ensure(ctx, ctx->bEf, (size_t)bp * mp * 8));
    F = ctx->bF.d();
    HIPCHK(hipMemsetAsync(F, 0, (size_t)np * mp * 8, s));
    HIPCHK(hipMemsetAsync(gg, 0, (size_t)2 * np * 8, s));  // g and diag(Gblk)
  }
  HIPCHK(ensure(ctx, ctx->bT, (size_t)bp * mp * 8));
  // the fold covariances C_f = Λ_f + K_f B_{−f}⁻¹K_fᵀ (round 5, oracle.fitc_fold_cov): first every
  // local fold's S_g = K_gᵀΛ_g⁻¹K_g (one SYRK over its rows); B_{−f} is then K̃mm + Σ_{g≠f} S_g
  // (+ the other ranks' Σ S when sharded) — no subtraction of nearly equal b×b terms
  const int nfl = (int)fid.size();
  const int64_t mm = mp * mp;
  HIPCHK(ensure(ctx, ctx->bSg, (size_t)nfl * mm * 8));
  HIPCHK(ensure(ctx, ctx->bBf, (size_t)mm * 8));
  HIPCHK(ensure(ctx, ctx->bldf, (size_t)mp * 8));
  HIPCHK(ensure(ctx, ctx->bW, (size_t)bp * mp * 8));
  HIPCHK(ensure(ctx, ctx->bkv, (size_t)bp * 8));
  HIPCHK(ensure(ctx, ctx->W, std::max(ctx->W.cap, potrf_ws_doubles(mp) * 8)));
  if (ctx->bLf.cap < (size_t)mm * 8 || !factor_zeroed(ctx, ctx->bLf.d(), mp)) {
    HIPCHK(ensure(ctx, ctx->bLf, (size_t)mm * 8));
    HIPCHK(zero_factor(ctx, ctx->bLf.d(), mp, s));
  }
  HIPCHK(hipMemsetAsync(ctx->bSg.p, 0, (size_t)nfl * mm * 8, s));  // (upper tiles stay zero)
  for (int gl = 0; gl < nfl; ++gl) {
    const int64_t a = bnd[gl], b = bnd[gl + 1] - bnd[gl];
    HIPCHK(launch_pad_copy(ctx->Knm.d() + a * mp, mp, ctx->bT.d(), mp, (int)b, (int)mp, (int)bp,
                           (int)mp, 0, s));
    HIPCHK(launch_pad_copy(ctx->ilam.d() + a, 1, ctx->bkv.d(), 1, (int)b, 1, (int)bp, 1, 0, s));
    GemmParams p = gp0();
    p.A = ctx->bT.d(); p.lda = mp; p.B = ctx->bT.d(); p.ldb = mp; p.C = ctx->bSg.d() + gl * mm;
    p.ldc = mp; p.M = (int)mp; p.N = (int)mp; p.K = (int)bp; p.kscale = ctx->bkv.d(); p.lower_out = 1;
    if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, p))) return rc;
  }
  const double* remote = nullptr;
  // the other ranks' folds: Σ_all S − Σ_local S (m×m; all-reduced once).  The S_g are PSD with
  // comparable norms (folds of equal size), so ‖Σ_local‖ ≈ ‖Σ_all‖/P and the subtraction's
  // rounding is ε(‖Σ_all‖ + ‖Σ_local‖) ≤ ε·(P + 1)/(P − 1)·‖Σ_remote‖ — 3ε at P = 2, not the
  // cancellation of nearly equal terms; forming the remote sum without it would take
  // a P·m² exchange (each rank's slot all-reduced) instead of m².  test_gpu_shards' fold-sharded
  // block-LOO cases hold the result to the unsharded one within 30× its conditioning floor.
  if (shard) {
    HIPCHK(ensure(ctx, ctx->bRem, (size_t)mm * 8));
    HIPCHK(launch_fold_sum(ctx->bSg.d(), mm, nfl, -1, nullptr, nullptr, 1.0, ctx->bRem.d(), mm, s));
    if ((rc = allreduce_sum(ctx, ctx->bRem.d(), (size_t)mm, s))) return rc;
    HIPCHK(launch_fold_sum(ctx->bSg.d(), mm, nfl, -1, ctx->bRem.d(), nullptr, -1.0, ctx->bRem.d(), mm, s));
    remote = ctx->bRem.d();
  }
  // W_f = K_f L_{−f}⁻ᵀ into bW (bpp × mp) and −½log|C_f| (determinant lemma) into *hl
  auto getW = [&](int fl, int64_t a, int64_t b, int64_t bpp, double* hl) -> int {
    HIPCHK(launch_fold_sum(ctx->bSg.d(), mm, nfl, fl, ctx->Kmm.d(), remote, 1.0, ctx->bBf.d(), mm, s));
    if (int rc2 = potrf_inv(ctx, ctx->bBf.d(), mp, ctx->bLf.d(), ctx->W.d(), ctx->bldf.d(), (int)m,
                            nullptr))
      return rc2;
    HIPCHK(launch_pad_copy(ctx->Knm.d() + a * mp, mp, ctx->bT.d(), mp, (int)b, (int)mp, (int)bpp,
                           (int)mp, 0, s));
    GemmParams p = gp0();
    p.A = ctx->bT.d(); p.lda = mp; p.B = ctx->bLf.d(); p.ldb = mp; p.C = ctx->bW.d(); p.ldc = mp;
    p.M = (int)bpp; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_LE_J;
    if (int rc2 = gemm(ctx, LAY_N, LAY_T, EPI_STORE, p)) return rc2;
    HIPCHK(launch_fold_logdet(ctx->bldf.d(), ctx->ldb.d(), (int)m, ctx->lam.d() + a, (int)b, hl, s));
    return 0;
  };
  std::vector<double> fvl(fid.size()), fv((size_t)nfold, 0.0);
  if ((rc = fitc_lr_folds(ctx, bnd, objective, alpha, getW, U, ldr, want ? F : nullptr,
                          want ? gd : nullptr, want ? gg : nullptr, fvl.data())))
    return rc;
  for (size_t j = 0; j < fid.size(); ++j) fv[fid[j]] = fvl[j];
  if (shard) {  // every fold's value on every rank (each fold is computed by exactly one rank)
    HIPCHK(hipMemcpyAsync(ctx->bfv.p, fv.data(), (size_t)nfold * 8, hipMemcpyHostToDevice, s));
    if ((rc = allreduce_sum(ctx, ctx->bfv.d(), (size_t)nfold, s))) return rc;
    HIPCHK(hipMemcpyAsync(fv.data(), ctx->bfv.p, (size_t)nfold * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  double tot = 0.0;
  for (int f = 0; f < nfold; ++f) tot += fv[f];
  *value = tot;
  if (fold_values)
    for (int f = 0; f < nfold; ++f) fold_values[f] = fv[f];
  if (!want) return 0;
  // v = C⁻¹g = g/λ − Ũ(Ũᵀg)
  HIPCHK(ensure(ctx, ctx->fgm, (size_t)6 * mp * 8));
  double* mb = ctx->fgm.d();
  double *tku = mb, *what = mb + 2 * mp;
  HIPCHK(launch_vec_mul(gg, ctx->ilam.d(), (int)np, ulam, s));
  HIPCHK(launch_colred(U, ldr, (int)np, (int)mp, 0, gg, nullptr, tku, nullptr, ctx->fslab.d(), s));
  if ((rc = allreduce_sum(ctx, tku, (size_t)mp, s))) return rc;
  HIPCHK(launch_gemv_full(U, ldr, tku, zv, (int)np, (int)mp, s));
  HIPCHK(launch_fitc_grad_v(ulam, zv, nullptr, (int)n, v, s));
  {  // S̃ = ŨᵀF̃ (n·m²), all-reduced
    GemmParams q = gp0();
    q.A = U; q.lda = ldr; q.B = F; q.ldb = mp; q.C = Sm; q.ldc = mp;
    q.M = (int)mp; q.N = (int)mp; q.K = (int)np;
    if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, q))) return rc;
  }
  if ((rc = allreduce_sum(ctx, Sm, (size_t)mp * mp, s))) return rc;
  {  // ŨS̃ into slot 1
    GemmParams p = gp0();
    p.A = U; p.lda = ldr; p.B = Sm; p.ldb = mp; p.C = US; p.ldc = ldr;
    p.M = (int)np; p.N = (int)mp; p.K = (int)mp;
    if ((rc = gemm(ctx, LAY_N, LAY_N, EPI_STORE, p))) return rc;
  }
  {  // M_ii, the V Lm⁻¹ row scale, and Y = −2Λ⁻¹F̃ + 2ŨS̃ over slot 1 — one pass over F̃, ŨS̃, Ũ
    Prof pr(ctx, "blk_mdiag", 0, 32.0 * np * mp);
    HIPCHK(launch_blk_mdiag(F, mp, US, ldr, U, ldr, (int)mp, gd, ctx->lam.d(), v, alpha, (int)n,
                            (int)np, md, scl, US, ldr, s));
  }
  if ((rc = fitc_tri_right(ctx, US, ldr, ctx->Lb.d(), U, ldr, np))) return rc;  // Y Lb⁻¹ → slot 0
  if ((rc = fitc_knm_xt(ctx, ldr, ctx->Lm.d(), V))) return rc;                  // V = K Lm⁻ᵀ
  // ŵ = Lm⁻ᵀVᵀv;  Lm⁻ᵀ(Vᵀdiag(M_ii)V)Lm⁻¹;  Σ M_ii
  // [P | Σ M_ii | (pad) | Vᵀv]: P = Vᵀdiag(M_ii)V lower-packed (m(m+1)/2) when sharded, else
  // the padded lower tiles (gps_fitc_grad's layout)
  HIPCHK(ensure(ctx, ctx->fgred, (size_t)(mp * mp + 2 * mp + 64) * 8));
  const int64_t plen = shard ? m * (m + 1) / 2 : mp * mp;
  const int64_t off_tw = (plen + 2) / 2 * 2;
  double* red = ctx->fgred.d();
  double* smd = red + plen;
  double* tw = red + off_tw;
  HIPCHK(launch_colred(V, ldr, (int)np, (int)mp, 0, v, nullptr, tw, nullptr, ctx->fslab.d(), s));
  if ((rc = allreduce_sum(ctx, tw, (size_t)mp, s))) return rc;
  if ((rc = fitc_lt_vec(ctx, ctx->Lm.d(), tw, what))) return rc;  // ŵ = Lm⁻ᵀ Vᵀv
  if ((rc = fitc_syrk(ctx, md, nullptr, red, shard, V, ldr))) return rc;
  HIPCHK(launch_dot(md, nullptr, (int)np, smd, s));
  if ((rc = allreduce_sum(ctx, red, (size_t)(plen + 1), s))) return rc;
  double* Pfull = red;
  if (shard) {
    Pfull = ctx->fgB.d() + 4 * mp * mp;
    HIPCHK(launch_sym_unpack(red, (int)m, (int)mp, nullptr, 1, Pfull, s));
  } else {
    HIPCHK(launch_sym_mirror(red, mp, (int)mp, s));
  }
  if ((rc = fitc_tri_right(ctx, V, ldr, ctx->Lm.d(), US, ldr, np))) return rc;  // V Lm⁻¹ → slot 1
  if ((rc = fitc_tri_right(ctx, Pfull, mp, ctx->Lm.d(), T1, mp, mp))) return rc;
  if ((rc = fitc_tri_left_t(ctx, ctx->Lm.d(), T1, KmD))) return rc;
  if ((rc = fitc_tri_right(ctx, Sm, mp, ctx->Lb.d(), T1, mp, mp))) return rc;   // Lb⁻ᵀS̃Lb⁻¹
  if ((rc = fitc_tri_left_t(ctx, ctx->Lb.d(), T1, Sfin))) return rc;
  // contractions with ∂Knm/∂θ, ∂Knm/∂Z and ∂Kmm/∂θ, ∂Kmm/∂Z
  const int passes = fitc_contract_passes(d);
  const int64_t outlen = (int64_t)passes * 17 + m * d;
  HIPCHK(ensure(ctx, ctx->fgslab, (size_t)std::max(fitc_contract_slab_doubles((int)n, (int)mp, d),
                                               fitc_contract_slab_doubles((int)m, (int)mp, d)) * 8));
  HIPCHK(ensure(ctx, ctx->fgout, (size_t)(2 * outlen + 8) * 8));
  double* out1 = ctx->fgout.d();
  double* out2 = out1 + outlen;
  FitcContractParams cp;
  memset(&cp, 0, sizeof(cp));
  cp.d = d;
  cp.sf2 = th.sf2;
  for (int k = 0; k < d; ++k) cp.inv_ell[k] = th.inv_ell[k];
  cp.slab = ctx->fgslab.d();
  {
    FitcContractParams p = cp;
    p.xr = ctx->fX.d(); p.xc = ctx->Z.d(); p.nr = (int)n; p.nc = (int)m; p.nc_pad = (int)mp;
    p.R[0] = U; p.ldr[0] = ldr; p.coef[0] = 1.0;                  // Y Lb⁻¹
    p.R[1] = US; p.ldr[1] = ldr; p.coef[1] = 1.0; p.rs[1] = scl;  // −2diag(M_ii) V Lm⁻¹
    p.nt = 2;
    p.pc[0] = -1.0; p.pv[0] = v; p.qv[0] = ctx->c.d();
    p.pc[1] = -1.0; p.pv[1] = alpha; p.qv[1] = what;
    Prof pr(ctx, "fitc_grad_contract", 0, 8.0 * 2 * np * mp);
    HIPCHK(launch_fitc_grad_contract(p, out1, out1 + passes * 17, s));
  }
  if ((rc = allreduce_sum(ctx, out1, (size_t)outlen, s))) return rc;
  {  // the m×m contraction: every operand is global by now (replicated on every rank)
    FitcContractParams p = cp;
    p.xr = ctx->Z.d(); p.xc = ctx->Z.d(); p.nr = (int)m; p.nc = (int)m; p.nc_pad = (int)mp;
    p.R[0] = Sfin; p.ldr[0] = mp; p.coef[0] = 1.0;
    p.R[1] = KmD; p.ldr[1] = mp; p.coef[1] = 1.0;
    p.nt = 2;
    p.pc[0] = 0.5; p.pv[0] = what; p.qv[0] = ctx->c.d();
    p.pc[1] = 0.5; p.pv[1] = ctx->c.d(); p.qv[1] = what;
    Prof pr(ctx, "fitc_grad_contract_mm", 0, 8.0 * 2 * mp * mp);
    HIPCHK(launch_fitc_grad_contract(p, out2, out2 + passes * 17, s));
  }
  std::vector<double> hout((size_t)2 * outlen + 1);
  HIPCHK(hipMemcpyAsync(hout.data(), out1, (size_t)2 * outlen * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hout.data() + 2 * outlen, smd, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const double* h1 = hout.data();
  const double* h2 = h1 + outlen;
  const double sum_md = hout[2 * outlen];
  if (grad) {
    grad[0] = h1[0] + h2[0] + th.sf2 * sum_md;
    double gl = 0.0;
    for (int k = 0; k < d; ++k) {
      const size_t at = (size_t)(k / 16) * 17 + 1 + (k % 16);
      const double gk = h1[at] + h2[at];
      if (n_ell == d) grad[1 + k] = gk;
      gl += gk;
    }
    if (n_ell == 1) grad[1] = gl;
    grad[1 + n_ell] = th.sn2 * sum_md;
  }
  if (grad_z) {
    const double* z1 = h1 + passes * 17;
    const double* z2 = h2 + passes * 17;
    for (int64_t j = 0; j < m; ++j)
      for (int k = 0; k < d; ++k)
        grad_z[j * d + k] = (z1[j * d + k] + 2.0 * z2[j * d + k]) * th.inv_ell[k];
  }
  return 0;
}

}  // extern "C"
