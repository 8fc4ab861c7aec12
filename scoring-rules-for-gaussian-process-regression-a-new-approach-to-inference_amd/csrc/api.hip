// C-ABI of libgpscore.so (declared in include/gpscore.h), core: context, device buffers,
// options, profiling, the launch helpers and the recursive Cholesky + triangular-inverse driver,
// and the L1 blocks.  The paths live in api_full.hip / api_fitc.hip / api_block.hip /
// api_comm.hip (api_internal.h).  Host orchestration only; the arithmetic lives in kernels_*.hip.
//
// Full GP, one fit (KF:239-245 LOO-CRPS, KF:329-334 NLML, KF:416-424 LOO-LogS):
//   A = K(X,X) + σ²I (lower)  →  [L, L⁻¹] = potrf_inv(A)  →  β = L⁻¹y
//   → α = L⁻ᵀβ, d = diag(A⁻¹) = colsum(L⁻¹∘L⁻¹)  →  μ_loo = y − α/d, σ²_loo = 1/d
//   NLML = ½n log2π + Σ log L_ii + ½‖β‖²
// Full GP, predict (cal_mean_and_cov KF:121-126, diag only):
//   V = L⁻¹ K_f*  (never stored: fused column reductions)  μ* = Vᵀβ,
//   σ²* = σ² + sf2 − colsum(V∘V)
// FITC (K20:222-340 restated, O(n m²)):
//   λ = sf2 − ‖Lm⁻¹k_i‖² + σ², B = K̃mm + KmnΛ⁻¹Knm (split-K SYRK, RCCL all-reduce
//   across row shards), c = B⁻¹KmnΛ⁻¹y, diag((Q+Λ)⁻¹) = 1/λ − ‖Lb⁻¹k_i‖²/λ²,
//   log|Q+Λ| = Σlogλ + log|B| − log|K̃mm|.
//
// potrf_inv (recursive, all O(n³) work in the MFMA GEMM):
//   [L11, L11⁻¹] = rec(A11);  L21 = A21 L11⁻ᵀ;  A22 −= L21 L21ᵀ;
//   T = L21 L11⁻¹ (into A21);  [L22, L22⁻¹] = rec(A22);  L⁻¹21 = −L22⁻¹ T
//   → n³/3 (potrf) + n³/3 (trtri) flops; base case: 128×128 LDS kernel.
#include "api_internal.h"

namespace gpsapi {

thread_local std::string g_err;  // (the last error of a call without a context)

int fail(gps_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  g_err = msg;
  return code;
}

// A cached factorisation graph bakes in the device addresses of the buffers its launches use
// (every one of them is in its key).  No graph may outlive such a buffer: before a buffer is
// freed (grown by ensure, or released), every graph whose key holds an address inside it is
// destroyed — after this context's streams drain, so none is in flight.  (Round 3 kept graphs
// alive for the context's lifetime instead, after destroying an exec that referenced freed
// buffers segfaulted the host and a replay read stale counters)
hipError_t sync_ctx_streams(gps_ctx* ctx) {
  for (hipStream_t st : {ctx->stream, ctx->side, ctx->aux[0], ctx->aux[1]})
    if (st) {
      const hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

hipError_t drop_graphs_in(gps_ctx* ctx, const void* p, size_t bytes) {
  if (!ctx || !p || ctx->pgraphs.empty()) return hipSuccess;
  const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
  bool synced = false;
  for (size_t i = 0; i < ctx->pgraphs.size();) {
    bool hit = false;
    for (uintptr_t v : ctx->pgraphs[i].key) hit |= v >= lo && v < hi;
    if (!hit) { ++i; continue; }
    if (!synced) {
      const hipError_t e = sync_ctx_streams(ctx);
      if (e != hipSuccess) return e;
      synced = true;
    }
    const hipError_t e = hipGraphExecDestroy(ctx->pgraphs[i].exec);
    ctx->pgraphs.erase(ctx->pgraphs.begin() + (ptrdiff_t)i);
    ++ctx->graph_dropped;
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

void forget_zeroed(gps_ctx* ctx, const void* p, size_t bytes) {
  const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
  for (auto it = ctx->zeroed.lower_bound(lo); it != ctx->zeroed.end() && it->first < hi;)
    it = ctx->zeroed.erase(it);
}

hipError_t ensure(gps_ctx* ctx, DBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return hipSuccess;
  if (b.p) {
    forget_zeroed(ctx, b.p, b.cap);
    hipError_t e = drop_graphs_in(ctx, b.p, b.cap);
    if (e != hipSuccess) return e;
    e = hipFree(b.p);
    if (e != hipSuccess) return e;
  }
  b.p = nullptr;
  b.cap = 0;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e == hipSuccess) b.cap = bytes;
  return e;
}
void release(gps_ctx* ctx, DBuf& b) {
  if (b.p) {
    forget_zeroed(ctx, b.p, b.cap);
    (void)drop_graphs_in(ctx, b.p, b.cap);
    (void)hipFree(b.p);
  }
  b.p = nullptr;
  b.cap = 0;
}

// ------------------------------------------------------------------ profiling
int get_event(gps_ctx* c) {
  if (c->ev_used == c->ev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    c->ev.push_back(e);
  }
  return (int)c->ev_used++;
}


// phase timing (gps_phase_enable): a timing event from the phase pool recorded on st
int phase_event(gps_ctx* c, hipStream_t st) {
  if (c->ph_used == c->ph_ev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    c->ph_ev.push_back(e);
  }
  const int i = (int)c->ph_used++;
  return hipEventRecord(c->ph_ev[i], st) == hipSuccess ? i : -1;
}
void phase_mark(gps_ctx* c, const char* name) {
  if (!c->phase) return;
  const int e = phase_event(c, c->stream);
  if (e >= 0) c->ph_marks.push_back({name, e});
}

// fork/join event from a per-call pool (reset by potrf_inv)
hipEvent_t sync_event(gps_ctx* c) {
  if (c->sync_used == c->sync_ev.size()) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    c->sync_ev.push_back(e);
  }
  return c->sync_ev[c->sync_used++];
}

// --------------------------------------------------------------- launch helpers

GemmParams gp0() {
  GemmParams p;
  memset(&p, 0, sizeof(p));
  p.alpha = 1.0;
  p.ksplit = 1;
  return p;
}

// profiling tag: operation + size class (s: < 16 output tiles, m: < 256, l: >= 256)
const char* gemm_tag(int al, int bl, int epi, const GemmParams& p) {
  (void)al;
  (void)bl;
  if (epi == EPI_COLRED) return "gemm_trmm_colred";
  if (epi == EPI_ROWSQ || epi == EPI_ROWSQ_DOT) return "gemm_rowsq";
  const int64_t tiles = (int64_t)(p.M / GPS_TILE) * (p.N / GPS_TILE) / (p.lower_out ? 2 : 1);
  const int cls = tiles < 16 ? 0 : (tiles < 256 ? 1 : 2);
  static const char* syrk[3] = {"gemm_syrk_s", "gemm_syrk_m", "gemm_syrk_l"};
  static const char* trmm[3] = {"gemm_trmm_s", "gemm_trmm_m", "gemm_trmm_l"};
  static const char* plain[3] = {"gemm_s", "gemm_m", "gemm_l"};
  if (p.lower_out) return p.ksplit > 1 ? "gemm_syrk_splitk" : syrk[cls];
  return p.tri ? trmm[cls] : plain[cls];
}

// algorithmic flops of one launch (triangular operands counted at their nonzero half)
double gemm_flops(const GemmParams& p) {
  const double M = p.M, N = p.N, K = p.K;
  if (p.lower_out && p.tri == TRI_K_GE_I) {  // L⁻ᵀL⁻¹ (LAUUM): k >= i over the lower half
    double f = 0.0;
    for (int64_t i = 0; i < p.M; i += GPS_TILE) f += (double)(i + GPS_TILE) * (K - i);
    return 2.0 * GPS_TILE * f;
  }
  if (p.lower_out) return M * (M + 1) * K;  // SYRK, lower half
  if ((p.tri == TRI_K_LE_I || p.tri == TRI_K_LE_J) && p.tri_off) {
    // rows (K_LE_I) / columns (K_LE_J) [off, off + len) of a larger triangular product
    const double len = p.tri == TRI_K_LE_I ? M : N, other = p.tri == TRI_K_LE_I ? N : M;
    const double o = p.tri_off, e = std::min<double>(K, o + len);
    return other * (e * e - o * o) + 2.0 * other * K * std::max(0.0, o + len - e);
  }
  if (p.tri) return M * N * K;              // triangular operand: half of 2MNK
  return 2.0 * M * N * K;
}

int gemm(gps_ctx* ctx, int al, int bl, int epi, const GemmParams& p, hipStream_t st) {
  if (!st) st = ctx->stream;
  GemmParams q = p;
  if (q.map_mode == 0) q.map_mode = ctx->gemm_map;
  // the stream's slabs: gemm_plan may split K on small grids; an explicit 64-tile split uses them
  if (epi == EPI_STORE && (q.ksplit == 1 || q.tile == 64) && !q.ws) {
    DBuf& ws = st == ctx->side      ? ctx->ws_side
               : st == ctx->aux[0] ? ctx->ws_aux[0]
               : st == ctx->aux[1] ? ctx->ws_aux[1]
                                   : ctx->ws_main;
    HIPCHK(ensure(ctx, ws, (size_t)kSplitWsDoubles * 8));
    q.ws = ws.d();
    q.ws_cap = kSplitWsDoubles;
    if (st == ctx->stream && ctx->sk_cnt.p) {  // the stream-K tail's tickets (main stream only)
      q.sk_cnt = static_cast<int*>(ctx->sk_cnt.p);
      q.sk_slots = 2 * ctx->ncu;
    }
  }
  std::string tag = gemm_tag(al, bl, epi, p);
  if (ctx->prof > 1) {  // per-shape accounting (gps_prof_enable(ctx, 2))
    const GemmPlan plan = gemm_plan(epi, q, q.ws ? q.ws_cap : 0);
    char buf[160];
    snprintf(buf, sizeof(buf), " %c%c %dx%dx%d tri%d t%d ks%d ld%lld", al ? 'T' : 'N',
             bl ? 'T' : 'N', p.M, p.N, p.K, (int)p.tri, plan.tile, plan.ksplit, (long long)p.lda);
    tag += buf;
  }
  Prof pr(ctx, tag, gemm_flops(p), 0, st);
  HIPCHK(launch_gemm(al, bl, epi, q, st));
  return 0;
}

int gram(gps_ctx* ctx, const char* tag, const double* x, int n, const double* xp, int m, int d,
         const Theta& th, double diag_add, int lower, int pad_identity, double* out, int64_t ldo,
         int M, int N, hipStream_t st) {
  GramParams g;
  memset(&g, 0, sizeof(g));
  g.x = x;
  g.xp = xp;
  g.out = out;
  g.ldo = ldo;
  g.n = n;
  g.m = m;
  g.M = M;
  g.N = N;
  g.d = d;
  g.sf2 = th.sf2;
  g.diag_add = diag_add;
  g.lower = lower;
  g.pad_identity = pad_identity;
  for (int k = 0; k < d; ++k) g.inv_ell[k] = th.inv_ell[k];
  const double elems = lower ? 0.5 * (double)M * (M + 1) : (double)M * N;
  Prof pr(ctx, tag, 0, 8.0 * elems, st);
  HIPCHK(launch_gram(g, st ? st : ctx->stream));
  return 0;
}

// Rows [r0, r1) of the predictive product V = L⁻¹K_f* (cal_mean_and_cov KF:121-126; V is
// never stored): per 128-row tile the column partials Σ_rows w·V and Σ_rows V∘V go to pslab
// rows [r0/128, r1/128); row r needs L⁻¹ columns ≤ r only (K clipped at tri_off + row).
// (Forming rows [0, n1) during the factorisation, as FITC does with q, measured 1.3 % slower
// on C3: profiles/r2_ab_pred_pre.txt.)
int pred_rows(gps_ctx* ctx, int64_t r0, int64_t r1, const double* w, hipStream_t st) {
  const int64_t np = ctx->n_pad, ntp = ctx->nt_pad, tiles_m = np / GPS_TILE;
  GemmParams p = gp0();
  p.A = ctx->Linv.d() + r0 * np; p.lda = np; p.B = ctx->Ksf.d(); p.ldb = np;
  p.M = (int)(r1 - r0); p.N = (int)ntp; p.K = (int)r1; p.tri = TRI_K_LE_I; p.tri_off = (int)r0;
  p.w = w + r0;
  p.out0 = ctx->pslab.d() + (r0 / GPS_TILE) * ntp;
  p.out1 = ctx->pslab.d() + (tiles_m + r0 / GPS_TILE) * ntp;
  p.ld_out = ntp;
  return gemm(ctx, LAY_N, LAY_T, EPI_COLRED, p, st);
}

// FITC row norms ‖L⁻¹k_i‖² (K20:222-234 restated): output column tiles [c0, c1) of Knm·L⁻ᵀ
// (rows [c0, c1) of the triangular L⁻¹, K clipped at the column) into fslab rows [c0/128,
// c1/128); columns [0, n1) need only the top-level L11⁻¹.
int fitc_rowsq_cols(gps_ctx* ctx, const double* Lx, int64_t c0, int64_t c1, hipStream_t st) {
  const int64_t np = ctx->fn_pad, mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = ctx->Knm.d(); p.lda = mp; p.B = Lx + c0 * mp; p.ldb = mp;
  p.M = (int)np; p.N = (int)(c1 - c0); p.K = (int)c1; p.tri = TRI_K_LE_J; p.tri_off = (int)c0;
  p.kend = (int)pad_to(ctx->m, 16);
  p.out0 = ctx->fslab.d() + (c0 / GPS_TILE) * np; p.ld_out = np;
  return gemm(ctx, LAY_N, LAY_T, EPI_ROWSQ, p, st);
}

// The FITC row norms behind a running m×m factorisation (GPS_OPT_FITC_DEP): output
// column tiles [0, ncols) of Knm·L⁻ᵀ (L⁻¹ in L, its first nb_dag row tiles being written by a
// persistent launch of the context's FITC width whose row signals are sig: the whole factorisation
// (C4) or the top-level L11 block of a recursive one (C5)).  mode 1: the dependent launch — each column tile
// as soon as its row of L⁻¹ is final; mode 2: the completion launch after the factorisation — the
// tiles mode 1 left.  Both write fslab's row-norm partials as fitc_rowsq_cols does, so the sums
// that read them are unchanged.
int fitc_rowsq_dep(gps_ctx* ctx, const double* L, int* sig, int64_t ncols, int mode,
                   hipStream_t st, int64_t nb_dag) {
  const int64_t np = ctx->fn_pad, mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = ctx->Knm.d(); p.lda = mp; p.B = L; p.ldb = mp;
  p.M = (int)np; p.N = (int)ncols; p.K = (int)ncols; p.tri = TRI_K_LE_J;
  p.kend = (int)pad_to(ctx->m, 16);
  p.out0 = ctx->fslab.d(); p.ld_out = np;
  p.dep_sig = sig; p.dep_q = sig + kSigQueue; p.dep_err = static_cast<int*>(ctx->info.p) + 1;
  p.dep_grid = dag_width(ctx, nb_dag, true); p.dep_mode = mode;
  return gemm(ctx, LAY_N, LAY_T, EPI_ROWSQ, p, st);
}

// the task list of an nb-tile persistent block under the context's options
int dag_list_key(const gps_ctx* ctx, int64_t nb) {
  return (int)(3 * nb + ctx->dag_order);
}

// a block of nb 128-tiles goes to the persistent factorisation (GPS_OPT_DAG)
bool dag_block(const gps_ctx* ctx, int64_t nb) { return ctx->dag && nb >= 2 && nb <= ctx->dag_tiles; }

// the block sizes the recursion of an nb-tile factorisation hands to the persistent kernel, and
// how many counter ints all of them need together
void dag_blocks(const gps_ctx* ctx, int64_t nb, std::vector<int>& sizes, int64_t& cnt) {
  if (nb <= 1) return;
  if (dag_block(ctx, nb)) {
    sizes.push_back((int)nb);
    cnt += dag_cnt_ints((int)nb);
    return;
  }
  dag_blocks(ctx, nb / 2, sizes, cnt);
  dag_blocks(ctx, nb - nb / 2, sizes, cnt);
}

// workgroups of a persistent launch of nb tiles: one per CU, or half the CUs for the FITC m×m
// factorisations, whose chain needs ~70 workgroups at m = 2048 and whose side streams (the row
// norms, the test pre-pass) then get the other half (C4 12.72 -> 12.29 ms; the full GP's blocks
// want every CU: 124.2 vs 126.1 ms, profiles/r3_dag_width_ab.txt); with the dependent q launch
// beside Lm's factorisation (GPS_OPT_FITC_DEP) half stays best within noise: 112 / 96 workgroups
// measured 11.71 / 11.73 against 11.56 ms (profiles/r6i_fitc_dep_ab_c4_phases.txt)
int dag_width(const gps_ctx* ctx, int64_t nb, bool half) {
  const int auto_w = half ? std::max(4, ctx->ncu / 2) : ctx->ncu;
  return (int)std::min<int64_t>(ctx->dag_wgs > 0 ? ctx->dag_wgs : auto_w, std::max<int64_t>(4, 2 * nb * nb));
}

// recursive Cholesky + inverse on a padded (multiple of 128) SPD block.
// W is this level's workspace (n1·n2 doubles); deeper levels on the A22 side get
// the region after it, so a concurrent GEMM that still reads this level's W never
// races with them.
//
// T = L21 L11⁻¹ only feeds the final L⁻¹21 product, so (ctx->overlap) it runs on the
// side stream (fork / join events) concurrently with the trailing update and rec(A22).
// Measured on C3 and dropped from the build (round 1): a lookahead split of the trailing
// update, CU-masked side streams and split-K fill of the top-level SYRK — each neutral or
// slower end to end, because the side stream's T product already fills the idle slots.
int potrf_inv_rec(gps_ctx* ctx, double* A, int64_t lda, double* Linv, int64_t ldl, double* W,
                  int nb, double* logdiag, int* info, int base, int nreal, double* Lout,
                  int64_t ldlo, bool top) {
  hipStream_t s = ctx->stream;
  if (nb == 1) {
    Prof pr(ctx, "potrf_diag128", 2.0 * 128 * 128 * 128 / 3.0, 0);
    HIPCHK(launch_potrf_leaf(A, lda, Linv, ldl, Lout, ldlo, logdiag, info, base, nreal, s));
    return 0;
  }
  if (dag_block(ctx, nb)) {  // the whole block in one persistent launch (kernels_potrf.hip)
    auto it = ctx->dag_lists.find(dag_list_key(ctx, nb));
    const int64_t need = dag_cnt_ints(nb);
    if (it == ctx->dag_lists.end() || ctx->dag_cnt_used + need > (int64_t)(ctx->dag_cnt.cap / 4))
      return fail(ctx, -2, "persistent factorisation: task list / counters not prepared");
    DagParams d;
    d.A = A; d.lda = lda; d.Linv = Linv; d.ldl = ldl; d.Lout = Lout; d.ldlo = ldlo;
    d.logdiag = logdiag; d.info = info; d.base = base; d.nreal = nreal; d.T = nb;
    d.tasks = static_cast<const uint32_t*>(it->second.first.p); d.ntasks = it->second.second;
    d.cnt = static_cast<int*>(ctx->dag_cnt.p) + ctx->dag_cnt_used;
    d.spin_ticks = 200000000ull;  // 2 s at the 100 MHz real-time clock
    d.group = ctx->dag_group;
    d.sig = ctx->dag_sig;  // (a dependent row-norm launch reads its rows: the first block only)
    ctx->dag_sig = nullptr;
    ctx->dag_cnt_used += need;
    const double nn = 128.0 * nb;
    Prof pr(ctx, "potrf_dag", 2.0 * nn * nn * nn / 3.0, 0);
    HIPCHK(launch_potrf_dag(d, dag_width(ctx, nb, ctx->dag_half), s));
    return 0;
  }
  const int n1b = nb / 2, n2b = nb - n1b;
  const int n1 = n1b * GPS_TILE, n2 = n2b * GPS_TILE;
  double* A21 = A + (int64_t)n1 * lda;
  double* A22 = A21 + n1;
  double* Li21 = Linv + (int64_t)n1 * ldl;
  double* Li22 = Li21 + n1;
  int rc;
  // top level with a pre-pass request whose L11 block is one persistent launch and a signal block
  // (GPS_OPT_FITC_DEP, C5): the pre-pass's column tiles start beside that launch, each as soon as
  // its row of L11⁻¹ is final, and a completion launch takes the rest once L11⁻¹ is (below)
  const bool pre_here = top && ctx->pre.kind == PRE_FITC_Q && ctx->pre.n1 == n1;
  const bool pre_dep = pre_here && ctx->pre.sig && ctx->overlap && dag_block(ctx, n1b);
  // (on aux[1]: aux[0] may still hold the test-side pre-pass, FIFO ahead of it)
  // (an error return after the fork joins aux[1] first: no launch of this call may still run
  //  beside the context's next one)
  auto join_dep = [&]() {
    if (!pre_dep) return;
    hipEvent_t j = sync_event(ctx);
    if (j && hipEventRecord(j, ctx->aux[1]) == hipSuccess) (void)hipStreamWaitEvent(s, j, 0);
  };
  if (pre_dep) {
    hipEvent_t f = sync_event(ctx);
    if (!f) return fail(ctx, -2, "hipEventCreate failed");
    HIPCHK(hipEventRecord(f, s));
    HIPCHK(hipStreamWaitEvent(ctx->aux[1], f, 0));
    if ((rc = fitc_rowsq_dep(ctx, Linv, ctx->pre.sig, n1, 1, ctx->aux[1], n1b))) {
      join_dep();
      return rc;
    }
    ctx->dag_sig = ctx->pre.sig;  // (consumed by rec(A11)'s persistent launch)
  }
  rc = potrf_inv_rec(ctx, A, lda, Linv, ldl, W, n1b, logdiag, info, base, nreal, Lout, ldlo);
  ctx->dag_sig = nullptr;
  if (rc) {
    join_dep();
    return rc;
  }
  {  // W = L21 = A21 · L11⁻ᵀ
    GemmParams p = gp0();
    p.A = A21; p.lda = lda; p.B = Linv; p.ldb = ldl; p.C = W; p.ldc = n1;
    p.M = n2; p.N = n1; p.K = n1; p.tri = TRI_K_LE_J;
    if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_STORE, p))) return rc;
  }
  if (Lout) HIPCHK(hipMemcpy2DAsync(Lout + (int64_t)n1 * ldlo, ldlo * 8, W, (size_t)n1 * 8,
                                    (size_t)n1 * 8, n2, hipMemcpyDeviceToDevice, s));
  // an event fork + join costs ~13 us of dependent-chain latency (tools/launch_latency.hip)
  const bool forked = ctx->overlap;
  hipStream_t ts = forked ? ctx->side : s;
  hipEvent_t fork = sync_event(ctx), join = sync_event(ctx);
  if (!fork || !join) return fail(ctx, -2, "hipEventCreate failed");
  if (forked) {
    HIPCHK(hipEventRecord(fork, s));
    HIPCHK(hipStreamWaitEvent(ts, fork, 0));
  }
  {  // trailing update A22 -= L21 L21ᵀ (lower tiles); alone (nothing forked) it takes the
     // stream-K tail for its last round of workgroup slots
    GemmParams p = gp0();
    p.A = W; p.lda = n1; p.B = W; p.ldb = n1; p.C = A22; p.ldc = lda;
    p.M = n2; p.N = n2; p.K = n1; p.alpha = -1.0; p.beta = 1.0; p.lower_out = 1;
    p.sk_alone = forked ? 0 : 1;
    if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_STORE, p))) return rc;
  }
  {  // T = L21 · L11⁻¹ → A21 (off the critical path)
    GemmParams p = gp0();
    p.A = W; p.lda = n1; p.B = Linv; p.ldb = ldl; p.C = A21; p.ldc = lda;
    p.M = n2; p.N = n1; p.K = n1; p.tri = TRI_K_GE_J;
    if ((rc = gemm(ctx, LAY_N, LAY_N, EPI_STORE, p, ts))) return rc;
  }
  if (forked) HIPCHK(hipEventRecord(join, ts));
  // top level with a pre-pass request: L11⁻¹ is final now, so the product that needs only its
  // rows (FITC: the q column tiles [0, n1)) runs on aux[0] while rec(A22) — mostly
  // latency-bound launches at m ≤ 4k — runs
  if (pre_here) {
    hipStream_t ps = !ctx->overlap ? s : pre_dep ? ctx->aux[1] : ctx->aux[0];
    if (ps != s) {
      hipEvent_t f = sync_event(ctx);
      ctx->pre.join = sync_event(ctx);
      if (!f || !ctx->pre.join) return fail(ctx, -2, "hipEventCreate failed");
      HIPCHK(hipEventRecord(f, s));
      HIPCHK(hipStreamWaitEvent(ps, f, 0));
    }
    if ((rc = pre_dep ? fitc_rowsq_dep(ctx, Linv, ctx->pre.sig, n1, 2, ps, n1b)
                      : fitc_rowsq_cols(ctx, Linv, 0, n1, ps)))
      return rc;
    if (ps != s) HIPCHK(hipEventRecord(ctx->pre.join, ps));
  }
  if ((rc = potrf_inv_rec(ctx, A22, lda, Li22, ldl, W + (int64_t)n1 * n2, n2b, logdiag + n1, info,
                          base + n1, nreal - n1, Lout ? Lout + (int64_t)n1 * ldlo + n1 : nullptr,
                          ldlo)))
    return rc;
  if (forked) HIPCHK(hipStreamWaitEvent(s, join, 0));
  {  // L⁻¹21 = −L22⁻¹ · T
    GemmParams p = gp0();
    p.A = Li22; p.lda = ldl; p.B = A21; p.ldb = lda; p.C = Li21; p.ldc = ldl;
    p.M = n2; p.N = n1; p.K = n2; p.alpha = -1.0; p.tri = TRI_K_LE_I;
    if ((rc = gemm(ctx, LAY_N, LAY_N, EPI_STORE, p))) return rc;
  }
  if (top && ctx->pre.join) {
    HIPCHK(hipStreamWaitEvent(s, ctx->pre.join, 0));
    ctx->pre.join = nullptr;
  }
  return 0;
}

// workspace of potrf_inv_rec: this level's n1·n2 plus, recursively, the A22 side
size_t potrf_ws_doubles(int64_t n_pad) {
  int64_t nb = n_pad / GPS_TILE, tot = 0;
  while (nb > 1) {
    const int64_t n1 = (nb / 2) * GPS_TILE, n2 = (nb - nb / 2) * GPS_TILE;
    tot += n1 * n2;
    nb = nb - nb / 2;
  }
  return (size_t)std::max<int64_t>(tot, GPS_TILE * GPS_TILE);
}

// factor the padded SPD matrix in A (destroyed) into Linv, logdiag (n_pad).  Linv (and Lout)
// must hold zeros above the diagonal already — every caller memsets the buffer when it allocates
// or resizes it; the factorisation writes the lower triangle only, the diagonal 16×16 tiles of
// the leaves included.  Returns 0 or the LAPACK-style info (> 0).
int reset_info(gps_ctx* ctx) {  // [first non-PD minor, persistent-kernel error]
  HIPCHK(hipMemsetAsync(ctx->info.p, 0x7f, 2 * sizeof(int), ctx->stream));
  return 0;
}

// The recursion issues ~7 host calls per 128-block (launches, fork/join events): at the
// bottom levels, where each GEMM is a few µs of GPU time, the host's ~3-4 µs per call
// became the bound.  With GPS_OPT_GRAPH (default) the whole sequence is captured once per
// (buffers, sizes, streams, options) into a hipGraph and replayed with one launch; the
// eager path remains for profiling (per-launch events) and as the option's off state.

// an n_pad × n_pad factor buffer at p, zeroed (stream-ordered on s) and recorded for potrf_inv
hipError_t zero_factor(gps_ctx* ctx, double* p, int64_t n_pad, hipStream_t s) {
  const hipError_t e = hipMemsetAsync(p, 0, (size_t)n_pad * n_pad * 8, s);
  if (e == hipSuccess) ctx->zeroed[(uintptr_t)p] = n_pad;
  return e;
}
bool factor_zeroed(const gps_ctx* ctx, const double* p, int64_t n_pad) {
  const auto it = ctx->zeroed.find((uintptr_t)p);
  return it != ctx->zeroed.end() && it->second == n_pad;
}

int potrf_inv(gps_ctx* ctx, double* A, int64_t n_pad, double* Linv, double* W, double* logdiag,
              int nreal, double* Lout) {
  // the leaves and strip tasks write the lower triangles only: the strict-upper 128-tiles of
  // Linv / Lout must already be zero for THIS layout (n_pad is the row stride)
  if (!factor_zeroed(ctx, Linv, n_pad) || (Lout && !factor_zeroed(ctx, Lout, n_pad)))
    return fail(ctx, -1, "potrf_inv: factor buffer not zeroed for this size (internal contract)");
  // persistent blocks: task lists per size (uploaded once, before any capture) and one counter
  // region per launch of this call.  The regions are zero when a launch starts: zeroed once when
  // the buffer is allocated (synchronously, outside any capture) and reset by each launch's last
  // workgroup on its way out, so the captured sequence holds kernel nodes only.  (A memset node
  // ahead of the sequence, the first design, was replayed with garbage in the counters after
  // ~60 other captures on the GPU suite's context: pointer-valued words in the head counter,
  // then a no-op or a dependency wait that timed out; the r3 suite runs 3c-3e.)
  std::vector<int> dsizes;
  int64_t dcnt = 0;
  dag_blocks(ctx, n_pad / GPS_TILE, dsizes, dcnt);
  for (int T : dsizes) {
    const int lk = dag_list_key(ctx, T);
    if (ctx->dag_lists.count(lk)) continue;
    const std::vector<uint32_t> tl = dag_task_list(T, ctx->dag_order, true);
    auto& e = ctx->dag_lists[lk];
    HIPCHK(ensure(ctx, e.first, tl.size() * 4));
    // (stream-ordered, never the legacy stream: another context of this process may be
    // capturing a graph on its own thread, and a legacy-stream call then fails)
    HIPCHK(hipMemcpyAsync(e.first.p, tl.data(), tl.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    e.second = (int)tl.size();
  }
  if (dcnt && ctx->dag_cnt.cap < (size_t)dcnt * 4) {
    HIPCHK(hipStreamSynchronize(ctx->stream));  // no launch of this context still uses the old one
    HIPCHK(ensure(ctx, ctx->dag_cnt, std::max<size_t>((size_t)dcnt * 4, (size_t)1 << 20)));
    HIPCHK(hipMemsetAsync(ctx->dag_cnt.p, 0, ctx->dag_cnt.cap, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  auto eager = [&]() {
    ctx->sync_used = 0;
    ctx->pre.join = nullptr;
    ctx->dag_cnt_used = 0;
    return potrf_inv_rec(ctx, A, n_pad, Linv, n_pad, W, (int)(n_pad / GPS_TILE), logdiag,
                         static_cast<int*>(ctx->info.p), 0, nreal, Lout, n_pad, true);
  };
  if (!ctx->graphs || ctx->prof || n_pad <= GPS_TILE) return eager();
  // capture: everything the recursion allocates must exist beforehand (no allocation inside a
  // capture), and the key names the buffers the sequence bakes in: the split-K workspaces first
  HIPCHK(ensure(ctx, ctx->ws_main, (size_t)kSplitWsDoubles * 8));
  HIPCHK(ensure(ctx, ctx->ws_side, (size_t)kSplitWsDoubles * 8));
  const bool pre = ctx->pre.kind == PRE_FITC_Q;
  std::vector<uintptr_t> key = {
      (uintptr_t)A, (uintptr_t)n_pad, (uintptr_t)Linv, (uintptr_t)W, (uintptr_t)logdiag,
      (uintptr_t)nreal, (uintptr_t)Lout, (uintptr_t)ctx->stream, (uintptr_t)ctx->side,
      (uintptr_t)ctx->overlap, (uintptr_t)ctx->gemm_map,
      (uintptr_t)g_tiny_gemm, (uintptr_t)g_stream_k, (uintptr_t)g_slab_xcd, (uintptr_t)ctx->info.p, (uintptr_t)ctx->ws_main.p,
      (uintptr_t)ctx->ws_side.p, (uintptr_t)pre,
      // the pre-pass's operands (only when it is part of the sequence)
      pre ? (uintptr_t)ctx->pre.n1 : 0, pre ? (uintptr_t)ctx->aux[0] : 0,
      pre ? (uintptr_t)ctx->Knm.p : 0, pre ? (uintptr_t)ctx->fslab.p : 0,
      pre ? (uintptr_t)ctx->fn_pad : 0, pre ? (uintptr_t)ctx->m_pad : 0, pre ? (uintptr_t)ctx->pre.sig : 0,
      (uintptr_t)ctx->dag, (uintptr_t)ctx->dag_tiles, (uintptr_t)ctx->dag_group, (uintptr_t)ctx->dag_wgs, (uintptr_t)ctx->dag_half,
      (uintptr_t)ctx->dag_cnt.p, (uintptr_t)ctx->sk_cnt.p, (uintptr_t)ctx->dag_sig};
  for (int T : dsizes) key.push_back((uintptr_t)ctx->dag_lists[dag_list_key(ctx, T)].first.p);  // the task lists
  for (auto& g : ctx->pgraphs)
    if (g.key == key) {
      g.last_use = ++ctx->graph_tick;
      HIPCHK(hipGraphLaunch(g.exec, ctx->stream));
      return 0;
    }
  // Full cache: the least recently used exec is destroyed (after the context's streams drain).
  // Every buffer it bakes in is still allocated — a buffer is never freed while a graph that
  // uses it lives (drop_graphs_in) — which is what round 3's host segfault on destroy lacked.
  if (ctx->pgraphs.size() >= kMaxGraphs) {
    size_t lru = 0;
    for (size_t i = 1; i < ctx->pgraphs.size(); ++i)
      if (ctx->pgraphs[i].last_use < ctx->pgraphs[lru].last_use) lru = i;
    HIPCHK(sync_ctx_streams(ctx));
    const hipError_t e = hipGraphExecDestroy(ctx->pgraphs[lru].exec);
    ctx->pgraphs.erase(ctx->pgraphs.begin() + (ptrdiff_t)lru);
    ++ctx->graph_evicted;
    HIPCHK(e);
  }
  // ... and the fork/join event pool
  const size_t nev = 2 * (size_t)(n_pad / GPS_TILE) + 8;
  while (ctx->sync_ev.size() < nev) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->sync_ev.push_back(e);
  }
  HIPCHK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
  int rc = eager();
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(ctx->stream, &graph);
  if (rc || ec != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    if (rc) return rc;
    HIPCHK(ec);
  }
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  HIPCHK(ei);
  ctx->pgraphs.push_back({key, exec, ++ctx->graph_tick});
  HIPCHK(hipGraphLaunch(exec, ctx->stream));
  return 0;
}

int check_info(gps_ctx* ctx) {
  HIPCHK(hipMemcpyAsync(ctx->hinfo, ctx->info.p, 2 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (ctx->hinfo[1] == 2)
    return fail(ctx, -4, "persistent factorisation: the task queue did not run to completion "
                         "(counters not zero at launch; internal error)");
  if (ctx->hinfo[1] != 0x7f7f7f7f)
    return fail(ctx, -4, "persistent factorisation: a task's dependency wait timed out (internal error)");
  const int info = *ctx->hinfo;
  if (info != 0x7f7f7f7f) {
    char buf[160];
    snprintf(buf, sizeof(buf),
             "cholesky: the leading minor of order %d is not positive definite", info);
    return fail(ctx, info, buf);
  }
  return 0;
}

int set_theta(gps_ctx* ctx, Theta& th, int kind, const double* theta, int n_ell, int d) {
  ARGCHK(theta != nullptr, "theta is NULL");
  ARGCHK(kind == GPS_ARD || kind == GPS_RBF, "kind must be GPS_ARD or GPS_RBF");
  ARGCHK(n_ell == 1 || n_ell == d, "n_ell must be 1 or d");
  th.kind = kind;
  th.sf2 = std::exp(theta[0]);
  th.sn2 = std::exp(theta[1 + n_ell]);
  for (int k = 0; k < d; ++k) {
    const double b = theta[1 + (n_ell == 1 ? 0 : k)];
    th.inv_ell[k] = kind == GPS_ARD ? std::exp(-b) : std::exp(-0.5 * b);
  }
  return 0;
}

int upload(gps_ctx* ctx, DBuf& b, const double* h, int64_t rows, int64_t cols, int64_t rows_pad) {
  HIPCHK(ensure(ctx, b, (size_t)rows_pad * cols * 8));
  HIPCHK(hipMemsetAsync(b.p, 0, (size_t)rows_pad * cols * 8, ctx->stream));
  if (rows * cols)
    HIPCHK(hipMemcpyAsync(b.p, h, (size_t)rows * cols * 8, hipMemcpyHostToDevice, ctx->stream));
  return 0;
}

void score_bundle(const double* sums, double nt, double out[GPS_N_SC]) {
  out[GPS_SC_CRPS] = sums[0] / nt;
  out[GPS_SC_LOGS] = sums[1] / nt;
  out[GPS_SC_MSLL] = sums[2] / nt;
  out[GPS_SC_SMSE] = sums[3] / sums[4];
  out[GPS_SC_MSE] = sums[3] / nt;
  out[GPS_SC_COVER] = sums[5] / nt;
}

int bind(gps_ctx* ctx) {
  if (!ctx) {
    g_err = "NULL context";
    return -1;
  }
  HIPCHK(hipSetDevice(ctx->device));
  return 0;
}

bool sharded(const gps_ctx* ctx) { return ctx->comm != nullptr || ctx->lgroup != nullptr; }



// =============================================================================
// every device buffer a context owns (destroy, gps_ctx_stats)
std::vector<DBuf*> ctx_buffers(gps_ctx* ctx) {
  return {&ctx->info, &ctx->small, &ctx->X, &ctx->y, &ctx->Xt, &ctx->yt, &ctx->A,
                 &ctx->Linv, &ctx->W, &ctx->logdiag, &ctx->beta, &ctx->alpha, &ctx->dinv,
                 &ctx->slab, &ctx->mu_loo, &ctx->var_loo, &ctx->Ksf, &ctx->s1, &ctx->s2,
                 &ctx->mu, &ctx->var, &ctx->Lout, &ctx->pslab, &ctx->fX, &ctx->fy, &ctx->fXt, &ctx->fyt,
                 &ctx->Z, &ctx->Kmm, &ctx->Am, &ctx->Lm, &ctx->Lb, &ctx->ldm, &ctx->ldb,
                 &ctx->Knm, &ctx->q, &ctx->lam, &ctx->ilam, &ctx->ys, &ctx->slabB, &ctx->red,
                 &ctx->c, &ctx->tvec, &ctx->r, &ctx->g, &ctx->fmu_loo, &ctx->fvar_loo,
                 &ctx->Ksm, &ctx->qm, &ctx->qb, &ctx->fmu, &ctx->fvar, &ctx->fslab, &ctx->fslab_pre, &ctx->t0,
                 &ctx->t1, &ctx->t2, &ctx->t3, &ctx->t4, &ctx->ws_main, &ctx->ws_side, &ctx->ws_aux[0], &ctx->ws_aux[1],
                 &ctx->gu, &ctx->gct, &ctx->gv, &ctx->Mx, &ctx->gslab, &ctx->gout, &ctx->fgv,
                 &ctx->fgm, &ctx->fgB, &ctx->fR, &ctx->fgred, &ctx->fgslab, &ctx->fgout, &ctx->bP,
                 &ctx->bL, &ctx->bPI, &ctx->bH, &ctx->bvec, &ctx->bGblk, &ctx->bT, &ctx->bkr,
                 &ctx->bEf, &ctx->bF, &ctx->ebuf, &ctx->edraws,
                 &ctx->bSg, &ctx->bBf, &ctx->bLf, &ctx->bldf, &ctx->bRem, &ctx->bW, &ctx->bkv,
                 &ctx->bLR, &ctx->bLRv,
                 &ctx->ebuf_aux[0], &ctx->ebuf_aux[1], &ctx->ebuf_aux[2], &ctx->bPIs, &ctx->bRW, &ctx->escale, &ctx->bfv, &ctx->rpart, &ctx->dag_cnt, &ctx->sk_cnt, &ctx->dsig};
}


std::mutex g_groups_mu;
std::map<long long, std::weak_ptr<LocalGroup>> g_groups;

}  // namespace gpsapi

extern "C" {

int gps_version(void) { return GPS_ABI_VERSION; }


// the off-critical-path streams: side (T products of the factorisation) and aux[0..1]
// (with side, the concurrent energy-score folds)
int make_aux_streams(gps_ctx* ctx) {
  for (hipStream_t* a : {&ctx->side, &ctx->aux[0], &ctx->aux[1]})
    HIPCHK(hipStreamCreateWithFlags(a, hipStreamNonBlocking));
  return 0;
}
int gps_ctx_create(int device, gps_ctx** out) {
  gps_ctx* ctx = nullptr;
  if (!out) return fail(nullptr, -1, "out is NULL");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return fail(nullptr, -2, std::string("no HIP device: ") + hipGetErrorString(e));
  if (device < 0 || device >= ndev) return fail(nullptr, -1, "device index out of range");
  ctx = new gps_ctx();
  ctx->device = device;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  HIPCHK(hipDeviceGetAttribute(&ctx->ncu, hipDeviceAttributeMultiprocessorCount, device));
  if (int rc = make_aux_streams(ctx)) return rc;
  HIPCHK(hipHostMalloc((void**)&ctx->hsmall, 256 * sizeof(double), hipHostMallocDefault));
  HIPCHK(hipHostMalloc((void**)&ctx->hinfo, 16, hipHostMallocDefault));
  HIPCHK(ensure(ctx, ctx->info, 16));
  HIPCHK(ensure(ctx, ctx->small, 256 * sizeof(double)));
  HIPCHK(ensure(ctx, ctx->sk_cnt, (size_t)kStreamKTiles * sizeof(int)));
  HIPCHK(hipMemsetAsync(ctx->sk_cnt.p, 0, (size_t)kStreamKTiles * sizeof(int), ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  *out = ctx;
  return 0;
}

int gps_ctx_destroy(gps_ctx* ctx) {
  if (!ctx) return 0;
  (void)hipSetDevice(ctx->device);
  // this context's own streams only (a device-wide synchronize would also wait on, and under a
  // capture interfere with, other contexts of the process)
  for (hipStream_t st : {ctx->stream, ctx->side, ctx->aux[0], ctx->aux[1]})
    if (st) (void)hipStreamSynchronize(st);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  leave_local_group(ctx);
  for (auto& g : ctx->pgraphs) (void)hipGraphExecDestroy(g.exec);  // before the buffers they use
  ctx->pgraphs.clear();
  for (DBuf* b : ctx_buffers(ctx)) release(ctx, *b);
  for (auto& kv : ctx->dag_lists) release(ctx, kv.second.first);
  for (hipEvent_t e : ctx->ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->ph_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->sync_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->ar_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : {ctx->pre_fork, ctx->pre_join, ctx->preb_fork, ctx->kn_fork, ctx->kn_join,
                       ctx->b_fork, ctx->b_join})
    if (e) (void)hipEventDestroy(e);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  for (hipStream_t l : ctx->aux)
    if (l) (void)hipStreamDestroy(l);
  if (ctx->hsmall) (void)hipHostFree(ctx->hsmall);
  if (ctx->hinfo) (void)hipHostFree(ctx->hinfo);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return 0;
}

const char* gps_last_error(gps_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int gps_ctx_set_stream(gps_ctx* ctx, void* hip_stream) {
  if (int rc = bind(ctx)) return rc;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (ctx->own_stream && ctx->stream) HIPCHK(hipStreamDestroy(ctx->stream));
  if (hip_stream) {
    ctx->stream = static_cast<hipStream_t>(hip_stream);
    ctx->own_stream = false;
  } else {
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    ctx->own_stream = true;
  }
  return 0;
}

int gps_ctx_set_option(gps_ctx* ctx, int key, int value) {
  if (int rc = bind(ctx)) return rc;
  switch (key) {
    case GPS_OPT_OVERLAP: ctx->overlap = value != 0; return 0;
    case GPS_OPT_GEMM_MAP:
      ARGCHK(value >= 0 && value <= 6, "GPS_OPT_GEMM_MAP must be in 0..6");
      ctx->gemm_map = value;
      return 0;
    case GPS_OPT_AR_CHUNKS:
      ARGCHK(value >= 1 && value <= 64, "GPS_OPT_AR_CHUNKS must be in 1..64");
      ctx->ar_chunks = value;
      return 0;
    case GPS_OPT_TINY_GEMM: g_tiny_gemm = value != 0; return 0;
    case GPS_OPT_STREAM_K:
      ARGCHK(value >= 0 && value <= 2, "GPS_OPT_STREAM_K must be 0, 1 or 2");
      g_stream_k = value;
      return 0;
    case GPS_OPT_SLAB_XCD: g_slab_xcd = value != 0; return 0;
    case GPS_OPT_GRAM_REG:
      ARGCHK(value >= 0 && value <= 2, "GPS_OPT_GRAM_REG must be 0, 1 or 2");
      g_gram_reg = value;
      return 0;
    case GPS_OPT_GRAPH: ctx->graphs = value != 0; return 0;
    case GPS_OPT_PRED_PRE: ctx->pred_pre = value != 0; return 0;
    case GPS_OPT_DAG: ctx->dag = value != 0; return 0;
    case GPS_OPT_DAG_WGS:
      ARGCHK(value >= 0, "GPS_OPT_DAG_WGS must be >= 0");
      ctx->dag_wgs = value;
      return 0;
    case GPS_OPT_FITC_DEP: ctx->fitc_dep = value != 0; return 0;
    case GPS_OPT_DAG_ORDER:
      ARGCHK(value >= 0 && value <= 2, "GPS_OPT_DAG_ORDER must be 0, 1 or 2");
      ctx->dag_order = value;
      return 0;
    case GPS_OPT_DAG_GROUP:
      ARGCHK(value >= 2 && value <= 4, "GPS_OPT_DAG_GROUP must be 2, 3 or 4");
      ctx->dag_group = value;
      return 0;
    case GPS_OPT_DAG_TILES:
      ARGCHK(value >= 2 && value <= 64, "GPS_OPT_DAG_TILES must be in 2..64");
      ctx->dag_tiles = value;
      return 0;
    default: return fail(ctx, -1, "unknown option");
  }
}

void* gps_ctx_stream(gps_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int gps_ctx_synchronize(gps_ctx* ctx) {
  if (int rc = bind(ctx)) return rc;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gps_ctx_stats(gps_ctx* ctx, int64_t* out, int cap) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(out != nullptr && cap >= 0, "out is NULL or cap < 0");
  size_t bytes = 0;
  for (DBuf* b : ctx_buffers(ctx)) bytes += b->cap;
  int64_t v[GPS_N_STATS];
  v[GPS_STAT_GRAPHS] = (int64_t)ctx->pgraphs.size();
  v[GPS_STAT_GRAPH_CAP] = (int64_t)kMaxGraphs;
  v[GPS_STAT_GRAPH_OVERFLOW] = ctx->graph_overflow;
  v[GPS_STAT_GRAPH_DROPPED] = ctx->graph_dropped;
  v[GPS_STAT_GRAPH_EVICTED] = ctx->graph_evicted;
  v[GPS_STAT_DEVICE_BYTES] = (int64_t)bytes;
  for (int i = 0; i < cap && i < GPS_N_STATS; ++i) out[i] = v[i];  // never past the caller's array
  return GPS_N_STATS;
}

int gps_dag_task_list(int T, int flags, uint32_t* out, int cap) {
  if (T < 2 || T > 64 || cap < 0 || (cap > 0 && !out) || (flags & ~13))
    return fail(nullptr, -1, "bad arguments");
  const std::vector<uint32_t> tl = dag_task_list(T, (flags >> 2 & 3) == 0 ? 1 : (flags >> 2 & 3) == 3 ? 0 : flags >> 2 & 3,
                                                 (flags & 1) != 0);
  for (int i = 0; i < cap && i < (int)tl.size(); ++i) out[i] = tl[i];
  return (int)tl.size();
}

int gps_phase_enable(gps_ctx* ctx, int on) {
  if (int rc = bind(ctx)) return rc;
  ctx->phase = on != 0;
  return 0;
}

int gps_phase_collect(gps_ctx* ctx, char* json_out, int64_t cap) {
  if (int rc = bind(ctx)) return rc;
  HIPCHK(sync_ctx_streams(ctx));
  std::map<std::string, std::pair<int, double>> agg;
  std::vector<std::string> order;
  for (size_t i = 1; i < ctx->ph_marks.size(); ++i) {
    const auto& m = ctx->ph_marks[i];
    if (m.first == "start") continue;  // a new forward: no phase ends here
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ph_ev[ctx->ph_marks[i - 1].second], ctx->ph_ev[m.second]));
    if (!agg.count(m.first)) order.push_back(m.first);
    agg[m.first].first += 1;
    agg[m.first].second += ms;
  }
  std::string js = "{\"phases\": {";
  for (size_t i = 0; i < order.size(); ++i) {
    char buf[160];
    snprintf(buf, sizeof(buf), "%s\"%s\": {\"count\": %d, \"ms\": %.6f}", i ? ", " : "",
             order[i].c_str(), agg[order[i]].first, agg[order[i]].second);
    js += buf;
  }
  js += "}, \"allreduce\": [";
  for (size_t i = 0; i < ctx->ph_ar.size(); ++i) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ph_ev[ctx->ph_ar[i].e0], ctx->ph_ev[ctx->ph_ar[i].e1]));
    char buf[96];
    snprintf(buf, sizeof(buf), "%s[%.0f, %.6f]", i ? ", " : "", ctx->ph_ar[i].bytes, ms);
    js += buf;
  }
  js += "]}";
  ctx->ph_marks.clear();
  ctx->ph_ar.clear();
  ctx->ph_used = 0;
  if (!json_out || cap <= (int64_t)js.size()) return fail(ctx, -1, "json buffer too small");
  memcpy(json_out, js.c_str(), js.size() + 1);
  return 0;
}

int gps_rccl_info(int* version, char* path, int cap) {
  if (!version || !path || cap < 1) return fail(nullptr, -1, "bad arguments");
  *version = 0;
  if (ncclGetVersion(version) != ncclSuccess) return fail(nullptr, -3, "ncclGetVersion failed");
  Dl_info di;
  memset(&di, 0, sizeof(di));
  const char* f = dladdr(reinterpret_cast<void*>(&ncclAllReduce), &di) && di.dli_fname ? di.dli_fname : "";
  snprintf(path, (size_t)cap, "%s", f);
  return 0;
}

int gps_prof_enable(gps_ctx* ctx, int on) {
  if (int rc = bind(ctx)) return rc;
  ctx->prof = on;
  return 0;
}

int gps_prof_collect(gps_ctx* ctx, char* json_out, int64_t cap) {
  if (int rc = bind(ctx)) return rc;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  struct Agg { int count = 0; double ms = 0, flop = 0, bytes = 0; };
  std::map<std::string, Agg> agg;
  for (const ProfRec& r : ctx->recs) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev[r.e0], ctx->ev[r.e1]));
    Agg& a = agg[r.tag];
    a.count++;
    a.ms += ms;
    a.flop += r.flop;
    a.bytes += r.bytes;
  }
  ctx->recs.clear();
  ctx->ev_used = 0;
  std::string js = "{";
  bool first = true;
  for (auto& kv : agg) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s\"%s\": {\"count\": %d, \"ms\": %.6f, \"flop\": %.6e, \"bytes\": %.6e}",
             first ? "" : ", ", kv.first.c_str(), kv.second.count, kv.second.ms, kv.second.flop,
             kv.second.bytes);
    js += buf;
    first = false;
  }
  js += "}";
  if (!json_out || cap <= (int64_t)js.size()) return fail(ctx, -1, "json buffer too small");
  memcpy(json_out, js.c_str(), js.size() + 1);
  return 0;
}

// ------------------------------------------------------------------ L1 blocks
int gps_gram(gps_ctx* ctx, int kind, const double* X, int64_t n, const double* Xp, int64_t m, int d,
             double log_sf2, const double* log_ell, int n_ell, double diag_add, int uplo,
             double* out) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(X && Xp && out && log_ell, "NULL argument");
  ARGCHK(n > 0 && m > 0 && d >= 1 && d <= GPS_MAX_D, "bad shape");
  ARGCHK(uplo == GPS_FULL || (uplo == GPS_LOWER && n == m), "uplo=LOWER needs a square Gram");
  std::vector<double> theta(n_ell + 2);
  theta[0] = log_sf2;
  for (int k = 0; k < n_ell; ++k) theta[1 + k] = log_ell[k];
  theta[1 + n_ell] = 0.0;
  Theta th;
  if (int rc = set_theta(ctx, th, kind, theta.data(), n_ell, d)) return rc;
  const int64_t M = pad_to(n, 32), N = pad_to(m);
  if (int rc = upload(ctx, ctx->t0, X, n, d, n)) return rc;
  if (int rc = upload(ctx, ctx->t1, Xp, m, d, m)) return rc;
  HIPCHK(ensure(ctx, ctx->t2, (size_t)M * N * 8));
  HIPCHK(hipMemsetAsync(ctx->t2.p, 0, (size_t)M * N * 8, ctx->stream));
  if (int rc = gram(ctx, "gram_user", ctx->t0.d(), (int)n, ctx->t1.d(), (int)m, d, th, diag_add,
                    uplo == GPS_LOWER, 0, ctx->t2.d(), N, (int)M, (int)N))
    return rc;
  HIPCHK(hipMemcpy2DAsync(out, (size_t)m * 8, ctx->t2.p, (size_t)N * 8, (size_t)m * 8, n,
                          hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// helper: bring a user SPD matrix to the device padded with identity, factor it
int factor_user(gps_ctx* ctx, int64_t n, const double* A, int64_t lda, bool want_L) {
  ARGCHK(A && n > 0 && lda >= n, "bad matrix argument");
  const int64_t np = pad_to(n);
  HIPCHK(ensure(ctx, ctx->t0, (size_t)n * lda * 8));
  HIPCHK(hipMemcpyAsync(ctx->t0.p, A, (size_t)n * lda * 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ensure(ctx, ctx->t1, (size_t)np * np * 8));
  HIPCHK(launch_pad_copy(ctx->t0.d(), lda, ctx->t1.d(), np, (int)n, (int)n, (int)np, (int)np, 1,
                         ctx->stream));
  HIPCHK(ensure(ctx, ctx->t2, (size_t)np * np * 8));
  HIPCHK(zero_factor(ctx, ctx->t2.d(), np, ctx->stream));  // L⁻¹ upper tiles = 0
  HIPCHK(ensure(ctx, ctx->t3, potrf_ws_doubles(np) * 8));
  HIPCHK(ensure(ctx, ctx->t4, (size_t)np * 8 * (want_L ? np + 1 : 1)));
  double* logdiag = ctx->t4.d();
  double* Lout = want_L ? ctx->t4.d() + np : nullptr;
  if (want_L) HIPCHK(zero_factor(ctx, Lout, np, ctx->stream));
  if (int rc = reset_info(ctx)) return rc;
  if (int rc = potrf_inv(ctx, ctx->t1.d(), np, ctx->t2.d(), ctx->t3.d(), logdiag, (int)n, Lout))
    return rc;
  return check_info(ctx);
}

int gps_potrf(gps_ctx* ctx, int64_t n, double* A, int64_t lda, double* logdet) {
  if (int rc = bind(ctx)) return rc;
  if (int rc = factor_user(ctx, n, A, lda, true)) return rc;
  const int64_t np = pad_to(n);
  HIPCHK(launch_dot(ctx->t4.d(), nullptr, (int)np, ctx->small.d(), ctx->stream));
  HIPCHK(hipMemcpy2DAsync(A, (size_t)lda * 8, ctx->t4.d() + np, (size_t)np * 8, (size_t)n * 8, n,
                          hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->hsmall, ctx->small.p, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (logdet) *logdet = 2.0 * ctx->hsmall[0];
  return 0;
}

int gps_potrs(gps_ctx* ctx, int64_t n, int64_t nrhs, const double* A, int64_t lda, const double* B,
              int64_t ldb, double* X, int64_t ldx) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(B && X && nrhs > 0 && ldb >= nrhs && ldx >= nrhs, "bad rhs argument");
  if (int rc = factor_user(ctx, n, A, lda, false)) return rc;
  const int64_t np = pad_to(n), rp = pad_to(nrhs);
  // B padded into t0 (reuse), Y = L⁻¹B into t1, X = L⁻ᵀY into t3
  HIPCHK(ensure(ctx, ctx->t0, (size_t)n * ldb * 8));
  HIPCHK(hipMemcpyAsync(ctx->t0.p, B, (size_t)n * ldb * 8, hipMemcpyHostToDevice, ctx->stream));
  DBuf Bp, Y;
  HIPCHK(ensure(ctx, Bp, (size_t)np * rp * 8));
  HIPCHK(ensure(ctx, Y, (size_t)np * rp * 8));
  int rc = 0;
  do {
    hipError_t e = launch_pad_copy(ctx->t0.d(), ldb, Bp.d(), rp, (int)n, (int)nrhs, (int)np,
                                   (int)rp, 0, ctx->stream);
    if (e != hipSuccess) { rc = fail(ctx, -2, hipGetErrorString(e)); break; }
    GemmParams p = gp0();
    p.A = ctx->t2.d(); p.lda = np; p.B = Bp.d(); p.ldb = rp; p.C = Y.d(); p.ldc = rp;
    p.M = (int)np; p.N = (int)rp; p.K = (int)np; p.tri = TRI_K_LE_I;
    if ((rc = gemm(ctx, LAY_N, LAY_N, EPI_STORE, p))) break;
    GemmParams q = gp0();
    q.A = ctx->t2.d(); q.lda = np; q.B = Y.d(); q.ldb = rp; q.C = Bp.d(); q.ldc = rp;
    q.M = (int)np; q.N = (int)rp; q.K = (int)np; q.tri = TRI_K_GE_I;
    if ((rc = gemm(ctx, LAY_T, LAY_N, EPI_STORE, q))) break;
    e = hipMemcpy2DAsync(X, (size_t)ldx * 8, Bp.p, (size_t)rp * 8, (size_t)nrhs * 8, n,
                         hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) rc = fail(ctx, -2, hipGetErrorString(e));
  } while (0);
  release(ctx, Bp);
  release(ctx, Y);
  return rc;
}

int gps_diag_inv(gps_ctx* ctx, int64_t n, const double* A, int64_t lda, double* dinv) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(dinv, "dinv is NULL");
  if (int rc = factor_user(ctx, n, A, lda, false)) return rc;
  const int64_t np = pad_to(n);
  const int64_t nchunk = (np + 255) / 256;
  HIPCHK(ensure(ctx, ctx->t0, (size_t)(nchunk * np * 2 + np) * 8));
  double* out = ctx->t0.d() + nchunk * np * 2;
  HIPCHK(launch_colred(ctx->t2.d(), np, (int)np, (int)np, 1, nullptr, nullptr, nullptr, out,
                       ctx->t0.d(), ctx->stream));
  HIPCHK(hipMemcpyAsync(dinv, out, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gps_gemm(gps_ctx* ctx, int transA, int transB, int64_t M, int64_t N, int64_t K, double alpha,
             const double* A, int64_t lda, const double* B, int64_t ldb, double beta, double* C,
             int64_t ldc) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(A && B && C && M > 0 && N > 0 && K > 0, "bad gemm argument");
  const int64_t Mp = pad_to(M), Np = pad_to(N), Kp = pad_to(K);
  // stored shapes of A and B
  const int64_t ar = transA ? K : M, ac = transA ? M : K, arp = transA ? Kp : Mp, acp = transA ? Mp : Kp;
  const int64_t br = transB ? N : K, bc = transB ? K : N, brp = transB ? Np : Kp, bcp = transB ? Kp : Np;
  ARGCHK(lda >= ac && ldb >= bc && ldc >= N, "leading dimension too small");
  HIPCHK(ensure(ctx, ctx->t0, (size_t)(ar * lda + br * ldb + M * ldc) * 8));
  double* rawA = ctx->t0.d();
  double* rawB = rawA + ar * lda;
  double* rawC = rawB + br * ldb;
  HIPCHK(hipMemcpyAsync(rawA, A, (size_t)ar * lda * 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(rawB, B, (size_t)br * ldb * 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ensure(ctx, ctx->t1, (size_t)(arp * acp + brp * bcp + Mp * Np) * 8));
  double* pA = ctx->t1.d();
  double* pB = pA + arp * acp;
  double* pC = pB + brp * bcp;
  HIPCHK(launch_pad_copy(rawA, lda, pA, acp, (int)ar, (int)ac, (int)arp, (int)acp, 0, ctx->stream));
  HIPCHK(launch_pad_copy(rawB, ldb, pB, bcp, (int)br, (int)bc, (int)brp, (int)bcp, 0, ctx->stream));
  if (beta != 0.0) {
    HIPCHK(hipMemcpyAsync(rawC, C, (size_t)M * ldc * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(launch_pad_copy(rawC, ldc, pC, Np, (int)M, (int)N, (int)Mp, (int)Np, 0, ctx->stream));
  }
  GemmParams p = gp0();
  p.A = pA; p.lda = acp; p.B = pB; p.ldb = bcp; p.C = pC; p.ldc = Np;
  p.M = (int)Mp; p.N = (int)Np; p.K = (int)Kp; p.alpha = alpha; p.beta = beta;
  if (int rc = gemm(ctx, transA ? LAY_T : LAY_N, transB ? LAY_T : LAY_N, EPI_STORE, p)) return rc;
  HIPCHK(hipMemcpy2DAsync(C, (size_t)ldc * 8, pC, (size_t)Np * 8, (size_t)N * 8, M,
                          hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// scratch for the row finalisers' per-workgroup partials (kernels_vec.hip): nv per 256 rows
double* row_part(gps_ctx* ctx, int64_t rows, int nv) {
  if (ensure(ctx, ctx->rpart, (size_t)(std::max<int64_t>(rows, 1) + 255) / 256 * nv * 8) != hipSuccess)
    return nullptr;
  return ctx->rpart.d();
}

int gps_scores(gps_ctx* ctx, const double* mu, const double* var, const double* y, int64_t nt,
               double ytr_mean, double ytr_var_unbiased, double out[GPS_N_SC]) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(mu && var && y && out && nt > 0, "bad argument");
  if (int rc = upload(ctx, ctx->t0, mu, nt, 1, nt)) return rc;
  if (int rc = upload(ctx, ctx->t1, var, nt, 1, nt)) return rc;
  if (int rc = upload(ctx, ctx->t2, y, nt, 1, nt)) return rc;
  double* part = row_part(ctx, nt, 6);
  ARGCHK(part != nullptr, "out of device memory");
  HIPCHK(launch_score_sums(ctx->t0.d(), ctx->t1.d(), ctx->t2.d(), (int)nt, ytr_mean,
                           ytr_var_unbiased, ctx->small.d(), part, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->hsmall, ctx->small.p, 6 * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  score_bundle(ctx->hsmall, (double)nt, out);
  return 0;
}

}  // extern "C"
