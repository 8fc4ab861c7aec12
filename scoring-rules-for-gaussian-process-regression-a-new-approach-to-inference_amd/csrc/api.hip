// C-ABI of libgpscore.so (declared in include/gpscore.h): context, device
// buffers, the recursive Cholesky + triangular-inverse driver, and the fused
// full-GP / FITC pipelines.  Host orchestration only; the arithmetic lives in
// kernels_*.hip.
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
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gps_internal.h"
#include "gpscore.h"

using namespace gps;

namespace {

struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  double* d() const { return static_cast<double*>(p); }
};

struct ProfRec {
  std::string tag;
  int e0, e1;
  double flop, bytes;
};

struct Theta {
  int kind = GPS_ARD;
  double sf2 = 1.0, sn2 = 1.0;
  double inv_ell[GPS_MAX_D];
};

// In-process stand-in for the RCCL communicator (gps_comm_init_local): nranks contexts of one
// process, each driven by its own host thread, meet at every all-reduce of the row-sharded
// FITC path.  Same call sites, extents and streams as ncclAllReduce.  Contexts on one device
// (round 5) sum on the device, stream-ordered like RCCL: each rank copies its partial into a
// group staging buffer on the calling stream and records an event, the ranks meet on the host
// (no GPU wait), then each rank's stream waits for every rank's event and sums the staging
// buffers in rank order into its own buffer — so the stream / event ordering of the sharded
// sequence (the chunked B exchange on the comm stream beside the SYRK) runs as it would over
// RCCL, without a host synchronisation.  Contexts on different devices sum on the host.
struct LocalGroup {
  std::mutex mu;
  std::condition_variable cv;
  int n = 0, arrived = 0;
  uint64_t gen = 0;
  size_t count = 0;
  bool mismatch = false, last_mismatch = false;
  bool aborted = false;  // a member left (comm destroy / context destroy): waits fail at once
  std::vector<std::vector<double>> in;
  std::vector<double> sum;
  std::vector<char> taken;  // ranks held by a live context (a second context may not join as one)
  int joined = 0;           // ranks that have joined; the reduction path is read only once all n
                            // have (a rank that summed before a member on another
                            // device joined would have taken the device path, that member the
                            // host path, and one generation would have mixed the two)
  // the device path: one device for every member, ≤ kLocalSumMax ranks (final once joined == n)
  int device = -1;
  bool device_ok = true;
  std::vector<double*> stage;   // per rank, written only by its owner (grown after every reader)
  std::vector<size_t> stage_cap;
  std::vector<hipEvent_t> ready, done;  // per rank: partial staged / staging buffers read
  ~LocalGroup() {
    for (hipEvent_t e : done)
      if (e) (void)hipEventSynchronize(e);
    for (hipEvent_t e : ready)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : done)
      if (e) (void)hipEventDestroy(e);
    for (double* p : stage)
      if (p) (void)hipFree(p);
  }
};
std::mutex g_groups_mu;
std::map<long long, std::weak_ptr<LocalGroup>> g_groups;

}  // namespace

enum { PRE_NONE = 0, PRE_FITC_Q = 1 };

struct gps_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  hipStream_t side = nullptr;          // second stream for off-critical-path GEMMs
  hipStream_t aux[2] = {nullptr, nullptr};  // two more streams (concurrent energy-score folds)
  bool overlap = true;                 // GPS_OPT_OVERLAP
  int gemm_map = 0;                    // GPS_OPT_GEMM_MAP: tile-order override (A/B measurements)
  int fork_min = 1;                    // GPS_OPT_FORK_MIN: smallest n1 (in 128-blocks) whose T GEMM
  int fork_max = 0;                    // GPS_OPT_FORK_MAX: largest such n1 (0: no limit)
  bool side_low = false;               // GPS_OPT_SIDE_PRIO: side stream at the lowest priority
  int ar_chunks = 4;                   // GPS_OPT_AR_CHUNKS: row blocks of the FITC B all-reduce
  std::vector<hipEvent_t> ar_ev;       // their hand-offs to the comm stream (aux[1])
                                       // goes to the side stream (a fork/join costs ~13 us, but
                                       // forking every level measured best: 128.3 vs 129.1 ms)
  int ncu = 0;
  std::vector<hipEvent_t> sync_ev;     // fork/join events (timing disabled)
  size_t sync_used = 0;
  bool graphs = true;                  // GPS_OPT_GRAPH: replay the factorisation from a hipGraph
  bool pred_pre = true;                // GPS_OPT_PRED_PRE
  bool dag = true;                     // GPS_OPT_DAG: persistent factorisation of the bottom blocks
  int dag_tiles = 20;                  // GPS_OPT_DAG_TILES
  int dag_group = 3;                   // GPS_OPT_DAG_GROUP
  int dag_wgs = 0;                     // GPS_OPT_DAG_WGS (0: automatic, see dag_width)
  bool dag_fine = true;                // GPS_OPT_DAG_FINE
  int dag_order = 1;                   // GPS_OPT_DAG_ORDER
  bool dag_half = false;               // this factorisation leaves half the CUs to a side stream
  int fitc_dep = 1;                    // GPS_OPT_FITC_DEP: FITC row norms behind the m×m factorisations
                                       // (1: q behind Lm's; 2: and r behind Lb's, g by a GEMV)
  int* dag_sig = nullptr;              // the top-level persistent launch's row signals (kSig*), if any
  DBuf dsig;                           // the FITC signal blocks: Lm's, Lb's (kSigInts ints each)
  std::map<int, std::pair<DBuf, int>> dag_lists;  // per 2(3T + order) + fine: device task list, length
  // factor buffers (L⁻¹, L) known to hold zeros for a padded size: potrf_inv writes their lower
  // triangles only and refuses a buffer without an entry here (zero_factor); freeing or growing
  // a buffer forgets its entries (the zero-upper contract is checked, not assumed)
  std::map<uintptr_t, int64_t> zeroed;
  DBuf dag_cnt;                        // arrival counters of every persistent launch of a call
  DBuf sk_cnt;                         // stream-K tail tickets of the main stream's GEMMs (zero)
  int64_t dag_cnt_used = 0;
  struct PrePass {                     // work potrf_inv launches on aux[0] once the top-level
    int kind = 0;                      // L11⁻¹ is final: PRE_FITC_Q (the q column tiles [0, n1))
    int64_t n1 = 0;
    const double* L = nullptr;         // the top-level L⁻¹
    hipEvent_t join = nullptr;         // waited by the top-level call before it returns
  } pre;
  struct PotrfGraph {                  // one captured potrf_inv launch sequence
    std::vector<uintptr_t> key;
    hipGraphExec_t exec = nullptr;
    uint64_t last_use = 0;
  };
  std::vector<PotrfGraph> pgraphs;     // keyed by buffers, sizes, streams, options; least recently
                                       // used evicted past kMaxGraphs; dropped with their buffers
  uint64_t graph_tick = 0;
  int64_t graph_overflow = 0;          // (kept for the stats layout: always 0 since round 4)
  int64_t graph_dropped = 0;           // execs destroyed because a buffer they bake in was freed
  int64_t graph_evicted = 0;           // execs destroyed by the LRU cap
  std::string err;
  // profiling
  int prof = 0;  // 1: per-tag timing, 2: per-shape tags
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  std::vector<ProfRec> recs;
  // phase timing of the FITC forward on the production schedule (gps_phase_enable)
  bool phase = false;
  std::vector<hipEvent_t> ph_ev;
  size_t ph_used = 0;
  std::vector<std::pair<std::string, int>> ph_marks;          // (phase, event) on the main stream
  struct PhAr { double bytes; int e0, e1; };
  std::vector<PhAr> ph_ar;                                    // one per all-reduce
  // pinned host staging for small results
  double* hsmall = nullptr;
  int* hinfo = nullptr;
  // generic scratch
  DBuf info, small;
  // ---- full GP state
  DBuf X, y, Xt, yt, A, Linv, W, logdiag, beta, alpha, dinv, slab, mu_loo, var_loo, Ksf, s1, s2,
      mu, var, Lout, pslab;
  int n_ell = 1;
  DBuf gu, gct, gv, Mx, gslab, gout;  // gradient scratch
  int64_t n = 0, n_pad = 0, nt = 0, nt_pad = 0;
  int d = 0;
  double ytr_mean = 0, ytr_var = 1;
  bool have_data = false, have_test = false, fitted = false;
  Theta th;
  // ---- FITC state
  DBuf fX, fy, fXt, fyt, Z, Kmm, Am, Lm, Lb, ldm, ldb, Knm, q, lam, ilam, ys, slabB, red, c, tvec,
      r, g, fmu_loo, fvar_loo, Ksm, qm, qb, fmu, fvar, fslab;
  DBuf fgv, fgm, fgB, fR, fgred, fgslab, fgout;  // FITC gradient scratch
  // block-LOO scratch (per fold, reused): P, its L⁻¹ / P⁻¹ / H, vectors; full-GP Gblk, T;
  // FITC gradient: the fold's G_f, E_f, G_fE_f and F = Gblk E; energy score: work area, draws
  DBuf bP, bL, bPI, bH, bvec, bGblk, bT, bkr, bEf, bF, ebuf, edraws;
  // FITC block-LOO fold covariances (fitc_fold_cov): the folds' K_gᵀΛ_g⁻¹K_g slabs, B_{−f} and its
  // L⁻¹ / log-diagonal, the remote ranks' sum, W_f = K_f L_{−f}⁻ᵀ, the fold's padded 1/λ
  DBuf bSg, bBf, bLf, bldf, bRem, bW, bkv;
  DBuf bLR, bLRv;                      // FITC block-LOO in low rank: b×m products, fold vectors
  DBuf ebuf_aux[3], bPIs, bRW;  // concurrent ES folds: work areas of the aux streams, C_f, r_f / w_f
  DBuf escale;                  // ES: per fold ‖C_f‖∞, then the row-sum scratch
  DBuf bfv;                       // sharded FITC block-LOO: row counts, then the fold values
  DBuf rpart;                     // per-workgroup partials of the row finalisers (main stream)
  int64_t fn = 0, fn_pad = 0, fnt = 0, fnt_pad = 0, m = 0, m_pad = 0, fn_total = 0, fnt_total = 0;
  int fd = 0;
  double f_ytr_mean = 0, f_ytr_var = 1;
  bool f_data = false, f_test = false, f_z = false, f_fitted = false;
  // test-side ‖Lm⁻¹k_*‖² formed by gps_fitc_fit on aux[0] during Lb's factorisation
  bool f_pre = false;
  bool f_pre_b = false;  // ... and ‖Lb⁻¹k_*‖², beside the r pass (fitc_test_prepass_b)
  hipEvent_t pre_fork = nullptr, pre_join = nullptr, preb_fork = nullptr;
  hipEvent_t kn_fork = nullptr, kn_join = nullptr;  // the FITC Knm Gram beside Lm's factorisation
  hipEvent_t b_fork = nullptr, b_join = nullptr;    // the FITC b pass beside B's SYRK
  hipEvent_t r_fork = nullptr, r_join = nullptr;    // the FITC r pass behind Lb's factorisation
  DBuf fslab_pre;
  Theta fth;
  // ---- comm: RCCL (gps_comm_init) or the in-process group (gps_comm_init_local)
  ncclComm_t comm = nullptr;
  std::shared_ptr<LocalGroup> lgroup;
  int nranks = 1, rank = 0;
  // ---- compat scratch (gps_gram / potrf / potrs / diag_inv / scores)
  DBuf t0, t1, t2, t3, t4;
  // ---- split-K slabs, one per stream (GEMMs on different streams run concurrently)
  DBuf ws_main, ws_side, ws_aux[2];
};

namespace {

thread_local std::string g_err;

int fail(gps_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return fail(ctx, -2, std::string(#expr) + " failed: " + hipGetErrorString(_e));   \
  } while (0)

#define NCCLCHK(expr)                                                                     \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess)                                                                \
      return fail(ctx, -3, std::string(#expr) + " failed: " + ncclGetErrorString(_r));  \
  } while (0)

#define ARGCHK(cond, msg)                  \
  do {                                     \
    if (!(cond)) return fail(ctx, -1, msg); \
  } while (0)

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

struct Prof {
  gps_ctx* c;
  hipStream_t st;
  int e0 = -1;
  std::string tag;
  double flop, bytes;
  Prof(gps_ctx* c_, std::string t, double f, double b, hipStream_t s_ = nullptr)
      : c(c_), st(s_ ? s_ : c_->stream), tag(t), flop(f), bytes(b) {
    if (c->prof && (e0 = get_event(c)) >= 0) (void)hipEventRecord(c->ev[e0], st);
  }
  ~Prof() {
    if (!c->prof || e0 < 0) return;
    const int e1 = get_event(c);
    if (e1 < 0) return;
    (void)hipEventRecord(c->ev[e1], st);
    c->recs.push_back({tag, e0, e1, flop, bytes});
  }
};

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
constexpr int64_t kSplitWsDoubles = 32ll << 20;  // 256 MiB of split-K slabs per stream

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

int gemm(gps_ctx* ctx, int al, int bl, int epi, const GemmParams& p, hipStream_t st = nullptr) {
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
         int M, int N, hipStream_t st = nullptr) {
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
// column tiles [0, ncols) of Knm·L⁻ᵀ (L⁻¹ in L, being written by a persistent launch of the
// context's FITC width whose row signals are sig).  mode 1: the dependent launch (EPI_ROWSQ) —
// each column tile as soon as its row of L⁻¹ is final; mode 2: the completion launch after the
// factorisation — the tiles mode 1 left, and with w / dot the last column tile's row dot g = Knm·w
// (EPI_ROWSQ_DOT, as fitc_fit_core's r pass).  Both write fslab's row-norm partials as
// fitc_rowsq_cols does, so the sums that read them are unchanged.
int dag_width(const gps_ctx* ctx, int64_t nb, bool half);
int fitc_rowsq_dep(gps_ctx* ctx, const double* L, int* sig, int64_t ncols, int mode,
                   hipStream_t st, const double* w = nullptr, double* dot = nullptr) {
  const int64_t np = ctx->fn_pad, mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = ctx->Knm.d(); p.lda = mp; p.B = L; p.ldb = mp;
  p.M = (int)np; p.N = (int)ncols; p.K = (int)ncols; p.tri = TRI_K_LE_J;
  p.kend = (int)pad_to(ctx->m, 16);
  p.out0 = ctx->fslab.d(); p.ld_out = np;
  p.dep_sig = sig; p.dep_q = sig + kSigQueue; p.dep_err = static_cast<int*>(ctx->info.p) + 1;
  p.dep_grid = dag_width(ctx, mp / GPS_TILE, true); p.dep_mode = mode;
  p.w = w; p.out1 = dot;
  return gemm(ctx, LAY_N, LAY_T, dot ? EPI_ROWSQ_DOT : EPI_ROWSQ, p, st);
}

// the task list of an nb-tile persistent block under the context's options
int dag_list_key(const gps_ctx* ctx, int64_t nb) {
  return (int)(2 * (3 * nb + ctx->dag_order) + (ctx->dag_fine ? 1 : 0));
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
// want every CU: 124.2 vs 126.1 ms, profiles/r3_dag_width_ab.txt)
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
                  int64_t ldlo, bool top = false) {
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
    d.sig = top ? ctx->dag_sig : nullptr;  // (a dependent row-norm launch reads its rows)
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
  if ((rc = potrf_inv_rec(ctx, A, lda, Linv, ldl, W, n1b, logdiag, info, base, nreal, Lout, ldlo)))
    return rc;
  {  // W = L21 = A21 · L11⁻ᵀ
    GemmParams p = gp0();
    p.A = A21; p.lda = lda; p.B = Linv; p.ldb = ldl; p.C = W; p.ldc = n1;
    p.M = n2; p.N = n1; p.K = n1; p.tri = TRI_K_LE_J;
    if ((rc = gemm(ctx, LAY_N, LAY_T, EPI_STORE, p))) return rc;
  }
  if (Lout) HIPCHK(hipMemcpy2DAsync(Lout + (int64_t)n1 * ldlo, ldlo * 8, W, (size_t)n1 * 8,
                                    (size_t)n1 * 8, n2, hipMemcpyDeviceToDevice, s));
  // an event fork + join costs ~13 us of dependent-chain latency (tools/launch_latency.hip)
  const bool forked = ctx->overlap && n1b >= ctx->fork_min && (!ctx->fork_max || n1b <= ctx->fork_max);
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
  if (top && ctx->pre.kind == PRE_FITC_Q && ctx->pre.n1 == n1) {
    hipStream_t ps = ctx->overlap ? ctx->aux[0] : s;
    if (ps != s) {
      hipEvent_t f = sync_event(ctx);
      ctx->pre.join = sync_event(ctx);
      if (!f || !ctx->pre.join) return fail(ctx, -2, "hipEventCreate failed");
      HIPCHK(hipEventRecord(f, s));
      HIPCHK(hipStreamWaitEvent(ps, f, 0));
    }
    if ((rc = fitc_rowsq_cols(ctx, Linv, 0, n1, ps))) return rc;
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
constexpr size_t kMaxGraphs = 64;

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
    const std::vector<uint32_t> tl = dag_task_list(T, ctx->dag_order, ctx->dag_fine);
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
      (uintptr_t)ctx->overlap, (uintptr_t)ctx->fork_min, (uintptr_t)ctx->fork_max, (uintptr_t)ctx->gemm_map,
      (uintptr_t)g_tiny_gemm, (uintptr_t)g_stream_k, (uintptr_t)g_gemm_prio, (uintptr_t)g_slab_xcd, (uintptr_t)ctx->info.p, (uintptr_t)ctx->ws_main.p,
      (uintptr_t)ctx->ws_side.p, (uintptr_t)pre,
      // the pre-pass's operands (only when it is part of the sequence)
      pre ? (uintptr_t)ctx->pre.n1 : 0, pre ? (uintptr_t)ctx->aux[0] : 0,
      pre ? (uintptr_t)ctx->Knm.p : 0, pre ? (uintptr_t)ctx->fslab.p : 0,
      pre ? (uintptr_t)ctx->fn_pad : 0, pre ? (uintptr_t)ctx->m_pad : 0,
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

// A member leaving marks the group aborted: ranks waiting in (or later entering) one of
// its all-reduces fail at once instead of waiting for a rank that will never arrive.
void leave_local_group(gps_ctx* ctx) {
  if (!ctx->lgroup) return;
  {
    std::lock_guard<std::mutex> lk(ctx->lgroup->mu);
    ctx->lgroup->aborted = true;
    ctx->lgroup->taken[ctx->rank] = 0;
  }
  ctx->lgroup->cv.notify_all();
  ctx->lgroup.reset();
}

// one host-side rendezvous of the group's ranks (no GPU wait); every rank passes the same count
int group_barrier(gps_ctx* ctx, LocalGroup& G, size_t count) {
  std::unique_lock<std::mutex> lk(G.mu);
  if (G.aborted) return fail(ctx, -3, "local all-reduce: another rank left the group");
  if (G.arrived == 0) {
    G.count = count;
    G.mismatch = false;
  } else if (G.count != count) {
    G.mismatch = true;
  }
  const uint64_t my = G.gen;
  if (++G.arrived == G.n) {
    G.last_mismatch = G.mismatch;
    G.arrived = 0;
    ++G.gen;
    G.cv.notify_all();
  } else if (!G.cv.wait_for(lk, std::chrono::seconds(60), [&] { return G.gen != my || G.aborted; })) {
    G.aborted = true;  // (as in the host path below: the whole group fails the same way)
    G.cv.notify_all();
    return fail(ctx, -3, "local all-reduce: timed out waiting for the other ranks (group aborted)");
  } else if (G.gen == my) {
    return fail(ctx, -3, "local all-reduce: another rank left the group");
  }
  if (G.last_mismatch) return fail(ctx, -3, "local all-reduce: ranks passed different element counts");
  return 0;
}

// Σ over the ranks of `count` doubles at buf (device, in place, stream s): ncclAllReduce on
// the RCCL communicator, or the in-process group's sum (on the device when every member shares
// one); a no-op on one rank.
int allreduce_sum_impl(gps_ctx* ctx, double* buf, size_t count, hipStream_t s);
int allreduce_sum(gps_ctx* ctx, double* buf, size_t count, hipStream_t s) {
  if (!ctx->phase || !sharded(ctx)) return allreduce_sum_impl(ctx, buf, count, s);
  const int e0 = phase_event(ctx, s);
  const int rc = allreduce_sum_impl(ctx, buf, count, s);
  const int e1 = phase_event(ctx, s);
  if (e0 >= 0 && e1 >= 0) ctx->ph_ar.push_back({8.0 * (double)count, e0, e1});
  return rc;
}
int allreduce_sum_impl(gps_ctx* ctx, double* buf, size_t count, hipStream_t s) {
  if (ctx->comm) {
    NCCLCHK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, ctx->comm, s));
    return 0;
  }
  if (!ctx->lgroup) return 0;
  LocalGroup& G = *ctx->lgroup;
  bool on_device;
  {  // the path is fixed once every rank has joined: wait for the late joiners (as a barrier would)
    std::unique_lock<std::mutex> lk(G.mu);
    if (!G.cv.wait_for(lk, std::chrono::seconds(60), [&] { return G.joined == G.n || G.aborted; })) {
      G.aborted = true;
      G.cv.notify_all();
      return fail(ctx, -3, "local all-reduce: timed out waiting for the other ranks to join (group aborted)");
    }
    if (G.aborted) return fail(ctx, -3, "local all-reduce: another rank left the group");
    on_device = G.device_ok;
  }
  if (on_device) {
    const int r = ctx->rank;
    if (G.stage_cap[r] < count) {  // grow: every earlier sum that read the old buffer is done
      for (int q = 0; q < G.n; ++q) HIPCHK(hipEventSynchronize(G.done[q]));
      if (G.stage[r]) HIPCHK(hipFree(G.stage[r]));
      G.stage[r] = nullptr;
      G.stage_cap[r] = 0;
      HIPCHK(hipMalloc(&G.stage[r], count * 8));
      G.stage_cap[r] = count;
    }
    // (the previous sums of the other ranks read this rank's staging buffer: wait for them)
    for (int q = 0; q < G.n; ++q)
      if (q != r) HIPCHK(hipStreamWaitEvent(s, G.done[q], 0));
    HIPCHK(hipMemcpyAsync(G.stage[r], buf, count * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipEventRecord(G.ready[r], s));
    if (int rc = group_barrier(ctx, G, count)) return rc;  // every rank's ready event recorded
    LocalSumPtrs sp;
    memset(&sp, 0, sizeof(sp));
    for (int q = 0; q < G.n; ++q) {
      sp.p[q] = G.stage[q];
      if (q != r) HIPCHK(hipStreamWaitEvent(s, G.ready[q], 0));
    }
    HIPCHK(launch_local_sum(sp, G.n, (int64_t)count, buf, s));
    HIPCHK(hipEventRecord(G.done[r], s));
    return group_barrier(ctx, G, count);  // every rank's done event recorded before the next use
  }
  std::vector<double> mine(count);
  HIPCHK(hipMemcpyAsync(mine.data(), buf, count * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::vector<double> out;
  bool bad;
  {
    std::unique_lock<std::mutex> lk(G.mu);
    if (G.arrived == 0) {
      G.count = count;
      G.mismatch = false;
    } else if (G.count != count) {
      G.mismatch = true;
    }
    G.in[ctx->rank] = std::move(mine);
    const uint64_t my = G.gen;
    if (++G.arrived == G.n) {
      G.sum.assign(G.count, 0.0);
      for (int r = 0; r < G.n; ++r)  // rank order: deterministic
        for (size_t i = 0; i < std::min(G.count, G.in[r].size()); ++i) G.sum[i] += G.in[r][i];
      G.last_mismatch = G.mismatch;
      G.arrived = 0;
      ++G.gen;
      G.cv.notify_all();
    } else if (!G.cv.wait_for(lk, std::chrono::seconds(60),
                              [&] { return G.gen != my || G.aborted; })) {
      // a timed-out rank aborts the group, so every member (including a late arriver, which
      // would otherwise complete this generation with a rank that has left) fails the same way
      G.aborted = true;
      G.cv.notify_all();
      return fail(ctx, -3, "local all-reduce: timed out waiting for the other ranks (group aborted)");
    } else if (G.gen == my) {
      return fail(ctx, -3, "local all-reduce: another rank left the group");
    }
    out = G.sum;
    bad = G.last_mismatch;
  }
  if (bad || out.size() != count)
    return fail(ctx, -3, "local all-reduce: ranks passed different element counts");
  HIPCHK(hipMemcpyAsync(buf, out.data(), count * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}

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
}  // namespace

// =============================================================================
// every device buffer a context owns (destroy, gps_ctx_stats)
static std::vector<DBuf*> ctx_buffers(gps_ctx* ctx) {
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
                       ctx->b_fork, ctx->b_join, ctx->r_fork, ctx->r_join})
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
    case GPS_OPT_FORK_MIN: ctx->fork_min = value < 1 ? 1 : value; return 0;
    case GPS_OPT_FORK_MAX: ctx->fork_max = value < 0 ? 0 : value; return 0;
    case GPS_OPT_SIDE_PRIO: {  // the side stream at the lowest queue priority (or back)
      if ((value != 0) == ctx->side_low) return 0;
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      // the replacement first: if its creation fails, the context keeps its working side stream
      // (never the legacy null stream, which would serialise against other contexts' captures)
      hipStream_t ns = nullptr;
      if (value) HIPCHK(hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, least));
      else HIPCHK(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
      const hipError_t es = hipStreamSynchronize(ctx->side);
      if (es != hipSuccess) (void)hipStreamDestroy(ns);
      HIPCHK(es);
      (void)hipStreamDestroy(ctx->side);
      ctx->side = ns;
      ctx->side_low = value != 0;
      return 0;
    }
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
    case GPS_OPT_GEMM_PRIO: g_gemm_prio = value < 0 ? 0 : value > 2 ? 2 : value; return 0;
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
    case GPS_OPT_DAG_FINE: ctx->dag_fine = value != 0; return 0;
    case GPS_OPT_FITC_DEP:
      ARGCHK(value >= 0 && value <= 2, "GPS_OPT_FITC_DEP must be 0, 1 or 2");
      ctx->fitc_dep = value;
      return 0;
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
static int factor_user(gps_ctx* ctx, int64_t n, const double* A, int64_t lda, bool want_L) {
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
static double* row_part(gps_ctx* ctx, int64_t rows, int nv) {
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
              bool packed = false, const double* A = nullptr, int64_t lda = 0) {
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
                  bool pre_test = false) {
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
  int* sig_m = nullptr;
  int* sig_b = nullptr;
  if (dep) {  // (zeroed, stream-ordered before both launches of each pair)
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
  if (dep && (rc = fitc_rowsq_dep(ctx, ctx->Lm.d(), sig_m, mp, 1, ctx->aux[0]))) {
    (void)hipStreamWaitEvent(s, ctx->kn_join, 0);
    return rc;
  }
  if (kside) HIPCHK(hipEventRecord(ctx->kn_join, ctx->aux[0]));
  const int64_t qn1 = preq ? (mp / GPS_TILE / 2) * GPS_TILE : 0;
  ctx->pre.kind = preq ? PRE_FITC_Q : PRE_NONE;
  ctx->pre.n1 = qn1;
  ctx->pre.L = ctx->Lm.d();
  ctx->dag_half = true;  // (the FITC m×m factorisations: see potrf_inv_rec's width)
  ctx->dag_sig = sig_m;
  rc = potrf_inv(ctx, ctx->Am.d(), mp, ctx->Lm.d(), ctx->W.d(), ctx->ldm.d(), (int)m, nullptr);
  ctx->dag_sig = nullptr;
  ctx->dag_half = false;
  ctx->pre.kind = PRE_NONE;
  phase_mark(ctx, "kmm_lm");
  if (kside) HIPCHK(hipStreamWaitEvent(s, ctx->kn_join, 0));  // (before any return: Knm in flight)
  if (rc) return rc;
  phase_mark(ctx, "knm");
  HIPCHK(launch_dot(ctx->ldm.d(), nullptr, (int)mp, sm + 0, s));
  // q_i = ‖Lm⁻¹ k_i‖²: the tiles the dependent launch left, or the remaining column tiles
  if ((rc = dep ? fitc_rowsq_dep(ctx, ctx->Lm.d(), sig_m, mp, 2, s)
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
  // GPS_OPT_FITC_DEP 2: the r pass behind Lb's factorisation too, on aux[1] (every column tile;
  // g = Knm c, which needs c = B⁻¹b, then by a GEMV)
  const bool rdep = dep && ctx->fitc_dep == 2;
  if (rdep) {
    for (hipEvent_t* e : {&ctx->r_fork, &ctx->r_join})
      if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->r_fork, s));
    HIPCHK(hipStreamWaitEvent(ctx->aux[1], ctx->r_fork, 0));
    if ((rc = fitc_rowsq_dep(ctx, ctx->Lb.d(), sig_b, mp, 1, ctx->aux[1]))) return rc;
    HIPCHK(hipEventRecord(ctx->r_join, ctx->aux[1]));
  }
  ctx->dag_half = true;
  ctx->dag_sig = rdep ? sig_b : nullptr;
  rc = potrf_inv(ctx, ctx->Am.d(), mp, ctx->Lb.d(), ctx->W.d(), ctx->ldb.d(), (int)m, nullptr);
  ctx->dag_sig = nullptr;
  ctx->dag_half = false;
  ctx->pre.kind = PRE_NONE;
  if (rc) {
    if (rdep) (void)hipStreamWaitEvent(s, ctx->r_join, 0);  // (r in flight)
    return rc;
  }
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
  if (rdep) {  // g = Knm c (a GEMV beside the dependent r launch's tail), then the r tiles it left
    HIPCHK(launch_gemv_full(ctx->Knm.d(), mp, ctx->c.d(), ctx->g.d(), (int)np, (int)mp, s));
    HIPCHK(hipStreamWaitEvent(s, ctx->r_join, 0));
    if ((rc = fitc_rowsq_dep(ctx, ctx->Lb.d(), sig_b, mp, 2, s))) return rc;
  } else {  // r_i = ‖Lb⁻¹ k_i‖² (the column tiles [qn1, mp): the rest came with B's factorisation),
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
static int fitc_knm_xt(gps_ctx* ctx, int64_t ldc, const double* X, double* C) {
  const int64_t mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = ctx->Knm.d(); p.lda = mp; p.B = X; p.ldb = mp; p.C = C; p.ldc = ldc;
  p.M = (int)ctx->fn_pad; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_LE_J;
  return gemm(ctx, LAY_N, LAY_T, EPI_STORE, p);
}
// y (m_pad) = Xᵀ x for a stored lower X (m_pad²): the column reductions of X weighted by x, in
// 256-row chunks through fslab (one chunk per 256 rows when fslab holds their partials)
static int fitc_lt_vec(gps_ctx* ctx, const double* X, const double* x, double* y) {
  const int64_t mp = ctx->m_pad;
  const int64_t cap = (int64_t)(ctx->fslab.cap / 8);
  int crows = 256;
  while ((mp + crows - 1) / crows * mp * 2 > cap) crows *= 2;
  HIPCHK(launch_colred(X, mp, (int)mp, (int)mp, 0, x, nullptr, y, nullptr, ctx->fslab.d(),
                       ctx->stream, crows));
  return 0;
}
// C (rows × m_pad) = A · X, X lower (k >= j)
static int fitc_tri_right(gps_ctx* ctx, const double* A, int64_t lda, const double* X, double* C,
                          int64_t ldc, int64_t rows) {
  const int64_t mp = ctx->m_pad;
  GemmParams p = gp0();
  p.A = A; p.lda = lda; p.B = X; p.ldb = mp; p.C = C; p.ldc = ldc;
  p.M = (int)rows; p.N = (int)mp; p.K = (int)mp; p.tri = TRI_K_GE_J;
  return gemm(ctx, LAY_N, LAY_N, EPI_STORE, p);
}
// C (m_pad²) = Xᵀ · B, X lower
static int fitc_tri_left_t(gps_ctx* ctx, const double* X, const double* B, double* C) {
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
  if (shard) {  // the other ranks' folds: Σ_all S − Σ_local S (m×m; all-reduced once)
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

// ---------------------------------------------------------------------- comm
int gps_comm_unique_id(char uid[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  gps_ctx* ctx = nullptr;
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  memcpy(uid, &id, 128);
  return 0;
}

int gps_comm_init(gps_ctx* ctx, int nranks, int rank, const char uid[128]) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(nranks >= 1 && rank >= 0 && rank < nranks && uid, "bad communicator arguments");
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  leave_local_group(ctx);
  ncclUniqueId id;
  memcpy(&id, uid, 128);
  NCCLCHK(ncclCommInitRank(&ctx->comm, nranks, id, rank));
  ctx->nranks = nranks;
  ctx->rank = rank;
  return 0;
}

int gps_comm_init_local(gps_ctx* ctx, int nranks, int rank, long long group) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(nranks >= 1 && rank >= 0 && rank < nranks, "bad communicator arguments");
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  leave_local_group(ctx);
  std::lock_guard<std::mutex> lk(g_groups_mu);
  std::shared_ptr<LocalGroup> G = g_groups[group].lock();
  bool dead = false;
  if (G) {
    std::lock_guard<std::mutex> gl(G->mu);
    dead = G->aborted;
  }
  if (!G || dead) {  // an aborted group is never rejoined: the key gets a fresh group
    G = std::make_shared<LocalGroup>();
    G->n = nranks;
    G->in.resize(nranks);
    G->taken.assign(nranks, 0);
    G->device = ctx->device;
    G->device_ok = nranks <= kLocalSumMax;
    G->stage.assign(nranks, nullptr);
    G->stage_cap.assign(nranks, 0);
    G->ready.assign(nranks, nullptr);
    G->done.assign(nranks, nullptr);
    if (G->device_ok)
      for (int q = 0; q < nranks; ++q) {
        HIPCHK(hipEventCreateWithFlags(&G->ready[q], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&G->done[q], hipEventDisableTiming));
      }
    g_groups[group] = G;
  }
  ARGCHK(G->n == nranks, "local group: nranks differs from the group's");
  {
    std::lock_guard<std::mutex> gl(G->mu);
    ARGCHK(!G->taken[rank], "local group: another live context already holds this rank");
    G->taken[rank] = 1;
    if (ctx->device != G->device) G->device_ok = false;  // members on two devices: host sums
    if (++G->joined == G->n) G->cv.notify_all();        // the path is final: release the waiters
  }
  ctx->lgroup = G;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return 0;
}

int gps_comm_info(gps_ctx* ctx, int* nranks, int* rank, int* kind) {
  if (int rc = bind(ctx)) return rc;
  ARGCHK(nranks && rank && kind, "out pointer is NULL");
  if (ctx->comm) {  // what the RCCL communicator itself holds, not what the caller asked for
    NCCLCHK(ncclCommCount(ctx->comm, nranks));
    NCCLCHK(ncclCommUserRank(ctx->comm, rank));
    *kind = GPS_COMM_RCCL;
  } else if (ctx->lgroup) {
    *nranks = ctx->lgroup->n;
    *rank = ctx->rank;
    *kind = GPS_COMM_LOCAL;
  } else {
    *nranks = 1;
    *rank = 0;
    *kind = GPS_COMM_NONE;
  }
  return 0;
}

int gps_comm_destroy(gps_ctx* ctx) {
  if (int rc = bind(ctx)) return rc;
  if (ctx->comm) NCCLCHK(ncclCommDestroy(ctx->comm));
  ctx->comm = nullptr;
  leave_local_group(ctx);
  ctx->nranks = 1;
  ctx->rank = 0;
  return 0;
}

}  // extern "C"
