// Internal header of the C-ABI layer (api*.hip): the context, its device buffers, the launch
// helpers every path shares and the non-exported functions one path calls in another.  The
// translation units split by path (round 6): api.hip (context, options, profiling,
// launch helpers, the recursive factorisation driver, L1 blocks), api_full.hip (full GP, CP.R
// surfaces), api_fitc.hip (FITC fit / gradients / predict), api_block.hip (block-LOO and the
// energy score), api_comm.hip (RCCL and the in-process communicator).
#pragma once
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

namespace gpsapi {


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

extern std::mutex g_groups_mu;
extern std::map<long long, std::weak_ptr<LocalGroup>> g_groups;

}  // namespace gpsapi
using namespace gpsapi;


enum { PRE_NONE = 0, PRE_FITC_Q = 1 };

struct gps_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  hipStream_t side = nullptr;          // second stream for off-critical-path GEMMs
  hipStream_t aux[2] = {nullptr, nullptr};  // two more streams (concurrent energy-score folds)
  bool overlap = true;                 // GPS_OPT_OVERLAP
  int gemm_map = 0;                    // GPS_OPT_GEMM_MAP: tile-order override (A/B measurements)
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
  int dag_order = 1;                   // GPS_OPT_DAG_ORDER
  bool dag_half = false;               // this factorisation leaves half the CUs to a side stream
  bool fitc_dep = true;                // GPS_OPT_FITC_DEP: the q row norms behind Lm's factorisation
  int* dag_sig = nullptr;              // the top-level persistent launch's row signals (kSig*), if any
  DBuf dsig;                           // the FITC signal block of Lm's factorisation (kSigInts ints)
  std::map<int, std::pair<DBuf, int>> dag_lists;  // per 3T + order: device task list, length
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
    int* sig = nullptr;                // row signals: the pre-pass runs behind the L11 block
                                       // (GPS_OPT_FITC_DEP; zeroed by the caller)
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


namespace gpsapi {

extern thread_local std::string g_err;
int fail(gps_ctx* ctx, int code, const std::string& msg);

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

constexpr int64_t kSplitWsDoubles = 32ll << 20;  // 256 MiB of split-K slabs per stream
constexpr size_t kMaxGraphs = 64;                // cached factorisation graphs per context

int get_event(gps_ctx* c);
// per-launch hipEvent timing of a tagged region (gps_prof_enable)
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

hipError_t sync_ctx_streams(gps_ctx* ctx);
hipError_t drop_graphs_in(gps_ctx* ctx, const void* p, size_t bytes);
void forget_zeroed(gps_ctx* ctx, const void* p, size_t bytes);
hipError_t ensure(gps_ctx* ctx, DBuf& b, size_t bytes);
void release(gps_ctx* ctx, DBuf& b);
int get_event(gps_ctx* c);
int phase_event(gps_ctx* c, hipStream_t st);
void phase_mark(gps_ctx* c, const char* name);
hipEvent_t sync_event(gps_ctx* c);
GemmParams gp0();
const char* gemm_tag(int al, int bl, int epi, const GemmParams& p);
double gemm_flops(const GemmParams& p);
int gemm(gps_ctx* ctx, int al, int bl, int epi, const GemmParams& p, hipStream_t st = nullptr);
int gram(gps_ctx* ctx, const char* tag, const double* x, int n, const double* xp, int m, int d,
         const Theta& th, double diag_add, int lower, int pad_identity, double* out, int64_t ldo,
         int M, int N, hipStream_t st = nullptr);
int pred_rows(gps_ctx* ctx, int64_t r0, int64_t r1, const double* w, hipStream_t st);
int fitc_rowsq_cols(gps_ctx* ctx, const double* Lx, int64_t c0, int64_t c1, hipStream_t st);
int fitc_rowsq_dep(gps_ctx* ctx, const double* L, int* sig, int64_t ncols, int mode,
                   hipStream_t st, int64_t nb_dag);
int dag_list_key(const gps_ctx* ctx, int64_t nb);
bool dag_block(const gps_ctx* ctx, int64_t nb);
void dag_blocks(const gps_ctx* ctx, int64_t nb, std::vector<int>& sizes, int64_t& cnt);
int dag_width(const gps_ctx* ctx, int64_t nb, bool half);
int potrf_inv_rec(gps_ctx* ctx, double* A, int64_t lda, double* Linv, int64_t ldl, double* W,
                  int nb, double* logdiag, int* info, int base, int nreal, double* Lout,
                  int64_t ldlo, bool top = false);
size_t potrf_ws_doubles(int64_t n_pad);
int reset_info(gps_ctx* ctx);
hipError_t zero_factor(gps_ctx* ctx, double* p, int64_t n_pad, hipStream_t s);
bool factor_zeroed(const gps_ctx* ctx, const double* p, int64_t n_pad);
int potrf_inv(gps_ctx* ctx, double* A, int64_t n_pad, double* Linv, double* W, double* logdiag,
              int nreal, double* Lout);
int check_info(gps_ctx* ctx);
int set_theta(gps_ctx* ctx, Theta& th, int kind, const double* theta, int n_ell, int d);
int upload(gps_ctx* ctx, DBuf& b, const double* h, int64_t rows, int64_t cols, int64_t rows_pad);
void score_bundle(const double* sums, double nt, double out[GPS_N_SC]);
int bind(gps_ctx* ctx);
bool sharded(const gps_ctx* ctx);
std::vector<DBuf*> ctx_buffers(gps_ctx* ctx);
// api_comm.hip
void leave_local_group(gps_ctx* ctx);
int group_barrier(gps_ctx* ctx, LocalGroup& G, size_t count);
int allreduce_sum(gps_ctx* ctx, double* buf, size_t count, hipStream_t s);
int allreduce_sum_impl(gps_ctx* ctx, double* buf, size_t count, hipStream_t s);

}  // namespace gpsapi

// the non-exported functions of the C-ABI files (C linkage, as they were in the one file)
extern "C" {
int make_aux_streams(gps_ctx* ctx);
int factor_user(gps_ctx* ctx, int64_t n, const double* A, int64_t lda, bool want_L);
double* row_part(gps_ctx* ctx, int64_t rows, int nv);
int full_fit_core(gps_ctx* ctx, int kind, const double* theta, int n_ell);
int fitc_syrk_ks(const gps_ctx* ctx);
int fitc_syrk_rows(gps_ctx* ctx, const double* kscale, int ks, int64_t R0, int64_t R1);
int fitc_syrk(gps_ctx* ctx, const double* kscale, const double* base, double* dst,
              bool packed = false, const double* A = nullptr, int64_t lda = 0);
int fitc_syrk_allreduce(gps_ctx* ctx, double* red, int64_t blen, int64_t tail);
int fitc_test_prepass(gps_ctx* ctx);
int fitc_test_prepass_b(gps_ctx* ctx);
int fitc_fit_core(gps_ctx* ctx, const double* theta, int n_ell, double obj[GPS_N_OBJ],
                  bool pre_test = false);
int fitc_knm_xt(gps_ctx* ctx, int64_t ldc, const double* X, double* C);
int fitc_lt_vec(gps_ctx* ctx, const double* X, const double* x, double* y);
int fitc_tri_right(gps_ctx* ctx, const double* A, int64_t lda, const double* X, double* C,
                   int64_t ldc, int64_t rows);
int fitc_tri_left_t(gps_ctx* ctx, const double* X, const double* B, double* C);
}
