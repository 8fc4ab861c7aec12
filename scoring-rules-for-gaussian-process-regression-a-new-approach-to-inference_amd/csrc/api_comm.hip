// C-ABI, multi-GPU: the RCCL communicator and the in-process stand-in (gps_comm_init_local), and
// the all-reduce every row-sharded FITC path calls.
#include "api_internal.h"

namespace gpsapi {

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

}  // namespace gpsapi

extern "C" {

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
