// FP64 MFMA GEMM for gfx950 — the one genuinely dense contraction of the GP hot path.
//
// Every O(n^3) / O(n m^2) step of the build reduces to this kernel:
//   * Cholesky trailing update  A22 -= L21 L21ᵀ        (SYRK, lower tiles only)
//   * TRSM as a product with the diagonal inverse       L21 = A21 L11⁻ᵀ
//   * triangular inverse off-diagonal blocks            L⁻¹21 = -L22⁻¹ (L21 L11⁻¹)
//   * predictive TRMM with fused column reductions      colsum((L⁻¹K_f*)²), (L⁻¹K_f*)ᵀβ
//   * FITC: ‖Lm⁻¹k_i‖² / ‖Lb⁻¹k_i‖² row reductions, B = Kmnᵀ Λ⁻¹ Knm (split-K SYRK)
// (reference: chol_solve KF:25-29, half-logdet KF:332, cal_mean_and_cov KF:121-126,
//  Q KF:32-39, spgp_cal_mean_and_cov K20:76-83 — all LAPACK/BLAS on the CPU there).
//
// Geometry: a TILE×TILE output tile per 256-thread workgroup (TILE = 128 for
// large grids, 64 for the latency-bound small grids at the bottom of the
// recursion); 4 waves, each a (TILE/2)² sub-tile of v_mfma_f64_16x16x4_f64
// blocks.  K is staged through LDS in 16-deep slices, double-buffered
// (global→register prefetch of slice k+1 while slice k is multiplied).  LDS
// images are k-major [k][TILE + 16]: a fragment read (16 consecutive doubles per
// k row, 4 k rows per wave instruction) hits all 64 banks without conflict (row
// stride ≡ 32 dwords mod 64).
//
// f64 MFMA operand map (cdna_hip_programming.md §3; checked on the box by
// tools/mfma_f64_probe.hip): lane l supplies A[i = l&15][k = l>>4] and
// B[k = l>>4][j = l&15]; accumulator register r of lane l is
// C[row = (l>>4) + 4r][col = l&15].  Built with -mllvm -amdgpu-mfma-vgpr-form=1:
// without it hipcc keeps the accumulators in VGPRs and copies them to AGPRs and
// back around every MFMA chain (measured: 35 TF/s instead of 77 on a pure MFMA
// loop, tools/mfma_f64_sweep.hip).
//
// Triangular operands are handled by clipping the K range per output tile (the
// diagonal 128-blocks of a triangular factor are stored with explicit zeros
// above the diagonal, so clipping at 64 or 128 granularity never drops a
// nonzero) — no multiply touches a structurally zero tile.
#include "gps_internal.h"

namespace gps {

typedef double d4 __attribute__((ext_vector_type(4)));
// staging registers: a native vector type, not HIP's double2 struct — struct copies
// lower to memcpy through a private alloca that SROA cannot promote, which put the
// B staging registers in scratch (80 B/lane of spills in the k-major-B kernels)
typedef double dv2 __attribute__((ext_vector_type(2)));

constexpr int BK = 16;
constexpr int GROUP_M = 8;

// logical tile id -> (ti, tj).  Lower-triangular enumeration for SYRK outputs
// (uniform work per tile); otherwise a grouped raster (GROUP_M tile rows at a
// time, column-major inside the group) so the tiles resident together share A
// and B panels in L2.
//
// Triangular operands (work per tile grows linearly along one tile index) are
// issued heaviest-first and WITHOUT the XCD-contiguous remap.  Measured on
// MI355X (tools/gemm_bench.cpp, 20096×5120×20096 TRMM): remap + any order
// 35-45 TF/s, plain grouped order 64.6, heaviest-first 68.9.  Workgroups are
// dealt to XCDs in block order, so an XCD whose slots are all held by long tiles
// stalls the dispatch of every later block; equal-work neighbours in block order
// (which land on different XCDs) avoid that.  Map 3 (the default for triangular
// operands since the microbenchmark below) keeps that equal-work-per-XCD property
// but gives each XCD a compact band of tiles: 70.7 TF/s on the same TRMM.
__device__ __forceinline__ bool tile_of(const GemmParams& p, int t, int& ti, int& tj) {
  if (p.lower_out) {
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    ti = r;
    tj = t - r * (r + 1) / 2;
    return true;
  }
  if (p.map_mode == 3) {
    // XCD-banded heaviest-first (triangular operands): block b runs on XCD b % 8;
    // XCD x owns a contiguous band of the index that does NOT carry the triangular
    // work and walks the other index heaviest-first, so every XCD gets the same work
    // profile (balanced under in-order dispatch) while its ~64 resident tiles form a
    // compact 2-D patch (both operand panels reused from its own L2).  Positions past
    // the matrix edge are holes (the workgroup exits at once).
    const int x = t & 7, i = t >> 3;
    if (p.tri == TRI_K_LE_I || p.tri == TRI_K_GE_I) {  // work grows/shrinks with ti
      const int bw = (p.tiles_n + 7) >> 3;
      const int ri = i / bw;
      tj = x * bw + i % bw;
      ti = p.tri == TRI_K_LE_I ? p.tiles_m - 1 - ri : ri;
      return tj < p.tiles_n && ri < p.tiles_m;
    }
    const int bh = (p.tiles_m + 7) >> 3;  // TRI_K_LE_J / TRI_K_GE_J: work follows tj
    const int cj = i / bh;
    ti = x * bh + i % bh;
    tj = p.tri == TRI_K_LE_J ? p.tiles_n - 1 - cj : cj;
    return ti < p.tiles_m && cj < p.tiles_n;
  }
  if (p.map_mode == 5) {
    // XCD-banded 8×8 patches (the automatic order of the FITC row norms): as map 3, XCD x owns
    // a band of the index that does not carry the triangular work, but its resident tiles form 8 (band) × 8
    // (work index) patches, the work index walked heaviest-first patch by patch, so an 8×8
    // group of tiles with neighbouring K ranges shares both operand panels in its L2.
    const int x = t & 7, i = t >> 3;
    const bool wi = p.tri == TRI_K_LE_I || p.tri == TRI_K_GE_I;  // work follows ti
    const int nb = wi ? p.tiles_n : p.tiles_m, nw = wi ? p.tiles_m : p.tiles_n;
    const int bb = (nb + 7) >> 3, per = ((bb + 7) >> 3) * 64;
    const int wg = i / per, rem = i - wg * per, w = rem & 63;
    const int bi = x * bb + (rem >> 6) * 8 + (w & 7), wk = wg * 8 + (w >> 3);
    if (bi >= min(nb, x * bb + bb) || wk >= nw) return false;
    const int widx = (p.tri == TRI_K_LE_I || p.tri == TRI_K_LE_J) ? nw - 1 - wk : wk;
    ti = wi ? widx : bi;
    tj = wi ? bi : widx;
    return true;
  }
  const int per_group = GROUP_M * p.tiles_n;
  const int g = t / per_group;
  const int first = g * GROUP_M;
  const int gm = min(GROUP_M, p.tiles_m - first);
  const int tt = t - g * per_group;
  ti = first + tt % gm;
  tj = tt / gm;
  if (p.map_mode != 0) return true;
  if (p.tri == TRI_K_LE_I) ti = p.tiles_m - 1 - ti;       // K grows with ti
  else if (p.tri == TRI_K_LE_J) tj = p.tiles_n - 1 - tj;  // K grows with tj
  // TRI_K_GE_I / TRI_K_GE_J: K shrinks with the index, natural order is heaviest-first
  return true;
}

// bijective XCD-contiguous remap: blocks b, b+8, b+16, ... (one XCD under the
// observed round-robin dispatch) get consecutive logical tile ids.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Row norms behind a running persistent factorisation (GemmParams::dep_mode).
// Row tiles are dealt to the 8 XCDs in contiguous bands; the dependent launch's workgroup takes,
// heaviest first, a column tile whose row of L⁻¹ is final, from its own XCD's band (then the
// others'), through one agent-scope ticket per (XCD, column).  It waits for a row only while
// every workgroup of the factorisation is known to have started (they are then resident and the
// factorisation finishes whatever this launch holds); before that it spins at most ~20 µs and
// then leaves its tile to the completion launch.  Waits are bounded (2 s without progress, then
// dep_err = 3) and give up when the factorisation reports an error.  Returns the tile (ti, tj) or
// false.  (Lane 0 decides; the other lanes wait at the barrier.)
__device__ __forceinline__ int dep_band0(int tm, int x) { return (int)((int64_t)tm * x / 8); }
__device__ __forceinline__ int dep_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ bool dep_take(const GemmParams& p, double* smem, int& ti, int& tj) {
  const int T = p.tiles_n, tm = p.tiles_m;
  if (p.dep_mode == 2) {  // the completion launch: the tiles the dependent launch left
    const int b = (int)blockIdx.x;
    tj = T - 1 - b / tm;
    ti = b - (b / tm) * tm;
    if (tj < 0) return false;
    int x = 7;
    while (x > 0 && dep_band0(tm, x) > ti) --x;
    const int len = dep_band0(tm, x + 1) - dep_band0(tm, x);
    return ti - dep_band0(tm, x) >= min(p.dep_q[x * 64 + tj], len);
  }
  // The take runs on wave 0's 64 lanes: one load per column state (lane j reads column j's)
  // and one per band counter (lane l reads band me + l's) per round instead of a lane-0 walk that
  // issued up to 9 dependent L2 round trips per exhausted column (round 5's dep_take; late in
  // the launch a workgroup walked ~10 of them before finding work).  Column state in kSigRdy:
  // 0 row not final, 1 final (the factorisation's store), 2 final and every band taken (set by
  // the workgroup that found all eight counters at their band length; counters only grow).
  int* sh = reinterpret_cast<int*>(smem);
  if (threadIdx.x < 64) {
    const int lane = (int)threadIdx.x;
    unsigned int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const int me = (int)(xcc & 7);
    int* st = p.dep_sig + kSigRdy;
    const int xb = (me + lane) & 7;  // lane l < 8: band me + l (this XCD's own band first)
    const int b0 = dep_band0(tm, xb), len = dep_band0(tm, xb + 1) - b0;
    int res = -1;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int seen = -1;
    unsigned int polls = 0;
    for (;;) {
      const int sv = lane < T ? dep_ld(st + lane) : 0;
      const unsigned long long ready = __ballot(sv != 0);
      unsigned long long cand = __ballot(sv == 1);
      while (cand && res < 0) {
        const int j = 63 - __builtin_clzll(cand);  // the heaviest final column not known taken
        cand &= ~(1ull << j);
        int* qj = p.dep_q + xb * 64 + j;
        const int qv = lane < 8 ? dep_ld(qj) : 0;
        unsigned long long open = __ballot(lane < 8 && qv < len);
        while (open && res < 0) {
          const int l = __builtin_ctzll(open);
          open &= open - 1;
          int r = 0;
          if (lane == l) r = __hip_atomic_fetch_add(qj, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          r = __shfl(r, l);
          const int lb0 = __shfl(b0, l), llen = __shfl(len, l);
          if (r < llen) res = (lb0 + r) << 8 | j;
        }
        if (res < 0 && lane == 0)
          __hip_atomic_store(st + j, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int nready = __popcll(ready);
      if (res >= 0 || nready == T) break;  // (all rows final and nothing left: the launch's tail)
      if (dep_ld(p.dep_err) != 0x7f7f7f7f) break;  // the factorisation failed: leave the tile
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (dep_ld(p.dep_sig + kSigStarted) < p.dep_grid) {  // not all resident yet: ≤ 20 µs
        if (now - t0 > 2000) break;
      } else {  // wait for the next row (bounded: 2 s without a new row and 1e5 polls)
        if (nready != seen) {
          seen = nready;
          t0 = now;
          polls = 0;
        } else if (++polls > 100000u && now - t0 > 200000000ull) {
          if (lane == 0) __hip_atomic_store(p.dep_err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // agent-scope acquire: the rows' payload (stored write-through and drained before the
    // factorisation's arrivals) is visible to the operand loads after the barrier
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (lane == 0) sh[0] = res;
  }
  __syncthreads();
  const int res = __builtin_amdgcn_readfirstlane(sh[0]);
  __syncthreads();  // (gemm_tile's first LDS stores overwrite sh)
  if (res < 0) return false;
  ti = res >> 8;
  tj = res & 255;
  return true;
}

template <int ALAY, int BLAY, int EPI, int TILE>
__device__ __forceinline__ void gemm_tile(const GemmParams& p, int ti, int tj, int kslice,
                                          double* smem, int kb_o = -1, int ke_o = -1,
                                          double* part = nullptr);
template <int ALAY, int BLAY>
__device__ void gemm_sk_block(const GemmParams& p, int s, double* smem);

template <int ALAY, int BLAY, int EPI, int TILE>
__global__ __launch_bounds__(256) void gemm_f64_kernel(GemmParams p) {
  constexpr int LS = TILE + 16;          // LDS row stride (doubles)
  constexpr int STAGE = 2 * BK * LS;     // one buffer: A image + B image
  __shared__ __attribute__((aligned(16))) double smem[2 * STAGE];
  const bool remap = p.map_mode == 2 || (p.map_mode == 0 && p.tri == TRI_NONE);
  // (map_mode 1 also disables the remap for lower-triangular SYRK grids)
  if constexpr (EPI == EPI_STORE && TILE == 128) {
    if (p.sk_wgs > 0 && (int)blockIdx.x >= p.sk_dp) {  // the stream-K tail (launch_gemm)
      gemm_sk_block<ALAY, BLAY>(p, (int)blockIdx.x - p.sk_dp, smem);
      return;
    }
  }
  if constexpr (EPI == EPI_ROWSQ) {
    if (p.dep_mode) {  // behind a running factorisation (dep_take)
      int ti, tj;
      if (dep_take(p, smem, ti, tj)) gemm_tile<ALAY, BLAY, EPI, TILE>(p, ti, tj, 0, smem);
      return;
    }
  }
  if constexpr (EPI == EPI_ROWSQ || EPI == EPI_ROWSQ_DOT) {
    if (p.map_mode == 6) {
      // paired column tiles (row norms over a triangular L⁻¹, work ∝ tj + 1): workgroup (ti, q)
      // runs column tile T−1−q and then q, so every workgroup has the same K, (T + 1)·TILE — the
      // grid is uniform like a square product's — in a grouped raster over XCD-contiguous ids
      const int np = (p.tiles_n + 1) >> 1;
      const int l = xcd_remap(blockIdx.x, gridDim.x);
      const int per_group = GROUP_M * np, g = l / per_group, first = g * GROUP_M;
      const int gm = min(GROUP_M, p.tiles_m - first), tt = l - g * per_group;
      const int ri = first + tt % gm, q = tt / gm, qh = p.tiles_n - 1 - q;
      gemm_tile<ALAY, BLAY, EPI, TILE>(p, ri, qh, 0, smem);
      if (q < qh) {
        __syncthreads();  // (the first tile's reduction still reads the LDS the second stages into)
        gemm_tile<ALAY, BLAY, EPI, TILE>(p, ri, q, 0, smem);
      }
      return;
    }
  }
  int ti, tj;
  if (p.slab_xcd) {
    // split-K, slice-major per XCD: the grid's (tile, slice) pairs in slice-major order, each XCD
    // a contiguous run of them, so the workgroups resident on an XCD share one K slice's rows of
    // both operands in its L2 (the tile-major remap spreads an XCD over every slice)
    const int nt = (int)gridDim.x;
    const int l = xcd_remap((int)(blockIdx.x + blockIdx.y * gridDim.x), nt * (int)gridDim.y);
    if (!tile_of(p, l % nt, ti, tj)) return;
    gemm_tile<ALAY, BLAY, EPI, TILE>(p, ti, tj, l / nt, smem);
    return;
  }
  const int nblk = p.sk_wgs > 0 ? p.sk_dp : (int)gridDim.x;
  if (!tile_of(p, remap ? xcd_remap(blockIdx.x, nblk) : (int)blockIdx.x, ti, tj)) return;
  gemm_tile<ALAY, BLAY, EPI, TILE>(p, ti, tj, blockIdx.y, smem);
}

// EPI_STORE epilogue: C = alpha·acc (+ beta·C) for this thread's accumulators
template <int TILE>
__device__ __forceinline__ void store_acc(const GemmParams& p, int ti, int tj, int kslice,
                                          const d4 (&acc)[TILE / 32][TILE / 32]) {
  constexpr int WT = TILE / 2, MI = WT / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int lrow = lane >> 4, lcol = lane & 15;
  const int row0 = ti * TILE, col0 = tj * TILE;
  double* Cb = p.C + (int64_t)kslice * p.c_kslice_stride;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + wr * WT + mi * 16 + lrow + 4 * r;
      double* crow = Cb + (int64_t)row * p.ldc + col0 + wc * WT + lcol;
#pragma unroll
      for (int ni = 0; ni < MI; ++ni) {
        double v = p.alpha * acc[mi][ni][r];
        if (p.beta != 0.0) v = fma(p.beta, crow[ni * 16], v);
        crow[ni * 16] = v;
      }
    }
}

// Stream-K tail of a 128-tile EPI_STORE launch with uniform K ranges (launch_gemm decides): the
// tiles [sk_dp, tiles) that would fill only part of a last round of workgroup slots are cut
// into sk_wgs equal runs of 16-deep K slices, one per workgroup (block s runs iterations
// [s·I/S, (s+1)·I/S) of the I = tiles·K/16 of the tail).  A run that covers part of a tile
// writes its partial accumulators to workspace slot (tile + s) — distinct for every (tile,
// block) pair, since runs are contiguous and ordered — publishes them (stores drained, agent
// release, relaxed ticket) and the last arriver of the tile (agent acquire) sums the partials
// in block order and runs the C epilogue: a fixed summation order, so the result is bitwise
// reproducible (cdna_hip_programming.md §5 "In-launch split-K reduction", plain-store recipe).
// The last arriver also zeroes the tile's ticket for the next launch.
template <int ALAY, int BLAY>
__device__ void gemm_sk_block(const GemmParams& p, int s, double* smem) {
  constexpr int TILE = 128, MI = TILE / 32, TT = TILE * TILE;
  const int tiles = p.lower_out ? p.tiles_m * (p.tiles_m + 1) / 2 : p.tiles_m * p.tiles_n;
  const int nk = p.K / BK;
  const int64_t I = (int64_t)(tiles - p.sk_dp) * nk, S = p.sk_wgs;
  auto bnd = [&](int64_t q) { return q * I / S; };
  auto owner = [&](int64_t x) {  // the block whose run holds iteration x
    int64_t q = x * S / I;
    while (q + 1 < S && bnd(q + 1) <= x) ++q;
    while (q > 0 && bnd(q) > x) --q;
    return (int)q;
  };
  const int tid = threadIdx.x;
  int64_t it = bnd(s);
  const int64_t it1 = bnd(s + 1);
  while (it < it1) {
    const int u = (int)(it / nk);
    const int k0 = (int)(it - (int64_t)u * nk);
    const int k1 = (int)min<int64_t>(nk, k0 + (it1 - it));
    int ti, tj;
    tile_of(p, p.sk_dp + u, ti, tj);
    const int s0 = owner((int64_t)u * nk), s1 = owner((int64_t)u * nk + nk - 1);
    if (s0 == s1) {  // the whole tile in this run
      gemm_tile<ALAY, BLAY, EPI_STORE, TILE>(p, ti, tj, 0, smem);
      __syncthreads();  // (its last slice is still being read when the next run stages)
    } else {
      gemm_tile<ALAY, BLAY, EPI_STORE, TILE>(p, ti, tj, 0, smem, k0 * BK, k1 * BK,
                                             p.ws + (int64_t)(u + s) * TT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      unsigned int* flag = reinterpret_cast<unsigned int*>(smem);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int t = __hip_atomic_fetch_add(p.sk_cnt + u, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int last = t == s1 - s0 ? 1u : 0u;
        if (last) {
          __hip_atomic_store(p.sk_cnt + u, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag[0] = last;
      }
      __syncthreads();
      const unsigned int last = __builtin_amdgcn_readfirstlane(flag[0]);
      __syncthreads();  // (the next run's first LDS stores may overwrite the flag)
      if (last) {
        d4 acc[MI][MI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < MI; ++ni) acc[mi][ni] = (d4){0.0, 0.0, 0.0, 0.0};
        for (int q = s0; q <= s1; ++q) {  // block order: deterministic
          const double* src = p.ws + (int64_t)(u + q) * TT + tid;
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < MI; ++ni)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[mi][ni][r] += src[((mi * MI + ni) * 4 + r) * 256];
        }
        store_acc<TILE>(p, ti, tj, 0, acc);
      }
    }
    it += k1 - k0;
  }
}

template <int ALAY, int BLAY, int EPI, int TILE>
__device__ __forceinline__ void gemm_tile(const GemmParams& p, int ti, int tj, int kslice,
                                          double* smem, int kb_o, int ke_o, double* part) {
  constexpr int LS = TILE + 16;          // LDS row stride (doubles)
  constexpr int STAGE = 2 * BK * LS;     // one buffer: A image + B image
  constexpr int WT = TILE / 2;           // per-wave sub-tile edge
  constexpr int MI = WT / 16;            // MFMA blocks per wave edge
  constexpr int PER = TILE * BK / 256;   // doubles of one operand slice per thread (8 or 4)
  constexpr int NQ = PER / 2;            // 16-byte loads per operand per thread
  constexpr int TPR = TILE / PER;        // threads per k-row for k-major sources (each thread
                                         // owns NQ 16-byte chunks 2·TPR doubles apart, so a
                                         // ds_write_b128 covers contiguous bytes: no conflicts)
  constexpr int TPI = BK / PER;          // threads per i-row for i-major sources
  // Image row k starts 4·(k >> 2) doubles in (skew SK on both images): the lanes that transpose
  // one i-major source row store to k rows PER apart, which the skew puts on different banks
  // (2-way / 4-way conflicts on every transposing store without it); the 4 rows one MFMA step
  // reads share a skew, so fragment reads stay conflict-free.  Applied where it measured faster
  // (profiles/r2_lds_skew_ab.txt): NT +1-5 % and every 64-tile shape +3-6 %; NN -2-5 % and
  // TN -1 % at TILE = 128, which keep the plain images.
  constexpr bool SK = TILE == 64 || (ALAY == LAY_N && BLAY == LAY_T);
  auto rowoff = [](int k) { return k * LS + (SK ? 4 * (k >> 2) : 0); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int row0 = ti * TILE, col0 = tj * TILE;

  int kb = 0, ke = p.K;
  switch (p.tri) {
    case TRI_K_LE_I: ke = min(ke, p.tri_off + row0 + TILE); break;
    case TRI_K_LE_J: ke = min(ke, p.tri_off + col0 + TILE); break;
    case TRI_K_GE_J: kb = p.tri_off + col0; break;
    case TRI_K_GE_I: kb = p.tri_off + row0; break;
    case TRI_KR_J:
      kb = p.kr[2 * (col0 / 16)];
      ke = p.kr[2 * ((col0 + TILE) / 16 - 1) + 1];
      break;
    default: break;
  }
  if (p.kend > 0 && ke > p.kend) ke = p.kend;  // (A's columns beyond kend are zero)
  if (kb_o >= 0) {  // a stream-K run: an explicit slice range of a uniform-K tile
    kb = kb_o;
    ke = ke_o;
  } else if (p.ksplit > 1) {
    const int nk = ke > kb ? (ke - kb) / BK : 0;
    const int s = kslice, q = nk / p.ksplit, r = nk % p.ksplit;
    const int s0 = s * q + min(s, r), s1 = s0 + q + (s < r ? 1 : 0);
    ke = kb + s1 * BK;
    kb = kb + s0 * BK;
  }
  const int nk = ke > kb ? (ke - kb) / BK : 0;

  // ---- global -> register staging (PER doubles of A and of B per thread) ----
  dv2 ra[NQ], rb[NQ];
  auto load_tile = [&](int k0) {
    if constexpr (ALAY == LAY_T) {  // A stored [k][i]
      const int k = tid / TPR, i = (tid % TPR) * 2;
      const dv2* src = reinterpret_cast<const dv2*>(p.A + (int64_t)(k0 + k) * p.lda + row0 + i);
#pragma unroll
      for (int q = 0; q < NQ; ++q) ra[q] = src[q * TPR];
      if (p.kscale) {
        const double sc = p.kscale[k0 + k];
#pragma unroll
        for (int q = 0; q < NQ; ++q) { ra[q].x *= sc; ra[q].y *= sc; }
      }
    } else {  // A stored [i][k]
      const int i = tid / TPI, k = (tid % TPI) * PER;
      const dv2* src = reinterpret_cast<const dv2*>(p.A + (int64_t)(row0 + i) * p.lda + k0 + k);
#pragma unroll
      for (int q = 0; q < NQ; ++q) ra[q] = src[q];
      if (p.kscale) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          ra[q].x *= p.kscale[k0 + k + 2 * q];
          ra[q].y *= p.kscale[k0 + k + 2 * q + 1];
        }
      }
    }
    if constexpr (BLAY == LAY_N) {  // B stored [k][j]
      const int k = tid / TPR, j = (tid % TPR) * 2;
      const dv2* src = reinterpret_cast<const dv2*>(p.B + (int64_t)(k0 + k) * p.ldb + col0 + j);
#pragma unroll
      for (int q = 0; q < NQ; ++q) rb[q] = src[q * TPR];
    } else {  // B stored [j][k]
      const int j = tid / TPI, k = (tid % TPI) * PER;
      const dv2* src = reinterpret_cast<const dv2*>(p.B + (int64_t)(col0 + j) * p.ldb + k0 + k);
#pragma unroll
      for (int q = 0; q < NQ; ++q) rb[q] = src[q];
    }
  };
  auto store_tile = [&](int buf) {
    double* As = smem + buf * STAGE;
    double* Bs = As + BK * LS;
    if constexpr (ALAY == LAY_T) {
      const int k = tid / TPR, i = (tid % TPR) * 2;
#pragma unroll
      for (int q = 0; q < NQ; ++q) *reinterpret_cast<dv2*>(&As[rowoff(k) + i + 2 * TPR * q]) = ra[q];
    } else {
      const int i = tid / TPI, k = (tid % TPI) * PER;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        As[rowoff(k + 2 * q) + i] = ra[q].x;
        As[rowoff(k + 2 * q + 1) + i] = ra[q].y;
      }
    }
    if constexpr (BLAY == LAY_N) {
      const int k = tid / TPR, j = (tid % TPR) * 2;
#pragma unroll
      for (int q = 0; q < NQ; ++q) *reinterpret_cast<dv2*>(&Bs[rowoff(k) + j + 2 * TPR * q]) = rb[q];
    } else {
      const int j = tid / TPI, k = (tid % TPI) * PER;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        Bs[rowoff(k + 2 * q) + j] = rb[q].x;
        Bs[rowoff(k + 2 * q + 1) + j] = rb[q].y;
      }
    }
  };

  d4 acc[MI][MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < MI; ++ni) acc[mi][ni] = (d4){0.0, 0.0, 0.0, 0.0};

  auto compute = [&](int buf) {
    const double* As = smem + buf * STAGE;
    const double* Bs = As + BK * LS;
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int krow = rowoff(kk * 4 + (lane >> 4)) + (lane & 15);
      double a[MI], b[MI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) a[mi] = As[krow + wr * WT + mi * 16];
#pragma unroll
      for (int ni = 0; ni < MI; ++ni) b[ni] = Bs[krow + wc * WT + ni * 16];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  // EPI_ROWSQ_DOT: the last column tile spans the full K range, so its A rows also give
  // A[row,:]·w — threads 0..TILE-1 take one row each from the slice image in LDS (w read
  // wave-uniform), which spares the caller a separate pass over A (FITC g = Knm c)
  const bool rdot = EPI == EPI_ROWSQ_DOT && tj == p.tiles_n - 1 && kb == 0;
  double dacc = 0.0;
  auto row_dot = [&](int buf, int k0) {
    if constexpr (EPI == EPI_ROWSQ_DOT) {
      if (rdot && tid < TILE) {
        const double* As = smem + buf * STAGE;
#pragma unroll
        for (int k = 0; k < BK; ++k) dacc = fma(As[rowoff(k) + tid], p.w[k0 + k], dacc);
      }
    }
  };

  if (nk > 0) {
    load_tile(kb);
    store_tile(0);
    __syncthreads();
    // steady state: prefetch slice it+1 into registers, multiply slice it, then
    // park the prefetched slice in the other LDS buffer (no branches in the body)
    for (int it = 0; it < nk - 1; ++it) {
      load_tile(kb + (it + 1) * BK);
      if (p.prio) __builtin_amdgcn_s_setprio(1);
      compute(it & 1);
      if (p.prio) __builtin_amdgcn_s_setprio(0);
      row_dot(it & 1, kb + it * BK);
      store_tile((it + 1) & 1);
      __syncthreads();
    }
    compute((nk - 1) & 1);
    row_dot((nk - 1) & 1, kb + (nk - 1) * BK);
  }
  if constexpr (EPI == EPI_ROWSQ_DOT) {
    if (rdot && tid < TILE) p.out1[row0 + tid] = dacc;
  }

  const int lrow = lane >> 4, lcol = lane & 15;
  if constexpr (EPI == EPI_STORE) {
    if (part) {  // stream-K partial: this thread's accumulators, coalesced ([element][thread])
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) part[((mi * MI + ni) * 4 + r) * 256 + tid] = acc[mi][ni][r];
      return;
    }
    store_acc<TILE>(p, ti, tj, kslice, acc);
  } else if constexpr (EPI == EPI_ROWSQ || EPI == EPI_ROWSQ_DOT) {
    // out0[tj][row] = sum over this tile's columns of (alpha*acc)^2
    double* red = smem;  // [2 (wc)][TILE rows]
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) s = fma(acc[mi][ni][r], acc[mi][ni][r], s);
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 8);
        if (lcol == 0) red[wc * TILE + wr * WT + mi * 16 + lrow + 4 * r] = s;
      }
    __syncthreads();
    if (tid < TILE)
      p.out0[(int64_t)tj * p.ld_out + row0 + tid] = p.alpha * p.alpha * (red[tid] + red[TILE + tid]);
  } else {  // EPI_COLRED: out0[ti][col] = sum_rows w[row]*acc, out1[ti][col] = sum_rows acc^2
    double* red = smem;  // [2 (wr)][2][TILE]
    __syncthreads();
    double wv[MI][4];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) wv[mi][r] = p.w[row0 + wr * WT + mi * 16 + lrow + 4 * r];
#pragma unroll
    for (int ni = 0; ni < MI; ++ni) {
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1 = fma(acc[mi][ni][r], wv[mi][r], s1);
          s2 = fma(acc[mi][ni][r], acc[mi][ni][r], s2);
        }
      s1 += __shfl_xor(s1, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 16);
      s2 += __shfl_xor(s2, 32);
      if (lrow == 0) {
        red[wr * 2 * TILE + wc * WT + ni * 16 + lcol] = s1;
        red[wr * 2 * TILE + TILE + wc * WT + ni * 16 + lcol] = s2;
      }
    }
    __syncthreads();
    if (tid < TILE) {
      p.out0[(int64_t)ti * p.ld_out + col0 + tid] = p.alpha * (red[tid] + red[2 * TILE + tid]);
      p.out1[(int64_t)ti * p.ld_out + col0 + tid] =
          p.alpha * p.alpha * (red[TILE + tid] + red[3 * TILE + tid]);
    }
  }
}

// Latency-optimised GEMM for the bottom of the recursion: no LDS staging, no split-K slabs,
// no reduction launch.  A wave owns a (16R)×(16R) output block (R·R accumulators of
// v_mfma_f64_16x16x4) over its share of K; WPT waves of one workgroup split K between them
// and the partial sums meet in LDS (fixed order: bitwise reproducible).  Operands stream
// straight from L2 into MFMA registers: for a 16-deep K chunk lane l (r = l & 15,
// g = l >> 4) feeds MFMA step kk with k = 4g + kk of A row r and B column r — a fixed
// permutation of k inside the chunk shared by both operands, so row-major A / Bᵀ fragments
// are one contiguous 32-byte load per lane.  Loads are issued G chunks at a time, one group
// ahead of the MFMAs, so a K range of ≤ G chunks per wave costs ONE memory latency (the
// one-chunk-ahead predecessor paid one per chunk: ~6-7 µs at K = 128, profiles/r2_kernel_stats).
// lower_out enumerates the blocks of the lower 64-tiles (diagonal 64-tiles whole, as the
// 64/128-tile kernels write them).
template <int ALAY, int BLAY, int R, int WPT>
__global__ __launch_bounds__(256) void gemm_f64_small_kernel(GemmParams p) {
  constexpr int TE = 16 * R;         // output block edge per tile
  constexpr int TPB = 4 / WPT;       // tiles per workgroup
  constexpr int G = R == 1 ? 4 : 2;  // 16-deep chunks per load group (64 VGPRs per group)
  constexpr int NACC = R * R * 4;    // doubles of accumulator per lane
  __shared__ double red[WPT > 1 ? 4 * NACC * 64 : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = wave / WPT, part = wave - slot * WPT;
  const int t = blockIdx.x * TPB + slot;
  const int tm = p.M / TE, tn = p.N / TE;
  int ti = 0, tj = 0;
  bool valid;
  if (p.lower_out) {  // blocks (ti, tj) with tj/u <= ti/u, u = 64/TE, row-major over ti
    constexpr int u = 64 / TE;
    auto pre = [](int r) { const int a = r / u, b = r % u; return u * (u * a * (a + 1) / 2 + b * (a + 1)); };
    valid = t < pre(tm);
    if (valid) {
      int lo = 0, hi = tm;
      while (hi - lo > 1) { const int mid = (lo + hi) / 2; if (pre(mid) <= t) lo = mid; else hi = mid; }
      ti = lo;
      tj = t - pre(ti);
    }
  } else {
    valid = t < tm * tn;
    if (valid) { ti = t / tn; tj = t - ti * tn; }
  }
  if (WPT == 1 && !valid) return;  // (with WPT > 1 every wave reaches the LDS barrier)
  const int row0 = ti * TE, col0 = tj * TE;
  int kb = 0, ke = p.K;
  switch (p.tri) {
    case TRI_K_LE_I: ke = min(ke, p.tri_off + row0 + TE); break;
    case TRI_K_LE_J: ke = min(ke, p.tri_off + col0 + TE); break;
    case TRI_K_GE_J: kb = p.tri_off + col0; break;
    case TRI_K_GE_I: kb = p.tri_off + row0; break;
    case TRI_KR_J:
      kb = p.kr[2 * (col0 / 16)];
      ke = p.kr[2 * ((col0 + TE) / 16 - 1) + 1];
      break;
    default: break;
  }
  const int nk = valid && ke > kb ? (ke - kb) / 16 : 0;
  const int q = nk / WPT, rr = nk - q * WPT;
  const int c0 = part * q + min(part, rr), c1 = c0 + q + (part < rr ? 1 : 0);
  const int r = lane & 15, g = lane >> 4;

  typedef double Frag[G][R][4];
  auto load_chunk = [&](int c, double (&a)[R][4], double (&b)[R][4]) {
    const int k = kb + 16 * c + 4 * g;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + 16 * i + r;
      if constexpr (ALAY == LAY_N) {
        const dv2* s = reinterpret_cast<const dv2*>(p.A + (int64_t)row * p.lda + k);
        const dv2 u0 = s[0], u1 = s[1];
        a[i][0] = u0.x; a[i][1] = u0.y; a[i][2] = u1.x; a[i][3] = u1.y;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) a[i][e] = p.A[(int64_t)(k + e) * p.lda + row];
      }
      const int col = col0 + 16 * i + r;
      if constexpr (BLAY == LAY_T) {
        const dv2* s = reinterpret_cast<const dv2*>(p.B + (int64_t)col * p.ldb + k);
        const dv2 u0 = s[0], u1 = s[1];
        b[i][0] = u0.x; b[i][1] = u0.y; b[i][2] = u1.x; b[i][3] = u1.y;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) b[i][e] = p.B[(int64_t)(k + e) * p.ldb + col];
      }
    }
  };
  d4 acc[R][R];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  auto load_group = [&](int c, Frag& a, Frag& b) {
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (c + j < c1) load_chunk(c + j, a[j], b[j]);
  };
  auto mma_group = [&](int c, const Frag& a, const Frag& b) {
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (c + j < c1) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int jj = 0; jj < R; ++jj)
              acc[i][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j][i][kk], b[j][jj][kk], acc[i][jj], 0, 0, 0);
      }
  };
  Frag fa0, fb0, fa1, fb1;
  int c = c0;
  if (c < c1) load_group(c, fa0, fb0);
  while (c < c1) {
    if (c + G < c1) load_group(c + G, fa1, fb1);
    mma_group(c, fa0, fb0);
    c += G;
    if (c >= c1) break;
    if (c + G < c1) load_group(c + G, fa0, fb0);
    mma_group(c, fa1, fb1);
    c += G;
  }
  if constexpr (WPT > 1) {  // partial sums of the K parts meet in LDS, summed in part order
    double* mine = red + (int64_t)wave * NACC * 64 + lane;
    if (part > 0) {
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) mine[((i * R + j) * 4 + e) * 64] = acc[i][j][e];
    }
    __syncthreads();
    if (part > 0 || !valid) return;
#pragma unroll
    for (int w = 1; w < WPT; ++w) {
      const double* o = mine + w * NACC * 64;
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] += o[((i * R + j) * 4 + e) * 64];
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      double* crow = p.C + (int64_t)(row0 + 16 * i + g + 4 * e) * p.ldc + col0 + r;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        double v = p.alpha * acc[i][j][e];
        if (p.beta != 0.0) v = fma(p.beta, crow[16 * j], v);
        crow[16 * j] = v;
      }
    }
}

// output blocks of the small kernel at edge te (lower_out: the blocks of the lower 64-tiles)
static int64_t small_tiles(const GemmParams& p, int te) {
  const int64_t tm = p.M / te, tn = p.N / te;
  if (!p.lower_out) return tm * tn;
  const int64_t u = 64 / te, a = tm / u;
  return u * u * a * (a + 1) / 2;
}

// C = beta*C + alpha * sum_s slab_s, slabs summed in slice order (deterministic);
// lower_tile > 0: only tiles with tj <= ti at that tile edge (the rest of a SYRK slab is unwritten)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const double* __restrict__ ws, int ks,
                                                            int M, int N, int lower_tile,
                                                            double alpha, double beta,
                                                            double* __restrict__ C, int64_t ldc) {
  const int64_t e = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (e >= (int64_t)M * N) return;
  const int i = (int)(e / N), j = (int)(e - (int64_t)i * N);
  if (lower_tile && j / lower_tile > i / lower_tile) return;
  const int64_t slab = (int64_t)M * N;
  dv2 s = *reinterpret_cast<const dv2*>(ws + e);
  for (int q = 1; q < ks; ++q) s += *reinterpret_cast<const dv2*>(ws + q * slab + e);
  dv2* c = reinterpret_cast<dv2*>(C + (int64_t)i * ldc + j);
  dv2 v = alpha * s;
  if (beta != 0.0) v += beta * *c;
  *c = v;
}

// The split-K reduction of a symmetric result (GemmParams::mirror): per lower 32-tile (r >= c)
// the slices summed in order (the values splitk_reduce_kernel writes), the tile stored and, below
// the diagonal, its transpose through LDS into tile (c, r) — sym_mirror's copy without a launch
// (the energy score's Newton–Schulz chains: one launch fewer per product).
__global__ __launch_bounds__(256) void splitk_reduce_sym_kernel(const double* __restrict__ ws, int ks,
                                                                int N, double alpha, double beta,
                                                                double* __restrict__ C, int64_t ldc) {
  __shared__ double t[32][33];
  const int b = blockIdx.x;
  int r = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= b) ++r;
  while (r * (r + 1) / 2 > b) --r;
  const int c = b - r * (r + 1) / 2;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t slab = (int64_t)N * N;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = r * 32 + ty + 8 * k, j = c * 32 + tx;
    const int64_t e = (int64_t)i * N + j;
    double sum = ws[e];
    for (int q = 1; q < ks; ++q) sum += ws[q * slab + e];
    double v = alpha * sum;
    double* cp = C + (int64_t)i * ldc + j;
    if (beta != 0.0) v += beta * *cp;
    *cp = v;
    t[ty + 8 * k][tx] = v;
  }
  if (r == c) return;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) C[(int64_t)(c * 32 + ty + 8 * k) * ldc + r * 32 + tx] = t[tx][ty + 8 * k];
}

int g_tiny_gemm = 1;  // GPS_OPT_TINY_GEMM (process-wide; set through gps_ctx_set_option)
// GPS_OPT_SLAB_XCD (process-wide): split-K launches slice-major per XCD.  The FITC SYRK's L2-fabric
// bytes 4.48 -> 1.91 GB per C4 launch (7x -> 2.9x its Knm operand), time neutral (C4 11.86 -> 11.83,
// C3 / C5 within noise: profiles/r4_slab_xcd_ab.txt) — the SYRK is not fabric-bound
int g_slab_xcd = 1;
// GPS_OPT_STREAM_K (process-wide): 2 (default) — the stream-K tail for launches that run alone (the
// trailing update with nothing forked beside it: overlap off or below the fork level), where the
// last round's idle slots are otherwise lost; with the side stream's T product beside the SYRK the
// tail is already filled and the split only costs
int g_stream_k = 2;

// waves per output block of the small kernel: K split 4 ways whenever there are 4 chunks
static int small_wpt(int K) { return K >= 64 ? 4 : (K >= 32 ? 2 : 1); }

static int64_t tiles_for(const GemmParams& p, int tile) {
  const int64_t tm = p.M / tile, tn = p.N / tile;
  return p.lower_out ? tm * (tm + 1) / 2 : tm * tn;
}

// Launch shape.  The 128-tile kernel holds 2 workgroups per CU (512 slots on 256 CUs).
// Below two full waves of 128-tiles the grid leaves CUs idle or unevenly loaded, so
// the GEMM switches to 64-tiles (4x the tiles) and splits K until the grid has about
// 1024 workgroups (2048 for SYRK, whose tiles are uniform), with at least 64 of K per
// slice and ks*M*N within the caller's workspace.  Row/column epilogues keep 128
// (their partial sums are laid out per 128-tile).  Thresholds from the
// tools/gemm_bench.cpp sweep on MI355X (profiles/r1_gemm_sweep.txt): e.g. a
// 1280-level triangular product 161 us -> 58 us, 2560-level 31 -> 47 TF/s.
// The bottom of the recursion goes to the small kernel (profiles/r2_small_gemm.txt,
// per launch incl. the boundary): 16-blocks up to M·N = 256² (128³: 7.6 -> 3.4 µs),
// 32-blocks for triangular products up to the 1280 level (640³ 23.5 -> 15-19 µs,
// 1024³ 45 -> 35 µs) and for SYRKs up to 640 (640² K=640 17.1 -> 14.2 µs); the
// LDS-tiled 64-tile kernel stays ahead for larger SYRKs (less L2 traffic per flop).
GemmPlan gemm_plan(int epi, const GemmParams& p, int64_t ws_cap) {
  if (p.tile) return {p.tile, p.ksplit > 1 ? p.ksplit : 1};
  if (epi != EPI_STORE || p.ksplit > 1) return {128, p.ksplit > 1 ? p.ksplit : 1};
  if (g_tiny_gemm && !p.kscale && p.K <= 1280) {
    const int64_t mn = (int64_t)p.M * p.N;
    if ((mn <= 256 * 256 && p.K <= 1024) || (p.lower_out && p.M <= 384 && p.K <= 640))
      return {16, small_wpt(p.K)};
    if (p.lower_out ? (p.M <= 640 && p.K <= 640) : (mn <= 1280 * 1280 && (p.tri || p.K <= 640)))
      return {32, small_wpt(p.K)};
  }
  // 128-tiles from 512 of them (the 5k-level trailing SYRK, 780 lower tiles, left the 64-tile
  // path: C3 -0.7 %; 256 was slower — the 2.5k-level TRMMs want 64-tiles: profiles/r2_t128_ab.txt)
  if (tiles_for(p, 128) >= 512) return {128, 1};
  const int64_t t64 = tiles_for(p, 64);
  const int64_t target = p.lower_out ? 2048 : 1024;
  int ks = 1;
  while (ks < 8 && t64 * ks < target && p.K / (2 * ks) >= 64 &&
         (int64_t)(2 * ks) * p.M * p.N <= ws_cap)
    ks *= 2;
  return {64, ks};
}

hipError_t launch_gemm(int alay, int blay, int epi, const GemmParams& pin, hipStream_t s) {
  GemmParams p = pin;
  if (p.M % GPS_TILE || p.N % GPS_TILE || p.K % BK || p.M <= 0 || p.N <= 0)
    return hipErrorInvalidValue;
  if ((p.lda & 1) || (p.ldb & 1) || (p.ldc & 1)) return hipErrorInvalidValue;
  if (p.lower_out && p.M != p.N) return hipErrorInvalidValue;
  if (p.mirror && (!p.lower_out || p.M % 32)) return hipErrorInvalidValue;
  if (p.ksplit < 1) p.ksplit = 1;
  // the row dot comes from the last column tile, which must span the whole K range (columns
  // [tri_off, tri_off + N) of a larger triangular product whose last column is K)
  if (epi == EPI_ROWSQ_DOT &&
      (!p.w || !p.out1 || p.tri != TRI_K_LE_J || p.tri_off < 0 || p.K != p.tri_off + p.N ||
       p.ksplit != 1))
    return hipErrorInvalidValue;
  const GemmPlan plan = gemm_plan(epi, p, p.ws ? p.ws_cap : 0);
  const int tile = plan.tile;
  if (tile == 16 || tile == 32) {  // small kernel: tile = block edge, ksplit = waves per block
    if (epi != EPI_STORE || p.kscale) return hipErrorInvalidValue;
    const int wpt = plan.ksplit;
    if (wpt != 1 && wpt != 2 && wpt != 4) return hipErrorInvalidValue;
    const int64_t tt = small_tiles(p, tile);
    const dim3 grid((unsigned)((tt * wpt + 3) / 4)), block(256);
    hipError_t err = hipErrorInvalidValue;
#define GPS_SMALL_CASE(AL, BL, RR, W)                                                           \
    if (err == hipErrorInvalidValue && alay == AL && blay == BL && tile == 16 * RR && wpt == W) { \
      hipLaunchKernelGGL((gemm_f64_small_kernel<AL, BL, RR, W>), grid, block, 0, s, p);           \
      err = hipGetLastError();                                                                    \
    }
#define GPS_SMALL_LAYOUTS(RR, W)                                                                \
    GPS_SMALL_CASE(LAY_N, LAY_T, RR, W) GPS_SMALL_CASE(LAY_N, LAY_N, RR, W)                     \
    GPS_SMALL_CASE(LAY_T, LAY_N, RR, W) GPS_SMALL_CASE(LAY_T, LAY_T, RR, W)
    GPS_SMALL_LAYOUTS(1, 1) GPS_SMALL_LAYOUTS(1, 2) GPS_SMALL_LAYOUTS(1, 4)
    GPS_SMALL_LAYOUTS(2, 1) GPS_SMALL_LAYOUTS(2, 2) GPS_SMALL_LAYOUTS(2, 4)
#undef GPS_SMALL_LAYOUTS
#undef GPS_SMALL_CASE
    if (err == hipSuccess && p.mirror) err = launch_sym_mirror(p.C, p.ldc, p.M, s);
    return err;
  }
  if (tile != 64 && tile != 128) return hipErrorInvalidValue;
  if (tile == 64 && epi != EPI_STORE) return hipErrorInvalidValue;
  p.ksplit = plan.ksplit;
  // split-K: with a workspace, slices go to slabs and an ordered reduction applies
  // alpha/beta; without one (legacy FITC path) slice s writes C + s*c_kslice_stride
  const bool slabbed = p.ksplit > 1 && p.ws != nullptr;
  if (p.ksplit > 1 && !slabbed && (epi != EPI_STORE || p.beta != 0.0)) return hipErrorInvalidValue;
  // a symmetric result is mirrored from the one reduced C; unslabbed slices land in separate
  // C + s·c_kslice_stride blocks, so there is nothing whole to mirror
  if (p.ksplit > 1 && !slabbed && p.mirror) return hipErrorInvalidValue;
  GemmParams q = p;
  if (slabbed) {
    if (epi != EPI_STORE) return hipErrorInvalidValue;
    q.C = p.ws;
    q.ldc = p.N;
    q.c_kslice_stride = (int64_t)p.M * p.N;
    q.alpha = 1.0;
    q.beta = 0.0;
  }
  q.tiles_m = q.M / tile;
  q.tiles_n = q.N / tile;
  int tiles = (int)tiles_for(q, tile);
  // triangular operands default to the XCD-banded heaviest-first order (map 3):
  // measured +2-4% over plain heaviest-first on every 10k-level shape of the C3 build.  The FITC
  // row norms (EPI_ROWSQ*) over a triangular L⁻¹ default to paired column tiles (map 6: uniform
  // work per workgroup; C4 11.82 → 11.72 ms, C5 neutral, profiles/r5h_rowsq_pairs.txt), before
  // that to the 8×8-patch order (map 5: C5 174.0 vs 181.5 ms against map 3 in round 2, while the
  // patch order on the factorisation / predictive TRMMs cost C3 27 %, profiles/r2_map5_ab.txt;
  // maps 3 and 7 for the row norms: profiles/r4_rowsq_map_ab.txt)
  const bool rowsq = epi == EPI_ROWSQ || epi == EPI_ROWSQ_DOT;
  if (q.dep_mode) {  // behind a factorisation: one workgroup per tile, tiles from dep_take
    if (epi != EPI_ROWSQ || alay != LAY_N || blay != LAY_T || q.tri != TRI_K_LE_J || q.tri_off != 0 ||
        tile != 128 || q.ksplit != 1 || q.tiles_n > 64 || !q.dep_sig || !q.dep_q || !q.dep_err ||
        q.dep_mode > 2 || q.K != q.N)
      return hipErrorInvalidValue;
    q.map_mode = 0;
    q.prio = 0;
    q.slab_xcd = 0;
    q.sk_dp = q.sk_wgs = 0;
    const dim3 grid((unsigned)(q.tiles_m * q.tiles_n)), block(256);
    hipLaunchKernelGGL((gemm_f64_kernel<LAY_N, LAY_T, EPI_ROWSQ, 128>), grid, block, 0, s, q);
    return hipGetLastError();
  }
  const bool pairable = rowsq && q.tri == TRI_K_LE_J && tile == 128 && q.ksplit == 1;
  if (q.map_mode == 6 && !pairable) q.map_mode = 0;  // (an override of 6 leaves the rest automatic)
  // pairs for every pairable launch since round 6: round 5 kept the smaller grids (< 2048 pairs)
  // in map 5 — C4's test-side norms ran 1097 µs paired against 961 then
  // (profiles/r5k_rowsq_pairs_prof.txt) — but on the round-6 library the same 10 112-row shape
  // runs 49.6 TF/s paired against 45.0 in map 5 (tools/gemm_bench rowsq_iso), and pairs on the
  // small grids (the test-side norms, C5's pre-pass at 25 000 rows) measured C4 11.64 → 11.44 ms
  // and C5r8 28.47 → 27.25 (profiles/r6q_rowsq_pairs_all_ab.txt)
  const bool paired = pairable;
  if (q.map_mode == 0 && q.tri != TRI_NONE && q.tri != TRI_KR_J && !q.lower_out)
    q.map_mode = rowsq ? (paired ? 6 : 5) : 3;
  else if (q.map_mode == 4) q.map_mode = 0;  // 4: the previous automatic order (A/B runs)
  if (q.map_mode == 6) tiles = q.tiles_m * ((q.tiles_n + 1) / 2);
  if (q.map_mode == 5 && (q.lower_out || q.tri == TRI_NONE || q.tri == TRI_KR_J)) q.map_mode = 0;
  if (q.map_mode == 5) {  // 8 XCDs × ceil(work / 8) groups × the band's 8-wide groups × 64
    const bool wi = q.tri == TRI_K_LE_I || q.tri == TRI_K_GE_I;
    const int nb = wi ? q.tiles_n : q.tiles_m, nw = wi ? q.tiles_m : q.tiles_n;
    tiles = 8 * ((nw + 7) / 8) * (((nb + 7) / 8 + 7) / 8) * 64;
  }
  if (q.map_mode == 3) {
    if (q.lower_out || q.tri == TRI_NONE || q.tri == TRI_KR_J) return hipErrorInvalidValue;
    tiles = (q.tri == TRI_K_LE_I || q.tri == TRI_K_GE_I) ? 8 * ((q.tiles_n + 7) / 8) * q.tiles_m
                                                          : 8 * ((q.tiles_m + 7) / 8) * q.tiles_n;
  }
  // stream-K tail (gemm_sk_block): a 128-tile EPI_STORE launch with uniform K ranges whose last
  // round of workgroup slots would be at most 3/4 full runs that round's tiles as equal K runs
  // over every slot instead
  q.sk_dp = q.sk_wgs = 0;
  if ((g_stream_k == 1 || (g_stream_k == 2 && q.sk_alone)) && epi == EPI_STORE && tile == 128 &&
      q.ksplit == 1 && q.sk_cnt && q.ws &&
      q.sk_slots > 0 && q.tri == TRI_NONE && (q.lower_out || q.map_mode == 0 || q.map_mode == 2)) {
    const int slots = q.sk_slots, rem = tiles % slots;
    if (tiles >= slots && rem > 0 && 4 * rem <= 3 * slots && rem <= kStreamKTiles &&
        (int64_t)(rem + slots) * 128 * 128 <= q.ws_cap && q.K / BK >= 2) {
      q.sk_dp = tiles - rem;
      q.sk_wgs = slots;
      tiles = q.sk_dp + slots;
    }
  }
  // raised MFMA-phase priority: 1 = the product / column-reduction launches only (C3 −1.3 %;
  // the FITC row-norm launches and the Λ-scaled SYRK ran 0.4 % slower with it), 2 = every launch
  // (GPS_OPT_GEMM_PRIO 0 and 2 measured slower and were removed in round 6: DESIGN §6.31)
  q.prio = (epi == EPI_STORE || epi == EPI_COLRED) && !q.kscale;
  // slice-major per XCD: split-K launches whose tile index is the plain (or remapped) raster
  q.slab_xcd = g_slab_xcd && q.ksplit > 1 && q.sk_wgs == 0 &&
               (q.map_mode == 0 || q.map_mode == 2) && (q.lower_out || q.tri == TRI_NONE);
  dim3 grid(tiles, q.ksplit), block(256);
  hipError_t err = hipErrorInvalidValue;
#define GPS_GEMM_CASE(AL, BL, EP, T)                                                        \
  if (err == hipErrorInvalidValue && alay == AL && blay == BL && epi == EP && tile == T) { \
    hipLaunchKernelGGL((gemm_f64_kernel<AL, BL, EP, T>), grid, block, 0, s, q);            \
    err = hipGetLastError();                                                                \
  }
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_STORE, 128)
  GPS_GEMM_CASE(LAY_N, LAY_N, EPI_STORE, 128)
  GPS_GEMM_CASE(LAY_T, LAY_N, EPI_STORE, 128)
  GPS_GEMM_CASE(LAY_T, LAY_T, EPI_STORE, 128)
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_ROWSQ, 128)
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_ROWSQ_DOT, 128)
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_COLRED, 128)
  GPS_GEMM_CASE(LAY_N, LAY_T, EPI_STORE, 64)
  GPS_GEMM_CASE(LAY_N, LAY_N, EPI_STORE, 64)
  GPS_GEMM_CASE(LAY_T, LAY_N, EPI_STORE, 64)
  GPS_GEMM_CASE(LAY_T, LAY_T, EPI_STORE, 64)
#undef GPS_GEMM_CASE
  if (err != hipSuccess) return err;
  if (!slabbed) return p.mirror ? launch_sym_mirror(p.C, p.ldc, p.M, s) : hipSuccess;
  if (p.mirror) {
    const int64_t t32 = p.M / 32;
    hipLaunchKernelGGL(splitk_reduce_sym_kernel, dim3((unsigned)(t32 * (t32 + 1) / 2)), dim3(256), 0,
                       s, p.ws, p.ksplit, p.N, p.alpha, p.beta, p.C, p.ldc);
    return hipGetLastError();
  }
  const int64_t pairs = (int64_t)p.M * p.N / 2;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, s,
                     p.ws, p.ksplit, p.M, p.N, p.lower_out ? tile : 0, p.alpha, p.beta, p.C, p.ldc);
  return hipGetLastError();
}

}  // namespace gps
