// HIP kernels (gfx950) for Coverage-v0's greedy expert, batched over B envs.
//
// Reference (gym_flock/envs/spatial/coverage.py): construct_time_matrix :621-653 and
// controller(greedy=True) :800-872.
//
// Time matrix. The reference relaxes hop counts column-wise over the motion edges in
// list order, in place (Gauss-Seidel), for all sources at once, and sweeps while some
// entry changed AND some entry is still infinite, at most horizon+1 sweeps. Rows
// (sources) are independent within a sweep; only the stop rule couples them. So:
//   - one wave per 64 sources of one env; each lane owns one source's row, kept in LDS
//     as uint16 (0xFFFF = inf) in column-major order, so a lane only ever touches its
//     own entries and a sweep needs no barrier;
//   - edge order within a sweep: two relaxations commute unless one writes a column
//     the other reads or writes, so any order that keeps every such pair in list order
//     gives bit-identical results (tests/test_coverage_greedy_gpu.py checks it against
//     the reference's matrices). cov_tm_schedule_kernel levels the edge list by those
//     conflicts and packs each level into batches of 8 mutually independent edges
//     (padded with no-ops on a dummy column): a batch's 16 column loads and 8 stores
//     issue back to back, without branches;
//   - pass A sweeps to the horizon (or to the wave's own fixed point), writes cost rows
//     and predecessors, and records per sweep whether its rows changed / hold an inf;
//   - pass B derives the reference's sweep count K* from every chunk's flags; only a
//     chunk that pass A swept past K* (the env-wide stop came first) is recomputed.
//
// Greedy step: 8 lanes per robot scan its node's cost row (16-byte uint16 loads, several
// in flight) for the first-index argmin over masked targets, then look one predecessor up.
#include "coverage_internal.h"

namespace gf {

namespace {

#ifndef GF_TM_DIAG
#define GF_TM_DIAG 0  // timing ablations only (wrong results): 1 no early stop, 2 schedule window, 4 no predecessor stores
#endif
constexpr int kTmLanes = 64;            // sources per wave (one wave per workgroup)
constexpr int kBatch = 8;               // independent edges per batch (16 measured slower)
constexpr uint32_t kInf = 0xFFFF;  // uint16 cost matrix: unreachable
constexpr int kMaxCost = 1000;          // MAX_COST :68

// Conflict levels of one env's motion-edge list, then the batched schedule: sched[b]
// holds nslots[b] (a multiple of kBatch) words s | q << 16 (target-local), level by
// level, no-op slots s = q = T (the dummy column). The levels are computed 64 edges at a
// time (below); the counts, offsets and the scatter run on the whole wave. Edges of one
// level are mutually independent, so their order inside the level does not change any
// result.
__global__ __launch_bounds__(64) void cov_tm_schedule_kernel(CovTmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = a.envs[blockIdx.x];
  const int T = a.ntg[b], E = a.n_motion[b], R = a.R, E4 = 4 * a.M;
  const int lane = threadIdx.x;
  int* shared2 = reinterpret_cast<int*>(smem);  // the level count, the slot count
  int* lw = shared2 + 2;                          // [T] last level writing the column
  int* lr = lw + T;                               // [T] last level reading it
  uint32_t* sq = reinterpret_cast<uint32_t*>(lr + T);  // [E] the edges, s | q << 16
  int* level = reinterpret_cast<int*>(sq + E);          // [E]
  int* fill = level + E;                                // [E + 1] per-level counts, then offsets
  int* base = fill + E + 1;                             // [E + 1] the levels' padded offsets
  const int32_t* snd = a.senders + (size_t)b * E4;
  const int32_t* rcv = a.receivers + (size_t)b * E4;
  for (int k = lane; k < T; k += 64) lw[k] = lr[k] = 0;
  for (int k = lane; k <= E; k += 64) fill[k] = 0;
  for (int e = lane; e < E; e += 64) sq[e] = (uint32_t)(snd[e] - R) | ((uint32_t)(rcv[e] - R) << 16);
  __syncthreads();
  // 64 edges at a time, lane i taking edge e0 + i: its level from the columns' state
  // before the window, then raised past every earlier edge of the window it conflicts
  // with, in window order (a broadcast per edge); the window's levels then go into the
  // columns' state with LDS maxima (order-free). The same levels as one serial pass.
  int nlev_w = 0;
  for (int e0 = 0; e0 < E; e0 += 64) {
    const int e = e0 + lane;
    const bool ve = e < E;
    const uint32_t w = ve ? sq[e] : 0xFFFEFFFFu;  // past E: columns no edge has
    const int s = w & 0xFFFF, q = w >> 16;
    int L = ve ? max(max(lw[s], lw[q]), lr[q]) + 1 : 0;
    const int n = min(64, E - e0);
    for (int j = 0; j + 1 < n; ++j) {
      const int sj = __builtin_amdgcn_readlane(s, j), qj = __builtin_amdgcn_readlane(q, j);
      const int Lj = __builtin_amdgcn_readlane(L, j);
      // edge j writes a column this edge reads or writes, or reads the column it writes
      if (lane > j && (qj == s || qj == q || sj == q)) L = max(L, Lj + 1);
    }
    __syncthreads();  // every lane has read the state the window started from
    if (ve) {
      level[e] = L;
      atomicMax(&lw[q], L);
      atomicMax(&lr[s], L);
      atomicMax(&lr[q], L);
      nlev_w = max(nlev_w, L);
    }
    __syncthreads();
  }
  for (int o = 32; o >= 1; o >>= 1) nlev_w = max(nlev_w, __shfl_xor(nlev_w, o));
  if (lane == 0) shared2[0] = nlev_w;
  __syncthreads();
  const int nlev = shared2[0];
  for (int e = lane; e < E; e += 64) atomicAdd(&fill[level[e] - 1], 1);
  __syncthreads();
  if (lane == 0) {
    int off = 0;
    for (int L = 0; L < nlev; ++L) {
      const int n = fill[L];
      fill[L] = base[L] = off;
      off += (n + kBatch - 1) / kBatch * kBatch;
    }
    base[nlev] = off;
    shared2[1] = off;
  }
  __syncthreads();
  const int off = shared2[1];
  uint32_t* out = a.sched + (size_t)b * a.sched_stride;
  for (int e = lane; e < E; e += 64) out[atomicAdd(&fill[level[e] - 1], 1)] = sq[e];
  __syncthreads();
  // each level's padding (past its edges) holds no-ops: words no edge was stored to
  const uint32_t noop = (uint32_t)T | ((uint32_t)T << 16);
  for (int L = lane; L < nlev; L += 64)
    for (int k = fill[L]; k < base[L + 1]; ++k) out[k] = noop;
  if (a.lev_off)  // the levels' slot offsets (cov_time_matrix_mw_kernel)
    for (int L = lane; L <= nlev; L += 64) a.lev_off[(size_t)b * a.lev_stride + L] = base[L];
  if (lane == 0) {
    a.nslots[b] = off;
    a.nlev[b] = nlev;
    a.overflow[b] = 0;
  }
}

// Per-lane scan of its own row after a sweep: any entry still inf, and the largest
// finite entry (the uint8 variant's overflow guard).
template <typename V>
__device__ __forceinline__ void tm_scan(const V* col, int T, int lane, bool valid, bool& any_inf, uint32_t& mx) {
  constexpr uint32_t inf = (V)~(V)0;
  any_inf = false;
  mx = 0;
  if (!valid) return;
  for (int t = 0; t < T; ++t) {
    const uint32_t v = col[t * kTmLanes + lane];
    any_inf = any_inf || v == inf;
    mx = v != inf && v > mx ? v : mx;
  }
}

// Time matrix of one 64-source chunk with entries of type V (uint8_t: inf = 255;
// uint16_t: inf = 0xFFFF). One sweep raises the largest finite entry by at most the
// schedule's level count (a value moves one hop per level), so the uint8 variant runs a
// sweep only while max + nlev < 255 and otherwise flags the env for the uint16 rerun.
template <typename V, bool PASS_B>
__global__ __launch_bounds__(kTmLanes) void cov_time_matrix_kernel(CovTmArgs a, const uint32_t* __restrict__ sched_all) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr uint32_t inf = (V)~(V)0;
  const int b = a.envs[blockIdx.y];
  const int chunk = blockIdx.x;
  const int T = a.ntg[b];
  const int src0 = chunk * kTmLanes;
  if (src0 >= T) return;  // uniform
  const int Tm = a.Tmax;
  const int lane = threadIdx.x;
  const int src = src0 + lane;
  const bool valid = src < T;
  const int kmax = a.horizon > -1 ? a.horizon + 1 : a.kcap;
  const int nlev = a.nlev[b];
  uint8_t* flags = a.flags + ((size_t)b * a.nchunk + chunk) * a.kcap;
  int K = T > 1 ? kmax : 0;
  if (PASS_B) {
    if (a.overflow[b]) return;  // the uint16 pass redoes this env
    // the reference's sweep count: stop after sweep k once no entry of the env changed
    // or none is infinite (the while test), or after horizon+1 sweeps (the break)
    const uint8_t* fenv = a.flags + (size_t)b * a.nchunk * a.kcap;
    const int nch = (T + kTmLanes - 1) / kTmLanes;
    for (int k = 0; k < kmax && K == kmax && T > 1; ++k) {
      int f = 0;
      for (int c = 0; c < nch; ++c) f |= fenv[(size_t)c * a.kcap + k];
      if (!(f & 1) || !(f & 2)) K = k + 1;
    }
    // pass A's output is the state after min(kmax, fixed point) sweeps (a sweep k that
    // changed nothing means the state after k sweeps is final): redo only if K is less
    int kvalid = kmax;
    for (int k = 0; k < kmax; ++k)
      if (!(flags[k] & 1)) {
        kvalid = k;
        break;
      }
    if (T <= 1 || K >= kvalid) return;
  }
  V* col = reinterpret_cast<V*>(smem);  // [T + 1][64], column T = dummy inf
  for (int t = 0; t <= T; ++t) col[t * kTmLanes + lane] = (t == src) ? 0 : (V)inf;
  int16_t* prevT = a.prevT + (size_t)b * Tm * Tm;  // [q][src]
  // raw buffer over the env's [Tm][Tm] predecessors (stride 0: offsets range-checked
  // against Tm * Tm * 2 bytes; dword 3 = gfx9's data format)
  const __amdgpu_buffer_rsrc_t prv = __builtin_amdgcn_make_buffer_rsrc(prevT, 0, Tm * Tm * 2, 0x00020000);
  if (valid)
    for (int q = 0; q < T; ++q) prevT[(size_t)q * Tm + src] = -1;
  const uint32_t* sched = sched_all + (size_t)b * a.sched_stride;
  const int nslots = a.nslots[b];
  uint32_t mx = 0;
  // lanes past T relax too (their rows stay inf, so nothing changes and they never
  // store a predecessor)
  for (int sweep = 0; sweep < K; ++sweep) {
    if (sizeof(V) == 1 && __ballot(mx + (uint32_t)nlev >= inf) != 0) {
      if (lane == 0) a.overflow[b] = 1;
      return;
    }
    int changed = 0;
    uint32_t nxt[kBatch];
#pragma unroll
    for (int k = 0; k < kBatch; ++k) nxt[k] = sched[k];
    for (int j = 0; j < nslots; j += kBatch) {
      uint32_t w[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) w[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)nxt[k]);
#if GF_TM_DIAG & 2
#pragma unroll
      for (int k = 0; k < kBatch; ++k) nxt[k] = sched[((j + kBatch) & 56) + k];
#else
#pragma unroll
      for (int k = 0; k < kBatch; ++k) nxt[k] = sched[j + kBatch + k];  // next batch (slack in the stride)
#endif
      uint32_t vs[kBatch], vq[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {
        vs[k] = col[(w[k] & 0xFFFF) * kTmLanes + lane];
        vq[k] = col[(w[k] >> 16) * kTmLanes + lane];
      }
      bool better[kBatch];
      bool bany = false;
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {
        const uint32_t via = vs[k] + 1u;  // inf + 1 never wins
        better[k] = via < vq[k];
        col[(w[k] >> 16) * kTmLanes + lane] = (V)(via < vq[k] ? via : vq[k]);
        bany = bany || better[k];
      }
      changed |= bany ? 1 : 0;
      // the predecessors, branch-free: a lane that did not improve stores past the end of
      // the buffer's range, which the hardware drops (no exec-mask branch per edge: 8.63 ->
      // 8.05-8.11 ms for 512 maps, profiles/r06/ab_tm_branchfree.txt); a batch no lane of
      // the wave improved skips its 8 stores on one uniform branch (the later sweeps' usual
      // case: 8.29 -> 7.69-7.76 ms, profiles/r06/ab_tm_store_skip.txt; a branch per edge,
      // 8.54-8.58, and 16-edge schedule loads on top, 7.87-7.90, were slower)
      if (__ballot(bany) != 0) {
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
#if !(GF_TM_DIAG & 4)
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(w[k] & 0xFFFF), prv,
                                                better[k] ? (int)(((w[k] >> 16) * (uint32_t)Tm + src) * 2) : (int)0x7FFFFFF0,
                                                0, 0);
#endif
        }
      }
    }
    if (!PASS_B || sizeof(V) == 1) {
      bool any_inf_lane;
      tm_scan(col, T, lane, valid, any_inf_lane, mx);
      if (!PASS_B) {
        const bool any_changed = __ballot(changed) != 0;
        const bool any_inf = __ballot(any_inf_lane) != 0;
        if (lane == 0) flags[sweep] = (any_changed ? 1 : 0) | (any_inf ? 2 : 0);
        if (!any_changed && !(GF_TM_DIAG & 1)) {  // a fixed point: later sweeps change nothing
          for (int k = sweep + 1 + lane; k < a.kcap; k += kTmLanes) flags[k] = any_inf ? 2 : 0;
          break;
        }
      }
    }
  }
  // cost rows, row-major [src][t] as uint16 (inf = 0xFFFF); 4 entries per 8-byte store
  if (valid) {
    auto ent = [&](int t) -> uint64_t {
      const uint32_t v = col[t * kTmLanes + lane];
      return v == inf ? 0xFFFFull : (uint64_t)v;
    };
    uint16_t* row = a.cost + ((size_t)b * Tm + src) * Tm;
    int t = 0;
    if ((Tm & 3) == 0)
      for (; t + 4 <= T; t += 4)
        *reinterpret_cast<uint64_t*>(row + t) = ent(t) | (ent(t + 1) << 16) | (ent(t + 2) << 32) | (ent(t + 3) << 48);
    for (; t < T; ++t) row[t] = (uint16_t)ent(t);
    if (sizeof(V) == 1 && a.cost8) {  // the greedy step's copy: one byte per entry, inf = 255
      uint8_t* row8 = a.cost8 + ((size_t)b * Tm + src) * Tm;
      t = 0;
      if ((Tm & 7) == 0)
        for (; t + 8 <= T; t += 8) {
          uint64_t w = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) w |= (uint64_t)col[(t + k) * kTmLanes + lane] << (8 * k);
          *reinterpret_cast<uint64_t*>(row8 + t) = w;
        }
      for (; t < T; ++t) row8[t] = (uint8_t)col[t * kTmLanes + lane];
    }
  }
}

// The same passes with kTmWaves waves per 64-source chunk, for launches of few chunks
// (the drop-in env's map: one env, ~9 chunks, where one wave per chunk leaves the sweep a
// chain of ~230 dependent batches). The waves split each conflict level's batches (its
// edges are mutually independent: disjoint written columns, none read by another) and
// meet at a barrier between levels; the sweep's flags and the row scan are combined over
// the workgroup. The predecessors are kept in LDS too (the waves' global stores to one
// entry would not be ordered by the barriers) and written out at the end. Same results
// as cov_time_matrix_kernel.
#ifndef GF_TM_WAVES
#define GF_TM_WAVES 8  // 8 per chunk: the drop-in first step 5-7 % below 4 waves (profiles/r06/ab_tm_waves_per_chunk.txt)
#endif
constexpr int kTmWaves = GF_TM_WAVES;
constexpr size_t kTmFewChunks = 256;  // launches of at most this many chunks (one per CU) take it

template <typename V, bool PASS_B>
__global__ __launch_bounds__(kTmLanes * kTmWaves) void cov_time_matrix_mw_kernel(CovTmArgs a, const uint32_t* __restrict__ sched_all) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr uint32_t inf = (V)~(V)0;
  const int b = a.envs[blockIdx.y];
  const int chunk = blockIdx.x;
  const int T = a.ntg[b];
  const int src0 = chunk * kTmLanes;
  if (src0 >= T) return;  // uniform
  const int Tm = a.Tmax;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int src = src0 + lane;
  const bool valid = src < T;
  const int kmax = a.horizon > -1 ? a.horizon + 1 : a.kcap;
  const int nlev = a.nlev[b];
  uint8_t* flags = a.flags + ((size_t)b * a.nchunk + chunk) * a.kcap;
  int K = T > 1 ? kmax : 0;
  if (PASS_B) {
    if (a.overflow[b]) return;
    const uint8_t* fenv = a.flags + (size_t)b * a.nchunk * a.kcap;
    const int nch = (T + kTmLanes - 1) / kTmLanes;
    for (int k = 0; k < kmax && K == kmax && T > 1; ++k) {
      int f = 0;
      for (int c = 0; c < nch; ++c) f |= fenv[(size_t)c * a.kcap + k];
      if (!(f & 1) || !(f & 2)) K = k + 1;
    }
    int kvalid = kmax;
    for (int k = 0; k < kmax; ++k)
      if (!(flags[k] & 1)) {
        kvalid = k;
        break;
      }
    if (T <= 1 || K >= kvalid) return;
  }
  V* col = reinterpret_cast<V*>(smem);  // [T + 1][64], column T = dummy inf
  const size_t col_bytes = ((size_t)(a.t_lds + 1) * kTmLanes * sizeof(V) + 15) & ~(size_t)15;
  int16_t* pl = reinterpret_cast<int16_t*>(smem + col_bytes);  // [T + 1][64] predecessors
  int* loff = reinterpret_cast<int*>(smem + col_bytes + ((((size_t)a.t_lds + 1) * kTmLanes * 2 + 15) & ~(size_t)15));
  for (int t = wv; t <= T; t += kTmWaves) {
    col[t * kTmLanes + lane] = (t == src) ? 0 : (V)inf;
    pl[t * kTmLanes + lane] = -1;
  }
  for (int k = tid; k <= nlev; k += kTmLanes * kTmWaves) loff[k] = a.lev_off[(size_t)b * a.lev_stride + k];
  const uint32_t* sched = sched_all + (size_t)b * a.sched_stride;
  __syncthreads();
  uint32_t mx = 0;  // this wave's share of the lane's row (columns wv, wv + kTmWaves, ...)
  for (int sweep = 0; sweep < K; ++sweep) {
    if (sizeof(V) == 1 && __syncthreads_or(mx + (uint32_t)nlev >= inf)) {
      if (tid == 0) a.overflow[b] = 1;
      return;
    }
    int changed = 0;
    for (int L = 0; L < nlev; ++L) {
      const int s0 = __builtin_amdgcn_readfirstlane(loff[L]), s1 = __builtin_amdgcn_readfirstlane(loff[L + 1]);
      for (int j = s0 + wv * kBatch; j < s1; j += kBatch * kTmWaves) {
        uint32_t w[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) w[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)sched[j + k]);
        uint32_t vs[kBatch], vq[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
          vs[k] = col[(w[k] & 0xFFFF) * kTmLanes + lane];
          vq[k] = col[(w[k] >> 16) * kTmLanes + lane];
        }
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
          const uint32_t via = vs[k] + 1u;
          const bool better = via < vq[k];
          col[(w[k] >> 16) * kTmLanes + lane] = (V)(via < vq[k] ? via : vq[k]);
          changed |= better ? 1 : 0;
          // branch-free: a lane that did not improve writes the dummy column T (the drop-in
          // first step 4-6 % shorter than a branch per edge, profiles/r06/ab_tm_mw_pl_select.txt)
          pl[(better ? (w[k] >> 16) : (uint32_t)T) * kTmLanes + lane] = (int16_t)(w[k] & 0xFFFF);
        }
      }
      __syncthreads();  // the next level reads what this one wrote
    }
    if (!PASS_B || sizeof(V) == 1) {
      bool any_inf_lane = false;
      mx = 0;
      if (valid)
        for (int t = wv; t < T; t += kTmWaves) {
          const uint32_t v = col[t * kTmLanes + lane];
          any_inf_lane = any_inf_lane || v == inf;
          mx = v != inf && v > mx ? v : mx;
        }
      if (!PASS_B) {
        const bool any_changed = __syncthreads_or(changed) != 0;
        const bool any_inf = __syncthreads_or(any_inf_lane) != 0;
        if (tid == 0) flags[sweep] = (any_changed ? 1 : 0) | (any_inf ? 2 : 0);
        if (!any_changed) {
          for (int k = sweep + 1 + tid; k < a.kcap; k += kTmLanes * kTmWaves) flags[k] = any_inf ? 2 : 0;
          break;
        }
      }
    }
  }
  // predecessors [q][src] (consecutive sources per wave: one 128-byte row piece per q)
  // and cost rows, row-major [src][t] as uint16 (inf = 0xFFFF); the waves take groups of
  // 4 (uint8 copy: 8) entries in turn
  if (valid) {
    int16_t* prevT = a.prevT + (size_t)b * Tm * Tm;
    for (int q = wv; q < T; q += kTmWaves) prevT[(size_t)q * Tm + src] = pl[q * kTmLanes + lane];
    auto ent = [&](int t) -> uint64_t {
      const uint32_t v = col[t * kTmLanes + lane];
      return v == inf ? 0xFFFFull : (uint64_t)v;
    };
    uint16_t* row = a.cost + ((size_t)b * Tm + src) * Tm;
    const int t4 = (Tm & 3) == 0 ? (T & ~3) : 0;
    for (int t = 4 * wv; t < t4; t += 4 * kTmWaves)
      *reinterpret_cast<uint64_t*>(row + t) = ent(t) | (ent(t + 1) << 16) | (ent(t + 2) << 32) | (ent(t + 3) << 48);
    for (int t = t4 + wv; t < T; t += kTmWaves) row[t] = (uint16_t)ent(t);
    if (sizeof(V) == 1 && a.cost8) {
      uint8_t* row8 = a.cost8 + ((size_t)b * Tm + src) * Tm;
      const int t8 = (Tm & 7) == 0 ? (T & ~7) : 0;
      for (int t = 8 * wv; t < t8; t += 8 * kTmWaves) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) w |= (uint64_t)col[(t + k) * kTmLanes + lane] << (8 * k);
        *reinterpret_cast<uint64_t*>(row8 + t) = w;
      }
      for (int t = t8 + wv; t < T; t += kTmWaves) row8[t] = (uint8_t)col[t * kTmLanes + lane];
    }
  }
}

// Minimum over aligned groups of L lanes (L = 4, 8, 16): DPP swaps inside rows of 16
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror).
template <int L>
__device__ __forceinline__ uint32_t group_min_u32(uint32_t w) {
  w = min(w, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false));
  w = min(w, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false));
  if (L > 4) w = min(w, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false));
  if (L > 8) w = min(w, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x140, 0xF, 0xF, false));
  return w;
}

// controller(greedy=True) without the random draws: 8 lanes per robot, 8 robots per
// wave, 32 per workgroup. A wave per robot left ~100k waves, each a chain of dependent
// loads, for 512 envs x 200 robots: 47.1 -> 33.4 us per expert step with 16 lanes, 32.4
// with 8.
constexpr int kGreedyLanes = 8;
constexpr int kGreedyRobotsPerBlock = 256 / kGreedyLanes;
constexpr int kGreedyInFlight = 4;  // rounds of 16-byte loads issued together

// uint8 rows are searched four targets per 32-bit operation (SWAR)
// 0/1 bytes -> 0/255 bytes: (f << 8) - f, byte by byte without carries (two full-rate
// operations; a 32-bit multiply by 255 issues at a quarter of the rate)
__device__ __forceinline__ uint32_t ff_bytes(uint32_t f) { return (f << 8) - f; }
// First byte of w equal to v (w must hold one): the zero-byte test on w ^ v..v, whose
// lowest flagged byte is exact (borrows only flag bytes above a zero byte).
__device__ __forceinline__ int first_byte_eq(uint32_t w, uint32_t v) {
  const uint32_t x = w ^ (v * 0x01010101u);
  return __builtin_ctz((x - 0x01010101u) & ~x & 0x80808080u) >> 3;
}

__global__ __launch_bounds__(256) void cov_greedy_kernel(CovGreedyArgs a) {
  const int b = blockIdx.x;
  const int sl = threadIdx.x & (kGreedyLanes - 1);
  const int i = blockIdx.y * kGreedyRobotsPerBlock + (int)(threadIdx.x / kGreedyLanes);
  // robots past R compute on robot 0 and write nothing (every lane takes part in the DPP)
  const bool vr = i < a.R;
  const int ir = vr ? i : 0;
  const int R = a.R, Tm = a.Tmax;
  const int T = a.ntg[b];
  const bool swar = a.cost8 && !a.wide[b];
  int c;
  if (a.dirty[b]) {  // robots were placed externally: closest_targets (:427-432)
    const double* tg = a.tgt + (size_t)b * Tm * 2;
    const double px = a.xr[((size_t)b * R + ir) * 2], py = a.xr[((size_t)b * R + ir) * 2 + 1];
    double best = __builtin_inf();
    int arg = T;
    for (int t = sl; t < T; t += kGreedyLanes) {
      const double dx = px - tg[2 * t], dy = py - tg[2 * t + 1];
      const double d = sqrt(dx * dx + dy * dy);
      if (d < best) {
        best = d;
        arg = t;
      }
    }
    for (int off = kGreedyLanes / 2; off > 0; off >>= 1) {
      const double ob = __shfl_xor(best, off);
      const int oa = __shfl_xor(arg, off);
      if (ob < best || (ob == best && oa < arg)) {
        best = ob;
        arg = oa;
      }
    }
    c = arg;
  } else {
    c = a.cur[(size_t)b * R + ir] - R;
  }
  // r = graph_cost[c, :] with visited targets masked (:817-818) — and, the reference
  // indexing with np.where's (rows, cols) tuple on the (T,1) visited column, target 0
  // as well whenever any target is visited
  const uint8_t* vis = a.visited + (size_t)b * Tm;
  const bool any_vis = a.nvisited[b] > 0;
  uint32_t key = 0xFFFFFFFFu;
  auto consider = [&](uint32_t v, uint32_t visited, int t, uint32_t inf) {
    if (v == inf || visited || (t == 0 && any_vis)) v = kMaxCost;
    const uint32_t kt = (v << 16) | (uint32_t)t;  // min value, then first index (np.argmin)
    key = kt < key ? kt : key;
  };
  if (swar) {
    // One byte per entry; masked (visited, inf = 255, target 0 once anything is visited)
    // entries become 255, above every hop count (<= 254 here), so the argmin of the
    // masked row in bytes is the reference's (min value, then first index). Each lane
    // takes four targets per 32-bit operation: the masked word c | 255 * visited, its
    // smallest byte, and the first word (in t order) holding the lane's minimum; the
    // group's minimum value m and the first index of m follow from those words.
    const uint8_t* row8 = a.cost8 + ((size_t)b * Tm + c) * Tm;
    uint32_t lmin = 0x100u, lword = 0xFFFFFFFFu;
    int lpos = 0;
    auto word = [&](uint32_t m, int tb) {
      const uint32_t dm = min(min(m & 0xFFu, (m >> 8) & 0xFFu), min((m >> 16) & 0xFFu, m >> 24));
      if (dm < lmin) {  // strict: the lane's first word holding its minimum
        lmin = dm;
        lword = m;
        lpos = tb;
      }
    };
    constexpr int kStride = 16 * kGreedyLanes;
    int t0 = 0;
    if ((Tm & 15) == 0) {
      for (; t0 + kGreedyInFlight * kStride <= T; t0 += kGreedyInFlight * kStride) {
        uint4 cv[kGreedyInFlight], fv[kGreedyInFlight];
#pragma unroll
        for (int k = 0; k < kGreedyInFlight; ++k) {
          const int t = t0 + k * kStride + 16 * sl;
          cv[k] = *reinterpret_cast<const uint4*>(row8 + t);
          fv[k] = *reinterpret_cast<const uint4*>(vis + t);
        }
        if (t0 == 0 && sl == 0 && any_vis) fv[0].x |= 1u;  // target 0 (the np.where quirk)
#pragma unroll
        for (int k = 0; k < kGreedyInFlight; ++k) {
          const int t = t0 + k * kStride + 16 * sl;
          word(cv[k].x | ff_bytes(fv[k].x), t);
          word(cv[k].y | ff_bytes(fv[k].y), t + 4);
          word(cv[k].z | ff_bytes(fv[k].z), t + 8);
          word(cv[k].w | ff_bytes(fv[k].w), t + 12);
        }
      }
    }
    for (int t = t0 + sl; t < T; t += kGreedyLanes) {  // the rest, one target per word
      const bool msk = vis[t] || (t == 0 && any_vis);
      word((msk ? 0xFFu : (uint32_t)row8[t]) | 0xFFFFFF00u, t);
    }
    const uint32_t m = group_min_u32<kGreedyLanes>(lmin);
    const uint32_t cand = (lmin == m && m <= 0xFFu) ? (uint32_t)(lpos + first_byte_eq(lword, m)) : 0xFFFFu;
    const uint32_t goal = group_min_u32<kGreedyLanes>(cand);
    key = ((m >= 0xFFu ? (uint32_t)kMaxCost : m) << 16) | goal;
  } else if (a.cost8 && !a.wide[b]) {  // one byte per entry (inf = 255): 16 targets per load
    const uint8_t* row8 = a.cost8 + ((size_t)b * Tm + c) * Tm;
    constexpr int kStride = 16 * kGreedyLanes;
    int t0 = 0;
    if ((Tm & 15) == 0) {
      for (; t0 + kGreedyInFlight * kStride <= T; t0 += kGreedyInFlight * kStride) {
        uint4 cv[kGreedyInFlight], fv[kGreedyInFlight];
#pragma unroll
        for (int k = 0; k < kGreedyInFlight; ++k) {
          const int t = t0 + k * kStride + 16 * sl;
          cv[k] = *reinterpret_cast<const uint4*>(row8 + t);
          fv[k] = *reinterpret_cast<const uint4*>(vis + t);
        }
#pragma unroll
        for (int k = 0; k < kGreedyInFlight; ++k) {
          const int t = t0 + k * kStride + 16 * sl;
          const uint32_t c4[4] = {cv[k].x, cv[k].y, cv[k].z, cv[k].w};
          const uint32_t f4[4] = {fv[k].x, fv[k].y, fv[k].z, fv[k].w};
#pragma unroll
          for (int q = 0; q < 16; ++q)
            consider((c4[q >> 2] >> (8 * (q & 3))) & 0xFF, (f4[q >> 2] >> (8 * (q & 3))) & 0xFF, t + q, 0xFF);
        }
      }
    }
    for (int t = t0 + sl; t < T; t += kGreedyLanes) consider(row8[t], vis[t], t, 0xFF);
  } else {  // two bytes per entry: 8 targets per load
    const uint16_t* row = a.cost + ((size_t)b * Tm + c) * Tm;
    constexpr int kStride = 8 * kGreedyLanes;
    int t0 = 0;
    if ((Tm & 7) == 0) {
      for (; t0 + kGreedyInFlight * kStride <= T; t0 += kGreedyInFlight * kStride) {
        uint4 cv[kGreedyInFlight];
        uint2 fv[kGreedyInFlight];
#pragma unroll
        for (int k = 0; k < kGreedyInFlight; ++k) {
          const int t = t0 + k * kStride + 8 * sl;
          cv[k] = *reinterpret_cast<const uint4*>(row + t);
          fv[k] = *reinterpret_cast<const uint2*>(vis + t);
        }
#pragma unroll
        for (int k = 0; k < kGreedyInFlight; ++k) {
          const int t = t0 + k * kStride + 8 * sl;
          const uint32_t c4[4] = {cv[k].x, cv[k].y, cv[k].z, cv[k].w};
          const uint32_t f2[2] = {fv[k].x, fv[k].y};
#pragma unroll
          for (int q = 0; q < 8; ++q)
            consider((c4[q >> 1] >> (16 * (q & 1))) & 0xFFFF, (f2[q >> 2] >> (8 * (q & 3))) & 0xFF, t + q, kInf);
        }
      }
    }
    for (int t = t0 + sl; t < T; t += kGreedyLanes) consider(row[t], vis[t], t, kInf);
  }
  key = group_min_u32<kGreedyLanes>(key);
  if (sl != 0 || !vr) return;
  const int goal = key & 0xFFFF;
  const int cost = key >> 16;
  int act = 0;
  bool rnd = cost == kMaxCost;  // no unvisited target within the horizon (:821-823)
  if (!rnd) {
    const int p = a.prevT[((size_t)b * Tm + c) * Tm + goal];  // graph_previous[goal, c]
    if (p < 0) {
      rnd = true;  // :863
    } else {
      // index of the next hop among the robot's action targets (:869)
      const int* nb = a.nbr + ((size_t)b * Tm + c) * 4;
      const int n = a.cnt[(size_t)b * Tm + c];
      act = -1;
      for (int k = n - 1; k >= 0; --k)
        if (nb[k] == p) act = k;
      if (act < 0) {  // the reference's np.where(..)[0][0] raises IndexError
        atomicOr(a.err, 8);
        act = 0;
      }
    }
  }
  a.actions[(size_t)b * R + i] = act;
  a.needs_random[(size_t)b * R + i] = rnd ? 1 : 0;
}

}  // namespace

size_t cov_time_matrix_lds_bytes(int t_lds, bool wide) { return (size_t)(t_lds + 1) * kTmLanes * (wide ? 2 : 1); }

size_t cov_tm_schedule_lds_bytes(int t_lds, int e_max) { return (size_t)(2 * t_lds + 4 * e_max + 4) * 4; }

hipError_t launch_cov_tm_schedule(const CovTmArgs& a, int n_envs_sel, int e_max, hipStream_t s) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cov_tm_schedule_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cov_tm_schedule_kernel, dim3(n_envs_sel), dim3(64), cov_tm_schedule_lds_bytes(a.t_lds, e_max), s, a);
  return hipGetLastError();
}

template <typename V>
static hipError_t launch_tm_passes(const CovTmArgs& a, int n_envs_sel, hipStream_t s) {
  const dim3 grid((a.t_lds + kTmLanes - 1) / kTmLanes, n_envs_sel);
  const size_t lds = cov_time_matrix_lds_bytes(a.t_lds, sizeof(V) == 2);
  const size_t lds_mw = ((lds + 15) & ~(size_t)15) + ((((size_t)a.t_lds + 1) * kTmLanes * 2 + 15) & ~(size_t)15) +
                        (size_t)a.lev_stride * sizeof(int32_t);
  // (pass A's block-wide reductions take 256 bytes of static LDS)
  if (a.lev_off && (size_t)grid.x * grid.y <= kTmFewChunks && lds_mw <= 160 * 1024 - 256) {
    // few chunks (the drop-in env): kTmWaves waves per chunk, the levels' offsets in LDS
    for (const void* f : {reinterpret_cast<const void*>(&cov_time_matrix_mw_kernel<V, false>),
                          reinterpret_cast<const void*>(&cov_time_matrix_mw_kernel<V, true>)}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((cov_time_matrix_mw_kernel<V, false>), grid, dim3(kTmLanes * kTmWaves), lds_mw, s, a, a.sched);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((cov_time_matrix_mw_kernel<V, true>), grid, dim3(kTmLanes * kTmWaves), lds_mw, s, a, a.sched);
    return hipGetLastError();
  }
  for (const void* f : {reinterpret_cast<const void*>(&cov_time_matrix_kernel<V, false>),
                        reinterpret_cast<const void*>(&cov_time_matrix_kernel<V, true>)}) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((cov_time_matrix_kernel<V, false>), grid, dim3(kTmLanes), lds, s, a, a.sched);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((cov_time_matrix_kernel<V, true>), grid, dim3(kTmLanes), lds, s, a, a.sched);
  return hipGetLastError();
}

hipError_t launch_cov_time_matrix(const CovTmArgs& a, int n_envs_sel, bool wide, hipStream_t s) {
  return wide ? launch_tm_passes<uint16_t>(a, n_envs_sel, s) : launch_tm_passes<uint8_t>(a, n_envs_sel, s);
}


namespace {

// One wave per source node c of a selected env: its greedy list (coverage_internal.h),
// a counting sort of the row's targets in (hop count, t) order, np.argmin's (min value,
// then first index) order: an entry's slot is the number of listed entries with a
// smaller count plus those with its count and a smaller t. The row's counts and entries
// and the count bins sit in the wave's own LDS region (a wave's LDS operations run in
// order: no barrier); the bin counts are order-free atomics, the offsets a scan of 16
// bins per lane, and each 64-target chunk's lanes of one count find each other with 10
// ballots on its bits. (Round 5 visited the distinct counts one by one, a pass over the
// row per count: ~100 passes on a map's longer rows, 5.7 ms for 512 maps.)
constexpr int kListBins = 1024;  // hop counts 0 .. MAX_COST - 1
// bin v's LDS word: one pad word per 16 bins, so the scan's lane-contiguous runs of 16
// bins sit in distinct banks (lane l's run starts at word 17 l)
__device__ __forceinline__ uint32_t list_bin(uint32_t v) { return v + (v >> 4); }

__global__ __launch_bounds__(256) void cov_greedy_list_kernel(CovTmArgs a) {
  __shared__ uint32_t bins_s[4][kListBins + kListBins / 16];
  __shared__ uint16_t vv_s[4][kGreedyListMaxT], ee_s[4][kGreedyListMaxT];
  const int b = a.envs[blockIdx.x];
  const int c = blockIdx.y * 4 + (int)(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int T = a.ntg[b], Tm = a.Tmax;
  if (c >= T) return;  // wave-uniform
  uint32_t* bins = bins_s[threadIdx.x >> 6];
  uint16_t* vv = vv_s[threadIdx.x >> 6];
  uint16_t* ee = ee_s[threadIdx.x >> 6];
  const size_t row = (size_t)b * Tm + c;
  const uint16_t* cost = a.cost + row * Tm;
  const int16_t* prev = a.prevT + row * Tm;  // graph_previous[t, c] at t
  const int32_t* nb = a.nbr + row * 4;
  const int n = a.cnt[row];
  const int nb0 = nb[0], nb1 = nb[1], nb2 = nb[2], nb3 = nb[3];
  for (int q = lane; q < kListBins + kListBins / 16; q += 64) bins[q] = 0u;
  for (int t = lane; t < T; t += 64) {
    const uint32_t v = cost[t];
    const bool listed = v != kInf && v < (uint32_t)kMaxCost;  // inf -> MAX_COST: never argmin-chosen
    const int p = prev[t];
    uint32_t flag = 0, act = 0;
    if (p < 0) {
      flag = kGreedyRnd;  // :863
    } else {  // the first of the node's action targets equal to the next hop (:869)
      act = (n > 3 && nb3 == p) ? 3u : 4u;
      act = (n > 2 && nb2 == p) ? 2u : act;
      act = (n > 1 && nb1 == p) ? 1u : act;
      act = (n > 0 && nb0 == p) ? 0u : act;
      if (act == 4u) {
        flag = kGreedyErr;
        act = 0;
      }
    }
    vv[t] = listed ? (uint16_t)v : (uint16_t)0xFFFFu;
    ee[t] = (uint16_t)((uint32_t)t | act << 10 | flag << 12);
    if (listed) atomicAdd(&bins[list_bin(v)], 1u);
  }
  constexpr int BPL = kListBins / 64;  // bins per lane
  uint32_t run = 0;
  for (int q = 0; q < BPL; ++q) run += bins[lane * (BPL + 1) + q];
  uint32_t incl = run;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
    if (lane >= d) incl += y;
  }
  const uint32_t len = (uint32_t)__shfl((int)incl, 63, 64);
  uint32_t off = incl - run;
  for (int q = 0; q < BPL; ++q) {
    const uint32_t k = bins[lane * (BPL + 1) + q];
    bins[lane * (BPL + 1) + q] = off;
    off += k;
  }
  uint16_t* out = a.glist + row * a.gstride;
  const uint64_t below_me = (1ull << lane) - 1ull;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    const uint32_t v = t < T ? vv[t] : 0xFFFFu;
    const bool listed = v != 0xFFFFu;
    uint64_t eq = __ballot(listed);
#pragma unroll
    for (int bit = 0; bit < 10; ++bit) {  // hop counts < MAX_COST = 1000 < 2^10
      const bool s = (v >> bit) & 1u;
      const uint64_t m = __ballot(s);
      eq &= s ? m : ~m;
    }
    uint32_t base = 0;
    if (listed) {
      base = bins[list_bin(v)];
      out[base + (uint32_t)__popcll(eq & below_me)] = ee[t];
    }
    // the class's lowest lane advances its offset after every lane of the class read it
    if (listed && (eq & below_me) == 0ull) bins[list_bin(v)] = base + (uint32_t)__popcll(eq);
  }
  if (lane == 0) a.glen[row] = (uint16_t)len;
}

// controller(greedy=True) from the greedy lists: one workgroup per env, one thread per
// robot; the env's visited flags staged in LDS as bits.
__global__ __launch_bounds__(256) void cov_greedy_list_step_kernel(CovGreedyArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* vbits = reinterpret_cast<uint32_t*>(smem);
  const int b = blockIdx.x;
  const int R = a.R, Tm = a.Tmax;
  const int T = a.ntg[b];
  const uint8_t* vis = a.visited + (size_t)b * Tm;
  for (int w = threadIdx.x; w < (Tm + 31) / 32; w += 256) vbits[w] = 0u;
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += 256)
    if (vis[t]) atomicOr(&vbits[t >> 5], 1u << (t & 31));
  __syncthreads();
  const bool any_vis = a.nvisited[b] > 0;
  // few targets left unvisited: the short candidate list instead of deep list scans
  int* ulist = reinterpret_cast<int*>(vbits + (Tm + 31) / 32);
  int* ucount = ulist + kGreedyDirectMax;
  const bool gdirect = T - a.nvisited[b] <= kGreedyDirectMax;
  if (gdirect) {
    greedy_direct_list(vbits, T, any_vis, ulist, ucount);
    __syncthreads();
  }
  const bool dirty = a.dirty[b] != 0;
  for (int i = threadIdx.x; i < R; i += 256) {
    int c;
    if (dirty) {  // robots were placed externally: closest_targets (:427-432)
      const double* tg = a.tgt + (size_t)b * Tm * 2;
      const double px = a.xr[((size_t)b * R + i) * 2], py = a.xr[((size_t)b * R + i) * 2 + 1];
      double best = __builtin_inf();
      c = 0;
      for (int t = 0; t < T; ++t) {
        const double dx = px - tg[2 * t], dy = py - tg[2 * t + 1];
        const double d = sqrt(dx * dx + dy * dy);
        if (d < best) {
          best = d;
          c = t;
        }
      }
    } else {
      c = a.cur[(size_t)b * R + i] - R;
    }
    const size_t row = (size_t)b * Tm + c;
    const int g = gdirect ? greedy_direct(a.cost + row * Tm, a.prevT + row * Tm, a.nbr + row * 4, a.cnt[row], ulist,
                                          *ucount)
                          : greedy_from_list(a.glist + row * a.gstride, a.glen + row, vbits, any_vis, a.nvisited[b] >= T);
    const uint32_t flag = (uint32_t)g >> 2;
    if (flag & kGreedyErr) atomicOr(a.err, 8);
    a.actions[(size_t)b * R + i] = (flag & kGreedyRnd) ? 0 : (g & 3);
    a.needs_random[(size_t)b * R + i] = (flag & kGreedyRnd) ? 1 : 0;
  }
}

}  // namespace

hipError_t launch_cov_greedy_lists(const CovTmArgs& a, int n_envs_sel, hipStream_t s) {
  hipLaunchKernelGGL(cov_greedy_list_kernel, dim3(n_envs_sel, (a.Tmax + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_cov_greedy(const CovGreedyArgs& a, hipStream_t s) {
  if (a.glist) {
    hipLaunchKernelGGL(cov_greedy_list_step_kernel, dim3(a.B), dim3(256),
                       ((a.Tmax + 31) / 32) * 4 + (kGreedyDirectMax + 1) * 4, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(cov_greedy_kernel, dim3(a.B, (a.R + kGreedyRobotsPerBlock - 1) / kGreedyRobotsPerBlock),
                     dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace gf
