// HIP kernels (gfx950) for gym-flock's Coverage-v0 step, batched over B envs.
//
// Reference (gym_flock/envs/spatial/): coverage.py step :174-204, get_action_edges
// :206-232, _get_obs_reward :234-364, closest_targets :427-432, _initialize_graph
// :529-594; utils.py _get_graph_edges :8-24.
//
// One workgroup per env. Node indices are global as in the reference: robots
// 0..R-1, targets R..R+T-1. The padded graph observation (nodes (M,3), edges (4M,1),
// senders/receivers (4M)) lives in HBM and is updated in place: the motion-graph part
// is written once per graph (cov_graph_kernel), each step rewrites the 8R action
// edges at the tail and flips the "unvisited" feature of newly visited nodes, which
// leaves the arrays equal to what the reference rebuilds every step.
#include <limits.h>

#include <cstring>
#include <type_traits>

#include "coverage_internal.h"

namespace gf {

namespace {

constexpr int kCovThreads = 256;

// Phase timeline (diagnostic builds only, -DGF_STAMPS): thread 0 of each workgroup
// records s_memrealtime (100 MHz) at: start (0), first round trip done (1), claims done
// (2), tail writes issued (3), all writes done (4), for scripts/cov_timeline.py.
#ifdef GF_STAMPS
__device__ unsigned long long gf_cov_stamp_buf[4096 * 8];
#define GF_COV_STAMP(k)                                                              \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                       \
      gf_cov_stamp_buf[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define GF_COV_STAMP(k) ((void)0)
#endif

__device__ __forceinline__ double dist2d(double ax, double ay, double bx, double by) {
  const double dx = ax - bx, dy = ay - by;
  return sqrt(dx * dx + dy * dy);  // np.linalg.norm of a 2-vector: sqrt(dx*dx + dy*dy)
}

// Motion graph of one env (utils.py:8-24 with self_loops=True, coverage.py:572-594):
// every ordered target pair with 0 < |p_i - p_j| <= radius, in row-major order, which
// per sender is ascending receiver order (what np.where returns in get_action_edges).
// The radius test of the motion graph, `0 < sqrt(dx*dx + dy*dy) <= r` exactly as dist2d
// rounds it, from the squared distance s: sqrt is correctly rounded and monotonic, so s at
// or below r2lo = r*r*(1 - 2^-50) always passes and s above r2hi = r*r*(1 + 2^-50) never
// does (the margins exceed the roundings of r*r and of the square root by far); only s
// between them takes the square root. 0 < sqrt(s) iff 0 < s; a NaN s fails both ways.
__device__ __forceinline__ bool within_radius(double s, double r, double r2lo, double r2hi) {
  return s > 0.0 && (s <= r2lo || (s <= r2hi && sqrt(s) <= r));
}

// Targets staged in LDS with a cell grid (GRID, when Tmax <= kGraphLdsTargets): cells of
// side h = radius (1 + 2^-20) over the targets' bounding box, so every target within the
// radius of a node lies in the 3 x 3 cells around it (the margin dwarfs the rounding of the
// cell coordinates); a node's in-radius targets are kept as its 4 smallest indices, the
// row-major scan order of the reference. Without the grid (too many cells, a non-finite
// coordinate, or GRID off) every node scans every target.
constexpr int kGraphLdsTargets = 4096;
constexpr int kGraphCells = 4096;

template <bool GRID>
__global__ __launch_bounds__(kCovThreads) void cov_graph_kernel(CovArgs a, const int32_t* envs, int n_envs_sel) {
  __shared__ int scan[kCovThreads];
  __shared__ int total_s;
  __shared__ double bb_s[kCovThreads / 64][4];
  __shared__ int grid_s[3];  // Gx, Gy (0: scan), cell count
  __shared__ double org_s[2];
  extern __shared__ __attribute__((aligned(16))) double2 tgs[];  // GRID: (Tm) targets, (cells + 1) runs, (Tm) by cell
  const int e = blockIdx.x;
  if (e >= n_envs_sel) return;
  const int b = envs ? envs[e] : e;
  const int R = a.R, M = a.M, Tm = a.Tmax, E = 4 * M;
  const int T = a.ntg[b];
  const double* tg = a.tgt + (size_t)b * Tm * 2;
  int32_t* nbr = a.nbr + (size_t)b * Tm * 4;
  int32_t* cnt = a.cnt + (size_t)b * Tm;
  const int tid = threadIdx.x;
  const double r = a.motion_radius, rr = r * r;
  const double r2lo = rr * (1.0 - 0x1p-50), r2hi = rr * (1.0 + 0x1p-50);
  const double2* tg2 = reinterpret_cast<const double2*>(tg);
  auto test = [&](double px, double py, double2 q) {
    const double dx = px - q.x, dy = py - q.y;
    return within_radius(dx * dx + dy * dy, r, r2lo, r2hi);
  };
  // 1. neighbour lists (<= 4 per node; more is the reference's "Increase MAX_EDGES")
  int Gx = 0, Gy = 0;
  int* cend = reinterpret_cast<int*>(tgs + Tm);  // (cells) end of each cell's run
  int* sidx = cend + kGraphCells;                 // (T) target indices in cell order
  double ox = 0.0, oy = 0.0;
  const double h = r * (1.0 + 0x1p-20);
  if (GRID) {
    double lo_x = __builtin_inf(), lo_y = __builtin_inf(), hi_x = -__builtin_inf(), hi_y = -__builtin_inf();
    bool finite = true;
    for (int j = tid; j < T; j += kCovThreads) {
      const double2 q = tg2[j];
      tgs[j] = q;
      finite = finite && isfinite(q.x) && isfinite(q.y);
      lo_x = fmin(lo_x, q.x), lo_y = fmin(lo_y, q.y), hi_x = fmax(hi_x, q.x), hi_y = fmax(hi_y, q.y);
    }
    if (!finite) lo_x = __builtin_nan("");  // poisons the box: scan
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const double o0 = __shfl_xor(lo_x, d, 64), o1 = __shfl_xor(lo_y, d, 64);
      const double o2 = __shfl_xor(hi_x, d, 64), o3 = __shfl_xor(hi_y, d, 64);
      lo_x = (isnan(o0) || isnan(lo_x)) ? __builtin_nan("") : fmin(lo_x, o0);
      lo_y = fmin(lo_y, o1), hi_x = fmax(hi_x, o2), hi_y = fmax(hi_y, o3);
    }
    if ((tid & 63) == 0) {
      bb_s[tid >> 6][0] = lo_x, bb_s[tid >> 6][1] = lo_y, bb_s[tid >> 6][2] = hi_x, bb_s[tid >> 6][3] = hi_y;
    }
    __syncthreads();
    if (tid == 0) {
      double x0 = bb_s[0][0], y0 = bb_s[0][1], x1 = bb_s[0][2], y1 = bb_s[0][3];
      bool nan = isnan(x0);
      for (int w = 1; w < kCovThreads / 64; ++w) {
        nan = nan || isnan(bb_s[w][0]);
        x0 = fmin(x0, bb_s[w][0]), y0 = fmin(y0, bb_s[w][1]), x1 = fmax(x1, bb_s[w][2]), y1 = fmax(y1, bb_s[w][3]);
      }
      const double fx = (x1 - x0) / h + 1.0, fy = (y1 - y0) / h + 1.0;
      int gx = 0, gy = 0;
      if (!nan && T > 0 && fx < (double)kGraphCells && fy < (double)kGraphCells && fx * fy < (double)kGraphCells) {
        gx = (int)fx, gy = (int)fy;
      }
      grid_s[0] = gx, grid_s[1] = gy;
      org_s[0] = x0, org_s[1] = y0;
    }
    __syncthreads();
    Gx = grid_s[0], Gy = grid_s[1];
    ox = org_s[0], oy = org_s[1];
  }
  // a target's cell: (x - ox) / h >= 0 for every target of the box
  auto cellx = [&](double v) { return min((int)((v - ox) / h), Gx - 1); };
  auto celly = [&](double v) { return min((int)((v - oy) / h), Gy - 1); };
  if (GRID && Gx > 0) {
    const int nc = Gx * Gy;
    for (int c = tid; c < nc; c += kCovThreads) cend[c] = 0;
    __syncthreads();
    for (int j = tid; j < T; j += kCovThreads) atomicAdd(&cend[cellx(tgs[j].x) * Gy + celly(tgs[j].y)], 1);
    __syncthreads();
    if (tid == 0) {  // cell starts (a few thousand cells at most)
      int run = 0;
      for (int c = 0; c < nc; ++c) {
        const int n = cend[c];
        cend[c] = run;
        run += n;
      }
    }
    __syncthreads();
    for (int j = tid; j < T; j += kCovThreads) sidx[atomicAdd(&cend[cellx(tgs[j].x) * Gy + celly(tgs[j].y)], 1)] = j;
    __syncthreads();  // cend[c] is now the end of cell c's run (the start of c + 1)
  }
  for (int i = tid; i < T; i += kCovThreads) {
    const double px = tg[2 * i], py = tg[2 * i + 1];
    int c = 0;
    if (GRID && Gx > 0) {
      // the in-radius targets of the 3 x 3 cells, the 4 smallest indices kept in order
      int n0 = INT_MAX, n1 = INT_MAX, n2 = INT_MAX, n3 = INT_MAX;
      const int ci = cellx(px), cj = celly(py);
      for (int gi = max(ci - 1, 0); gi <= min(ci + 1, Gx - 1); ++gi)
        for (int gj = max(cj - 1, 0); gj <= min(cj + 1, Gy - 1); ++gj) {
          const int cc = gi * Gy + gj, k1 = cend[cc];
          for (int k = cc > 0 ? cend[cc - 1] : 0; k < k1; ++k) {
            const int j = sidx[k];
            if (!test(px, py, tgs[j])) continue;
            ++c;
            int x = j, t;
            t = min(n0, x), x = max(n0, x), n0 = t;
            t = min(n1, x), x = max(n1, x), n1 = t;
            t = min(n2, x), x = max(n2, x), n2 = t;
            n3 = min(n3, x);
          }
        }
      nbr[4 * i] = n0;
      nbr[4 * i + 1] = n1;
      nbr[4 * i + 2] = n2;
      nbr[4 * i + 3] = n3;
    } else {
      for (int j = 0; j < T; ++j) {
        if (test(px, py, GRID ? tgs[j] : tg2[j])) {
          if (c < 4) nbr[4 * i + c] = j;
          ++c;
        }
      }
    }
    if (c > 4) atomicOr(a.err, 1);
    for (int k = c; k < 4; ++k) nbr[4 * i + k] = -1;
    cnt[i] = c > 4 ? 4 : c;
  }
  __syncthreads();
  // 2. exclusive scan of the degrees -> position of each node's edges in the list
  const int per = (T + kCovThreads - 1) / kCovThreads;
  const int i0 = tid * per, i1 = min(T, i0 + per);
  int local = 0;
  for (int i = i0; i < i1; ++i) local += cnt[i];
  scan[tid] = local;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int k = 0; k < kCovThreads; ++k) {
      const int v = scan[k];
      scan[k] = run;
      run += v;
    }
    total_s = run;
  }
  __syncthreads();
  const int n_motion = total_s;
  if (n_motion + 8 * R > E) atomicOr(a.err, 2);
  int32_t* snd = a.senders + (size_t)b * E;
  int32_t* rcv = a.receivers + (size_t)b * E;
  float* edg = a.edges + (size_t)b * E;
  // 3. static observation: motion edges, then -1 / 0 padding
  int off = scan[tid];
  for (int i = i0; i < i1; ++i) {
    for (int k = 0; k < cnt[i]; ++k) {
      const int j = nbr[4 * i + k];
      snd[off] = i + R;
      rcv[off] = j + R;
      edg[off] = static_cast<float>(dist2d(tg[2 * i], tg[2 * i + 1], tg[2 * j], tg[2 * j + 1]));
      ++off;
    }
  }
  for (int k = n_motion + tid; k < E; k += kCovThreads) {
    snd[k] = -1;
    rcv[k] = -1;
    edg[k] = 0.0f;
  }
  float* nodes = a.nodes + (size_t)b * M * 3;
  for (int k = tid; k < M; k += kCovThreads) {
    nodes[3 * k] = k < R ? 1.0f : 0.0f;
    nodes[3 * k + 1] = (k >= R && k < R + T) ? 1.0f : 0.0f;
    nodes[3 * k + 2] = 0.0f;
  }
  // coordinates of every node's 4 action targets (padding = the node itself), so a
  // step reads a moved robot's new action edges in one round trip
  double2* axy = reinterpret_cast<double2*>(a.axy) + (size_t)b * Tm * 4;
  for (int k = tid; k < 4 * T; k += kCovThreads) {
    const int t = k >> 2, ac = k & 3;
    const int q = ac < cnt[t] ? nbr[4 * t + ac] : t;
    axy[k] = make_double2(tg[2 * q], tg[2 * q + 1]);
  }
  // per node, the record a robot moving onto it needs (one 64-byte line): its 4 action
  // targets, the 4 action-edge features from its position (get_action_edges :206-232 with
  // the robot on the node, exactly as the step's full pass computes them) and the position
  float4* rec = reinterpret_cast<float4*>(a.nrec) + (size_t)b * Tm * 4;
  for (int t = tid; t < T; t += kCovThreads) {
    const int c = cnt[t], n = t + R;
    const double px = tg[2 * t], py = tg[2 * t + 1];
    int q[4];
    float d[4];
    for (int k = 0; k < 4; ++k) {
      const int j = k < c ? nbr[4 * t + k] : t;
      q[k] = k < c ? j + R : n;
      d[k] = static_cast<float>(dist2d(px, py, tg[2 * j], tg[2 * j + 1]) / a.res);
    }
    const double2 xy = make_double2(px, py);
    rec[4 * t] = make_float4(__int_as_float(q[0]), __int_as_float(q[1]), __int_as_float(q[2]), __int_as_float(q[3]));
    rec[4 * t + 1] = make_float4(d[0], d[1], d[2], d[3]);
    rec[4 * t + 2] = *reinterpret_cast<const float4*>(&xy);
    rec[4 * t + 3] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (tid == 0) {
    a.n_motion[b] = n_motion;
    a.dirty[b] = 1;  // a new graph: the next pass recomputes nodes and action edges
  }
}

// Action targets of a robot on node c (global): its out-neighbours, padded with c.
__device__ __forceinline__ int action_node(const int32_t* nbr, const int32_t* cnt, int c, int act, int R) {
  const int t = c - R;
  return act < cnt[t] ? nbr[4 * t + act] + R : c;
}

// One step (or, with a.actions == nullptr, the observation that reset() returns).
//
// Two dependent global round trips per env. (1) Each robot's node, action, and the 4
// action targets its node offers: the observation tail written by the previous pass
// already lists them (coverage.py:206-232), so the chosen node needs no neighbour
// lookup. (2) After the LDS-only claim resolution, each robot that moved reads its new
// node's position, visited flag, neighbours and their coordinates (cov_graph_kernel's
// table) together, and rewrites its 8 tail edges; a robot that stayed keeps its edges.
// After an external placement, a new graph or a reset, everything is recomputed.
// UIN (cov_step_host): the env batch's actions arrive in the kernel arguments (CovArgsU)
// instead of being read from memory, one dependent round trip fewer.
// One step of env a.env0 + blockIdx.x (the kernels below): MULTI also records the step's
// reward and done flag at [it][b] of reward_k / done_k.
template <int NT, bool MULTI>
__device__ __forceinline__ void cov_step_body(const CovArgs& a, [[maybe_unused]] int it,
                                              [[maybe_unused]] double* reward_k, [[maybe_unused]] uint8_t* done_k) {
  constexpr int RPT = kCovThreads / NT;  // robots per thread when R <= kCovThreads
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = a.env0 + blockIdx.x;
  const int R = a.R, M = a.M, Tm = a.Tmax, E = 4 * M;
  const int T = a.ntg[b];
  int* cur_s = reinterpret_cast<int*>(smem);          // R: node before the move
  int* new_s = cur_s + R;                             // R: node after the move
  int* chosen = new_s + R;                            // R: node the action points at
  unsigned* claim = reinterpret_cast<unsigned*>(chosen + R);  // (M+31)/32 claim bits
  unsigned* seen = claim + (M + 31) / 32;                      // visited-this-step bits
  int* counter = reinterpret_cast<int*>(seen + (M + 31) / 32);
  int* first = counter + 4;                                    // M: first claimer of each node
  uint32_t* gvis = reinterpret_cast<uint32_t*>(first + M);     // greedy: visited bits, 64 per 2 words
  int* ulist = reinterpret_cast<int*>(gvis + ((a.Tmax + 63) / 64) * 2);  // greedy_direct candidates
  int* ucount = ulist + kGreedyDirectMax;
  const int W = (M + 31) / 32;
  const int tid = threadIdx.x;
  const double* tg = a.tgt + (size_t)b * Tm * 2;
  const int32_t* nbr = a.nbr + (size_t)b * Tm * 4;
  const int32_t* cnt = a.cnt + (size_t)b * Tm;
  const double2* axy = reinterpret_cast<const double2*>(a.axy) + (size_t)b * Tm * 4;
  double* xr = a.xr + (size_t)b * R * 2;
  int32_t* cur = a.cur + (size_t)b * R;
  uint8_t* vis = a.visited + (size_t)b * Tm;
  int32_t* snd = a.senders + (size_t)b * E;
  int32_t* rcv = a.receivers + (size_t)b * E;
  float* edg = a.edges + (size_t)b * E;
  const int base = E - 8 * R;  // action edges: [base, base+4R) target->robot, then robot->target

  for (int k = tid; k < W; k += NT) {
    claim[k] = 0u;
    seen[k] = 0u;
  }
  if (a.actions || a.glist)
    for (int k = tid; k < M; k += NT) first[k] = INT_MAX;
  if (tid == 0) {
    counter[0] = 0;  // targets newly visited
    counter[1] = 0;  // COV_GREEDY_RNG: fallback robots
  }
  GF_COV_STAMP(0);
  const int32_t* act = a.actions ? a.actions + (size_t)b * R : nullptr;
  // COV_ACTIONS_GREEDY: controller(greedy=True) picks each robot's action in this launch
  const bool greedy = a.glist != nullptr && !a.next_greedy;
  const bool has_act = act || greedy;
  // One robot per thread (R <= NT): the data of the node a robot will end on
  // (if it moves: the chosen node; in a full pass: its node) is loaded right after the
  // chosen node is known, so that round trip runs under the claim resolution.
  const bool one = R <= kCovThreads;
  const float4* rec = reinterpret_cast<const float4*>(a.nrec) + (size_t)b * Tm * 4;
  // per robot slot: the chosen node's record (n = -1: none)
  struct Pf {
    int n;
    float4 r0, r1, r2;
    uint8_t was;
  };
  Pf pf[RPT];
  // a robot that stays in a full pass keeps its own position (xr, which after an external
  // placement need not be its node's): its edges come from the coordinate table
  auto load_node = [&](int t, uint8_t& was, int4& q4, int& nc, double2& c0, double2& c1, double2& c2,
                       double2& c3) {
    was = vis[t];
    q4 = *reinterpret_cast<const int4*>(nbr + 4 * t);
    nc = cnt[t];
    c0 = axy[4 * t];
    c1 = axy[4 * t + 1];
    c2 = axy[4 * t + 2];
    c3 = axy[4 * t + 3];
  };
  // robot i's loads: the node, the action and the 4 action targets offered at the node, i.e.
  // the tail of the last observation, read whether or not the env is dirty so that it is
  // not a dependent load
  struct Ld {
    int c, ai;
    int4 offer;
  };
  auto load = [&](int i) {
    Ld l;
    l.c = cur[i];
    l.ai = act ? act[i] : 0;
    l.offer = has_act ? *reinterpret_cast<const int4*>(snd + base + 4 * i) : make_int4(0, 0, 0, 0);
    return l;
  };
  Ld ld[RPT];  // R <= kCovThreads: every slot's loads issued first, before the env's words
  if (one) {
#pragma unroll
    for (int j = 0; j < RPT; ++j)
      if (tid + j * NT < R) ld[j] = load(tid + j * NT);
  }
  // the env's words, loaded up front so none of them costs a round trip of its own
  // COV_GREEDY_RNG: the env's MT19937 key, loaded now with the robots' loads (its words
  // are only written by this workgroup, below) so the fallback draws after the picks do
  // not wait for a global round trip of their own
  constexpr int kKeyPer = (kMtN + NT - 1) / NT;
  uint32_t kpre[kKeyPer];
  const bool rng_pre = a.glist != nullptr && !a.next_greedy && a.mt_key != nullptr;
  if (rng_pre) {
#pragma unroll
    for (int j = 0; j < kKeyPer; ++j) {
      const int k = tid + j * NT;
      kpre[j] = k < kMtN ? a.mt_key[(size_t)b * kMtN + k] : 0u;
    }
  }
  const bool dirty = a.dirty[b] != 0;
  const int nv0 = a.nvisited[b], sc0 = a.step_counter[b];
  const bool full = dirty || !has_act;  // recompute every robot's action edges
  const bool any_vis = nv0 > 0;
  if (greedy || a.next_greedy) {
    // the env's visited flags as bits, before this step marks any (ballots, no atomics),
    // read after the robots' loads are in flight
    const int lane = tid & 63, wv = tid >> 6;
    for (int t0 = wv * 64; t0 < Tm; t0 += NT) {
      const int t = t0 + lane;
      const uint64_t m = __ballot(t < T && vis[t]);
      if (lane == 0) {
        gvis[t0 >> 5] = static_cast<uint32_t>(m);
        gvis[(t0 >> 5) + 1] = static_cast<uint32_t>(m >> 32);
      }
    }
    if (rng_pre) {  // the prefetched key into its LDS words (read by the draws below)
      uint32_t* kb = reinterpret_cast<uint32_t*>(ulist + kGreedyDirectMax + 1);
#pragma unroll
      for (int j = 0; j < kKeyPer; ++j)
        if (tid + j * NT < kMtN) kb[tid + j * NT] = kpre[j];
    }
    __syncthreads();
  }
  // few targets left unvisited: the greedy actions from the short candidate list
  const bool gdirect = greedy && T - nv0 <= kGreedyDirectMax;
  if (gdirect) {
    greedy_direct_list(gvis, T, any_vis, ulist, ucount);
    __syncthreads();
  }
  // the node action ai of a robot on c points at (:184-200)
  auto aim = [&](int c, int ai, const int4& offer) {
    return dirty ? action_node(nbr, cnt, c, ai, R)
                 : (ai == 0 ? offer.x : ai == 1 ? offer.y : ai == 2 ? offer.z : offer.w);
  };
  auto prefetch = [&](Pf& p, int n) {
    const int t = n - R;
    p.n = n;
    p.r0 = rec[4 * t];
    p.r1 = rec[4 * t + 1];
    p.r2 = rec[4 * t + 2];
    p.was = vis[t];
  };
  // robot i: its node c and the node n its action points at (claiming c if n == c)
  auto pick = [&](int i, const Ld& l, int& c) {
    c = l.c;
    int ai = l.ai;
    const int4 offer = l.offer;
    if (dirty) {
      // closest_targets (:427-432): the robots were placed externally
      const double px = xr[2 * i], py = xr[2 * i + 1];
      double best = __builtin_inf();
      c = 0;
      for (int j = 0; j < T; ++j) {
        const double d = dist2d(px, py, tg[2 * j], tg[2 * j + 1]);
        if (d < best) {  // strict: first index on ties, like np.argmin
          best = d;
          c = j;
        }
      }
      c += R;
    }
    cur_s[i] = c;
    int n = c;
    if (greedy) {  // :814-869 from the node's greedy list; fallbacks: action 0 or drawn below
      const size_t row = (size_t)b * Tm + (c - R);
      const int g = gdirect ? greedy_direct(a.gcost + row * Tm, a.gprev + row * Tm, nbr + 4 * (c - R), cnt[c - R],
                                            ulist, *ucount)
                            : greedy_from_list(a.glist + row * a.gstride, a.glen + row, gvis, any_vis, nv0 >= T);
      const uint32_t flag = static_cast<uint32_t>(g) >> 2;
      if (flag & kGreedyErr) atomicOr(a.err, 8);
      const bool rnd = flag & kGreedyRnd;
      ai = rnd ? 0 : (g & 3);
      a.needs_random[(size_t)b * R + i] = rnd ? 1 : 0;
      if (rnd && a.mt_key) {  // COV_GREEDY_RNG: drawn in robot order after every pick
        chosen[i] = -1;
        atomicAdd(counter + 1, 1);
        return c;
      }
      a.gactions[(size_t)b * R + i] = ai;
    }
    if (has_act) {
      // step (:184-200): the node the action points at; robots that stay claim first
      if (ai < 0 || ai >= 4) {
        atomicOr(a.err, 4);
        ai = 0;
      }
      n = aim(c, ai, offer);
      chosen[i] = n;
      if (n == c) atomicOr(&claim[n >> 5], 1u << (n & 31));
    }
    return n;
  };
  if (one) {
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      pf[j].n = -1;
      const int i = tid + j * NT;
      if (i < R) {
        int c;
        const int n = pick(i, ld[j], c);
        if (n != c) pf[j].n = n;
      }
    }
    // then every slot's record: no wait for one slot's record before the next slot
#pragma unroll
    for (int j = 0; j < RPT; ++j)
      if (pf[j].n >= 0) prefetch(pf[j], pf[j].n);
  } else {
    for (int i = tid; i < R; i += NT) {
      int c;
      pick(i, load(i), c);
    }
  }
  __syncthreads();
  GF_COV_STAMP(1);

  if (greedy && a.mt_key && counter[1] > 0) {
    // COV_GREEDY_RNG: u_ind[i] = np_random.choice(4) for each fallback robot in robot
    // order (:861-864): the k-th fallback robot takes output pos + k of its env's stream.
    // The key goes through LDS; when pos + k passes 624 the key is regenerated in LDS
    // (the earlier words read first) and written back. R <= 624 (checked by the host):
    // at most one regeneration per step.
    uint32_t* kb = reinterpret_cast<uint32_t*>(ucount + 1);
    uint32_t* pm = kb + kMtN;  // fallback robots as bits, 32 per word
    uint32_t* key = a.mt_key + (size_t)b * kMtN;
    const int nfall = counter[1];
    const int pos = a.mt_pos[b];
    {
      const int lane = tid & 63, wv = tid >> 6;
      for (int k0 = wv * 64; k0 < R; k0 += NT) {
        const uint64_t m = __ballot(k0 + lane < R && chosen[k0 + lane] < 0);
        if (lane == 0) {
          pm[k0 >> 5] = static_cast<uint32_t>(m);
          pm[(k0 >> 5) + 1] = static_cast<uint32_t>(m >> 32);
        }
      }
    }
    __syncthreads();
    auto word = [&](int i) {  // the stream index of robot i's draw
      int r = __popc(pm[i >> 5] & ((1u << (i & 31)) - 1u));
      for (int w = 0; w < (i >> 5); ++w) r += __popc(pm[w]);
      return pos + r;
    };
    // the raw words parked in new_s, which the claim resolution below writes first
    for (int i = tid; i < R; i += NT)
      if (chosen[i] < 0 && word(i) < kMtN) new_s[i] = static_cast<int>(kb[word(i)]);
    if (pos + nfall > kMtN) {
      mt_regen<NT>(kb);  // its first barrier orders the reads above before its writes
      for (int i = tid; i < R; i += NT)
        if (chosen[i] < 0 && word(i) >= kMtN) new_s[i] = static_cast<int>(kb[word(i) - kMtN]);
      for (int k = tid; k < kMtN; k += NT) key[k] = kb[k];
    }
    if (tid == 0) a.mt_pos[b] = pos + nfall > kMtN ? pos + nfall - kMtN : pos + nfall;
    auto draw = [&](int i, const int4& offer, Pf* p) {
      const int c = cur_s[i];
      const int ai = static_cast<int>(mt_temper(static_cast<uint32_t>(new_s[i])) & 3u);
      a.gactions[(size_t)b * R + i] = ai;
      const int n = aim(c, ai, offer);
      chosen[i] = n;
      if (n == c) atomicOr(&claim[n >> 5], 1u << (n & 31));
      else if (p) prefetch(*p, n);
    };
    if (one) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int i = tid + j * NT;
        if (i < R && chosen[i] < 0) draw(i, ld[j].offer, &pf[j]);
      }
    } else {
      for (int i = tid; i < R; i += NT)
        if (chosen[i] < 0) draw(i, load(i).offer, nullptr);
    }
    __syncthreads();
  }

  if (has_act) {
    // then, in robot order, a move succeeds unless its node is already claimed; a
    // blocked robot stays and its node joins the claims. The reference walks the robots
    // serially; here every robot's outcome is re-evaluated in parallel from the current
    // guesses (the first claimer of each node by atomicMin) until nothing changes. A
    // robot's outcome depends only on lower-indexed robots, so after k rounds robots
    // 0..k-1 are final, and the fixed point is the serial walk's unique result.
    if (R <= 4 * 64) {
      // One wave, up to 4 robots per lane kept in registers; only first[] is in LDS.
      // A wave's LDS operations complete in order, so a round needs no workgroup
      // barrier, only waits for its own LDS operations.
      if (tid < 64) {
        // a wave's LDS instructions execute in issue order, so only the compiler must
        // keep them in order (the reads' results are waited for as used; a fence would
        // also wait for the node prefetch still in flight from global memory)
        auto lds_fence = [] { asm volatile("" ::: "memory"); };
        // four named robots, not an array: an array indexed in a loop stays in scratch
        struct Rb {
          int i, c, n, v;
          bool mv, fr;
        };
        auto init = [&](Rb& r, int i) {
          r.i = i;
          const bool valid = i < R;
          r.c = valid ? cur_s[i] : 0;
          r.n = valid ? chosen[i] : 0;
          r.mv = valid && r.n != r.c;
          r.fr = r.mv && !(claim[r.n >> 5] & (1u << (r.n & 31)));  // not a stayer's node
          r.v = r.n;  // guess: every move succeeds
        };
        // branch-free rounds: a robot that does not move adds INT_MAX (no-op).
        // A mover's claim sits on its chosen node or its own; both are cleared between
        // rounds (a non-mover's own node: no mover's test reads it, since movers onto it
        // are blocked by its stay claim; robots past R sit on node 0, a slot no target uses)
        auto put = [&](const Rb& r) { atomicMin(&first[r.v], r.mv ? r.i : INT_MAX); };
        auto clear = [&](const Rb& r) {
          first[r.n] = INT_MAX;
          first[r.c] = INT_MAX;
        };
        auto eval = [&](Rb& r, int f) {
          const int v = (r.fr && f >= r.i) ? r.n : r.c;  // r.fr implies r.mv
          const bool ch = v != r.v;
          r.v = v;
          return ch;
        };
        Rb r0, r1, r2, r3;
        init(r0, tid);
        init(r1, tid + 64);
        init(r2, tid + 128);
        init(r3, tid + 192);
        while (true) {
          put(r0), put(r1), put(r2), put(r3);
          lds_fence();
          const int f0 = first[r0.n], f1 = first[r1.n], f2 = first[r2.n], f3 = first[r3.n];
          // all four evaluated (no short circuit)
          const int changed = int(eval(r0, f0)) | int(eval(r1, f1)) | int(eval(r2, f2)) | int(eval(r3, f3));
          if (!__any(changed)) break;
          lds_fence();
          clear(r0), clear(r1), clear(r2), clear(r3);
          lds_fence();
        }
        if (r0.i < R) new_s[r0.i] = r0.v;
        if (r1.i < R) new_s[r1.i] = r1.v;
        if (r2.i < R) new_s[r2.i] = r2.v;
        if (r3.i < R) new_s[r3.i] = r3.v;
      }
      __syncthreads();
      GF_COV_STAMP(2);
    } else {
      for (int i = tid; i < R; i += NT) new_s[i] = chosen[i];  // guess: every move succeeds
      while (true) {
        __syncthreads();
        for (int i = tid; i < R; i += NT)
          if (chosen[i] != cur_s[i]) atomicMin(&first[new_s[i]], i);
        __syncthreads();
        int changed = 0;
        for (int i = tid; i < R; i += NT) {
          const int c = cur_s[i], n = chosen[i];
          if (n == c) continue;
          const bool ok = !(claim[n >> 5] & (1u << (n & 31))) && first[n] >= i;
          const int v = ok ? n : c;
          if (v != new_s[i]) {
            new_s[i] = v;
            changed = 1;
          }
        }
        if (!__syncthreads_or(changed)) break;
        for (int i = tid; i < R; i += NT)
          if (chosen[i] != cur_s[i]) {
            first[chosen[i]] = INT_MAX;
            first[cur_s[i]] = INT_MAX;
          }
      }
    }
  } else {
    for (int i = tid; i < R; i += NT) new_s[i] = cur_s[i];
    __syncthreads();
  }

  // move (:198), visit (:265-266, :359) and the observation tail (:259-323)
  float* nodes = a.nodes + (size_t)b * M * 3;
  auto finish = [&](int i, const Pf* p) {
    const int n = new_s[i];
    const int t = n - R;
    const bool moved = n != cur_s[i];
    if (!moved && !full) return;  // same node, same position: its edges stand
    cur[i] = n;
    uint8_t was;
    int4 q;
    float4 d;
    if (moved) {  // on its node's position: the node's record holds its edges
      float4 r0, r1, r2;
      if (p && n == p->n) {
        r0 = p->r0, r1 = p->r1, r2 = p->r2, was = p->was;
      } else {  // R > kCovThreads
        r0 = rec[4 * t], r1 = rec[4 * t + 1], r2 = rec[4 * t + 2], was = vis[t];
      }
      q = make_int4(__float_as_int(r0.x), __float_as_int(r0.y), __float_as_int(r0.z), __float_as_int(r0.w));
      d = r1;
      *reinterpret_cast<float4*>(xr + 2 * i) = r2;
    } else {  // a robot that does not move keeps its position (:198)
      int4 q4;
      int nc;
      double2 c0, c1, c2, c3;
      load_node(t, was, q4, nc, c0, c1, c2, c3);
      const double px = xr[2 * i], py = xr[2 * i + 1];
      q = make_int4(0 < nc ? q4.x + R : n, 1 < nc ? q4.y + R : n, 2 < nc ? q4.z + R : n, 3 < nc ? q4.w + R : n);
      d = make_float4(static_cast<float>(dist2d(px, py, c0.x, c0.y) / a.res),
                      static_cast<float>(dist2d(px, py, c1.x, c1.y) / a.res),
                      static_cast<float>(dist2d(px, py, c2.x, c2.y) / a.res),
                      static_cast<float>(dist2d(px, py, c3.x, c3.y) / a.res));
    }
    if (!was) {
      const unsigned old = atomicOr(&seen[n >> 5], 1u << (n & 31));
      if (!(old & (1u << (n & 31)))) {
        vis[t] = 1;
        nodes[3 * n + 2] = 0.0f;
        atomicAdd(counter, 1);
      }
    }
    // the robot's 4 action edges in both directions: six 16-byte stores (base and 4i are
    // multiples of 4 elements, so every group is 16-byte aligned)
    // (the robot's own index never changes: written by full passes only, so a step leaves
    // fewer dirty lines for the end-of-kernel L2 writeback)
    const int k = base + 4 * i;
    *reinterpret_cast<int4*>(snd + k) = q;
    *reinterpret_cast<int4*>(rcv + k + 4 * R) = q;
    if (full) {
      const int4 ii = make_int4(i, i, i, i);
      *reinterpret_cast<int4*>(snd + k + 4 * R) = ii;
      *reinterpret_cast<int4*>(rcv + k) = ii;
    }
    *reinterpret_cast<float4*>(edg + k) = d;
    *reinterpret_cast<float4*>(edg + k + 4 * R) = d;
  };
  if (one) {
#pragma unroll
    for (int j = 0; j < RPT; ++j)
      if (tid + j * NT < R) finish(tid + j * NT, &pf[j]);
  } else {
    for (int i = tid; i < R; i += NT) finish(i, nullptr);
  }
  GF_COV_STAMP(3);
  __syncthreads();
  const int newly = *counter;
  const int nv = nv0 + newly;
  if (tid == 0) {
    a.nvisited[b] = nv;
    a.obs_step[b] = sc0;
    a.step_counter[b] = sc0 + 1;
    a.reward[b] = static_cast<double>(newly);
    a.done[b] = (sc0 + 1 == a.episode_length || nv == T) ? 1 : 0;
    a.dirty[b] = 0;
    if (MULTI && reward_k) reward_k[(size_t)it * a.B + b] = static_cast<double>(newly);
    if (MULTI && done_k) done_k[(size_t)it * a.B + b] = (sc0 + 1 == a.episode_length || nv == T) ? 1 : 0;
  }
  if (a.next_greedy) {
    // controller(greedy=True) (:800-872) on the resulting state, for the next step of an
    // expert loop: this step's visits (the `seen` node bits) joined to the visited bits,
    // then each robot's first unmasked entry of its new node's greedy list
    for (int t = tid; t < T; t += NT) {
      const int n = t + R;
      if ((seen[n >> 5] >> (n & 31)) & 1u) atomicOr(&gvis[t >> 5], 1u << (t & 31));
    }
    __syncthreads();
    const bool ndirect = T - nv <= kGreedyDirectMax;
    if (ndirect) {
      greedy_direct_list(gvis, T, nv > 0, ulist, ucount);
      __syncthreads();
    }
    for (int i = tid; i < R; i += NT) {
      const int c = new_s[i];
      const size_t row = (size_t)b * Tm + (c - R);
      const int g = ndirect ? greedy_direct(a.gcost + row * Tm, a.gprev + row * Tm, nbr + 4 * (c - R), cnt[c - R],
                                            ulist, *ucount)
                            : greedy_from_list(a.glist + row * a.gstride, a.glen + row, gvis, nv > 0, nv >= T);
      const uint32_t flag = static_cast<uint32_t>(g) >> 2;
      if (flag & kGreedyErr) atomicOr(a.err, 8);
      const int ai = (flag & kGreedyRnd) ? 0 : (g & 3);
      const uint8_t nr = (flag & kGreedyRnd) ? 1 : 0;
      a.gactions[(size_t)b * R + i] = ai;
      a.needs_random[(size_t)b * R + i] = nr;
      if (a.h_next) a.h_next[(size_t)b * R + i] = ai;
      if (a.h_nrand) a.h_nrand[(size_t)b * R + i] = nr;
    }
  }
  if (a.h_nodes || a.h_edges || a.h_senders || a.h_receivers || a.h_closest || a.h_step || a.h_err) {
    // cov_step_host: the env's whole observation and step outputs to page-locked host
    // memory, 16-byte stores where both sides are aligned. The workgroup reads back what
    // its own waves wrote above: after the barrier those stores are visible to it.
    __syncthreads();
    auto put = [&](auto* dst, const auto* src, size_t n) {
      using T1 = typename std::remove_const<typename std::remove_pointer<decltype(src)>::type>::type;
      static_assert(sizeof(T1) == 4, "4-byte elements");
      if (!dst) return;
      if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        const size_t n4 = n >> 2;
        for (size_t k = tid; k < n4; k += NT) reinterpret_cast<int4*>(dst)[k] = reinterpret_cast<const int4*>(src)[k];
        for (size_t k = (n4 << 2) + tid; k < n; k += NT) dst[k] = src[k];
      } else {
        for (size_t k = tid; k < n; k += NT) dst[k] = src[k];
      }
    };
    put(a.h_nodes ? a.h_nodes + (size_t)b * M * 3 : nullptr, nodes, (size_t)M * 3);
    put(a.h_edges ? a.h_edges + (size_t)b * E : nullptr, edg, (size_t)E);
    put(a.h_senders ? a.h_senders + (size_t)b * E : nullptr, snd, (size_t)E);
    put(a.h_receivers ? a.h_receivers + (size_t)b * E : nullptr, rcv, (size_t)E);
    if (a.h_closest)
      for (int i = tid; i < R; i += NT) a.h_closest[(size_t)b * R + i] = new_s[i];
    if (tid == 0) {
      if (a.h_step) a.h_step[b] = sc0;
      if (a.h_reward) a.h_reward[b] = static_cast<double>(newly);
      if (a.h_done) a.h_done[b] = (sc0 + 1 == a.episode_length || nv == T) ? 1 : 0;
      if (a.h_err) a.h_err[b] = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int NT, bool UIN = false>
__global__ __launch_bounds__(NT) void cov_step_kernel(typename std::conditional<UIN, CovArgsU, CovArgs>::type p) {
  [[maybe_unused]] CovArgs uargs;
  if constexpr (UIN) {
    uargs = p.a;
    uargs.actions = p.u;
  }
  const CovArgs& a = *[&]() -> const CovArgs* {
    if constexpr (UIN) return &uargs;
    else return &p;
  }();
  cov_step_body<NT, false>(a, 0, nullptr, nullptr);
#ifdef GF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GF_COV_STAMP(4);
#endif
  signal_done(a.fin);  // cov_step_host: the host waits for this, not the stream
}

// cov_step_expert: k_steps steps of every env in one launch, each env's workgroup stepping
// its env k_steps times (the actions come from the device: the greedy lists and the env's
// MT19937 stream), each iteration exactly one cov_step. What an iteration reads of the
// previous one's global writes (robots' nodes, the tail's offers, visited flags, the env's
// words, the key) was written by this workgroup, and the barrier between iterations orders
// it. A kernel of its own: the loop would cost the one-step kernel registers.
template <int NT>
__global__ __launch_bounds__(NT) void cov_step_multi_kernel(CovArgsM p) {
  const int n = p.k_steps > 1 ? p.k_steps : 1;
  for (int it = 0; it < n; ++it) {
    cov_step_body<NT, true>(p.a, it, p.reward_k, p.done_k);
    __syncthreads();
  }
}

// reset (:405-424 after the random draws): robots onto their start targets, the
// unvisited flags, then the same observation pass as a step without actions.
__global__ __launch_bounds__(kCovThreads) void cov_reset_kernel(CovArgs a, const int32_t* start,
                                                                 const uint8_t* visited0) {
  const int b = blockIdx.x;
  const int R = a.R, M = a.M, Tm = a.Tmax;
  const int T = a.ntg[b];
  const double* tg = a.tgt + (size_t)b * Tm * 2;
  __shared__ int count;
  if (threadIdx.x == 0) count = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += kCovThreads) {
    const int t = start[(size_t)b * R + i];
    a.cur[(size_t)b * R + i] = t + R;
    a.xr[((size_t)b * R + i) * 2] = tg[2 * t];
    a.xr[((size_t)b * R + i) * 2 + 1] = tg[2 * t + 1];
  }
  float* nodes = a.nodes + (size_t)b * M * 3;
  int local = 0;
  for (int t = threadIdx.x; t < Tm; t += kCovThreads) {
    const uint8_t v = t < T ? (visited0[(size_t)b * Tm + t] ? 1 : 0) : 1;  // flags are 0 / 1
    a.visited[(size_t)b * Tm + t] = v;
    if (t < T) {
      nodes[3 * (t + R) + 2] = v ? 0.0f : 1.0f;
      local += v ? 1 : 0;
    }
  }
  atomicAdd(&count, local);
  __syncthreads();
  if (threadIdx.x == 0) {
    a.nvisited[b] = count;
    a.step_counter[b] = 0;
    a.dirty[b] = 0;
  }
}

// reset()'s draws (coverage.py:405-424) for env b as a reference env whose np_random was
// seeded seed0 + b: RandomState(seed) (mt19937_seed: the generator's init_genrand), then
// choice(arange(T), R, replace=False) for the start targets and choice(arange(T) + R,
// int(T * frac), replace=False) for the unvisited ones, each numpy's legacy permutation of
// the stream (Fisher-Yates from the top, random_interval's masked rejection: oracle/
// mt19937.py). The stream is left in mt_key / mt_pos for the fallback draws
// (COV_GREEDY_RNG). One wave per env: the draws are one chain, which every lane runs, then
// lane 0 swaps; the key regenerations and the tempering take the whole wave.
__global__ __launch_bounds__(64) void cov_seed_reset_kernel(CovArgs a, uint32_t seed0, double frac, int32_t* start,
                                                            uint8_t* visited0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* key = reinterpret_cast<uint32_t*>(smem);
  int32_t* perm = reinterpret_cast<int32_t*>(key + kMtN);
  int32_t* vseq = perm + a.Tmax;  // [Tm] the draws of one permutation, by i
  uint8_t* vis = reinterpret_cast<uint8_t*>(vseq + a.Tmax);
  const int b = blockIdx.x, lane = threadIdx.x;
  const int R = a.R, Tm = a.Tmax, T = a.ntg[b];
  if (lane == 0) {
    uint32_t s = seed0 + static_cast<uint32_t>(b);
    for (int p = 0; p < kMtN; ++p) {
      key[p] = s;
      s = 1812433253u * (s ^ (s >> 30)) + static_cast<uint32_t>(p + 1);
    }
  }
  __syncthreads();
  int pos = kMtN;  // wave-uniform
  // RandomState.permutation(n) into perm[0, n). The draws do not depend on the permutation,
  // so they come first: 64 tempered words per round (one LDS load per lane), consumed in
  // stream order by a register chain (readlane; the masked rejection of each i), the
  // accepted ones into vseq[i]; then lane 0 runs the swaps, one LDS round trip each (the
  // draws and swaps interleaved waited on two per swap; profiles/r06/ab_seed_reset_draws.txt)
  auto permute = [&](int n) {
    for (int k = lane; k < n; k += 64) perm[k] = k;
    int i = n - 1;  // wave-uniform
    while (i >= 1) {
      if (pos == kMtN) {
        mt_regen<64>(key);
        pos = 0;
      }
      const int avail = min(64, kMtN - pos);
      const uint32_t wl = lane < avail ? mt_temper(key[pos + lane]) : 0u;
      int u = 0;
      for (; u < avail && i >= 1; ++u) {
        const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(static_cast<uint32_t>(i));
        const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wl), u)) & mask;
        if (v <= static_cast<uint32_t>(i)) {
          if (lane == 0) vseq[i] = static_cast<int>(v);
          --i;
        }
      }
      pos += u;
    }
    __syncthreads();
    if (lane == 0 && n > 1) {  // one lane: its LDS reads and writes stay in program order
      // the next swap's draw is read with this swap's entries (vseq is not written here),
      // so a swap waits on one LDS round trip, not two
      int v = vseq[n - 1];
      for (int k = n - 1; k >= 1; --k) {
        const int vnext = vseq[k - 1];  // vseq[0]: read, never used
        const int t = perm[k];
        const int pv = perm[v];
        perm[k] = pv;
        perm[v] = t;
        v = vnext;
      }
    }
    __syncthreads();
  };
  permute(T);
  for (int k = lane; k < R; k += 64) start[(size_t)b * R + k] = perm[k];
  __syncthreads();
  permute(T);
  const int kdrop = static_cast<int>(static_cast<double>(T) * frac);  // Python's int(T * frac)
  for (int t = lane; t < Tm; t += 64) vis[t] = 1;
  __syncthreads();
  for (int k = lane; k < kdrop; k += 64) vis[perm[k]] = 0;
  __syncthreads();
  for (int t = lane; t < Tm; t += 64) visited0[(size_t)b * Tm + t] = vis[t];
  for (int k = lane; k < kMtN; k += 64) a.mt_key[(size_t)b * kMtN + k] = key[k];
  if (lane == 0) a.mt_pos[b] = pos;
}

// FlattenDictWrapper order (reference test.py:33, keys coverage.py:90): nodes (M,3),
// edges (4M,1), senders (4M), receivers (4M), step (1,1), concatenated per env. The
// wrapper's np.concatenate promotes to float64; every value here is exact in float32
// too (the Box the wrapper declares), so both widths are offered.
template <class V>
__global__ __launch_bounds__(kCovThreads) void cov_flat_obs_kernel(CovArgs a, V* dst) {
  const int b = blockIdx.y;
  const size_t M = a.M, E = 4 * M, L = 15 * M + 1;
  V* out = dst + (size_t)b * L;
  const float* nodes = a.nodes + (size_t)b * 3 * M;
  const float* edges = a.edges + (size_t)b * E;
  const int32_t* snd = a.senders + (size_t)b * E;
  const int32_t* rcv = a.receivers + (size_t)b * E;
  for (size_t k = (size_t)blockIdx.x * kCovThreads + threadIdx.x; k < L; k += (size_t)gridDim.x * kCovThreads) {
    V v;
    if (k < 3 * M)
      v = static_cast<V>(nodes[k]);
    else if (k < 7 * M)
      v = static_cast<V>(edges[k - 3 * M]);
    else if (k < 11 * M)
      v = static_cast<V>(snd[k - 7 * M]);
    else if (k < 15 * M)
      v = static_cast<V>(rcv[k - 11 * M]);
    else
      v = static_cast<V>(a.obs_step[b]);
    out[k] = v;
  }
}

// unpack_obs (coverage.py:689-741) on the batch: edges, senders and receivers of every
// graph concatenated in env order, node indices offset by b*M, padded edges dropped.
// The reference offsets the senders BEFORE testing them against -1, so only graph 0's
// padding is dropped (a padded sender of graph b > 0 reads b*M - 1); mask_all drops
// every graph's padding instead. Graph b's edges start at off[b].
__global__ __launch_bounds__(kCovThreads) void cov_graphs_kernel(CovArgs a, const int64_t* off, int mask_all,
                                                                 float* edges_out, int32_t* snd_out, int32_t* rcv_out) {
  const int b = blockIdx.y;
  const int M = a.M, E = 4 * M, tail0 = E - 8 * a.R;
  const int nm = a.n_motion[b];
  const bool keep_all = !mask_all && b > 0;
  const float* edges = a.edges + (size_t)b * E;
  const int32_t* snd = a.senders + (size_t)b * E;
  const int32_t* rcv = a.receivers + (size_t)b * E;
  const int64_t base = off[b];
  const int32_t shift = b * M;
  for (int k = blockIdx.x * kCovThreads + threadIdx.x; k < E; k += gridDim.x * kCovThreads) {
    int64_t dst;
    if (keep_all || k < nm)
      dst = base + k;
    else if (k >= tail0)
      dst = base + nm + (k - tail0);
    else
      continue;  // padding (sender -1)
    edges_out[dst] = edges[k];
    snd_out[dst] = snd[k] + shift;
    rcv_out[dst] = rcv[k] + shift;
  }
}

}  // namespace

hipError_t launch_cov_flat_obs(const CovArgs& a, void* dst, bool f32, hipStream_t s) {
  const size_t L = 15 * (size_t)a.M + 1;
  const dim3 grid((unsigned)((L + 4 * kCovThreads - 1) / (4 * kCovThreads)), a.B);
  if (f32)
    hipLaunchKernelGGL(cov_flat_obs_kernel<float>, grid, dim3(kCovThreads), 0, s, a, static_cast<float*>(dst));
  else
    hipLaunchKernelGGL(cov_flat_obs_kernel<double>, grid, dim3(kCovThreads), 0, s, a, static_cast<double*>(dst));
  return hipGetLastError();
}

hipError_t launch_cov_graphs(const CovArgs& a, const int64_t* off, bool mask_all, float* edges, int32_t* snd,
                             int32_t* rcv, hipStream_t s) {
  const int E = 4 * a.M;
  const dim3 grid((unsigned)((E + 4 * kCovThreads - 1) / (4 * kCovThreads)), a.B);
  hipLaunchKernelGGL(cov_graphs_kernel, grid, dim3(kCovThreads), 0, s, a, off, mask_all ? 1 : 0, edges, snd, rcv);
  return hipGetLastError();
}

size_t cov_step_lds_bytes(int R, int M) {
  return (size_t)3 * R * 4 + (size_t)2 * ((M + 31) / 32) * 4 + 16 + (size_t)M * 4 + (size_t)((M - R + 63) / 64) * 8 +
         (size_t)(kGreedyDirectMax + 1) * 4 + (size_t)kMtN * 4 + (size_t)((R + 63) / 64) * 8;
}

hipError_t launch_cov_graph(const CovArgs& a, const int32_t* envs, int n, hipStream_t s) {
  if (a.Tmax <= kGraphLdsTargets) {
    const size_t lds = (size_t)a.Tmax * 16 + (size_t)kGraphCells * 4 + (size_t)a.Tmax * 4;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cov_graph_kernel<true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cov_graph_kernel<true>, dim3(n), dim3(kCovThreads), lds, s, a, envs, n);
  } else {
    hipLaunchKernelGGL(cov_graph_kernel<false>, dim3(n), dim3(kCovThreads), 0, s, a, envs, n);
  }
  return hipGetLastError();
}

hipError_t launch_cov_seed_reset(const CovArgs& a, uint32_t seed0, double frac, int32_t* start, uint8_t* visited0,
                                 hipStream_t s) {
  const size_t lds = (size_t)kMtN * 4 + (size_t)a.Tmax * 9;
  hipLaunchKernelGGL(cov_seed_reset_kernel, dim3(a.B), dim3(64), lds, s, a, seed0, frac, start, visited0);
  return hipGetLastError();
}

hipError_t launch_cov_reset(const CovArgs& a, const int32_t* start, const uint8_t* visited0, hipStream_t s) {
  hipLaunchKernelGGL(cov_reset_kernel, dim3(a.B), dim3(kCovThreads), 0, s, a, start, visited0);
  return hipGetLastError();
}

hipError_t launch_cov_step_uin(const CovArgs& a, const int32_t* u, hipStream_t s) {
  const size_t bytes = (size_t)a.B * a.R * 4;
  if (bytes > (size_t)kCovUInlineBytes || !u) return hipErrorInvalidValue;
  CovArgsU p;
  p.a = a;
  p.a.actions = nullptr;
  std::memcpy(p.u, u, bytes);
  void* args[] = {&p};
  return hipLaunchKernel(reinterpret_cast<const void*>(&cov_step_kernel<kCovThreads, true>), dim3(a.B),
                         dim3(kCovThreads), args, cov_step_lds_bytes(a.R, a.M), s);
}

hipError_t launch_cov_step_multi(const CovArgsM& m, hipStream_t s) {
  void* args[] = {const_cast<CovArgsM*>(&m)};
  return hipLaunchKernel(reinterpret_cast<const void*>(&cov_step_multi_kernel<kCovThreads>), dim3(m.a.B),
                         dim3(kCovThreads), args, cov_step_lds_bytes(m.a.R, m.a.M), s);
}

hipError_t launch_cov_step(const CovArgs& a, hipStream_t s) {
  // hipLaunchKernel with the argument pointer: the step is host-bound at two launches
  // per step, and the hipLaunchKernelGGL wrapper's repacking measured ~0.15 us more per
  // launch (scripts/graphprobe.hip)
  void* args[] = {const_cast<CovArgs*>(&a)};
  return hipLaunchKernel(reinterpret_cast<const void*>(&cov_step_kernel<kCovThreads>), dim3(a.B), dim3(kCovThreads),
                         args, cov_step_lds_bytes(a.R, a.M), s);
}

#ifdef GF_STAMPS
extern "C" __attribute__((visibility("default"))) int cov_diag_stamps(unsigned long long* dst, int n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(gf_cov_stamp_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

}  // namespace gf
