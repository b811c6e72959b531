// Internal interface of the Coverage-v0 kernels (coverage_kernels.hip) for the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "done_flag.h"

namespace gf {

// Device buffers of a batch of B Coverage envs with R robots and room for M nodes
// (robots + targets), i.e. at most Tmax = M - R targets per env.
struct CovArgs {
  int B, R, M, Tmax, episode_length;
  int env0;               // cov_step_kernel: first env of this launch (split steps)
  double res, motion_radius;
  const double* tgt;      // (B,Tmax,2) target positions
  const int32_t* ntg;     // (B) targets per env
  int32_t* nbr;           // (B,Tmax,4) motion-graph neighbours (target-local), -1 padded
  int32_t* cnt;           // (B,Tmax) neighbour counts
  int32_t* n_motion;      // (B) motion edges per env
  double* xr;             // (B,R,2) robot positions
  int32_t* cur;           // (B,R) node each robot is on (global index)
  uint8_t* visited;       // (B,Tmax)
  int32_t* nvisited;      // (B)
  int32_t* step_counter;  // (B)
  uint8_t* dirty;         // (B) robots were placed externally: recompute closest nodes
  const int32_t* actions; // (B,R) in [0,4), or nullptr (observation only)
  double* reward;         // (B)
  uint8_t* done;          // (B)
  float* nodes;           // (B,M,3)
  float* edges;           // (B,4M)
  int32_t* senders;       // (B,4M)
  int32_t* receivers;     // (B,4M)
  int64_t* obs_step;      // (B)
  double* axy;            // (B,Tmax,4,2) coordinates of each node's 4 action targets
  float* nrec;            // (B,Tmax,16) per node, 64 B: its 4 action targets (global, padded
                          // with itself; int4), the 4 action-edge features of a robot on it
                          // (float4), its position (double2), 16 B pad
  int* err;               // device error bits: 1 degree > 4, 2 edges overflow, 4 bad action
  // fused greedy expert (cov_step with COV_ACTIONS_GREEDY): the step's actions are
  // controller(greedy=True)'s, taken from each node's greedy list (below)
  const uint16_t* glist;  // (B,Tmax,gstride) or nullptr: actions come from `actions`
  const uint16_t* glen;   // (B,Tmax)
  int gstride;
  const uint16_t* gcost;  // (B,Tmax,Tmax) hop counts [source][target] (greedy_direct)
  const int16_t* gprev;   // (B,Tmax,Tmax) graph_previous[t, c] at [c][t] (greedy_direct)
  int32_t* gactions;      // (B,R) the greedy actions taken (written)
  uint8_t* needs_random;  // (B,R) robots the reference hands to np_random.choice (action 0 here)
  // COV_GREEDY_RNG: those robots draw np_random.choice(4) (:863-864) from their env's
  // MT19937 stream instead, in robot order, as numpy's legacy RandomState does (nullptr:
  // action 0). The stream is RandomState.get_state()'s key words and position.
  uint32_t* mt_key;       // (B,624)
  int32_t* mt_pos;        // (B) in [0, 624]
  // cov_step_host: after the step, controller(greedy=True)'s actions of the RESULTING state
  // from the greedy lists (glist / glen / gstride) into gactions / needs_random (and the
  // host copies below), for the next step of an expert loop
  int next_greedy;
  // cov_step_host: every output of the env written by the step's own workgroup to page-
  // locked host memory (mapped device addresses) at its end; any may be nullptr
  float* h_nodes;         // (B,M,3)
  float* h_edges;         // (B,4M)
  int32_t* h_senders;     // (B,4M)
  int32_t* h_receivers;   // (B,4M)
  int64_t* h_step;        // (B)
  double* h_reward;       // (B)
  uint8_t* h_done;        // (B)
  int32_t* h_closest;     // (B,R) each robot's node after the step (closest_targets, global)
  int32_t* h_next;        // (B,R) next_greedy actions
  uint8_t* h_nrand;       // (B,R) next_greedy needs_random flags
  int32_t* h_err;         // (B) the device error word as this env's workgroup ends
  DoneFlag fin;           // cov_step_host: the grid's completion flag (done_flag.h)
};

// cov_step_expert: k_steps fused greedy expert steps in one launch, each env's workgroup
// stepping its env k_steps times; step s's rewards and done flags at [s][b] (a separate
// argument block, so the one-step kernel's arguments stay as they are)
struct CovArgsM {
  CovArgs a;
  int k_steps;
  double* reward_k;       // (k_steps,B) or nullptr
  uint8_t* done_k;        // (k_steps,B) or nullptr
};

// cov_step_host: one env's actions travel in the kernel arguments up to this many bytes
constexpr int kCovUInlineBytes = 2048;
struct CovArgsU {
  CovArgs a;
  alignas(16) int32_t u[kCovUInlineBytes / 4];
};

// Greedy lists (built with the time matrix, cov_greedy_list_kernel): for every source
// node c of an env, the targets t with a finite hop count cost[c][t] < MAX_COST, in
// (cost, t) order, i.e. the order of controller(greedy=True)'s np.argmin over the
// masked row (coverage.py:817-819). Entry = t | action << 10 | flag << 12: the index of
// the first hop (graph_previous[t, c], :863-869) among the node's action targets, flag
// 1 when the predecessor is -1 (the reference draws a random action), 2 when it is not
// among them (the reference raises IndexError). Needs Tmax <= 1024.
constexpr int kGreedyListMaxT = 1024;
constexpr uint32_t kGreedyRnd = 1, kGreedyErr = 2;

// The greedy action of a robot on target-local node c from its list row: the first
// entry whose target is unvisited (and is not target 0 once anything is visited: the
// reference masks visited targets through np.where on its (N,1) visited column, which
// also hits column 0). vbits: the env's visited flags as bits (LDS). Returns
// action | flag << 2; flag kGreedyRnd also when every listed target is masked (at once
// when the env has no unvisited target left: nv == T). The row's length and its first
// kGreedyListPad entries are loaded together, and each later round trip brings the next
// kGreedyListPad (four 16-byte loads): late in an episode, when most targets near a robot
// are visited, its scan runs deep into the list, and one 16-byte load per round trip made
// such robots' dependent loads the step's longest phase. Rows are padded to a multiple
// of kGreedyListPad entries (gstride).
constexpr int kGreedyListPad = 32;
__device__ __forceinline__ int greedy_from_list(const uint16_t* row, const uint16_t* lenp, const uint32_t* vbits,
                                                bool any_vis, bool none_left) {
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
  int len = *lenp;
  uint4 q[kGreedyListPad / 8];
#pragma unroll
  for (int c = 0; c < kGreedyListPad / 8; ++c) q[c] = r4[c];
  if (none_left) len = 0;
  for (int k0 = 0; k0 < len; k0 += kGreedyListPad) {
    if (k0 > 0) {
#pragma unroll
      for (int c = 0; c < kGreedyListPad / 8; ++c) q[c] = r4[k0 / 8 + c];
    }
#pragma unroll
    for (int j = 0; j < kGreedyListPad; ++j) {
      const uint4 v = q[j >> 3];
      const uint32_t w = (j & 7) < 2 ? v.x : (j & 7) < 4 ? v.y : (j & 7) < 6 ? v.z : v.w;
      const uint32_t e = (w >> (16 * (j & 1))) & 0xFFFFu;
      const int t = static_cast<int>(e & 1023u);
      const bool masked = ((vbits[t >> 5] >> (t & 31)) & 1u) || (t == 0 && any_vis);
      if (k0 + j < len && !masked) return static_cast<int>(e >> 10);
    }
  }
  return static_cast<int>(kGreedyRnd << 2);
}

// When few targets are left unvisited the list scan runs deep: late in an episode every
// target near a robot is visited and its list's first unvisited entry lies hundreds of
// entries in (a dependent load per 32 entries; 50-80 us steps at config 4). With at most
// kGreedyDirectMax unvisited targets (excluding target 0 once anything is visited, the
// reference's mask) the kernels take the minimum (hop count, target) over that short list
// directly from the robot's cost row instead: the same target, as the list is in that
// order. ulist: the env's unvisited candidates in ascending target order (LDS).
constexpr int kGreedyDirectMax = 32;
constexpr uint32_t kCostInf = 0xFFFF;   // uint16 cost matrix: unreachable
constexpr uint32_t kCostMax = 1000;     // MAX_COST (coverage.py:68)
__device__ __forceinline__ int greedy_direct(const uint16_t* crow, const int16_t* prow, const int32_t* nbr4,
                                             int n, const int* ulist, int U) {
  uint32_t key = 0xFFFFFFFFu;
  for (int k0 = 0; k0 < U; k0 += 8) {  // eight loads of the row in flight
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = k0 + k < U ? crow[ulist[k0 + k]] : kCostInf;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (v[k] != kCostInf && v[k] < kCostMax) key = min(key, v[k] << 10 | static_cast<uint32_t>(ulist[k0 + k]));
  }
  if (key == 0xFFFFFFFFu) return static_cast<int>(kGreedyRnd << 2);  // every candidate out of reach
  const int t = static_cast<int>(key & 1023u);
  const int p = prow[t];
  if (p < 0) return static_cast<int>(kGreedyRnd << 2);  // :863
  const int4 nb = *reinterpret_cast<const int4*>(nbr4);
  int act = (n > 3 && nb.w == p) ? 3 : 4;  // the first of the node's action targets equal to the next hop
  act = (n > 2 && nb.z == p) ? 2 : act;
  act = (n > 1 && nb.y == p) ? 1 : act;
  act = (n > 0 && nb.x == p) ? 0 : act;
  if (act == 4) return static_cast<int>(kGreedyErr << 2);
  return act;
}
// The candidates of greedy_direct from the visited bits (one wave: lane-ordered ballots
// keep ascending target order); returns their count (<= kGreedyDirectMax is the caller's
// condition: T - visited <= kGreedyDirectMax). Every wave calls it; wave 0 writes.
__device__ __forceinline__ void greedy_direct_list(const uint32_t* vbits, int T, bool any_vis, int* ulist, int* ucount) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  int cnt = 0;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    const bool cand = t < T && !((vbits[t >> 5] >> (t & 31)) & 1u) && !(t == 0 && any_vis);
    const uint64_t m = __ballot(cand);
    const int pos = cnt + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0));
    if (cand && pos < kGreedyDirectMax) ulist[pos] = t;
    cnt += __popcll(m);
  }
  if (lane == 0) *ucount = cnt;
}

// np_random's generator (numpy's legacy RandomState: MT19937, the published algorithm of
// Matsumoto & Nishimura). choice(4) with uniform p is randint(0, 4): one 32-bit output,
// masked to 2 bits (the mask equals the range, so no draw is ever rejected).
constexpr int kMtN = 624, kMtM = 397;
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y ^ (y >> 18);
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t next, uint32_t far) {
  const uint32_t y = (cur & 0x80000000u) | (next & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
// The key's regeneration (after 624 outputs) by the whole workgroup on a key in LDS. Word i
// mixes words i, i+1 and i+397 (mod 624, the wrapped ones already regenerated), so three
// passes of at most 227 independent words each, then word 623: [0,227) reads only old
// words, [227,454) reads the first pass's results, [454,623) the second's. Ends with a
// barrier. Every thread of the workgroup calls it.
template <int NT>
__device__ __forceinline__ void mt_regen(uint32_t* k) {
  constexpr int P = kMtN - kMtM;  // 227
  constexpr int S = (P + NT - 1) / NT;
  auto pass = [&](int lo, int hi) {
    uint32_t v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int i = lo + static_cast<int>(threadIdx.x) + s * NT;
      if (i < hi) v[s] = mt_mix(k[i], k[i + 1], k[i < P ? i + kMtM : i - P]);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int i = lo + static_cast<int>(threadIdx.x) + s * NT;
      if (i < hi) k[i] = v[s];
    }
    __syncthreads();
  };
  pass(0, P);
  pass(P, 2 * P);
  pass(2 * P, kMtN - 1);
  if (threadIdx.x == 0) k[kMtN - 1] = mt_mix(k[kMtN - 1], k[0], k[kMtM - 1]);
  __syncthreads();
}

// Greedy expert (coverage_expert.hip).
struct CovTmArgs {
  int R, M, Tmax, horizon;
  int kcap;                  // flag slots per chunk: horizon+1, or Tmax+1 when unbounded
  int nchunk;                // (Tmax + 63) / 64
  int t_lds;                 // largest target count among the selected envs
  const int32_t* envs;       // selected envs (blockIdx.y)
  const int32_t* ntg;        // (B)
  const int32_t* n_motion;   // (B)
  const int32_t* senders;    // (B,4M): motion edges first (global indices)
  const int32_t* receivers;  // (B,4M)
  uint8_t* flags;            // (B,nchunk,kcap): bit 0 changed, bit 1 some entry inf
  uint16_t* cost;            // (B,Tmax,Tmax) [source][target], 0xFFFF = inf
  uint8_t* cost8;            // (B,Tmax,Tmax) the same as uint8 (255 = inf), written by the
                             // uint8 pass only (envs whose hop counts all fit)
  int16_t* prevT;            // (B,Tmax,Tmax) [q][source] = graph_previous[source, q]
  uint32_t* sched;           // (B,sched_stride) batched edge schedule
  int32_t* nslots;           // (B) schedule length
  int32_t* nlev;             // (B) schedule levels
  uint8_t* overflow;         // (B) the uint8 pass could not bound an entry: rerun wide
  int sched_stride;
  int32_t* lev_off;          // (B,lev_stride) each level's first schedule slot, then nslots
  int lev_stride;
  // greedy lists (cov_greedy_list_kernel), when Tmax <= kGreedyListMaxT
  const uint8_t* wide;       // (B) which cost form holds the env's matrix
  const int32_t* nbr;        // (B,Tmax,4)
  const int32_t* cnt;        // (B,Tmax)
  uint16_t* glist;           // (B,Tmax,gstride)
  uint16_t* glen;            // (B,Tmax)
  int gstride;
};

struct CovGreedyArgs {
  int B, R, Tmax;
  const int32_t* ntg;
  const double* tgt;
  const double* xr;
  const uint8_t* dirty;
  const int32_t* cur;
  const uint16_t* cost;
  const uint8_t* cost8;      // used for envs with wide[b] == 0 (half the bytes per row)
  const uint8_t* wide;       // (B) 1: the env's matrix needed uint16 entries
  const int16_t* prevT;
  const uint8_t* visited;
  const int32_t* nvisited;
  const int32_t* nbr;
  const int32_t* cnt;
  int32_t* actions;        // (B,R)
  uint8_t* needs_random;   // (B,R)
  int* err;                // 8: next hop not among the robot's actions
  const uint16_t* glist;   // greedy lists (or nullptr: scan the cost rows)
  const uint16_t* glen;
  int gstride;
};

size_t cov_time_matrix_lds_bytes(int t_lds, bool wide);
size_t cov_tm_schedule_lds_bytes(int t_lds, int e_max);
hipError_t launch_cov_tm_schedule(const CovTmArgs& a, int n_envs_sel, int e_max, hipStream_t s);
// Pass A + pass B over the selected envs; wide = uint16 entries (else uint8, which sets
// overflow[b] for envs it cannot bound).
hipError_t launch_cov_time_matrix(const CovTmArgs& a, int n_envs_sel, bool wide, hipStream_t s);
hipError_t launch_cov_greedy(const CovGreedyArgs& a, hipStream_t s);
// the greedy lists of the selected envs (after their time matrices)
hipError_t launch_cov_greedy_lists(const CovTmArgs& a, int n_envs_sel, hipStream_t s);

// Per-episode target maps (coverage_maps.hip; coverage.py:516-527, make_map.py:30-67,
// :207-231). One workgroup per selected env.
struct CovMapArgs {
  int n_sel;
  const int32_t* envs;       // (n_sel) env of each workgroup
  int R, Tmax;
  int NC;                    // cities per map (<= kMapMaxCities)
  double lo, range;          // cities: lo + range * random_sample (np.random.uniform)
  double road_radius;        // waypoint spacing along each road (motion_radius)
  double near_radius;        // lattice points within it of a waypoint (motion_radius / 1.4)
  double link_radius;        // target radius graph (motion_radius)
  int L;                     // lattice points
  const double2* lat;        // (L) generate_lattice's points, [y, x] columns
  const int32_t* lat_cell;   // (L) each point's cell gi * NJ + gj
  const int32_t* cell;       // (NI * NJ) the lattice point of each cell, or -1
  int NI, NJ, K;             // cell grid, cells searched either side for a link
  int wcap;                  // waypoints the LDS holds
  int G;                     // waypoint grid (G x G cells of side gh from (gx0, gy0)) for the
  double gx0, gy0, gh;       //   near-road test; G = 0: every lattice point scans every waypoint
  double* cities;            // (B, kMapMaxCities, 2): drawn by cov_map_cities_kernel or uploaded
  uint32_t* mt_key;          // (B, 624) each env's map stream (the reference's global np.random)
  int32_t* mt_pos;           // (B)
  uint32_t seed0;            // seed: stream b := RandomState(seed0 + b)
  int seed;
  double* tgt;               // (B, Tmax, 2) out: the largest component's points, lattice order
  int32_t* ntg;              // (B) out: targets (0 when the map is refused)
  int32_t* nraw;             // (B) out: the largest component's size
  int32_t* status;           // (B) out: kMapNearDegenerate | kMapTooMany | kMapTooFew | kMapOverflow
};
constexpr int kMapMaxCities = 32;
constexpr int32_t kMapNearDegenerate = 1, kMapTooMany = 2, kMapTooFew = 4, kMapOverflow = 8;
size_t cov_map_lds_bytes(int L, int wcap, int G);
hipError_t launch_cov_map_cities(const CovMapArgs& a, hipStream_t s);
hipError_t launch_cov_map(const CovMapArgs& a, hipStream_t s);

size_t cov_step_lds_bytes(int R, int M);
// Observation wire formats: the flat FlattenDictWrapper rows (B, 15M+1) and the
// batched unpack_obs graph tuple (edges compacted at off[b]).
hipError_t launch_cov_flat_obs(const CovArgs& a, void* dst, bool f32, hipStream_t s);
hipError_t launch_cov_graphs(const CovArgs& a, const int64_t* off, bool mask_all, float* edges, int32_t* snd,
                             int32_t* rcv, hipStream_t s);
hipError_t launch_cov_graph(const CovArgs& a, const int32_t* envs, int n, hipStream_t s);
hipError_t launch_cov_reset(const CovArgs& a, const int32_t* start, const uint8_t* visited0, hipStream_t s);
// reset()'s random draws on the device for envs seeded seed0 + b (start (B,R), visited0
// (B,Tmax)), the streams left in a.mt_key / a.mt_pos
hipError_t launch_cov_seed_reset(const CovArgs& a, uint32_t seed0, double frac, int32_t* start, uint8_t* visited0,
                                 hipStream_t s);
hipError_t launch_cov_step(const CovArgs& a, hipStream_t s);
hipError_t launch_cov_step_multi(const CovArgsM& m, hipStream_t s);  // m.k_steps steps, one launch
// the step with a.actions read from `u` (host memory, copied into the kernel arguments;
// B * R * 4 <= kCovUInlineBytes)
hipError_t launch_cov_step_uin(const CovArgs& a, const int32_t* u, hipStream_t s);

}  // namespace gf
