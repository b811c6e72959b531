// HIP kernels (gfx950 / CDNA4) for gym-flock's FlockingRelative-v0 / Flocking-v0 step.
//
// Reference (paths relative to the reference root):
//   gym_flock/envs/flocking/flocking_relative.py  step :91-109, compute_helpers :111-134,
//     get_stats :136-143, instant_cost :145-147, controller/potential_grad :194-226
//   gym_flock/envs/flocking/flocking.py            get_observation :20-25 (k nearest)
//
// The reference materialises several (N,N,{4,6}) float64 temporaries per step. Here
// one launch does the whole step for B envs: each 256-thread workgroup owns R rows
// (agents i) of one env, stages the env's agents through LDS in tiles of up to 1024,
// and produces
//   - adjacency bits for its rows (wave64 ballots of r2 < comm_radius^2) kept in LDS,
//   - the neighbour features / controller gradients, evaluated only for the pairs
//     whose bit is set (lane per (row, word-slice), iterating set bits),
//   - the dense mean-pooled (N,N) network rows as 16-byte coalesced stores.
// The dense network write (4*N^2 bytes per env) is the roofline: the kernel is HBM
// write bound, not MFMA work.
//
// Numerics: the pair path is float64 with -ffp-contract=off so every r2 is the
// reference's bit pattern (dx*dx + dy*dy, two roundings then a sum); adjacency is
// therefore bit-exact, and features differ from NumPy only by summation order.
#include "flock_internal.h"

#include <float.h>
#include <limits.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>

#include <type_traits>

namespace gf {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

struct __attribute__((aligned(16))) St {
  double px, py, vx, vy;
};

// Workgroup -> (env, row block) with all row blocks of an env on one XCD
// (blocks b and b+8 share an XCD under round-robin dispatch; speed only).
__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int xcd = bid & 7, q = G >> 3, r = G & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// xcd_remap, then within each XCD's contiguous range the envs' first row blocks (the
// ones that also compute the reward) are dealt out first, so none of them is among
// the last workgroups to start. Needs whole envs per XCD (G % (8 * bpe) == 0);
// otherwise the plain remap.
__device__ __forceinline__ int xcd_remap_reward_first(int bid, int G, int bpe) {
  const int L = xcd_remap(bid, G);
  if (bpe < 2 || G % (8 * bpe) != 0) return L;
  const int per = G >> 3, nenv = per / bpe;
  const int base = (bid & 7) * per, k = L - base;
  if (k < nenv) return base + k * bpe;  // env k's block 0
  const int k2 = k - nenv, e = k2 / (bpe - 1);
  return base + e * bpe + 1 + (k2 - e * (bpe - 1));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Deterministic workgroup sum: butterfly inside each wave, then the 4 wave totals in
// a fixed tree. Every thread returns the same bits.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// State of agent `g` (flat index b*N + j) after the double-integrator update of
// flocking_relative.py:96-105, in the reference's operation order. With a float32 u
// the action terms are float32 arithmetic (NumPy keeps u*10.0, *dt, *0.5 in float32)
// and are widened when added to the float64 state.
template <class V>
__device__ __forceinline__ V clip_sym(V v, V c) {  // np.clip(v, -c, c); NaN stays NaN
  return v < -c ? -c : (v > c ? c : v);
}

// The variants' update (oracle/flocking_variants.integrate): optional clip, the
// step's own action scale, per-env dt, the frozen agents' float64 mask applied after
// the action arithmetic, and the stochastic env's state scaling around the update.
template <bool UF64>
__device__ St load_state_variant(const StepArgs& a, size_t g, double2 p, double2 v) {
  const int b = static_cast<int>(g / static_cast<size_t>(a.N));
  const int j = static_cast<int>(g - static_cast<size_t>(b) * a.N);
  const double dt = a.dt_env ? a.dt_env[b] : a.dt;
  const double m = j < a.n_frozen ? 0.0 : 1.0;
  const double S = a.x_scale;
  const double px = p.x * S, py = p.y * S, vx = v.x * S, vy = v.y * S;
  double apx, apy, avx, avy;
  if constexpr (UF64) {
    const double2 u = reinterpret_cast<const double2*>(a.u)[g];
    double ux = u.x, uy = u.y;
    if (a.u_clip > 0) {
      ux = clip_sym(ux, a.u_clip);
      uy = clip_sym(uy, a.u_clip);
    }
    ux *= a.u_scale;
    uy *= a.u_scale;
    apx = (((ux * dt) * dt) * 0.5) * m;
    apy = (((uy * dt) * dt) * 0.5) * m;
    avx = (ux * dt) * m;
    avy = (uy * dt) * m;
  } else {
    const float2 u = reinterpret_cast<const float2*>(a.u)[g];
    const float dtf = static_cast<float>(dt);
    float ux = u.x, uy = u.y;
    if (a.u_clip > 0) {
      ux = clip_sym(ux, a.uc_f);
      uy = clip_sym(uy, a.uc_f);
    }
    ux *= a.us_f;
    uy *= a.us_f;
    apx = static_cast<double>(((ux * dtf) * dtf) * 0.5f) * m;
    apy = static_cast<double>(((uy * dtf) * dtf) * 0.5f) * m;
    avx = static_cast<double>(ux * dtf) * m;
    avy = static_cast<double>(uy * dtf) * m;
  }
  St s;
  s.px = ((px + vx * dt) + apx) / S;
  s.py = ((py + vy * dt) + apy) / S;
  s.vx = (vx + avx) / S;
  s.vy = (vy + avy) / S;
  return s;
}

// The global loads behind one agent's post-update state, and the update itself: split
// so the tiled step can issue a tile's loads one tile ahead (PF) and apply the update
// when it stages the tile.
template <bool UF64>
struct RawState {
  double2 p, v;
  typename std::conditional<UF64, double2, float2>::type u;
};

template <bool DYN, bool UF64>
__device__ __forceinline__ RawState<UF64> load_raw(const StepArgs& a, size_t g) {
  using U = typename std::conditional<UF64, double2, float2>::type;
  const double2* xp = reinterpret_cast<const double2*>(a.x_in) + 2 * g;
  RawState<UF64> r;
  r.p = xp[0];
  r.v = xp[1];
  if constexpr (DYN) r.u = reinterpret_cast<const U*>(a.u)[g];
  return r;
}

template <bool DYN, bool UF64>
__device__ __forceinline__ St state_from_raw(const StepArgs& a, const RawState<UF64>& r) {
  const double2 p = r.p, v = r.v;
  St s{p.x, p.y, v.x, v.y};
  if constexpr (DYN) {
    if constexpr (UF64) {
      const double ux = r.u.x * a.action_scalar, uy = r.u.y * a.action_scalar;
      s.px = (p.x + v.x * a.dt) + ((ux * a.dt) * a.dt) * 0.5;
      s.py = (p.y + v.y * a.dt) + ((uy * a.dt) * a.dt) * 0.5;
      s.vx = v.x + ux * a.dt;
      s.vy = v.y + uy * a.dt;
    } else {
      const float ux = r.u.x * a.as_f, uy = r.u.y * a.as_f;
      const float apx = ((ux * a.dt_f) * a.dt_f) * 0.5f;
      const float apy = ((uy * a.dt_f) * a.dt_f) * 0.5f;
      s.px = (p.x + v.x * a.dt) + static_cast<double>(apx);
      s.py = (p.y + v.y * a.dt) + static_cast<double>(apy);
      s.vx = v.x + static_cast<double>(ux * a.dt_f);
      s.vy = v.y + static_cast<double>(uy * a.dt_f);
    }
  }
  return s;
}

template <bool DYN, bool UF64, bool VAR = false>
__device__ __forceinline__ St load_state(const StepArgs& a, size_t g) {
  if constexpr (DYN && VAR) {
    const double2* xp = reinterpret_cast<const double2*>(a.x_in) + 2 * g;
    return load_state_variant<UF64>(a, g, xp[0], xp[1]);
  } else {
    return state_from_raw<DYN, UF64>(a, load_raw<DYN, UF64>(a, g));
  }
}

// 1/r2 for the feature pair terms (float32 outputs) without the controller: v_rcp_f64
// refined by one Newton step (about 2^-50 relative, 3 float64 ops instead of the 10 of a
// correctly rounded division). The controller keeps the IEEE division.
__device__ __forceinline__ double recip_f64(double r2) {
  // one Newton step on v_rcp_f64; outside [2^-1000, 2^1000] (zero, denormals, huge,
  // inf, NaN) the raw v_rcp_f64 value, chosen without a branch
  const double x0 = __builtin_amdgcn_rcp(r2);
  const double e = fma(-r2, x0, 1.0);
  const double x1 = fma(x0, e, x0);
  return (r2 >= 0x1p-1000 && r2 <= 0x1p+1000) ? x1 : x0;
}

__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c) {
  unsigned r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Insert v into the ascending list k[0..L) keeping its L smallest (the largest drops
// off): new k[m] = median(k[m-1], k[m], v) from the top down, then k[0] = min(k[0], v):
// one v_med3_u32 per entry, in place (a min/max exchange chain needs two per entry
// plus the register copies the compiler adds to rotate its temporaries)
template <int L>
__device__ __forceinline__ void knn_list_insert(unsigned (&k)[L], unsigned v) {
#pragma unroll
  for (int m = L - 1; m >= 1; --m) k[m] = med3_u32(k[m - 1], k[m], v);
  k[0] = min(k[0], v);
}

template <int K>
__device__ __forceinline__ void knn_insert(double (&kr)[K], int (&kj)[K], double r2, int j) {
  if (r2 < kr[K - 1] || (r2 == kr[K - 1] && j < kj[K - 1])) {
    double cr = r2;
    int cj = j;
#pragma unroll
    for (int m = 0; m < K; ++m) {
      const bool sw = (cr < kr[m]) || (cr == kr[m] && cj < kj[m]);
      const double tr = sw ? kr[m] : cr;
      const int tj = sw ? kj[m] : cj;
      kr[m] = sw ? cr : kr[m];
      kj[m] = sw ? cj : kj[m];
      cr = tr;
      cj = tj;
    }
  }
}

// knn_insert for columns that arrive in ascending j with finite r2: a tie keeps the
// listed (lower) index first, so only the new entry is compared against the list.
template <int K>
__device__ __forceinline__ void knn_insert_asc(double (&kr)[K], int (&kj)[K], double r2, int j) {
  if (r2 < kr[K - 1]) {
    bool prev = false;
    double pr = 0.0;
    int pj = 0;
#pragma unroll
    for (int m = 0; m < K; ++m) {
      const bool sw = r2 < kr[m];
      const double om = kr[m];
      const int oj = kj[m];
      kr[m] = sw ? (prev ? pr : r2) : om;
      kj[m] = sw ? (prev ? pj : j) : oj;
      prev = sw;
      pr = om;
      pj = oj;
    }
  }
}

// A NaN r2 (a non-finite state: e.g. the controller's division by zero for coincident
// agents) enters as (inf, j + N): after every real (inf, j) and ordered by index, as the
// exact small-env ranking orders NaN keys above +inf (r2_key) and argsort puts NaN last;
// the writers map j + N back to j.
template <int K>
__device__ __forceinline__ void knn_consider(double (&kr)[K], int (&kj)[K], double pxi, double pyi, double2 p,
                                             int j, int N) {
  const double dx = pxi - p.x, dy = pyi - p.y;
  const double r2 = dx * dx + dy * dy;
  const bool nan = r2 != r2;
  knn_insert<K>(kr, kj, nan ? __builtin_inf() : r2, nan ? j + N : j);
}
// the column of a ranked slot: j, j + N (a NaN r2) or unfilled (the row itself)
__device__ __forceinline__ int knn_slot_col(int kj, int N, int row) {
  return kj < N ? kj : (kj < 2 * N ? kj - N : row);
}

// Row `i` of lane l, ranked by the whole wave: lanes scan columns lane, lane + 64, ...
// into lane-local K-lists, then K rounds of a wave-wide (r2, j) minimum merge them into
// lane l's (kr, kj). pos(j): the agent's position.
template <int K, class Pos>
__device__ __forceinline__ void knn_wave_scan(const Pos& pos, int N, int l, int i, double pxi, double pyi,
                                              double (&kr)[K], int (&kj)[K]) {
  const int lane = threadIdx.x & 63;
  const int row = __shfl(i, l);
  const double px = __shfl(pxi, l), py = __shfl(pyi, l);
  double lr[K];
  int lj[K];
#pragma unroll
  for (int m = 0; m < K; ++m) {
    lr[m] = __builtin_inf();
    lj[m] = INT_MAX;
  }
  constexpr int U = 4;  // positions of U columns in flight per lane
  for (int j0 = lane; j0 < N; j0 += U * 64) {
    double2 p[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (j0 + u * 64 < N) p[u] = pos(j0 + u * 64);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * 64;
      if (j < N && j != row) knn_consider<K>(lr, lj, px, py, p[u], j, N);
    }
  }
#pragma unroll
  for (int m = 0; m < K; ++m) {
    double br = lr[0];
    int bj = lj[0];
    for (int o = 32; o > 0; o >>= 1) {
      const double orr = __shfl_xor(br, o);
      const int oj = __shfl_xor(bj, o);
      if (orr < br || (orr == br && oj < bj)) {
        br = orr;
        bj = oj;
      }
    }
    if (lane == l) {
      kr[m] = br;
      kj[m] = bj;
    }
    if (lj[0] == bj) {  // the winner's lane pops its head (columns are disjoint per lane)
#pragma unroll
      for (int q = 0; q + 1 < K; ++q) {
        lr[q] = lr[q + 1];
        lj[q] = lj[q + 1];
      }
      lr[K - 1] = __builtin_inf();
      lj[K - 1] = INT_MAX;
    }
  }
}

// Inline rim of the fused kNN step: the wave's rows in `todo` (lane bits; lane l holds
// row il with post-update state me), one at a time. Each is scanned by the whole wave
// over every agent's post-update position (recomputed from x_in and u, bit-identical to
// the step's) exactly as knn_wave_scan does, but round m's winner stays in lane m, so
// lanes 0..K-1 write the row's outputs as knn_write_row does (self inserted last with
// r2 = inf, the k-th nearest r2 for the fused steps' candidate radius).
template <bool DYN, bool UF64, int KN>
__device__ __forceinline__ void step_inline_rim(const StepArgs& a, size_t env0, uint64_t todo, int il,
                                                const St& me) {
  const int N = a.N, lane = threadIdx.x & 63;
  for (; todo; todo &= todo - 1) {
    const int l = __builtin_ctzll(todo);
    const int row = __shfl(il, l);
    const double px = __shfl(me.px, l), py = __shfl(me.py, l);
    double lr[KN];
    int lj[KN];
#pragma unroll
    for (int m = 0; m < KN; ++m) {
      lr[m] = __builtin_inf();
      lj[m] = INT_MAX;
    }
    constexpr int U = kInlineRimU;  // columns in flight per lane
    for (int j0 = lane; j0 < N; j0 += U * 64) {
      St p[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j0 + u * 64 < N) p[u] = load_state<DYN, UF64>(a, env0 + j0 + u * 64);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * 64;
        if (j < N && j != row) knn_consider<KN>(lr, lj, px, py, make_double2(p[u].px, p[u].py), j, N);
      }
    }
    double rr = __builtin_inf();
    int rj = INT_MAX;
#pragma unroll
    for (int m = 0; m < KN; ++m) {
      double br = lr[0];
      int bj = lj[0];
      for (int o = 32; o > 0; o >>= 1) {
        const double orr = __shfl_xor(br, o);
        const int oj = __shfl_xor(bj, o);
        if (orr < br || (orr == br && oj < bj)) {
          br = orr;
          bj = oj;
        }
      }
      if (lane == m) {
        rr = br;
        rj = bj;
      }
      if (lj[0] == bj) {  // the winner's lane pops its head (columns are disjoint per lane)
#pragma unroll
        for (int q = 0; q + 1 < KN; ++q) {
          lr[q] = lr[q + 1];
          lj[q] = lj[q + 1];
        }
        lr[KN - 1] = __builtin_inf();
        lj[KN - 1] = INT_MAX;
      }
    }
    // self last, (inf, row) in (r2, j) order: lanes past its slot shift up by one
    const int pslot = __popcll(__ballot(lane < KN && (rr < __builtin_inf() || (rr == __builtin_inf() && rj < row))));
    const double ur = __shfl_up(rr, 1);
    const int uj = __shfl_up(rj, 1);
    if (lane > pslot) {
      rr = ur;
      rj = uj;
    } else if (lane == pslot) {
      rr = __builtin_inf();
      rj = row;
    }
    const double vx = __shfl(me.vx, l), vy = __shfl(me.vy, l);
    if (lane < KN) {
      const size_t g = env0 + row;
      if (lane == KN - 1 && a.knn_r2) a.knn_r2[g] = static_cast<float>(rr);
      const int j = knn_slot_col(rj, N, row);  // unfilled slots (non-finite r2 only): self
      a.knn_idx[g * KN + lane] = j;
      const St o = load_state<DYN, UF64>(a, env0 + j);
      float4 ob;
      ob.x = static_cast<float>(px - o.px);
      ob.y = static_cast<float>(py - o.py);
      ob.z = static_cast<float>(vx - o.vx);
      ob.w = static_cast<float>(vy - o.vy);
      reinterpret_cast<float4*>(a.knn_obs)[g * KN + lane] = ob;
    }
  }
}

__device__ __forceinline__ double clip10(double v) {  // np.clip(v, -10, 10); NaN stays NaN
  return v < -10.0 ? -10.0 : (v > 10.0 ? 10.0 : v);
}

// float32 prefilter band for one threshold: a pair whose float32 r2 (from float32-
// rounded positions) is < lo is below the threshold in float64 too, one >= hi is not;
// pairs in [lo, hi) are decided exactly in float64. For coordinates bounded by Pi, Pj
// the float32 r2 is within 2^-20 (Pi + Pj + 4) of the float64 one.
struct Band {
  float lo, hi;
};

__device__ __forceinline__ Band make_band(double thr, double delta) {
  const double lo = thr - delta, hi = thr + delta;
  float l = static_cast<float>(lo), h = static_cast<float>(hi);
  if (static_cast<double>(l) > lo) l = nextafterf(l, -__builtin_inff());
  if (static_cast<double>(h) < hi) h = nextafterf(h, __builtin_inff());
  return {l, h};
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// float32 position of a staged float64 state (reads px, py only)
__device__ __forceinline__ float2 pos32(const St& s) {
  const double2 p = *reinterpret_cast<const double2*>(&s);
  return make_float2(static_cast<float>(p.x), static_cast<float>(p.y));
}

// pass 1's float32 squared distance of a row (xi, yi) to a wave's two columns
__device__ __forceinline__ f2v d2_f32(float xi, float yi, f2v qx, f2v qy) {
  const f2v dx = xi - qx, dy = yi - qy;
  return __builtin_elementwise_fma(dx, dx, dy * dy);
}

// A value the whole wave holds (compiler-visible as scalar).
__device__ __forceinline__ float uniform_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// v_writelane_b32 through the LLVM intrinsic (this clang has no __builtin for it), so
// the compiler applies the constant-bus and lane-select hazard rules itself.
extern "C" __device__ int gf_writelane_i32(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
// float64 -> uint32, saturating (negative and NaN -> 0, >= 2^32 -> 2^32 - 1): the
// hardware conversion itself (a plain cast is undefined outside the range, and the
// compiler's saturating form adds two compares and two selects)
__device__ __forceinline__ unsigned gf_cvt_u32_sat(double v) {
  unsigned r;
  asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// Minimum over aligned groups of S lanes (S a power of two): DPP lane swaps inside rows
// of 16 (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), shuffles beyond.
__device__ __forceinline__ unsigned dpp_u32(unsigned v, int ctrl) {
  switch (ctrl) {  // the control word must be a compile-time constant
    case 0xB1: return static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false));
    case 0x4E: return static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false));
    case 0x141: return static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x141, 0xF, 0xF, false));
    default: return static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x140, 0xF, 0xF, false));
  }
}
// group_min_u32 with the group size a compile-time constant (the fused kNN merge: a
// runtime S left a branch around every DPP step)
template <int S>
__device__ __forceinline__ unsigned group_min_u32c(unsigned w) {
  if constexpr (S > 1) w = min(w, dpp_u32(w, 0xB1));
  if constexpr (S > 2) w = min(w, dpp_u32(w, 0x4E));
  if constexpr (S > 4) w = min(w, dpp_u32(w, 0x141));
  if constexpr (S > 8) w = min(w, dpp_u32(w, 0x140));
#pragma unroll
  for (int o = 16; o < S; o <<= 1) w = min(w, static_cast<unsigned>(__shfl_xor(static_cast<int>(w), o)));
  return w;
}
// Sum over groups of S consecutive lanes (S a power of two), the xor butterfly's tree:
// DPP lane swaps (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror) give each
// lane the same partial sums a shfl_xor by 1, 2, 4, 8 would (the lanes of each half group
// already agree), so every lane ends with identical bits and the same order of additions,
// without the LDS round trips of ds_bpermute.
__device__ __forceinline__ double dpp_f64(double v, int ctrl) {
  const int lo = static_cast<int>(dpp_u32(static_cast<unsigned>(__double2loint(v)), ctrl));
  const int hi = static_cast<int>(dpp_u32(static_cast<unsigned>(__double2hiint(v)), ctrl));
  return __hiloint2double(hi, lo);
}
template <int S, class V>
__device__ __forceinline__ V group_sum_c(V v) {
  if constexpr (sizeof(V) == 8) {
    if constexpr (S > 1) v += dpp_f64(v, 0xB1);
    if constexpr (S > 2) v += dpp_f64(v, 0x4E);
    if constexpr (S > 4) v += dpp_f64(v, 0x141);
    if constexpr (S > 8) v += dpp_f64(v, 0x140);
  } else {
    if constexpr (S > 1) v += static_cast<V>(dpp_u32(static_cast<unsigned>(v), 0xB1));
    if constexpr (S > 2) v += static_cast<V>(dpp_u32(static_cast<unsigned>(v), 0x4E));
    if constexpr (S > 4) v += static_cast<V>(dpp_u32(static_cast<unsigned>(v), 0x141));
    if constexpr (S > 8) v += static_cast<V>(dpp_u32(static_cast<unsigned>(v), 0x140));
  }
#pragma unroll
  for (int o = 16; o < S; o <<= 1) v += __shfl_xor(v, o);
  return v;
}
// Exact (r2, j) order of the small-env kNN (KX): a pair's key is the bit pattern of its
// float64 r2 (non-negative, so the bits order as the values; +inf for the diagonal, as
// the reference's r2, and every NaN as one canonical NaN above +inf, where argsort puts
// NaN), ties broken by the lower index.
__device__ __forceinline__ unsigned long long r2_key(double r2) {
  return r2 != r2 ? 0x7FF8000000000000ull : static_cast<unsigned long long>(__double_as_longlong(r2));
}
// Insert (key, j) into the ascending list (kk, kj) of L entries, keeping its L smallest;
// columns arrive in ascending j, so an equal key keeps the listed (lower) index first.
template <int L>
__device__ __forceinline__ void key_insert_asc(unsigned long long (&kk)[L], int (&kj)[L], unsigned long long key, int j) {
  if (key < kk[L - 1]) {
    bool prev = false;
    unsigned long long pk = 0;
    int pj = 0;
#pragma unroll
    for (int m = 0; m < L; ++m) {
      const bool sw = key < kk[m];
      const unsigned long long ok = kk[m];
      const int oj = kj[m];
      kk[m] = sw ? (prev ? pk : key) : ok;
      kj[m] = sw ? (prev ? pj : j) : oj;
      prev = sw;
      pk = ok;
      pj = oj;
    }
  }
}
// (key, j) minimum over aligned groups of S lanes (S a power of two): DPP lane swaps
// within rows of 16, shuffles beyond; every lane of a group ends with the group's minimum.
template <int S>
__device__ __forceinline__ void group_min_key(unsigned long long& k, int& j) {
  auto take = [&](unsigned long long ok, int oj) {
    if (ok < k || (ok == k && oj < j)) {
      k = ok;
      j = oj;
    }
  };
  auto dstep = [&](int ctrl) {
    const unsigned lo = dpp_u32(static_cast<unsigned>(k), ctrl), hi = dpp_u32(static_cast<unsigned>(k >> 32), ctrl);
    take((static_cast<unsigned long long>(hi) << 32) | lo, static_cast<int>(dpp_u32(static_cast<unsigned>(j), ctrl)));
  };
  if constexpr (S > 1) dstep(0xB1);
  if constexpr (S > 2) dstep(0x4E);
  if constexpr (S > 4) dstep(0x141);
  if constexpr (S > 8) dstep(0x140);
#pragma unroll
  for (int o = 16; o < S; o <<= 1) {
    const unsigned long long ok = __shfl_xor(k, o);
    take(ok, __shfl_xor(j, o));
  }
}
// f(std::integral_constant<int, S>) for the runtime slice count S in {4, 8, 16, 32, 64}
template <class F>
__device__ __forceinline__ void with_slices(int S, F&& f) {
  switch (S) {
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 16: f(std::integral_constant<int, 16>{}); break;
    case 32: f(std::integral_constant<int, 32>{}); break;
    default: f(std::integral_constant<int, 64>{}); break;
  }
}
__device__ __forceinline__ int wid_of(unsigned tid) { return __builtin_amdgcn_readfirstlane(tid >> 6); }

// Lane l of (w0, w1) takes the wave-uniform 64-bit mask m.
// Flocking-v0 predicted row's candidate bound: float32 d2 < bound covers every agent with
// r2 < th (float32 error of d2 at |d| <= sqrt(th): 2^-23 |d| (Pi + Pj + |d|) + 2^-22 r2,
// taken x8); -1 (no candidates) at huge coordinates (those rows go to the rim kNN)
__device__ __forceinline__ float cand_bound(float th, float pu) {
  float tcr = -1.f;
  if (th > 0.f && pu < 1.0e5f) {
    const double t = th;
    const double dc = ldexp((static_cast<double>(pu) + 4.0) * (sqrt(t) + 1.0) + t, -20);
    tcr = static_cast<float>(t + dc);
    if (static_cast<double>(tcr) < t + dc) tcr = nextafterf(tcr, __builtin_inff());
  }
  return tcr;
}

__device__ __forceinline__ void put_lane(unsigned& w0, unsigned& w1, uint64_t m, int l) {
  w0 = static_cast<unsigned>(gf_writelane_i32(static_cast<int>(m), l, static_cast<int>(w0)));
  w1 = static_cast<unsigned>(gf_writelane_i32(static_cast<int>(m >> 32), l, static_cast<int>(w1)));
}

// Dense network rows adj/deg of one row block (flocking_relative.py:120-122), 16-byte
// stores (1 KiB per wave instruction); the block's rows are one contiguous range
// starting at global row grow0.
__device__ __forceinline__ void store_network_rows(const StepArgs& a, const uint64_t* adj, const float* inv,
                                                   f4v* stab, int Wn, size_t grow0, int nrows, int wid, int lane,
                                                   bool knn) {
  const int N = a.N;
  const bool vec4 = (N & 3) == 0;
  // wave w writes the contiguous rows [w*R/4, (w+1)*R/4): the 4 waves' concurrent
  // stores land R/4 rows apart (212 vs 215 us with rows w, w+4, ... at config 2)
  const int per = (nrows + 3) >> 2;
  // fast form (N % 1024 == 0): every lane owns float4 columns lane + 64m of a row, so
  // its nibble sits at a fixed bit offset of 32-bit words 8 apart; four words are read
  // ahead and each nibble selects a float4 from the row's table (below).
  // The host picks it per kernel (StepArgs.store_fast; diag 64 / 128 force it off / on);
  // the fused-kNN step always takes it: 10 VALU per 4 KiB of a wave instead of ~64 (the
  // kNN step is bound by its VALU issue more than the plain step, which measured the
  // fast loop slower: 164.1 vs 161.5 us, the kNN step 195 vs 207, profiles/r04)
  const bool fast = (N & 1023) == 0 && !GF_ABLATE(a, (4 | 64)) && (a.store_fast || knn || GF_ABLATE(a, 128));
  const unsigned* bits32 = reinterpret_cast<const unsigned*>(adj);
  const int hl = lane & 15;
  const int wsel = 2 * (lane >> 4) + (hl >> 3);  // 32-bit word of column block m = 0
  const int o0 = (hl & 7) << 2;                  // bit offset of this lane's nibble
  for (int m = 0; m < per; ++m) {
    const int r = wid * per + m;
    if (r >= nrows) break;
    const float iv = inv[r];
    const uint64_t* bits = adj + (size_t)r * Wn;
    float* rowp = a.network + (grow0 + r) * (size_t)N;
    if (GF_ABLATE(a, 1024)) {  // timing only: constant rows, no bit reads
      f4v* r4 = reinterpret_cast<f4v*>(rowp);
      for (int q = lane; q < (N >> 2); q += 64) r4[q] = f4v{iv, 0.f, iv, 0.f};
      continue;
    }
    if (fast) {
      // the row's 16 float4 values by nibble in the wave's LDS table (a wave's LDS
      // operations run in order: the previous row's reads precede this write, and this
      // write the reads below), then per float4 one bit-field extract and one address
      f4v* tab = stab + wid * kStoreTab;
      if (lane < kStoreTab)
        tab[lane] = f4v{(lane & 1) ? iv : 0.0f, (lane & 2) ? iv : 0.0f, (lane & 4) ? iv : 0.0f, (lane & 8) ? iv : 0.0f};
      const unsigned* wr = bits32 + (size_t)r * 2 * Wn + wsel;
      f4v* dst = reinterpret_cast<f4v*>(rowp) + lane;
#pragma unroll 1
      for (int c = 0; c < (N >> 8); c += 4) {
        unsigned w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = wr[8 * (c + k)];
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[64 * (c + k)] = tab[__builtin_amdgcn_ubfe(w[k], o0, 4)];
      }
    } else if (vec4) {
      f4v* r4 = reinterpret_cast<f4v*>(rowp);
      const int nq = N >> 2;
      for (int q = lane; q < nq; q += 64) {
        const unsigned nib = static_cast<unsigned>(bits[q >> 4] >> ((q & 15) << 2)) & 0xFu;
        const f4v v = {(nib & 1u) ? iv : 0.0f, (nib & 2u) ? iv : 0.0f, (nib & 4u) ? iv : 0.0f,
                       (nib & 8u) ? iv : 0.0f};
        if (GF_ABLATE(a, 4))
          __builtin_nontemporal_store(v, &r4[q]);
        else
          r4[q] = v;
      }
    } else {
      for (int c = lane; c < N; c += 64) rowp[c] = ((bits[c >> 6] >> (c & 63)) & 1ull) ? iv : 0.0f;
    }
  }
}

// Per-row outputs of a row block once its features are summed: the S slices of each
// row combined, state_values (:124-129), the updated state, the controller (:194-226)
// and, by the env's first block, the reward (instant_cost :145-147). `writer` = the
// thread holding slice 0 of a valid row.
template <bool DYN, bool UF64, bool CTRL, bool VAR>
__device__ __forceinline__ void step_epilogue(const StepArgs& a, const St* tile, double* red, const St& me,
                                              double f0, double f1, double f2, double f3, double f4,
                                              double f5, double gx, double gy, double svx, double svy, int b,
                                              int i0, int i_row, bool writer, int S, int tid) {
  const int N = a.N, T = a.T;
  const size_t env0 = (size_t)b * N;
  // combine the S slices of each row (butterfly: identical bits in every lane)
  with_slices(S, [&](auto Sc) {
    constexpr int SS = decltype(Sc)::value;
    f0 = group_sum_c<SS>(f0);
    f1 = group_sum_c<SS>(f1);
    f2 = group_sum_c<SS>(f2);
    f3 = group_sum_c<SS>(f3);
    f4 = group_sum_c<SS>(f4);
    f5 = group_sum_c<SS>(f5);
    if constexpr (CTRL) {
      gx = group_sum_c<SS>(gx);
      gy = group_sum_c<SS>(gy);
    }
  });

  // every thread summed its share of the env's velocities while staging the tiles
  const double Svx = block_sum(svx, red), Svy = block_sum(svy, red);

  if (writer && !GF_ABLATE(a, 256)) {  // diag 256: skip the per-row outputs (timing only)
    const size_t g = env0 + i_row;
    if (a.state_values) {
      float* sv = a.state_values + g * 6;
      sv[0] = static_cast<float>(f0);
      sv[1] = static_cast<float>(f1);
      sv[2] = static_cast<float>(f2);
      sv[3] = static_cast<float>(f3);
      sv[4] = static_cast<float>(f4);
      sv[5] = static_cast<float>(f5);
    }
    if constexpr (DYN) {
      double2* xo = reinterpret_cast<double2*>(a.x_out) + 2 * g;
      xo[0] = double2{me.px, me.py};
      xo[1] = double2{me.vx, me.vy};
    }
    if constexpr (CTRL) {
      // centralized: sum over ALL j of (v_i - v_j) = N*v_i - sum_j v_j (:200-208)
      double p2 = a.centralized ? static_cast<double>(N) * me.vx - Svx : f0;
      double p3 = a.centralized ? static_cast<double>(N) * me.vy - Svy : f3;
      if (VAR && a.centralized && a.n_vel_zero > 0) {
        // obstacle variant: only pairs between free agents count (flocking_obstacle.py:79-80)
        const int nz = min(a.n_vel_zero, N);
        double zx = 0, zy = 0;
        for (int j = 0; j < nz; ++j) {
          const St s = load_state<DYN, UF64, VAR>(a, env0 + j);
          zx += s.vx;
          zy += s.vy;
        }
        const bool frozen = i_row < nz;
        p2 = frozen ? 0.0 : static_cast<double>(N - nz) * me.vx - (Svx - zx);
        p3 = frozen ? 0.0 : static_cast<double>(N - nz) * me.vy - (Svy - zy);
      }
      double2 u;
      u.x = clip10(-gx - p2) / a.action_scalar;  // (-p4 - p2), :209-211
      u.y = clip10(-p3 - gy) / a.action_scalar;  // (-p3 - p5)
      if (VAR && a.ctrl_clip > 0) {  // stochastic variant (flocking_stoch.py:44-45)
        u.x = clip_sym(u.x, a.ctrl_clip);
        u.y = clip_sym(u.y, a.ctrl_clip);
      }
      reinterpret_cast<double2*>(a.ctrl_out)[g] = u;
    }
  }

  // instant_cost (:145-147) = -(var(vx) + var(vy)), two-pass like np.var, by the env's
  // first row block; single-tile envs read the velocities from the LDS tile
  if (a.reward && i0 == 0 && !GF_ABLATE(a, 512)) {  // diag 512: skip the reward (timing only)
    const double mx = Svx / static_cast<double>(N), my = Svy / static_cast<double>(N);
    double qx = 0, qy = 0;
    if (N <= T) {
      for (int t = tid; t < N; t += kThreads) {
        const double ex = tile[t].vx - mx, ey = tile[t].vy - my;
        qx += ex * ex;
        qy += ey * ey;
      }
    } else {
      for (int j = tid; j < N; j += kThreads) {
        const St s = load_state<DYN, UF64, VAR>(a, env0 + j);
        const double ex = s.vx - mx, ey = s.vy - my;
        qx += ex * ex;
        qy += ey * ey;
      }
    }
    const double Qx = block_sum(qx, red);
    const double Qy = block_sum(qy, red);
    if (tid == 0) {
      const double rw = -1.0 * (Qx / static_cast<double>(N) + Qy / static_cast<double>(N));
      a.reward[b] = rw;
      if (a.reward2) a.reward2[b] = rw;
    }
  }
}

// ---------------------------------------------------------------------------------
// The fused step: DYN = apply dynamics (step) or not (compute_helpers on the current
// state: reset / standalone controller), UF64 = action dtype, CTRL = also controller().
// Waves per SIMD the register allocation must allow: 7 for the plain step (71 VGPRs,
// no spills; its LDS is floored to hold it at 6 workgroups per CU, see
// kStepLdsPlainFloor), 6 with the controller (79 VGPRs, 23.2 KiB of LDS: 6 per CU);
// variants are not capped (their extra state would spill).
#ifndef GF_WAVES_KNN  // register studies (scripts/vgpr_phases.sh) may raise it
#define GF_WAVES_KNN 5
#endif
constexpr int kWavesPlain = 6, kWavesPf = 4, kWavesCtrl = 6, kWavesKnn = GF_WAVES_KNN, kWavesKnnCtrl = 4;
// Phase timeline instrumentation (diagnostic builds only, -DGF_STAMPS): lane 0 of
// wave 0 records s_memrealtime (100 MHz) at phase boundaries of each workgroup, plus
// its HW_ID / XCC_ID, for scripts/phase_timeline.py. Product builds compile it out.
#ifdef GF_STAMPS
__device__ unsigned long long gf_stamp_buf[8192 * 16];
#define GF_STAMP(k)                                                                     \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                          \
      gf_stamp_buf[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime();           \
  } while (0)
#else
#define GF_STAMP(k) ((void)0)
#endif

// VAR: the flocking variants' switches (StepArgs.variant); without it the FlockingRelative
// path carries none of their instructions.
// PF (1 or 2): each tile's global loads are issued PF tiles ahead (raw x/u in registers,
// T <= 2 * kThreads), for envs of many tiles; its register budget is that of 4 waves.
// KN > 0 (Flocking-v0, flocking.py:20-25): each (row, slice) thread also keeps the KN
// smallest keys of its neighbours, the S slices of a row are merged after the last
// feature pass, and the row's k nearest indices and observation are written (below).
// UIN: the drop-in step of a small env with its actions in the kernel arguments
// (StepArgsU): they arrive with the dispatch instead of being read over the link from
// page-locked host memory, one dependent round trip per workgroup fewer.
// KX > 0 (Flocking-v0 in an env of one tile, N <= kStepExactKnnMax; KN == 0): after the
// epilogue every row is ranked exactly against the whole env, staged in LDS as the tile
// (below): no keys in the feature pass, no unranked rows, no rim kernel.
template <bool DYN, bool UF64, bool CTRL, bool VAR, int PF = 0, int KN = 0, bool UIN = false, int KX = 0>
__global__ __launch_bounds__(kThreads, VAR ? 1
                                           : (PF ? kWavesPf
                                                 : (KN ? (CTRL ? kWavesKnnCtrl : kWavesKnn)
                                                       : (CTRL ? kWavesCtrl : kWavesPlain))))
void flock_step_kernel(typename std::conditional<UIN, StepArgsU, StepArgs>::type p) {
  [[maybe_unused]] StepArgs uargs;
  if constexpr (UIN) {
    uargs = p.a;
    uargs.u = p.u;
  }
  const StepArgs& a = *[&]() -> const StepArgs* {
    if constexpr (UIN) return &uargs;
    else return &p;
  }();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N, R = a.R, T = a.T;
  const int Wn = (N + 63) >> 6;  // adjacency words per row (whole env)
  const int Wt = T >> 6;         // words per row of one tile
  // the plain step deals the reward blocks out first (195 vs 200 us at config 2; with
  // the controller it measured 1 us slower); diag 8192 forces the plain remap (A/B)
  const int L = (!CTRL && !GF_ABLATE(a, 8192)) ? xcd_remap_reward_first(blockIdx.x, gridDim.x, a.bpe)
                                            : xcd_remap(blockIdx.x, gridDim.x);
  const int b = L / a.bpe;
  const int i0 = (L - b * a.bpe) * R;
  f4v* stab = reinterpret_cast<f4v*>(smem);                    // 4 x 16 network-row table entries
  float2* rxy = reinterpret_cast<float2*>(stab + 4 * kStoreTab);  // R rows' float32 positions
  St* tile = reinterpret_cast<St*>(smem + 4 * kStoreTab * 16 + ((R * 8 + 31) & ~31));  // float64 state, T
  St* rows = tile + T;                                         // this block's rows, R
  uint64_t* adj = reinterpret_cast<uint64_t*>(rows + R);       // R x Wn adjacency bits
  // the controller without kNN (kOuter): pass 1 leaves in adj the float32 superset of both
  // the adjacency and the controller's "near" pairs, and the feature pass decides both
  // exactly in float64 (it computes every such pair's r2 anyway), writing the exact
  // adjacency words back; the fused-kNN controller keeps separate near bits
  constexpr bool kOuter = CTRL && KN == 0;
  // Flocking-v0 without the controller (kSupK): pass 1 leaves the float32 superset of the
  // adjacency (one compare per pair, no band sweep); the feature pass, which computes
  // every such pair's float64 r2 to rank it, decides the adjacency exactly and writes the
  // exact words back, so every tile's feature pass runs before the network stores
  constexpr bool kSupK = KN > 0 && !CTRL;
  constexpr bool kSup = kOuter || kSupK;
  uint64_t* nearb = adj + (size_t)R * Wn;                      // R x Wt controller bits (KN && CTRL)
  uint64_t* candb = nearb + ((CTRL && !kOuter) ? (size_t)R * Wt : 0);  // (predicted rows) x Wt kNN candidates
  double* red = reinterpret_cast<double*>(candb + (KN ? (size_t)R * Wt : 0));
  float* redf = reinterpret_cast<float*>(red + 4);
  float* inv = reinterpret_cast<float*>(red + 8);
  [[maybe_unused]] float* rthr = inv + R;                      // R kNN candidate radii^2 (0: none)
  // each wave's copy of the rows' candidate bounds (read as LDS broadcasts)
  // and the block's predicted rows in order (prow[p]: the p-th predicted row)
  [[maybe_unused]] float* ptc = rthr + R + wid_of(threadIdx.x) * R;
  [[maybe_unused]] int* prow = reinterpret_cast<int*>(rthr + 5 * R);

  const int nrows = min(R, N - i0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const size_t env0 = (size_t)b * N;
  GF_STAMP(0);
#ifdef GF_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 8192) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    gf_stamp_buf[blockIdx.x * 16 + 15] = (static_cast<unsigned long long>(xcc) << 32) | hw;
  }
#endif

  // PF: the loads of the tiles PF ahead are in flight (pfa: even tiles, pfb: odd ones
  // when PF == 2), the first ones issued before the rows' loads
  [[maybe_unused]] RawState<UF64> pfa[2], pfb[2];
  auto issue = [&](int j, RawState<UF64>(&pf)[2]) {
    const int tn = min(T, N - j);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (tid + k * kThreads < tn) pf[k] = load_raw<DYN, UF64>(a, env0 + j + tid + k * kThreads);
  };
  if constexpr (PF >= 1) issue(0, pfa);
  if constexpr (PF == 2) {
    if (T < N) issue(T, pfb);
  }

  // kNN: lane r's row's k-th nearest r2 two states back (predicted rows, below), loaded
  // before everything else: issued later, its round trip sat between the tile loads and
  // pass 1 of every workgroup
  [[maybe_unused]] float khist = 0.f;
  if constexpr (KN > 0) {
    if (lane < nrows && a.knn_r2) khist = a.knn_r2[env0 + i0 + lane];
  }

  // rows owned by this workgroup (post-update state). An env of one tile takes them from
  // the tile's staging instead (below): one dependent round trip fewer, which the
  // drop-in step pays over the link when its actions are read from page-locked host memory
  const bool one_tile = N <= T;
  if (!one_tile)
    for (int r = tid; r < nrows; r += kThreads) rows[r] = load_state<DYN, UF64, VAR>(a, env0 + i0 + r);

  // feature-pass thread mapping: S word-slices per row
  const int S = kThreads / R;
  const int fr = tid / S, fs = tid - fr * S;
  const bool frow = fr < nrows;
  double f0 = 0, f1 = 0, f2 = 0, f3 = 0, f4 = 0, f5 = 0, gx = 0, gy = 0;
  double svx = 0, svy = 0;  // partial sums of the env's velocities (controller, reward)
  float rx32 = 0.f, ry32 = 0.f, Pr = 0.f;  // lane r: row r's float32 position; rows' max |coord|
  // kNN rows predicted to lack k neighbours (their k-th nearest two states back was
  // at >= 0.8 comm_radius): predm (wave-uniform) marks them, rthr[r] holds row r's
  // candidate radius^2 thr
  [[maybe_unused]] uint64_t predm = 0;

  const int i_row = i0 + fr;  // global row of this thread's feature slice
  // Fused k-nearest selection (KN > 0). Every pair the feature pass visits is ranked:
  // the neighbours and, for a predicted row, its candidates: agents whose float32 d2
  // is below a bound covering every agent with r2 < thr (2.25 x the row's k-th nearest
  // r2 two states back, knn_r2). The ranked set thus holds every agent with
  // r2 < Tr = max(thr, comm_radius^2). A pair's key is
  //   (q << jbits) | j,  q = min(floor(r2 * 2^qbits / Tr), 2^qbits - 2),
  // a 32-bit integer whose order is (q, j): q never decreases as r2 grows, so keys of
  // different q are in true (r2, j) order. Each thread keeps its KL smallest keys sorted
  // (a min/max exchange chain, 2 VALU per entry, no branches); a slice with more keys
  // drops its largest. A drop matters only if the dropped key is among the row's KN + 1
  // smallest (agents indexed in spatial order put a row's nearest in one slice); the
  // merge detects the only way that can happen and leaves such a row unranked. (Lists
  // of 4 or 5 measured no faster: with 4, ~1 % of the rows hold 5 of their 8 nearest in
  // one slice and fall to the exact scan.)
  constexpr int KL = KN > 0 ? KN : 1;
  [[maybe_unused]] unsigned kk[KL];
  if constexpr (KN > 0) {
#pragma unroll
    for (int m = 0; m < KL; ++m) kk[m] = 0xFFFFFFFFu;
  }
  // one neighbour pair (row fr = me, tile column c): features and controller gradient.
  // The row's state is read from LDS per feature pass, so it holds no registers
  // through pass 1.
  auto pair_terms = [&](const St& me, int j0, int c, bool isadj, bool isnear, double ksc) {
    const St o = tile[c];
    const double dx = me.px - o.px, dy = me.py - o.py;
    const double r2 = dx * dx + dy * dy;
    if constexpr (kOuter) {  // a pass-1 candidate: both decisions exactly (:117, :225)
      isadj = r2 < a.cr2;
      isnear = r2 <= a.cr;
      if (!isadj && !isnear) return isadj;
    }
    if constexpr (kSupK) isadj = r2 < a.cr2;  // a superset or candidate bit: decided here (:117)
    if constexpr (KN > 0) {
      if (!GF_ABLATE(a, 0x200000)) {  // diag 0x200000: no insertion (timing only)
        // q = min(ceil(r2 * ksc), qmax): qmax - (qmax - r2 * ksc truncated; negative or
        // NaN converts to 0), so a NaN r2 ranks last. ceil or floor, q never decreases as
        // r2 grows, and q <= qmax - 2 still means r2 < Tr (the merge's test (a)).
        const unsigned q = a.knn_qmax - gf_cvt_u32_sat(fma(-r2, ksc, a.knn_qmaxd));
        knn_list_insert<KL>(kk, (q << a.knn_jbits) | static_cast<unsigned>(j0 + c));
      }
      if (!isadj && !(CTRL && isnear)) return isadj;  // a candidate only: no features
    }
    // one reciprocal per pair: q = d / r2, d / r2^2 from 1/r2 (a few ulp from the
    // reference's two divisions; far inside the float32 outputs' tolerance)
    // the controller (rtol 1e-9 on its output) keeps the IEEE division: v_rcp_f64 with one
    // or two Newton steps measured the same (174.3 / 175.0 / 174.6 us per config-2 step,
    // profiles/r04/ab_ctrl_recip.txt)
    // diag 2048: the controller with the plain step's reciprocal (instruction counts only)
    const double ir = (CTRL && !GF_ABLATE(a, 2048)) ? 1.0 / r2 : recip_f64(r2), irr = ir * ir;
    const double q1x = dx * irr, q2x = dx * ir;
    const double q1y = dy * irr, q2y = dy * ir;
    if (isadj) {
      // obstacle variant: no velocity difference for pairs touching agents < nvz
      const bool vz = VAR && (i_row < a.n_vel_zero || j0 + c < a.n_vel_zero);
      f0 += vz ? 0.0 : me.vx - o.vx;
      f1 += q1x;
      f2 += q2x;
      f3 += vz ? 0.0 : me.vy - o.vy;
      f4 += q1y;
      f5 += q2y;
    }
    if constexpr (CTRL) {
      if (isnear && (a.centralized || isadj) && !GF_ABLATE(a, 4096)) {  // diag 4096: no gradient sums
        gx += (-2.0 * q1x) + (2.0 * q2x);
        gy += (-2.0 * q1y) + (2.0 * q2y);
      }
    }
    return isadj;
  };

  // pass 2: features / gradients for the set bits of one tile, ascending j per slice.
  // (Dealing a row's bits round robin over its S threads balances the slices but its
  // cursor bookkeeping cost more than it saved: 266 vs 215 us, DESIGN.md.)
  auto feature_pass = [&](int j0, int nch) {
    if (!frow || GF_ABLATE(a, 2)) return;
    const St me = rows[fr];
    // kNN: this row's candidate words (predicted rows) and key scale 2^qbits / Tr
    [[maybe_unused]] const uint64_t* crow = nullptr;
    [[maybe_unused]] double ksc = 0.0;
    if constexpr (KN > 0) {
      const bool pr = (predm >> fr) & 1ull;
      crow = pr ? candb + (size_t)__popcll(predm & ((1ull << fr) - 1ull)) * Wt : nullptr;
      ksc = a.knn_qscale / (pr ? fmax(static_cast<double>(rthr[fr]), a.cr2) : a.cr2);
    }
    const int wpt = (nch + S - 1) / S;
    const int wb = fs * wpt, we = min(nch, wb + wpt);
    for (int w = wb; w < we; ++w) {
      uint64_t* aw = adj + (size_t)fr * Wn + (j0 >> 6) + w;
      const uint64_t am = *aw;
      if constexpr (kOuter) {  // candidates in, the exact adjacency word out
        uint64_t m = am, ex = 0;
        while (m) {
          const int k = __builtin_ctzll(m);
          m &= m - 1;
          if (pair_terms(me, j0, (w << 6) + k, false, false, ksc)) ex |= 1ull << k;
        }
        *aw = ex;
        continue;
      }
      const uint64_t cm = (KN && crow) ? crow[w] : 0ull;
      if constexpr (kSupK) {  // superset and candidates in, the exact adjacency word out
        // am covers the adjacency, so clearing the bit of every pair found not adjacent
        // (the rare float32 superset pairs past comm_radius, and a predicted row's
        // candidates, whose bits may not be set) leaves the exact word; an LDS atomic
        // keeps it a branch that no wave enters unless one of its lanes has such a pair
        uint64_t m = am | cm;
        while (m) {
          const int k = __builtin_ctzll(m);
          m &= m - 1;
          if (!pair_terms(me, j0, (w << 6) + k, false, false, ksc))
            __hip_atomic_fetch_and(aw, ~(1ull << k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        continue;
      }
      const uint64_t nm = CTRL ? nearb[(size_t)fr * Wt + w] : 0ull;
      uint64_t m = am | nm | cm;
      while (m) {
        const int k = __builtin_ctzll(m);
        m &= m - 1;
        // without the controller and the kNN candidates every iterated bit is a neighbour
        pair_terms(me, j0, (w << 6) + k, (!CTRL && KN == 0) || ((am >> k) & 1ull), CTRL && ((nm >> k) & 1ull), ksc);
      }
    }
  };

  auto tile_body = [&](const int j0, RawState<UF64>(&pf)[2]) {
    const int tc = min(T, N - j0);
    __syncthreads();  // previous tile fully consumed; rows[] visible on first pass
    [[maybe_unused]] const int ti = j0 / T;
    if (ti == 0) GF_STAMP(1);
    float pt = 0.f;
    auto stage = [&](int t, const St& s) {
      tile[t] = s;
      if (one_tile && static_cast<unsigned>(t - i0) < static_cast<unsigned>(nrows)) rows[t - i0] = s;
      const float fx = static_cast<float>(s.px), fy = static_cast<float>(s.py);
      pt = fmaxf(pt, fmaxf(fabsf(fx), fabsf(fy)));
      svx += s.vx;
      svy += s.vy;
    };
    if constexpr (PF >= 1) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (tid + k * kThreads < tc) stage(tid + k * kThreads, state_from_raw<DYN, UF64>(a, pf[k]));
      if (j0 + PF * T < N) issue(j0 + PF * T, pf);
    } else {
      for (int t = GF_ABLATE(a, 16) ? tc : tid; t < tc; t += kThreads)
        stage(t, load_state<DYN, UF64, VAR>(a, env0 + j0 + t));
    }
    if (j0 == 0) {
      if (one_tile) __syncthreads();  // rows[] written by the staging threads
      if (lane < nrows) {
        const St ri = rows[lane];
        rx32 = static_cast<float>(ri.px);
        ry32 = static_cast<float>(ri.py);
        if (wid == 0) rxy[lane] = make_float2(rx32, ry32);
      } else if ((!CTRL || kOuter) && wid == 0 && lane < ((nrows + 3) & ~3)) {
        rxy[lane] = make_float2(-1.0e18f, -1.0e18f);  // pass 1's padding rows (far away)
      }
      Pr = wave_max(fmaxf(fabsf(rx32), fabsf(ry32)));
      if constexpr (KN > 0) {
        const float h = khist;
        // diag 0x20000: no predicted rows (timing only)
        const bool pr = h >= static_cast<float>(0.64 * a.cr2) && h < 1.0e30f && !GF_ABLATE(a, 0x20000);
        predm = __ballot(pr);
        if (wid == 0 && lane < nrows) rthr[lane] = pr ? 2.25f * h : 0.f;
        if (wid == 0 && predm) {  // lane p: the p-th predicted row (published by block_max)
          int rp = 0, p = 0;
          for (uint64_t pm = predm; pm; pm &= pm - 1, ++p)
            if (lane == p) rp = __builtin_ctzll(pm);
          if (lane < nrows) prow[lane] = rp;
        }
      }
    }
    const float Pt = block_max(pt, redf);  // also the barrier that publishes the tile
    if (ti < 2) GF_STAMP(2 + 3 * ti);

    // pass 1: adjacency (and controller "near") bits. A wave takes 128 columns (lane
    // j and j+64, packed float32 math) and loops over the block's rows; the compare
    // masks are the bit words, collected so that lane r ends up holding row r's words.
    // float32 decides every pair outside the error band (make_band); if any pair of
    // the chunk falls inside it, the rows are swept again deciding those in float64.
    const int nch = (tc + 63) >> 6;
    const int npair = (nch + 1) >> 1;
    const float pu = uniform_f(Pr) + uniform_f(Pt);
    Band ba{-__builtin_inff(), __builtin_inff()}, bn = ba;  // huge/non-finite: all exact
    if (pu < 1.0e5f) {
      const double delta = ldexp(static_cast<double>(pu) * (1.0 + 1e-6) + 4.0, -20);
      ba = make_band(a.cr2, delta);
      bn = make_band(a.cr, delta);
    }
    ba.lo = uniform_f(ba.lo); ba.hi = uniform_f(ba.hi);
    bn.lo = uniform_f(bn.lo); bn.hi = uniform_f(bn.hi);
    // row r's float32 position: an LDS broadcast (no VALU)
    auto row_pos = [&](int r) { return rxy[r]; };
    for (int cp = GF_ABLATE(a, 8) ? npair : wid; cp < npair; cp += 4) {
      const int ca = cp << 1;
      const bool has_b = ca + 1 < nch;
      const int jta = (ca << 6) + lane, jtb = jta + 64;
      const bool va = jta < tc, vb = jtb < tc;
      // float32 positions from the tile's float64 states (no float32 copy is staged);
      // columns past the tile sit far away: never adjacent, never in the band
      const float2 qa = va ? pos32(tile[jta]) : make_float2(1.0e18f, 1.0e18f);
      const float2 qb = vb ? pos32(tile[jtb]) : make_float2(1.0e18f, 1.0e18f);
      const f2v qx = {qa.x, qb.x}, qy = {qa.y, qb.y};
      unsigned wa0 = 0, wa1 = 0, wb0 = 0, wb1 = 0, na0 = 0, na1 = 0, nb0 = 0, nb1 = 0;
      uint64_t band = 0;
      // most rows predicted: their candidate test rides on the adjacency loop's d2
      unsigned fca0 = 0, fca1 = 0, fcb0 = 0, fcb1 = 0;
      int fp = 0;
      bool fused = false;
      if constexpr (KN > 0) fused = 2 * __popcll(predm) >= nrows;
      // the rows' candidate bounds of this tile in the wave's LDS table
      [[maybe_unused]] float tcr_l = -1.f;
      if constexpr (KN > 0) {
        if (predm) {
          tcr_l = cand_bound(lane < nrows ? rthr[lane] : 0.f, pu);
          if (lane < nrows) ptc[lane] = tcr_l;  // read back by this wave only (in-order LDS)
        }
      }
      if constexpr (kSupK) {
        // one compare per column: the float32 superset of the adjacency (the feature pass
        // decides it exactly), plus the predicted rows' candidates when most rows are
        // predicted. Rows in pairs; the rows past nrows sit far away in rxy (columns past
        // the tile are masked: at huge coordinates ba.hi is +inf)
        const uint64_t vma = __ballot(va), vmb = __ballot(vb);
        auto srow = [&](int r, float2 pr) {
          const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
          put_lane(wa0, wa1, __ballot(!(d2.x >= ba.hi)) & vma, r);
          put_lane(wb0, wb1, __ballot(!(d2.y >= ba.hi)) & vmb, r);
          if (fused && ((predm >> r) & 1)) {  // wave-uniform
            const float tc = ptc[r];
            put_lane(fca0, fca1, __ballot(d2.x < tc), fp);
            put_lane(fcb0, fcb1, __ballot(d2.y < tc), fp);
            ++fp;
          }
        };
        const int nr4 = (nrows + 3) & ~3;
        for (int r = 0; r < nr4; r += 2) {
          const float2 p0 = rxy[r], p1 = rxy[r + 1];
          srow(r, p0);
          srow(r + 1, p1);
        }
      } else if (fused) {
        // rows in pairs (their LDS reads issued together), as the plain step; rows past
        // nrows sit far away in rxy and are never predicted
        auto frow = [&](int r, float2 pr) {
          const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
          const uint64_t Aa = __ballot(d2.x < ba.lo), Ab = __ballot(d2.y < ba.lo);
          const uint64_t Ma = __ballot(!(d2.x >= ba.hi)), Mb = __ballot(!(d2.y >= ba.hi));
          band |= (Aa ^ Ma) | (Ab ^ Mb);
          put_lane(wa0, wa1, Aa, r);
          put_lane(wb0, wb1, Ab, r);
          if constexpr (CTRL) {
            const uint64_t Na = __ballot(d2.x <= bn.lo), Nb = __ballot(d2.y <= bn.lo);
            const uint64_t NMa = __ballot(!(d2.x > bn.hi)), NMb = __ballot(!(d2.y > bn.hi));
            band |= (Na ^ NMa) | (Nb ^ NMb);
            put_lane(na0, na1, Na, r);
            put_lane(nb0, nb1, Nb, r);
          }
          if ((predm >> r) & 1) {  // wave-uniform
            const float tc = ptc[r];
            put_lane(fca0, fca1, __ballot(d2.x < tc), fp);
            put_lane(fcb0, fcb1, __ballot(d2.y < tc), fp);
            ++fp;
          }
        };
        if constexpr (!CTRL) {
          const int nr4 = (nrows + 3) & ~3;
          for (int r = 0; r < nr4; r += 2) {
            const float2 p0 = rxy[r], p1 = rxy[r + 1];
            frow(r, p0);
            frow(r + 1, p1);
          }
        } else {
          for (int r = 0; r < nrows; ++r) frow(r, row_pos(r));
        }
      } else if (kOuter) {
        // every pair within float32 reach of either threshold (r2 < cr^2 or r2 <= cr):
        // one compare per column, no band sweep; the feature pass decides them exactly.
        // Rows in pairs as the plain step; the rows past nrows sit far away in rxy.
        // (columns past the tile are masked: at huge coordinates ho is +inf)
        const float ho = uniform_f(fmaxf(ba.hi, bn.hi));
        const uint64_t vma = __ballot(va), vmb = __ballot(vb);
        auto orow = [&](int r, float2 pr) {
          const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
          put_lane(wa0, wa1, __ballot(!(d2.x > ho)) & vma, r);
          put_lane(wb0, wb1, __ballot(!(d2.y > ho)) & vmb, r);
        };
        const int nr4 = (nrows + 3) & ~3;
        for (int r = 0; r < nr4; r += 2) {
          const float2 p0 = rxy[r], p1 = rxy[r + 1];
          orow(r, p0);
          orow(r + 1, p1);
        }
      } else {
        auto row1 = [&](int r, float2 pr) {
          const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
          const uint64_t Aa = __ballot(d2.x < ba.lo), Ab = __ballot(d2.y < ba.lo);
          const uint64_t Ma = __ballot(!(d2.x >= ba.hi)), Mb = __ballot(!(d2.y >= ba.hi));
          band |= (Aa ^ Ma) | (Ab ^ Mb);
          put_lane(wa0, wa1, Aa, r);
          put_lane(wb0, wb1, Ab, r);
          if constexpr (CTRL) {
            const uint64_t Na = __ballot(d2.x <= bn.lo), Nb = __ballot(d2.y <= bn.lo);
            const uint64_t NMa = __ballot(!(d2.x > bn.hi)), NMb = __ballot(!(d2.y > bn.hi));
            band |= (Na ^ NMa) | (Nb ^ NMb);
            put_lane(na0, na1, Na, r);
            put_lane(nb0, nb1, Nb, r);
          }
        };
        if constexpr (!CTRL) {  // (the controller's budget would spill)
          // rows in pairs, their two LDS reads issued together (the compiler will not
          // unroll a loop of ballots by a runtime count); rows past nrows sit far away
          // in rxy: no bits, no band, and their lanes store nothing
          const int nr4 = (nrows + 3) & ~3;
          for (int r = 0; r < nr4; r += 2) {
            const float2 p0 = rxy[r], p1 = rxy[r + 1];
            row1(r, p0);
            row1(r + 1, p1);
          }
        } else {
          for (int r = 0; r < nrows; ++r) {
            const float2 pr = row_pos(r);
            const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
            const uint64_t Aa = __ballot(d2.x < ba.lo), Ab = __ballot(d2.y < ba.lo);
            const uint64_t Ma = __ballot(!(d2.x >= ba.hi)), Mb = __ballot(!(d2.y >= ba.hi));
            band |= (Aa ^ Ma) | (Ab ^ Mb);
            put_lane(wa0, wa1, Aa, r);
            put_lane(wb0, wb1, Ab, r);
            if constexpr (CTRL) {
              const uint64_t Na = __ballot(d2.x <= bn.lo), Nb = __ballot(d2.y <= bn.lo);
              const uint64_t NMa = __ballot(!(d2.x > bn.hi)), NMb = __ballot(!(d2.y > bn.hi));
              band |= (Na ^ NMa) | (Nb ^ NMb);
              put_lane(na0, na1, Na, r);
              put_lane(nb0, nb1, Nb, r);
            }
          }
        }
      }
      if (band) {  // rare: some pair is within the float32 error band of a threshold
        const St oa = va ? tile[jta] : St{1.0e300, 1.0e300, 0, 0};
        const St ob = vb ? tile[jtb] : St{1.0e300, 1.0e300, 0, 0};
        for (int r = 0; r < nrows; ++r) {
          const float2 pr = row_pos(r);
          const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
          const uint64_t Aa = __ballot(d2.x < ba.lo), Ab = __ballot(d2.y < ba.lo);
          const uint64_t Ma = __ballot(!(d2.x >= ba.hi)), Mb = __ballot(!(d2.y >= ba.hi));
          uint64_t Na = 0, Nb = 0, NMa = 0, NMb = 0;
          if constexpr (CTRL) {
            Na = __ballot(d2.x <= bn.lo);
            Nb = __ballot(d2.y <= bn.lo);
            NMa = __ballot(!(d2.x > bn.hi));
            NMb = __ballot(!(d2.y > bn.hi));
          }
          if ((Aa ^ Ma) | (Ab ^ Mb) | (Na ^ NMa) | (Nb ^ NMb)) {
            const St ri = rows[r];
            const double dxa = ri.px - oa.px, dya = ri.py - oa.py;
            const double dxb = ri.px - ob.px, dyb = ri.py - ob.py;
            const double r2a = dxa * dxa + dya * dya, r2b = dxb * dxb + dyb * dyb;
            put_lane(wa0, wa1, Aa | (__ballot(r2a < a.cr2) & (Aa ^ Ma)), r);
            put_lane(wb0, wb1, Ab | (__ballot(r2b < a.cr2) & (Ab ^ Mb)), r);
            if constexpr (CTRL) {
              put_lane(na0, na1, Na | (__ballot(r2a <= a.cr) & (Na ^ NMa)), r);
              put_lane(nb0, nb1, Nb | (__ballot(r2b <= a.cr) & (Nb ^ NMb)), r);
            }
          }
        }
      }
      if (lane < nrows) {
        // the diagonal (self, r2 = 0 here; inf in the reference) is never a neighbour
        const int dl = i0 + lane - (j0 + (ca << 6));
        const uint64_t ka = (static_cast<unsigned>(dl) < 64u) ? ~(1ull << dl) : ~0ull;
        const uint64_t kb = (static_cast<unsigned>(dl - 64) < 64u) ? ~(1ull << (dl - 64)) : ~0ull;
        uint64_t* arow = adj + (size_t)lane * Wn + (j0 >> 6) + ca;
        arow[0] = ((static_cast<uint64_t>(wa1) << 32) | wa0) & ka;
        if (has_b) arow[1] = ((static_cast<uint64_t>(wb1) << 32) | wb0) & kb;
        if constexpr (CTRL && !kOuter) {
          uint64_t* nrow = nearb + (size_t)lane * Wt + ca;
          nrow[0] = ((static_cast<uint64_t>(na1) << 32) | na0) & ka;
          if (has_b) nrow[1] = ((static_cast<uint64_t>(nb1) << 32) | nb0) & kb;
        }
      }
      if constexpr (KN > 0) {
        // the predicted rows' candidate words: lane p collects predicted row p's
        if (predm) {
          // row lane's candidate test: float32 d2 < tcr covers every agent with r2 < thr
          // (float32 error of d2 at |d| <= sqrt(thr): 2^-23 |d| (Pi + Pj + |d|) +
          // 2^-22 r2, taken x8); none at huge coordinates (those rows go to the rim kNN)
          unsigned ca0 = 0, ca1 = 0, cb0 = 0, cb1 = 0;
          int p = 0, rp = 0;
          if (fused) {
            ca0 = fca0; ca1 = fca1; cb0 = fcb0; cb1 = fcb1;
            p = fp;
          } else
          for (uint64_t pm = predm; pm; pm &= pm - 1, ++p) {
            const int r = __builtin_ctzll(pm);
            const float2 pr = row_pos(r);
            const float tc = ptc[r];
            const f2v d2 = d2_f32(pr.x, pr.y, qx, qy);
            put_lane(ca0, ca1, __ballot(d2.x < tc), p);
            put_lane(cb0, cb1, __ballot(d2.y < tc), p);
          }
          if (lane < p) {
            rp = prow[lane];
            const int dl = i0 + rp - (j0 + (ca << 6));
            const uint64_t ka = (static_cast<unsigned>(dl) < 64u) ? ~(1ull << dl) : ~0ull;
            const uint64_t kb = (static_cast<unsigned>(dl - 64) < 64u) ? ~(1ull << (dl - 64)) : ~0ull;
            uint64_t* crow = candb + (size_t)lane * Wt + ca;
            crow[0] = ((static_cast<uint64_t>(ca1) << 32) | ca0) & ka;
            if (has_b) crow[1] = ((static_cast<uint64_t>(cb1) << 32) | cb0) & kb;
          }
        }
      }
    }
    __syncthreads();
    if (ti < 2) GF_STAMP(3 + 3 * ti);

    // pass 2 (features) of every tile but the last runs here; the last tile's runs
    // after the network stores are issued, so the stores drain under it (kOuter: the
    // stores need the exact adjacency this pass writes, so every tile's runs here)
    if (kSup || j0 + T < N) {
      feature_pass(j0, nch);
      if (ti < 1) GF_STAMP(4);
    }
  };
  if constexpr (PF == 2) {
    for (int j0 = 0; j0 < N; j0 += 2 * T) {
      tile_body(j0, pfa);
      if (j0 + T < N) tile_body(j0 + T, pfb);
    }
  } else {
    for (int j0 = 0; j0 < N; j0 += T) tile_body(j0, pfa);
  }
  const int jl = ((N - 1) / T) * T;  // first column of the last tile (still in LDS)
  const int nchl = (N - jl + 63) >> 6;
  if constexpr (kSup) __syncthreads();  // the last feature pass's adjacency words

  // degree of each row -> 1/deg for the mean-pooled network (:120-122)
  {
    int deg = 0;
    if (frow) {
      const int wpt = (Wn + S - 1) / S;
      const int wb = fs * wpt, we = min(Wn, wb + wpt);
      for (int w = wb; w < we; ++w) deg += __popcll(adj[(size_t)fr * Wn + w]);
    }
    with_slices(S, [&](auto Sc) { deg = group_sum_c<decltype(Sc)::value>(deg); });
    if (frow && fs == 0) {
      inv[fr] = a.mean_pooling ? static_cast<float>(1.0 / static_cast<double>(deg == 0 ? 1 : deg)) : 1.0f;
      if (a.degree_out) a.degree_out[env0 + i0 + fr] = deg;
    }
  }
  // packed output: the block's R x Wn adjacency words are one contiguous range
  if (a.adj_bits) {
    uint64_t* dst = a.adj_bits + (env0 + i0) * (size_t)Wn;
    for (int k = tid; k < nrows * Wn; k += kThreads) dst[k] = adj[k];
  }
  __syncthreads();
  GF_STAMP(7);

  if (a.network) store_network_rows(a, adj, inv, stab, Wn, env0 + i0, nrows, wid, lane, KN > 0);

  GF_STAMP(8);
  if constexpr (!kSup) feature_pass(jl, nchl);
  GF_STAMP(9);

  [[maybe_unused]] RawState<UF64> kraw{};
  [[maybe_unused]] bool kgo = false;
  [[maybe_unused]] int kj = 0;
  [[maybe_unused]] bool kinl = false;  // this row is ranked by its wave at the end (inline rim)
  if constexpr (KN > 0) {
   if (!GF_ABLATE(a, 1)) {  // diag 1: no merge / kNN outputs (timing only)
    // Merge the S slices' lists of each row (S consecutive lanes): KN + 1 rounds of an
    // S-lane minimum; the lane whose head won pops it (keys are distinct: j differs).
    // Round m's winner is the row's m-th nearest; lane fs keeps winner fs. The result
    // is the reference's argsort order (ties to the lower index, as the kNN kernel)
    // when (a) the KN-th key has q <= 2^qbits - 4, so its r2 < Tr and every agent left
    // out of the ranking (r2 >= Tr) is farther, and (b) the KN + 1 smallest keys have
    // distinct q: then the top KN are strictly closer than every other agent and
    // strictly ordered among themselves; and (c) no slice that filled its list had all
    // of it popped: a slice's dropped keys exceed its kept ones, so only then can one
    // of them be among the KN + 1 smallest. Any other row (too few agents ranked, equal
    // q, (c)) is left unranked (inline scan or rim kernel).
    const int jb = a.knn_jbits;
    unsigned mine = 0xFFFFFFFFu, prevq = 0xFFFFFFFFu;
    bool slow = false;
    auto merge = [&](auto Sc) {
      constexpr int SS = decltype(Sc)::value;
      const bool kfull = kk[KL - 1] != 0xFFFFFFFFu;
#pragma unroll
      for (int m = 0; m <= KN; ++m) {
        const unsigned w = group_min_u32c<SS>(kk[0]);
        const bool pop = kk[0] == w;
#pragma unroll
        for (int q = 0; q + 1 < KL; ++q) kk[q] = pop ? kk[q + 1] : kk[q];
        kk[KL - 1] = pop ? 0xFFFFFFFFu : kk[KL - 1];
        const bool real = w != 0xFFFFFFFFu;
        const unsigned qw = w >> jb;
        if (m < KN) mine = (fs == m) ? w : mine;
        if (m == KN - 1) slow |= qw > a.knn_qmax - 2u;
        slow |= real && m > 0 && qw == prevq;
        prevq = qw;
      }
      slow |= group_min_u32c<SS>((kfull && kk[0] == 0xFFFFFFFFu) ? 0u : 1u) == 0u;  // (c)
    };
    with_slices(S, merge);  // S >= KN + 1 = 8 here (step_fused_knn_ok)
    // a wave with at most kStepInlineRim such rows ranks them itself after the epilogue
    // (an exact scan of the env, as the rim kernel's few-rows path); more go to the rim
    // kernel (idx = -1, block flagged)
    // diag 0x40000: every such row to the rim kernel (timing only)
    // (envs of at most kStepExactKnnMax agents take the KX instantiation instead)
    const bool inl = __popcll(__ballot(frow && slow && fs == 0)) <= kStepInlineRim && !GF_ABLATE(a, 0x40000);
    if (frow) {
      const size_t g = env0 + i_row;
      if (slow) {
        kinl = inl;
        if (fs == 0 && !inl) {
          a.knn_idx[g * KN] = -1;
          a.knn_rimflag[b * ((N + kThreads - 1) / kThreads) + i_row / kThreads] = 1;
        }
      } else if (fs < KN) {
        const int j = static_cast<int>(mine & ((1u << jb) - 1u));
        if (!GF_ABLATE(a, 0x20000000)) a.knn_idx[g * KN + fs] = j;  // diag: no idx/obs stores
        // the neighbour's state: its loads are issued here and used after the
        // epilogue, so their latency runs under the epilogue's sums
        if (!GF_ABLATE(a, 32)) {  // diag 32: no observation gather (timing only)
          kraw = load_raw<DYN, UF64>(a, env0 + j);
          kj = j;
          kgo = true;
        }
      }
    }
   }
  }

  const St me = frow ? rows[fr] : St{0, 0, 0, 0};
  step_epilogue<DYN, UF64, CTRL, VAR>(a, tile, red, me, f0, f1, f2, f3, f4, f5, gx, gy, svx, svy, b, i0, i_row,
                                      frow && fs == 0, S, tid);
  if constexpr (KN > 0) {
    // Flocking-v0 observation x_i - x_j of this lane's neighbour(s) (flocking.py:24)
    auto knn_out = [&](const St& o, int m) {
      if (m == KN - 1 && a.knn_r2) {  // the row's k-th nearest r2: candidate radius two steps on
        const double dx = me.px - o.px, dy = me.py - o.py;
        a.knn_r2[env0 + i_row] = static_cast<float>(dx * dx + dy * dy);
      }
      float4 ob;
      ob.x = static_cast<float>(me.px - o.px);
      ob.y = static_cast<float>(me.py - o.py);
      ob.z = static_cast<float>(me.vx - o.vx);
      ob.w = static_cast<float>(me.vy - o.vy);
      if (!GF_ABLATE(a, 0x20000000)) reinterpret_cast<float4*>(a.knn_obs)[(env0 + i_row) * KN + m] = ob;
    };
    if (kgo) knn_out(state_from_raw<DYN, UF64>(a, kraw), fs);
    // inline rim: the wave's remaining rows, each scanned by the whole wave over every
    // agent's post-update position (recomputed from x_in and u, bit-identical to the
    // step's), with the rim kernel's ranking and outputs (knn_wave_scan, knn_write_row)
    const uint64_t todo = __ballot(kinl && fs == 0);
    if (todo) step_inline_rim<DYN, UF64, KN>(a, env0, todo, i_row, me);
  }
  if constexpr (KX > 0) {
    // Flocking-v0 (flocking.py:20-25) in an env of one tile: the tile holds every agent's
    // post-update state, so each (row, slice) thread ranks the columns fs, fs + S, ... of
    // its row exactly (float64 r2 computed as the reference's, -ffp-contract=off; the
    // diagonal +inf) into a sorted list of KX (key, j), and KX rounds of an S-lane (key, j)
    // minimum leave winner m in the row's lane m: np.argsort's order with ties to the
    // lower index. The observation x_i - x_j comes from the same LDS tile.
    unsigned long long kk[KX];
    int kj[KX];
#pragma unroll
    for (int m = 0; m < KX; ++m) {
      kk[m] = ~0ull;
      kj[m] = INT_MAX;
    }
    if (frow) {
      for (int c = fs; c < N; c += S) {
        const double2 p = *reinterpret_cast<const double2*>(&tile[c]);
        const double dx = me.px - p.x, dy = me.py - p.y;
        const double r2 = c == i_row ? __builtin_inf() : dx * dx + dy * dy;
        key_insert_asc<KX>(kk, kj, r2_key(r2), c);
      }
    }
    unsigned long long wk = ~0ull;
    int wj = INT_MAX;
    with_slices(S, [&](auto Sc) {
      constexpr int SS = decltype(Sc)::value;
#pragma unroll
      for (int m = 0; m < KX; ++m) {
        unsigned long long k0 = kk[0];
        int j0 = kj[0];
        group_min_key<SS>(k0, j0);
        const bool pop = kj[0] == j0;  // j is unique among the group's listed entries
#pragma unroll
        for (int q = 0; q + 1 < KX; ++q) {
          kk[q] = pop ? kk[q + 1] : kk[q];
          kj[q] = pop ? kj[q + 1] : kj[q];
        }
        kk[KX - 1] = pop ? ~0ull : kk[KX - 1];
        kj[KX - 1] = pop ? INT_MAX : kj[KX - 1];
        if (fs == m) {
          wk = k0;
          wj = j0;
        }
      }
    });
    if (frow && fs < KX) {
      const size_t g = env0 + i_row;
      const int j = wj < N ? wj : i_row;  // (N >= KX: every winner is a real column)
      a.knn_idx[g * KX + fs] = j;
      const St o = tile[j];
      float4 ob;
      ob.x = static_cast<float>(me.px - o.px);
      ob.y = static_cast<float>(me.py - o.py);
      ob.z = static_cast<float>(me.vx - o.vx);
      ob.w = static_cast<float>(me.vy - o.vy);
      reinterpret_cast<float4*>(a.knn_obs)[g * KX + fs] = ob;
      if (fs == KX - 1 && a.knn_r2) a.knn_r2[g] = static_cast<float>(__longlong_as_double(static_cast<long long>(wk)));
    }
  }
  GF_STAMP(10);
#if defined(GF_STAMPS) && GF_STAMPS >= 2
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GF_STAMP(11);
#endif
  signal_done(a.fin);  // drop-in launches: the host waits for this, not the stream
}

// ---------------------------------------------------------------------------------
// Flocking-v0 observation (flocking.py:20-25): the K nearest agents by r2 (self
// excluded by its infinite r2), ties to the lower index. One thread per agent.
//  * Neighbour path: when the step left this state's adjacency behind (adj_bits) and
//    the agent has at least K neighbours, its K nearest are all neighbours (every
//    non-neighbour is farther: r2 >= comm_radius^2 > any neighbour's), so only its ~deg
//    set bits are ranked.
//  * Rim mode: the fused step already ranked every row it could (idx >= 0); only the
//    others are ranked here.
//  * Every remaining row is ranked through a uniform grid of the env's agents, built
//    in LDS by the workgroup (counting sort of agent indices by cell, ~2 agents per
//    cell): the row visits rings of cells around its own, Chebyshev distance d = 0, 1,
//    ..., ranking each agent there exactly (float64 r2, sorted (r2, j) insertion). An
//    agent in a ring beyond d is at least d*h - err away (h: cell size, err: the
//    rounding of cell assignment), so the row stops once its K-th r2 is below that
//    bound squared. The visiting order does not matter: the insertion is a total order
//    on (r2, j). Non-finite or extreme coordinates fall back to a scan of every column.
struct KnnGrid {
  double x0, y0, invh, bound_h, err;  // origin, 1/h, h, cell-assignment error (distance)
  int nx, ny;
};

__device__ __forceinline__ int knn_cell_x(const KnnGrid& G, double x) {
  return min(G.nx - 1, max(0, static_cast<int>((x - G.x0) * G.invh)));
}
__device__ __forceinline__ int knn_cell_y(const KnnGrid& G, double y) {
  return min(G.ny - 1, max(0, static_cast<int>((y - G.y0) * G.invh)));
}

// One ranked row's outputs: indices, observation x_i - x_j (flocking.py:24) and its k-th
// nearest r2 (the fused steps' candidate radius).
template <int K>
__device__ __forceinline__ void knn_write_row(const KnnArgs& a, const double* xb, size_t g, int i, int N,
                                              const double (&kr)[K], const int (&kj)[K]) {
  if (a.r2k) a.r2k[g] = static_cast<float>(kr[K - 1]);
  const double2* xi = reinterpret_cast<const double2*>(xb) + 2 * (size_t)i;
  const double2 pi = xi[0], vv = xi[1];
#pragma unroll
  for (int m = 0; m < K; ++m) {
    const int j = knn_slot_col(kj[m], N, i);  // unfilled slots (non-finite r2 only): self
    a.idx[g * K + m] = j;
    const double2* xj = reinterpret_cast<const double2*>(xb) + 2 * (size_t)j;
    const double2 pj = xj[0], vj = xj[1];
    float4 o;
    o.x = static_cast<float>(pi.x - pj.x);
    o.y = static_cast<float>(pi.y - pj.y);
    o.z = static_cast<float>(vv.x - vj.x);
    o.w = static_cast<float>(vv.y - vj.y);
    reinterpret_cast<float4*>(a.obs + g * 4 * K)[m] = o;
  }
}

// One 256-row block L (env L / bpe) of the kNN kernel.
template <int K, bool LDS>
__device__ __forceinline__ void knn_block(const KnnArgs& a, const int L, unsigned char* smem) {
  const int N = a.N;
  const int bpe = (N + kThreads - 1) / kThreads;
  const int b = L / bpe;
  const int i = (L - b * bpe) * kThreads + threadIdx.x;
  const int tid = threadIdx.x;
  const bool vi = i < N;
  const double* xb = a.x + (size_t)b * N * 4;
  const size_t g = (size_t)b * N + i;
  // rim mode: the fused step ranked every row but those it marked with idx = -1; a
  // workgroup without such rows leaves before staging anything
  if (GF_ABLATE(a, 0x0400)) return;  // ablation 0x0400: no kNN kernel work (timing only)
  // rim mode: only blocks the step flagged hold rows it left unranked
  if (a.rim && a.rimflag[L] == 0) return;
  const bool rim_done = a.rim && (!vi || a.idx[g * K] >= 0);
  const int nrim = a.rim ? __syncthreads_count(!rim_done) : 1;  // every thread has read the flag
  if (a.rim && threadIdx.x == 0) a.rimflag[L] = 0;
  if (nrim == 0) return;
  // positions: the whole env staged in LDS (N <= kKnnLdsMax), else read from L2
  const double2* gpos = reinterpret_cast<const double2*>(xb);
  double2* lpos = reinterpret_cast<double2*>(smem);
  int* cell_end = reinterpret_cast<int*>(lpos + N);                          // kKnnGridCells + 1
  unsigned short* sorted = reinterpret_cast<unsigned short*>(cell_end + kKnnGridCells + 1);  // N
  __shared__ double kred[4][4];
  __shared__ KnnGrid grid;
  __shared__ int grid_ok;
  double pxi = 0, pyi = 0;
  if (vi) {
    pxi = xb[4 * (size_t)i];
    pyi = xb[4 * (size_t)i + 1];
  }
  double kr[K];
  int kj[K];
#pragma unroll
  for (int m = 0; m < K; ++m) {
    kr[m] = __builtin_inf();
    kj[m] = INT_MAX;
  }
  const bool fast = vi && !a.rim && a.adj_bits && a.degree[g] >= K && !GF_ABLATE(a, 0x8000);
  const bool need = vi && !fast && !rim_done;  // ranked by a scan (few rows) or the grid
  const int nslow = __syncthreads_count(need);
  const int nfast = a.adj_bits ? __syncthreads_count(fast) : 0;
  // the env's positions go to LDS for the neighbour path and for the grid; a workgroup
  // with only a few rows to scan (the rim of a compact swarm) reads them from L2
  const bool staged = LDS && (nfast > 0 || nslow > kKnnFewSlow);
  double bx[4] = {-__builtin_inf(), -__builtin_inf(), -__builtin_inf(), -__builtin_inf()};
  bool finite = true;
  if (staged) {
    constexpr int U = 4;  // loads of U agents in flight per thread
    for (int t0 = tid; t0 < N; t0 += U * kThreads) {
      double2 p[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (t0 + u * kThreads < N) p[u] = gpos[2 * (size_t)(t0 + u * kThreads)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (t0 + u * kThreads >= N) break;
        lpos[t0 + u * kThreads] = p[u];
        finite &= __builtin_isfinite(p[u].x) && __builtin_isfinite(p[u].y);
        bx[0] = fmax(bx[0], -p[u].x);  // -min x
        bx[1] = fmax(bx[1], -p[u].y);
        bx[2] = fmax(bx[2], p[u].x);
        bx[3] = fmax(bx[3], p[u].y);
      }
    }
    finite = __syncthreads_and(finite);  // also publishes the staged positions
  }
  auto pos = [&](int j) -> double2 { return staged ? lpos[j] : gpos[2 * (size_t)j]; };
  if (fast) {  // rank the neighbours only
    const int Wn = (N + 63) >> 6;
    const uint64_t* bits = a.adj_bits + g * Wn;
    uint64_t nxt = bits[0];  // one word in flight ahead of the one being ranked
    for (int w = 0; w < Wn; ++w) {
      uint64_t m = nxt;
      if (w + 1 < Wn) nxt = bits[w + 1];
      while (m) {
        const int j = (w << 6) + __builtin_ctzll(m);
        m &= m - 1;
        const double2 p = pos(j);
        const double dx = pxi - p.x, dy = pyi - p.y;
        if (GF_ABLATE(a, 0x4000)) {  // ablation: no ranking (outputs: the last neighbour K times)
          kr[0] += dx * dx + dy * dy;
          kj[0] = j;
        } else {
          knn_insert_asc<K>(kr, kj, dx * dx + dy * dy, j);
        }
      }
    }
    if (GF_ABLATE(a, 0x4000)) {
#pragma unroll
      for (int m = 1; m < K; ++m) kj[m] = kj[0];
    }
  }
  if (nslow > 0 && nslow <= kKnnFewSlow) {
    // few rows: each is scanned by its whole wave (knn_wave_scan)
    uint64_t todo = __ballot(need);
    while (todo) {
      const int l = __builtin_ctzll(todo);
      todo &= todo - 1;
      knn_wave_scan<K>(pos, N, l, i, pxi, pyi, kr, kj);
    }
    if (need) knn_insert<K>(kr, kj, __builtin_inf(), i);  // self last (r2 = inf in the reference)
  } else if (nslow > 0) {
    bool use_grid = false;
    if (staged && finite) {
      // bounding box (workgroup max of -xmin, -ymin, xmax, ymax)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        for (int o = 32; o >= 1; o >>= 1) bx[q] = fmax(bx[q], __shfl_xor(bx[q], o));
      if ((tid & 63) == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) kred[tid >> 6][q] = bx[q];
      __syncthreads();
      if (tid == 0) {
        double e[4];
        for (int q = 0; q < 4; ++q) e[q] = fmax(fmax(kred[0][q], kred[1][q]), fmax(kred[2][q], kred[3][q]));
        const double x0 = -e[0], y0 = -e[1], ex = e[2] - x0, ey = e[3] - y0;
        const double P = fmax(fmax(fabs(x0), fabs(y0)), fmax(fabs(e[2]), fabs(e[3])));
        // ~2 agents per cell over the bounding box, at most kKnnGridCells cells
        const double nt = fmax(1.0, fmin(static_cast<double>(kKnnGridCells) / 3.0, 0.5 * N));
        double h = fmax(sqrt(ex * ey / nt), fmax(ex, ey) / nt);
        if (!(h > 0)) h = 1.0;
        int nx = 0, ny = 0;
        for (int it = 0; it < 64; ++it, h *= 1.25) {
          nx = static_cast<int>(ex / h) + 1;
          ny = static_cast<int>(ey / h) + 1;
          if ((long long)nx * ny <= kKnnGridCells) break;
        }
        // cell assignment error as a distance: (x - x0) and its product with 1/h are
        // rounded; 2^-40 (P + ex + ey) covers both agents' errors many times over
        const double err = ldexp(P + ex + ey, -40);
        grid = KnnGrid{x0, y0, 1.0 / h, h, err, nx, ny};
        grid_ok = (long long)nx * ny <= kKnnGridCells && err < 1e-3 * h && P < 1e15;
      }
      __syncthreads();
      use_grid = grid_ok;
    }
    if (GF_ABLATE(a, 0x2000)) use_grid = false;  // ablation: no grid, no search (timing only)
    if (use_grid) {
      const KnnGrid G = grid;
      const int ncell = G.nx * G.ny;
      // counting sort of the agents by cell: cell_end[c] = inclusive prefix count, then
      // each agent takes slot --cell_end[c], which leaves cell_end[c] = start of cell c
      for (int c = tid; c <= ncell; c += kThreads) cell_end[c] = 0;
      __syncthreads();
      for (int t = tid; t < N; t += kThreads) {
        const double2 p = lpos[t];
        atomicAdd(&cell_end[knn_cell_y(G, p.y) * G.nx + knn_cell_x(G, p.x)], 1);
      }
      __syncthreads();
      {  // inclusive scan over ncell counts: a contiguous chunk per thread
        const int per = (ncell + kThreads - 1) / kThreads;
        const int c0 = min(ncell, tid * per), c1 = min(ncell, c0 + per);
        int s = 0;
        for (int c = c0; c < c1; ++c) s += cell_end[c];
        int incl = s;  // workgroup inclusive scan of the chunk sums
        const int lane = tid & 63;
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o);
          if (lane >= o) incl += v;
        }
        __shared__ int wsum[4];
        if (lane == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        int base = incl - s;
        for (int w = 0; w < (tid >> 6); ++w) base += wsum[w];
        for (int c = c0; c < c1; ++c) {
          base += cell_end[c];
          cell_end[c] = base;
        }
      }
      if (tid == 0) cell_end[ncell] = N;
      __syncthreads();
      for (int t = tid; t < N; t += kThreads) {
        const double2 p = lpos[t];
        const int slot = atomicSub(&cell_end[knn_cell_y(G, p.y) * G.nx + knn_cell_x(G, p.x)], 1) - 1;
        sorted[slot] = static_cast<unsigned short>(t);
      }
      __syncthreads();
      if (need && !GF_ABLATE(a, 0x1000)) {  // ablation 0x1000: grid only, no search
        const int cx = knn_cell_x(G, pxi), cy = knn_cell_y(G, pyi);
        const int dmax = max(max(cx, G.nx - 1 - cx), max(cy, G.ny - 1 - cy));
        auto range = [&](int y, int xa, int xb2) {  // cells [xa, xb2] of grid row y
          xa = max(xa, 0);
          xb2 = min(xb2, G.nx - 1);
          if (y < 0 || y >= G.ny || xa > xb2) return;
          const int s0 = cell_end[y * G.nx + xa], s1 = cell_end[y * G.nx + xb2 + 1];
          for (int s = s0; s < s1; ++s) {
            const int j = sorted[s];
            if (j != i) knn_consider<K>(kr, kj, pxi, pyi, lpos[j], j, N);
          }
        };
        for (int d = 0; d <= dmax; ++d) {
          range(cy - d, cx - d, cx + d);
          if (d > 0) {
            range(cy + d, cx - d, cx + d);
            for (int y = cy - d + 1; y <= cy + d - 1; ++y) {
              range(y, cx - d, cx - d);
              range(y, cx + d, cx + d);
            }
          }
          // every agent not visited yet is >= d*h - 2 err away; r2 of such a pair, as
          // computed, is at least that squared (1 - 2^-40)
          const double lim = static_cast<double>(d) * G.bound_h - 2.0 * G.err;
          if (lim > 0 && kr[K - 1] < lim * lim * (1.0 - 0x1p-40)) break;
        }
      }
    } else if (need && !GF_ABLATE(a, 0x2000)) {
      for (int j = 0; j < N; ++j)
        if (j != i) knn_consider<K>(kr, kj, pxi, pyi, pos(j), j, N);
    }
    // self last (its r2 is inf in the reference), for k >= the agents with finite r2
    if (need) knn_insert<K>(kr, kj, __builtin_inf(), i);
  }
  if (!vi || rim_done || GF_ABLATE(a, 0x0800)) return;  // ablation 0x0800: no outputs
  knn_write_row<K>(a, xb, g, i, N, kr, kj);
}

// Rim mode runs a small grid that walks the blocks (kKnnRimGrid workgroups): it is
// enqueued beside the next step, whose workgroups hold most CU slots, and a full grid of
// mostly idle workgroups took ~150 us to drain between them. Other modes: one
// workgroup per block.
template <int K, bool LDS>
__global__ __launch_bounds__(kThreads) void flock_knn_kernel(KnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (a.rim) {
    const int nblk = a.B * ((a.N + kThreads - 1) / kThreads);
    for (int L = blockIdx.x; L < nblk; L += gridDim.x) {
      knn_block<K, LDS>(a, L, smem);
      __syncthreads();  // the block's LDS is free for the next one
    }
  } else {
    knn_block<K, LDS>(a, xcd_remap(blockIdx.x, gridDim.x), smem);
  }
  signal_done(a.fin);  // the drop-in step's rim kNN: the host waits for this, not the stream
}

// get_stats (:136-143): vel_diffs_i = |v_i - mean v|, min_dists_i = sqrt(min_j r2_ij)
// (r2 is exactly symmetric, so the reference's column min equals this row min), plus
// the degree used by reset()'s acceptance test (:177-184).
__global__ __launch_bounds__(kThreads) void flock_stats_kernel(StatsArgs a) {
  __shared__ St tile[kTileMax];
  __shared__ double red[8];
  const int N = a.N;
  const int bpe = (N + kThreads - 1) / kThreads;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int b = L / bpe;
  const int i = (L - b * bpe) * kThreads + threadIdx.x;
  const bool vi = i < N;
  const St* xb = reinterpret_cast<const St*>(a.x + (size_t)b * N * 4);
  St me{0, 0, 0, 0};
  if (vi) me = xb[i];
  double mn = __builtin_inf(), sx = 0, sy = 0;
  int deg = 0;
  for (int j0 = 0; j0 < N; j0 += kTileMax) {
    const int tc = min(kTileMax, N - j0);
    __syncthreads();
    for (int t = threadIdx.x; t < tc; t += kThreads) {
      const St s = xb[j0 + t];
      tile[t] = s;
      sx += s.vx;
      sy += s.vy;
    }
    __syncthreads();
    if (vi) {
      for (int t = 0; t < tc; ++t) {
        const double dx = me.px - tile[t].px, dy = me.py - tile[t].py;
        const double r2 = dx * dx + dy * dy;
        const bool other = j0 + t != i;
        if (other && r2 < mn) mn = r2;
        deg += (other && r2 < a.cr2) ? 1 : 0;
      }
    }
  }
  const double mx = block_sum(sx, red) / static_cast<double>(N);
  const double my = block_sum(sy, red) / static_cast<double>(N);
  if (!vi) return;
  const size_t g = (size_t)b * N + i;
  const double ex = me.vx - mx, ey = me.vy - my;
  a.vel_diffs[g] = sqrt(ex * ex + ey * ey);
  a.min_dists[g] = sqrt(mn);
  a.degree[g] = deg;
}


// get_stats() summaries per env for the multi-GPU metrics path: the
// means of vel_diffs and min_dists over the env's N agents (np.mean of the two arrays
// flocking_relative.py:140-142 returns), one workgroup per env, a fixed summation tree
// (deterministic bits; ulps from NumPy's pairwise order).
__global__ __launch_bounds__(kThreads) void flock_stats_summary_kernel(const double* vd, const double* md,
                                                                       double* out, int N) {
  __shared__ double red[8];
  const size_t e0 = (size_t)blockIdx.x * N;
  double s0 = 0, s1 = 0;
  for (int i = threadIdx.x; i < N; i += kThreads) {
    s0 += vd[e0 + i];
    s1 += md[e0 + i];
  }
  s0 = block_sum(s0, red);
  s1 = block_sum(s1, red);
  if (threadIdx.x == 0) {
    out[2 * (size_t)blockIdx.x] = s0 / static_cast<double>(N);
    out[2 * (size_t)blockIdx.x + 1] = s1 / static_cast<double>(N);
  }
}


}  // namespace

// ----------------------------------------------------------------------------- host
// Geometry measured on MI355X (scripts/ablate.py, N=1024 x 256 envs): 32-row blocks
// with 512-agent LDS tiles keep 6 workgroups per CU resident, which is what hides the
// per-block load/compute latency under the network stores: 190 us at 6 per CU, 193 at
// 5, 211 at 4, 206 at 7 (scripts/occprobe.hip measures what fits: <= 20 KiB -> 8,
// 24-26 KiB -> 6, 27-31 KiB -> 5, 32 KiB -> 4).
int step_rows_per_block(int N) {
  const int words = (N + 63) / 64;
  int R = 32;
  while (R > 4 && (size_t)R * words * 8 > 16384) R >>= 1;  // adjacency bits <= 16 KiB
  while (R > 4 && R / 2 >= N) R >>= 1;
  return R;
}

int step_tile(int N) {
  const int t = ((N + 63) / 64) * 64;
  return t < kTileDefault ? t : kTileDefault;
}

size_t step_lds_bytes(int N, int R, int T, bool ctrl, bool knn) {
  const size_t Wn = (N + 63) / 64, Wt = T / 64;
  size_t s = (size_t)T * sizeof(St) + (size_t)R * sizeof(St);
  s += (size_t)R * Wn * 8 + ((ctrl && knn) ? (size_t)R * Wt * 8 : 0) + (knn ? (size_t)R * Wt * 8 : 0);
  // inv (R floats); kNN: rthr (R), the waves' candidate-bound tables (4R), prow (R ints)
  s += 8 * sizeof(double) + (((size_t)R * 4 * (knn ? 7 : 1) + 15) / 16) * 16;
  s += 4 * kStoreTab * 16 + (((size_t)R * 8 + 31) & ~size_t(31));  // row table, rows' float32 positions
  return s;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): `done`
// holds one bit per device ordinal (a second handle on another device sets its own;
// concurrent first calls both set it, which is harmless).
hipError_t max_lds_once(const void* f, std::atomic<uint64_t>& done, int bytes) {
  int dev = 0;
  if (const hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? (1ull << dev) : 0ull;
  if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

template <bool DYN, bool UF64, bool CTRL, bool VAR, int PF = 0, int KN = 0, int KX = 0>
static hipError_t launch_step_tiled(const StepArgs& a, hipStream_t s) {
  size_t lds = step_lds_bytes(a.N, a.R, a.T, CTRL, KN > 0);
  // the plain step runs best at 6 workgroups per CU: 199 us vs 206 at the 7 its 21.2 KiB
  // would allow
  if (!CTRL && !VAR && lds < kStepLdsPlainFloor) lds = kStepLdsPlainFloor;
  static std::atomic<uint64_t> attr{0};
  if (const hipError_t e = max_lds_once(
          reinterpret_cast<const void*>(&flock_step_kernel<DYN, UF64, CTRL, VAR, PF, KN, false, KX>), attr, 160 * 1024);
      e != hipSuccess)
    return e;
  const int grid = a.B * a.bpe;
  hipLaunchKernelGGL((flock_step_kernel<DYN, UF64, CTRL, VAR, PF, KN, false, KX>), dim3(grid), dim3(kThreads), lds, s,
                     a);
  return hipGetLastError();
}

// the drop-in step with its actions copied from the host into the kernel arguments
template <bool UF64, bool CTRL, int KN = 0, int KX = 0>
static hipError_t launch_step_uin(const StepArgs& a, hipStream_t s) {
  const size_t bytes = (size_t)a.B * a.N * 2 * (UF64 ? 8 : 4);
  if (bytes > (size_t)kUInlineBytes || a.N > a.T) return hipErrorInvalidValue;
  size_t lds = step_lds_bytes(a.N, a.R, a.T, CTRL, KN > 0);
  if (!CTRL && KN == 0 && lds < kStepLdsPlainFloor) lds = kStepLdsPlainFloor;
  static std::atomic<uint64_t> attr{0};
  if (const hipError_t e = max_lds_once(
          reinterpret_cast<const void*>(&flock_step_kernel<true, UF64, CTRL, false, 0, KN, true, KX>), attr, 160 * 1024);
      e != hipSuccess)
    return e;
  StepArgsU p;
  p.a = a;
  p.a.u = nullptr;
  p.a.u_inline = 0;
  std::memcpy(p.u, a.u, bytes);
  hipLaunchKernelGGL((flock_step_kernel<true, UF64, CTRL, false, 0, KN, true, KX>), dim3(a.B * a.bpe), dim3(kThreads),
                     lds, s, p);
  return hipGetLastError();
}

bool step_fused_knn_ok(int N, int R, int K, bool variant, bool prefetch) {
  return K == kStepFusedK && !variant && !prefetch && kThreads / R >= K && N <= 65536;
}

bool step_knn_exact(int N, int T, int B) {
  return N <= T && (N <= kStepExactKnnMax || (B == 1 && N <= kStepExactKnnMaxOneEnv));
}

template <bool DYN, bool UF64, bool CTRL>
static hipError_t launch_step_t(const StepArgs& a, hipStream_t s) {
  if constexpr (DYN) {
    const bool exact = a.knn_idx && a.knn_exact;
    if (a.u_inline) {
      if (a.variant) return hipErrorInvalidValue;
      if (a.knn_idx) {  // the drop-in Flocking-v0 step (fe_step_host_knn*)
        if (kThreads / a.R < kStepFusedK) return hipErrorInvalidValue;
        if (exact) return launch_step_uin<UF64, CTRL, 0, kStepFusedK>(a, s);
        if constexpr (CTRL) return hipErrorInvalidValue;
        else return launch_step_uin<UF64, CTRL, kStepFusedK>(a, s);
      }
      return launch_step_uin<UF64, CTRL>(a, s);
    }
    if (a.knn_idx) {
      if (a.variant || (a.prefetch && a.T <= 2 * kThreads && a.N > a.T) || kThreads / a.R < kStepFusedK)
        return hipErrorInvalidValue;
      if (exact) return launch_step_tiled<DYN, UF64, CTRL, false, 0, 0, kStepFusedK>(a, s);
      return launch_step_tiled<DYN, UF64, CTRL, false, 0, kStepFusedK>(a, s);
    }
  }
  if (a.knn_idx) return hipErrorInvalidValue;
  if (a.variant) return launch_step_tiled<DYN, UF64, CTRL, true>(a, s);
  if (a.prefetch && a.T <= 2 * kThreads && a.N > a.T) return launch_step_tiled<DYN, UF64, CTRL, false, 1>(a, s);
  return launch_step_tiled<DYN, UF64, CTRL, false>(a, s);
}


hipError_t launch_step(const StepArgs& a, bool dyn, bool u_f64, bool ctrl, hipStream_t s) {
  if (dyn) {
    if (u_f64) return ctrl ? launch_step_t<true, true, true>(a, s) : launch_step_t<true, true, false>(a, s);
    return ctrl ? launch_step_t<true, false, true>(a, s) : launch_step_t<true, false, false>(a, s);
  }
  return ctrl ? launch_step_t<false, false, true>(a, s) : launch_step_t<false, false, false>(a, s);
}

hipError_t launch_knn(const KnnArgs& a, hipStream_t s) {
  int grid = a.B * ((a.N + kThreads - 1) / kThreads);
  if (a.rim) grid = min(grid, a.grid_cap > 0 ? a.grid_cap : kKnnRimGrid);
  const bool lds = a.N <= kKnnLdsMax;
  const size_t bytes = lds ? knn_lds_bytes(a.N) : 0;
  switch (a.K) {
#define GF_KNN_CASE(k)                                                                                  \
  case k:                                                                                               \
    if (lds) {                                                                                          \
      static std::atomic<uint64_t> attr_##k{0};                                                         \
      if (const hipError_t e = max_lds_once(reinterpret_cast<const void*>(&flock_knn_kernel<k, true>), \
                                            attr_##k, (int)knn_lds_bytes(kKnnLdsMax));                  \
          e != hipSuccess)                                                                              \
        return e;                                                                                       \
      hipLaunchKernelGGL((flock_knn_kernel<k, true>), dim3(grid), dim3(kThreads), bytes, s, a);        \
    } else                                                                                              \
      hipLaunchKernelGGL((flock_knn_kernel<k, false>), dim3(grid), dim3(kThreads), 0, s, a);           \
    break;
    GF_KNN_CASE(1) GF_KNN_CASE(2) GF_KNN_CASE(3) GF_KNN_CASE(4) GF_KNN_CASE(5) GF_KNN_CASE(6)
    GF_KNN_CASE(7) GF_KNN_CASE(8) GF_KNN_CASE(10) GF_KNN_CASE(12) GF_KNN_CASE(16)
#undef GF_KNN_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <bool NT>
__global__ __launch_bounds__(kThreads) void diag_fill_kernel(f4v* p, size_t n4) {
  const f4v v{1.0f, 0.0f, 0.5f, 0.0f};
  for (size_t k = blockIdx.x * (size_t)kThreads + threadIdx.x; k < n4; k += (size_t)gridDim.x * kThreads) {
    if (NT)
      __builtin_nontemporal_store(v, &p[k]);
    else
      p[k] = v;
  }
}

hipError_t launch_fill(void* p, size_t bytes, bool nt, hipStream_t s) {
  const size_t n4 = bytes / 16;
  const int grid = 256 * 16;
  if (nt)
    hipLaunchKernelGGL(diag_fill_kernel<true>, dim3(grid), dim3(kThreads), 0, s, (f4v*)p, n4);
  else
    hipLaunchKernelGGL(diag_fill_kernel<false>, dim3(grid), dim3(kThreads), 0, s, (f4v*)p, n4);
  return hipGetLastError();
}

#ifdef GF_STAMPS
extern "C" __attribute__((visibility("default"))) int fe_diag_stamps(unsigned long long* dst, int n) {
  if (n > 8192 * 16) n = 8192 * 16;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(gf_stamp_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_stats(const StatsArgs& a, hipStream_t s) {
  const int grid = a.B * ((a.N + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(flock_stats_kernel, dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_stats_summary(const StatsArgs& a, double* out, hipStream_t s) {
  hipLaunchKernelGGL(flock_stats_summary_kernel, dim3(a.B), dim3(kThreads), 0, s, a.vel_diffs, a.min_dists, out, a.N);
  return hipGetLastError();
}

}  // namespace gf
