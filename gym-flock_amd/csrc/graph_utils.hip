// Graph helpers of gym_flock/envs/spatial/utils.py on the device (SURVEY.md §8a row
// a14): _get_graph_edges :8-24 (radius graph), _nodes_within_radius :27-39 and
// _get_k_edges :60-88 (k-nearest graph), C-ABI gu_* (include/gymflock.h).
//
// One wave per sender row; the row's columns are swept 64 at a time and the per-column
// predicate is a ballot, so a row's edges come out in ascending receiver order, which
// is np.nonzero's row-major order. Distances are r = sqrt(dx*dx + dy*dy) in float64
// without contraction, exactly np.linalg.norm(diff, axis=2) on (n, n2, 2) differences
// (numpy: sqrt(add.reduce(x*x)) over the 2-wide axis), so the edge sets are bit-exact.
//
// The k-nearest rows pick the k (or k+1) smallest by (r, column), NaN above +inf: a
// wave-wide (key, column) minimum per pick, each pick the smallest pair above the last
// one. np.argpartition leaves the choice among EQUAL distances at the k-th boundary to
// its selection algorithm (introselect, or a SIMD kernel on AVX-512 hosts); the lowest
// column wins here. Untied boundaries match the reference exactly.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <string>

#include "gymflock.h"

namespace gf {
int set_error(int code, const std::string& msg);
}

namespace {

constexpr int kGuThreads = 256;
constexpr int kGuWaves = kGuThreads / 64;
constexpr uint64_t kNanKey = 0x7FF0000000000001ull;  // above +inf's bit pattern

struct GuArgs {
  const double* p1 = nullptr;  // (n1, 2) senders
  const double* p2 = nullptr;  // (n2, 2) receivers; == p1 for pos2=None
  int n1 = 0, n2 = 0;
  int same = 0;        // pos2 is None (the diagonal is the self pair)
  int self_loops = 0;  // keep the diagonal
  double rad = 0;
  int k = 0, allow_nearest = 0;
  int32_t* cnt = nullptr;   // (n1) edges per row
  int64_t* off = nullptr;   // (n1) first edge of each row
  int64_t* total = nullptr; // (1)
  int32_t* sel = nullptr;   // (n1, k+1) chosen columns (k-nearest)
  int32_t* snd = nullptr;
  int32_t* rcv = nullptr;
  double* r = nullptr;
  double* dx = nullptr;     // all dx, then
  double* dy = nullptr;     // all dy (the reference's np.hstack of the two columns)
  uint8_t* valid = nullptr; // (n2) _nodes_within_radius
};

__device__ inline double pair_r(const GuArgs& a, int i, int j, double& dx, double& dy) {
  dx = a.p1[2 * i] - a.p2[2 * j];
  dy = a.p1[2 * i + 1] - a.p2[2 * j + 1];
  return sqrt(dx * dx + dy * dy);
}

// _get_graph_edges: r[r > rad] = 0; without self loops the diagonal is zeroed; edges
// are the nonzero entries (NaN is nonzero and not > rad, so it stays an edge)
__device__ inline bool radius_keep(const GuArgs& a, int i, int j, double r) {
  if (a.same && !a.self_loops && i == j) return false;
  return !(r > a.rad) && r != 0.0;
}

// _get_k_edges: the diagonal is +inf without self loops (np.fill_diagonal(r, np.Inf))
__device__ inline double knn_r(const GuArgs& a, int i, int j, double& dx, double& dy) {
  const double r = pair_r(a, i, j, dx, dy);
  return (a.same && !a.self_loops && i == j) ? __builtin_inf() : r;
}

// order key of a distance (r >= +0 or NaN): the bit pattern, NaN above everything
__device__ inline uint64_t rkey(double r) {
  return r != r ? kNanKey : static_cast<uint64_t>(__double_as_longlong(r));
}

__device__ inline bool pair_less(uint64_t ka, int ja, uint64_t kb, int jb) {
  return ka < kb || (ka == kb && ja < jb);
}

__global__ __launch_bounds__(kGuThreads) void gu_radius_count_kernel(GuArgs a) {
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * kGuWaves + (threadIdx.x >> 6); i < a.n1; i += gridDim.x * kGuWaves) {
    int c = 0;
    for (int j0 = 0; j0 < a.n2; j0 += 64) {
      const int j = j0 + lane;
      bool keep = false;
      if (j < a.n2) {
        double dx, dy;
        keep = radius_keep(a, i, j, pair_r(a, i, j, dx, dy));
      }
      c += __popcll(__ballot(keep));
    }
    if (lane == 0) a.cnt[i] = c;
  }
}

__global__ __launch_bounds__(kGuThreads) void gu_radius_fill_kernel(GuArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int i = blockIdx.x * kGuWaves + (threadIdx.x >> 6); i < a.n1; i += gridDim.x * kGuWaves) {
    int64_t o = a.off[i];
    for (int j0 = 0; j0 < a.n2; j0 += 64) {
      const int j = j0 + lane;
      bool keep = false;
      double dx = 0, dy = 0, r = 0;
      if (j < a.n2) {
        r = pair_r(a, i, j, dx, dy);
        keep = radius_keep(a, i, j, r);
      }
      const uint64_t m = __ballot(keep);
      if (keep) {
        const int64_t e = o + __popcll(m & below);
        a.snd[e] = i;
        a.rcv[e] = j;
        a.r[e] = r;
        a.dx[e] = dx;
        a.dy[e] = dy;
      }
      o += __popcll(m);
    }
  }
}

// exclusive scan of the per-row counts (one workgroup; these graphs have at most a few
// thousand rows)
__global__ __launch_bounds__(1024) void gu_scan_kernel(GuArgs a) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x, per = (a.n1 + 1023) / 1024;
  const int b = min(a.n1, t * per), e = min(a.n1, b + per);
  int64_t s = 0;
  for (int i = b; i < e; ++i) s += a.cnt[i];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int q = 0; q < 1024; ++q) {
      const int64_t v = part[q];
      part[q] = run;
      run += v;
    }
    *a.total = run;
  }
  __syncthreads();
  int64_t run = part[t];
  for (int i = b; i < e; ++i) {
    a.off[i] = run;
    run += a.cnt[i];
  }
}

// _nodes_within_radius: column j is valid when the column sum of r (r > rad zeroed)
// is > 0, i.e. some 0 < r <= rad and no NaN in the column (a NaN sum is not > 0)
__global__ __launch_bounds__(kGuThreads) void gu_within_kernel(GuArgs a) {
  const int j = blockIdx.x * kGuThreads + threadIdx.x;
  if (j >= a.n2) return;
  bool any = false, nan = false;
  for (int i = 0; i < a.n1; ++i) {
    double dx, dy;
    const double r = pair_r(a, i, j, dx, dy);
    nan |= r != r;
    any |= r > 0.0 && r <= a.rad;
  }
  a.valid[j] = (any && !nan) ? 1 : 0;
}

// k-nearest selection: kp = k (allow_nearest) or k + 1 picks per row, each the smallest
// (key, column) above the previous pick; without allow_nearest the row's argmin (first
// NaN if any, np.argmin's rule; else the first pick) is then dropped if picked. The
// kept columns are sorted ascending (np.nonzero order) into sel.
__global__ __launch_bounds__(kGuThreads) void gu_knn_select_kernel(GuArgs a) {
  const int lane = threadIdx.x & 63;
  const int kp = a.allow_nearest ? a.k : a.k + 1;
  for (int i = blockIdx.x * kGuWaves + (threadIdx.x >> 6); i < a.n1; i += gridDim.x * kGuWaves) {
    int32_t* sel = a.sel + (size_t)i * (a.k + 1);
    uint64_t lk = 0;
    int lj = -1;
    int first_nan = INT_MAX;
    for (int s = 0; s < kp; ++s) {
      uint64_t bk = ~0ull;
      int bj = INT_MAX;
      for (int j = lane; j < a.n2; j += 64) {
        double dx, dy;
        const double r = knn_r(a, i, j, dx, dy);
        if (s == 0 && r != r) first_nan = min(first_nan, j);
        const uint64_t key = rkey(r);
        if (pair_less(lk, lj, key, j) && pair_less(key, j, bk, bj)) {
          bk = key;
          bj = j;
        }
      }
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t ok = __shfl_xor(bk, o);
        const int oj = __shfl_xor(bj, o);
        if (pair_less(ok, oj, bk, bj)) {
          bk = ok;
          bj = oj;
        }
      }
      lk = bk;
      lj = bj;
      if (lane == 0) sel[s] = bj;
    }
    for (int o = 32; o > 0; o >>= 1) first_nan = min(first_nan, __shfl_xor(first_nan, o));
    if (lane == 0) {
      int c = kp;
      if (!a.allow_nearest) {
        const int drop = first_nan != INT_MAX ? first_nan : sel[0];
        int w = 0;
        for (int s = 0; s < kp; ++s)
          if (sel[s] != drop) sel[w++] = sel[s];
        c = w;
      }
      for (int s = 1; s < c; ++s) {  // insertion sort, c <= k + 1
        const int v = sel[s];
        int q = s - 1;
        while (q >= 0 && sel[q] > v) {
          sel[q + 1] = sel[q];
          --q;
        }
        sel[q + 1] = v;
      }
      a.cnt[i] = c;
    }
  }
}

__global__ __launch_bounds__(kGuThreads) void gu_knn_fill_kernel(GuArgs a) {
  const int i = blockIdx.x * kGuThreads + threadIdx.x;
  if (i >= a.n1) return;
  const int32_t* sel = a.sel + (size_t)i * (a.k + 1);
  const int64_t o = a.off[i];
  for (int s = 0; s < a.cnt[i]; ++s) {
    const int j = sel[s];
    double dx, dy;
    const double r = knn_r(a, i, j, dx, dy);
    a.snd[o + s] = i;
    a.rcv[o + s] = j;
    a.r[o + s] = r;
    a.dx[o + s] = dx;
    a.dy[o + s] = dy;
  }
}

int gfail(int code, const std::string& m) { return gf::set_error(code, m); }

#define GU_HIP(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return gfail(GF_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

}  // namespace

struct gu_graph {
  int device = 0;
  hipStream_t stream = nullptr;
  void* buf[12] = {};      // device buffers, grown on demand
  size_t cap[12] = {};
  int64_t n_edges = 0;     // the last result
  GuArgs a{};
};

namespace {

enum { B_P1, B_P2, B_CNT, B_OFF, B_TOT, B_SEL, B_SND, B_RCV, B_R, B_DX, B_DY, B_VALID };

template <class T>
int grow(gu_graph* g, int slot, size_t n, T** out) {
  const size_t bytes = (n ? n : 1) * sizeof(T);
  if (g->cap[slot] < bytes) {
    if (g->buf[slot]) GU_HIP(hipFree(g->buf[slot]));
    g->buf[slot] = nullptr;
    g->cap[slot] = 0;
    if (hipMalloc(&g->buf[slot], bytes) != hipSuccess) return gfail(GF_ENOMEM, "hipMalloc (graph helpers)");
    g->cap[slot] = bytes;
  }
  *out = static_cast<T*>(g->buf[slot]);
  return GF_OK;
}

#define GU_TRY(expr)        \
  do {                      \
    const int rc_ = (expr); \
    if (rc_ != GF_OK) return rc_; \
  } while (0)

// common setup: positions to the device, the argument block
int stage(gu_graph* g, const double* pos1, int32_t n1, const double* pos2, int32_t n2) {
  if (!g) return gfail(GF_EINVAL, "null graph context");
  if (n1 < 0 || (pos2 && n2 < 0)) return gfail(GF_EINVAL, "negative point count");
  if (n1 > 0 && !pos1) return gfail(GF_EINVAL, "null positions");
  GU_HIP(hipSetDevice(g->device));
  GuArgs& a = g->a;
  a = GuArgs{};
  a.n1 = n1;
  a.same = pos2 == nullptr;
  a.n2 = a.same ? n1 : n2;
  double* d1 = nullptr;
  double* d2 = nullptr;
  GU_TRY(grow(g, B_P1, (size_t)2 * a.n1, &d1));
  if (a.n1) GU_HIP(hipMemcpyAsync(d1, pos1, sizeof(double) * 2 * a.n1, hipMemcpyHostToDevice, g->stream));
  if (a.same) {
    d2 = d1;
  } else {
    GU_TRY(grow(g, B_P2, (size_t)2 * a.n2, &d2));
    if (a.n2) GU_HIP(hipMemcpyAsync(d2, pos2, sizeof(double) * 2 * a.n2, hipMemcpyHostToDevice, g->stream));
  }
  a.p1 = d1;
  a.p2 = d2;
  GU_TRY(grow(g, B_CNT, (size_t)a.n1, &a.cnt));
  GU_TRY(grow(g, B_OFF, (size_t)a.n1, &a.off));
  GU_TRY(grow(g, B_TOT, 1, &a.total));
  g->n_edges = 0;
  return GF_OK;
}

int row_grid(int n1) { return n1 > 0 ? (n1 + kGuWaves - 1) / kGuWaves : 0; }

// scan the counts, size the outputs, run the fill
template <class Fill>
int finish(gu_graph* g, int64_t* n_edges, Fill launch_fill) {
  GuArgs& a = g->a;
  int64_t total = 0;
  if (a.n1 > 0) {
    gu_scan_kernel<<<1, 1024, 0, g->stream>>>(a);
    GU_HIP(hipGetLastError());
    GU_HIP(hipMemcpyAsync(&total, a.total, sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
    GU_HIP(hipStreamSynchronize(g->stream));
  }
  GU_TRY(grow(g, B_SND, (size_t)total, &a.snd));
  GU_TRY(grow(g, B_RCV, (size_t)total, &a.rcv));
  GU_TRY(grow(g, B_R, (size_t)total, &a.r));
  GU_TRY(grow(g, B_DX, (size_t)total, &a.dx));
  GU_TRY(grow(g, B_DY, (size_t)total, &a.dy));
  if (total > 0) {
    launch_fill();
    GU_HIP(hipGetLastError());
  }
  g->n_edges = total;
  if (n_edges) *n_edges = total;
  return GF_OK;
}

}  // namespace

extern "C" {

int gu_create(int device, gu_graph** out) {
  if (!out) return gfail(GF_EINVAL, "null output pointer");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return gfail(GF_EHIP, "no HIP device");
  if (device < 0 || device >= ndev) return gfail(GF_EINVAL, "device out of range");
  GU_HIP(hipSetDevice(device));
  gu_graph* g = new gu_graph();
  g->device = device;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    delete g;
    return gfail(GF_EHIP, "hipStreamCreate");
  }
  *out = g;
  return GF_OK;
}

int gu_destroy(gu_graph* g) {
  if (!g) return GF_OK;
  hipSetDevice(g->device);
  if (g->stream) hipStreamSynchronize(g->stream);
  for (void* p : g->buf)
    if (p) hipFree(p);
  if (g->stream) hipStreamDestroy(g->stream);
  delete g;
  return GF_OK;
}

int gu_radius_edges(gu_graph* g, const double* pos1, int32_t n1, const double* pos2, int32_t n2, double rad,
                    int self_loops, int64_t* n_edges) {
  GU_TRY(stage(g, pos1, n1, pos2, n2));
  GuArgs& a = g->a;
  a.rad = rad;
  a.self_loops = self_loops != 0;
  if (a.n1 > 0) {
    gu_radius_count_kernel<<<row_grid(a.n1), kGuThreads, 0, g->stream>>>(a);
    GU_HIP(hipGetLastError());
  }
  return finish(g, n_edges, [&] { gu_radius_fill_kernel<<<row_grid(a.n1), kGuThreads, 0, g->stream>>>(a); });
}

int gu_k_edges(gu_graph* g, int32_t k, const double* pos1, int32_t n1, const double* pos2, int32_t n2,
               int self_loops, int allow_nearest, int64_t* n_edges) {
  if (k < 1) return gfail(GF_EINVAL, "k must be >= 1");
  GU_TRY(stage(g, pos1, n1, pos2, n2));
  GuArgs& a = g->a;
  // np.argpartition(r, kth) needs kth < the row length (kth = k - 1 or k)
  const int kth = allow_nearest ? k - 1 : k;
  if (kth >= a.n2) return gfail(GF_EINVAL, "kth(=" + std::to_string(kth) + ") out of bounds (" + std::to_string(a.n2) + ")");
  a.k = k;
  a.allow_nearest = allow_nearest != 0;
  a.self_loops = self_loops != 0;
  GU_TRY(grow(g, B_SEL, (size_t)a.n1 * (k + 1), &a.sel));
  if (a.n1 > 0) {
    gu_knn_select_kernel<<<row_grid(a.n1), kGuThreads, 0, g->stream>>>(a);
    GU_HIP(hipGetLastError());
  }
  return finish(g, n_edges, [&] {
    gu_knn_fill_kernel<<<(a.n1 + kGuThreads - 1) / kGuThreads, kGuThreads, 0, g->stream>>>(a);
  });
}

int gu_get_edges(gu_graph* g, int32_t* senders, int32_t* receivers, double* r, double* diff) {
  if (!g) return gfail(GF_EINVAL, "null graph context");
  const int64_t E = g->n_edges;
  GU_HIP(hipSetDevice(g->device));
  if (E > 0) {
    const GuArgs& a = g->a;
    if (senders) GU_HIP(hipMemcpyAsync(senders, a.snd, sizeof(int32_t) * E, hipMemcpyDeviceToHost, g->stream));
    if (receivers) GU_HIP(hipMemcpyAsync(receivers, a.rcv, sizeof(int32_t) * E, hipMemcpyDeviceToHost, g->stream));
    if (r) GU_HIP(hipMemcpyAsync(r, a.r, sizeof(double) * E, hipMemcpyDeviceToHost, g->stream));
    if (diff) {
      GU_HIP(hipMemcpyAsync(diff, a.dx, sizeof(double) * E, hipMemcpyDeviceToHost, g->stream));
      GU_HIP(hipMemcpyAsync(diff + E, a.dy, sizeof(double) * E, hipMemcpyDeviceToHost, g->stream));
    }
  }
  GU_HIP(hipStreamSynchronize(g->stream));
  return GF_OK;
}

int gu_nodes_within_radius(gu_graph* g, const double* pos1, int32_t n1, const double* pos2, int32_t n2, double rad,
                           uint8_t* valid) {
  if (!pos2 || !valid) return gfail(GF_EINVAL, "pos2 and valid are required");
  GU_TRY(stage(g, pos1, n1, pos2, n2));
  GuArgs& a = g->a;
  a.rad = rad;
  GU_TRY(grow(g, B_VALID, (size_t)a.n2, &a.valid));
  if (a.n2 > 0) {
    gu_within_kernel<<<(a.n2 + kGuThreads - 1) / kGuThreads, kGuThreads, 0, g->stream>>>(a);
    GU_HIP(hipGetLastError());
    GU_HIP(hipMemcpyAsync(valid, a.valid, a.n2, hipMemcpyDeviceToHost, g->stream));
  }
  GU_HIP(hipStreamSynchronize(g->stream));
  return GF_OK;
}

}  // extern "C"
