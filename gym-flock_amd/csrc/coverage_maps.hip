// HIP kernels (gfx950) for Coverage-v0's per-episode target maps, batched over envs.
//
// Reference: CoverageEnv._generate_targets (gym_flock/envs/spatial/coverage.py:516-527),
// called by every reset() (:378-397), with generate_lattice (make_map.py:30-67) and
// generate_geometric_roads (make_map.py:207-231). Per env:
//   1. 12 cities U(-x_max, x_max)^2 from the global np.random (make_map.py:208): drawn
//      here from the env's own MT19937 stream (cov_map_cities_kernel), or given by the
//      caller (the drop-in env draws them from np.random itself);
//   2. the Delaunay edges of the cities (scipy/Qhull in the reference, :213-219): the
//      edges of every triangle whose circumcircle holds no other city strictly inside,
//      i.e. the unique triangulation of points in general position. Orientation and
//      incircle signs inside their rounding bound (Shewchuk's A bounds, x4) are not
//      decided here but reported (kMapNearDegenerate): Qhull's precision handling
//      decides those city sets (~1e-12 of maps);
//   3. waypoints p1 + (p2 - p1) / dist * k * road_radius, k < int(dist / road_radius),
//      dist = np.linalg.norm(p1 - p2) = sqrt(fma(dy, dy, dx * dx)) (OpenBLAS ddot's
//      fused multiply-add, :227), plus the cities themselves (:230);
//   4. lattice points whose nearest waypoint is within motion_radius / 1.4 (:521): the
//      root of the minimum squared norm (sqrt is monotone and correctly rounded);
//   5. their radius graph (0 < |p_i - p_j| <= motion_radius, :523-524) and its largest
//      connected component (:525-526): union-find in LDS, each component rooted at its
//      lowest node, so argmax(bincount(labels))'s first-label rule is the largest count
//      with the smallest root (scipy numbers components in order of their lowest node).
// The targets are that component's lattice points in lattice order (:526).
//
// One workgroup of 512 threads per env. The lattice (1,849 points at the defaults) is
// the same for every env and read through L2; waypoints, near flags, the union-find
// forest and the component counts live in LDS (~68 KB at the defaults). The link search
// walks the lattice's cell grid (a square lattice: K cells either side cover the link
// radius), not all pairs.
#include "coverage_internal.h"

namespace gf {

namespace {

constexpr int kMapThreads = 512;
constexpr int kMapWaves = kMapThreads / 64;
constexpr double kEps = 1.1102230246251565e-16;  // 2^-53
constexpr double kIccBound = 4.0 * (10.0 + 96.0 * kEps) * kEps;
constexpr double kCcwBound = 4.0 * (3.0 + 16.0 * kEps) * kEps;

// Exclusive scan of one int per thread over the workgroup; *total = the sum. wsum: LDS
// of kMapWaves + 1 ints. Every thread calls it.
__device__ int block_exscan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int k = 0; k < kMapWaves; ++k) {
      const int t = wsum[k];
      wsum[k] = run;
      run += t;
    }
    wsum[kMapWaves] = run;
  }
  __syncthreads();
  const int r = wsum[w] + x - v;
  *total = wsum[kMapWaves];
  __syncthreads();
  return r;
}

__device__ __forceinline__ int uf_find(volatile int32_t* p, int x) {
  for (int y = p[x]; y != x; y = p[x]) x = y;
  return x;
}

// Joins the trees of a and b: the larger root is hooked under the smaller, so a parent
// is always a lower index and each tree's root is its lowest node.
__device__ __forceinline__ void uf_unite(int32_t* p, int a, int b) {
  for (;;) {
    a = uf_find(p, a);
    b = uf_find(p, b);
    if (a == b) return;
    if (a > b) {
      const int t = a;
      a = b;
      b = t;
    }
    if (atomicCAS(&p[b], b, a) == b) return;
  }
}

// make_map.py:208 for env b: 2 * NC doubles of np.random.uniform from the env's stream
// (numpy's legacy random_sample: (a >> 5) * 2^26 + (b >> 6), over 2^53; then lo + range
// * u). One wave per env; every lane runs the draw chain, lane 0 writes.
__global__ __launch_bounds__(64) void cov_map_cities_kernel(CovMapArgs a) {
  __shared__ uint32_t key[kMtN];
  const int e = blockIdx.x;
  if (e >= a.n_sel) return;
  const int b = a.envs[e], lane = threadIdx.x;
  int pos;
  if (a.seed) {
    if (lane == 0) {
      uint32_t s = a.seed0 + static_cast<uint32_t>(b);
      for (int p = 0; p < kMtN; ++p) {
        key[p] = s;
        s = 1812433253u * (s ^ (s >> 30)) + static_cast<uint32_t>(p + 1);
      }
    }
    pos = kMtN;
  } else {
    for (int k = lane; k < kMtN; k += 64) key[k] = a.mt_key[(size_t)b * kMtN + k];
    pos = a.mt_pos[b];
  }
  __syncthreads();
  auto next = [&]() {
    if (pos == kMtN) {
      mt_regen<64>(key);
      pos = 0;
    }
    return mt_temper(key[pos++]);
  };
  double* out = a.cities + (size_t)b * kMapMaxCities * 2;
  for (int q = 0; q < 2 * a.NC; ++q) {
    const uint32_t hi = next() >> 5;
    const uint32_t lo = next() >> 6;
    const double u = (static_cast<double>(hi) * 67108864.0 + static_cast<double>(lo)) / 9007199254740992.0;
    if (lane == 0) out[q] = a.lo + a.range * u;
  }
  __syncthreads();
  for (int k = lane; k < kMtN; k += 64) a.mt_key[(size_t)b * kMtN + k] = key[k];
  if (lane == 0) a.mt_pos[b] = pos;
}

__global__ __launch_bounds__(kMapThreads) void cov_map_kernel(CovMapArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ double2 city[kMapMaxCities];
  __shared__ uint32_t adj[kMapMaxCities];
  __shared__ int2 elist[3 * kMapMaxCities];
  __shared__ int eoff[3 * kMapMaxCities + 1];
  __shared__ double edist[3 * kMapMaxCities];
  __shared__ int wsum[kMapWaves + 1];
  __shared__ int nedge_s, flags_s;
  __shared__ unsigned long long best_s;
  const int e = blockIdx.x;
  if (e >= a.n_sel) return;
  const int b = a.envs[e];
  const int tid = threadIdx.x, NC = a.NC, L = a.L;
  double2* wp = reinterpret_cast<double2*>(smem);      // (wcap) waypoints
  int32_t* parent = reinterpret_cast<int32_t*>(wp + a.wcap);  // (L) union-find forest
  int32_t* cnt = parent + L;                           // (L) component sizes by root
  int32_t* cidx = cnt + L;                             // (L) lattice point -> target node or -1
  int32_t* cend = cidx + L;                            // (G * G) waypoint grid: end of each cell's run
  int32_t* widx = cend + a.G * a.G;                    // (wcap) waypoints in cell order
  // 1. cities, no edges yet
  if (tid < NC) {
    const double* c = a.cities + ((size_t)b * kMapMaxCities + tid) * 2;
    city[tid] = make_double2(c[0], c[1]);
    adj[tid] = 0u;
  }
  if (tid == 0) {
    flags_s = 0;
    best_s = 0ull;
  }
  __syncthreads();
  // 2. Delaunay triangles: (i < j < k) with no city strictly inside their circumcircle
  for (int t = tid; t < NC * NC * NC; t += kMapThreads) {
    const int i = t / (NC * NC), j = (t / NC) % NC, k = t % NC;
    if (!(i < j && j < k)) continue;
    const double2 pa = city[i];
    double2 pb = city[j], pc = city[k];
    const double ol = (pa.x - pc.x) * (pb.y - pc.y), orr = (pa.y - pc.y) * (pb.x - pc.x);
    const double o = ol - orr;
    if (fabs(o) <= kCcwBound * (fabs(ol) + fabs(orr))) {
      atomicOr(&flags_s, kMapNearDegenerate);
      continue;
    }
    if (o < 0) {  // counter-clockwise (a, b, c): a positive incircle determinant is inside
      const double2 q = pb;
      pb = pc;
      pc = q;
    }
    bool inside = false, unsure = false;
    for (int m = 0; m < NC && !inside; ++m) {
      if (m == i || m == j || m == k) continue;
      const double2 d = city[m];
      const double adx = pa.x - d.x, ady = pa.y - d.y;
      const double bdx = pb.x - d.x, bdy = pb.y - d.y;
      const double cdx = pc.x - d.x, cdy = pc.y - d.y;
      const double bdxcdy = bdx * cdy, cdxbdy = cdx * bdy;
      const double cdxady = cdx * ady, adxcdy = adx * cdy;
      const double adxbdy = adx * bdy, bdxady = bdx * ady;
      const double alift = adx * adx + ady * ady;
      const double blift = bdx * bdx + bdy * bdy;
      const double clift = cdx * cdx + cdy * cdy;
      const double det = alift * (bdxcdy - cdxbdy) + blift * (cdxady - adxcdy) + clift * (adxbdy - bdxady);
      const double perm = (fabs(bdxcdy) + fabs(cdxbdy)) * alift + (fabs(cdxady) + fabs(adxcdy)) * blift +
                          (fabs(adxbdy) + fabs(bdxady)) * clift;
      const double bound = kIccBound * perm;
      if (det > bound) inside = true;
      else if (fabs(det) <= bound) unsure = true;
    }
    if (!inside) {
      if (unsure) atomicOr(&flags_s, kMapNearDegenerate);
      atomicOr(&adj[i], (1u << j) | (1u << k));
      atomicOr(&adj[j], (1u << i) | (1u << k));
      atomicOr(&adj[k], (1u << i) | (1u << j));
    }
  }
  __syncthreads();
  // 3. the roads (i < j, the reference's edge order; the order does not matter below)
  if (tid == 0) {
    int n = 0;
    for (int i = 0; i < NC; ++i)
      for (int j = i + 1; j < NC; ++j)
        if (((adj[i] >> j) & 1u) && n < 3 * kMapMaxCities) elist[n++] = make_int2(i, j);
    nedge_s = n;
  }
  __syncthreads();
  const int nedge = nedge_s;
  if (tid < nedge) {
    const double2 p1 = city[elist[tid].x], p2 = city[elist[tid].y];
    const double dx = p1.x - p2.x, dy = p1.y - p2.y;
    const double dist = sqrt(__fma_rn(dy, dy, dx * dx));
    edist[tid] = dist;
    eoff[tid + 1] = static_cast<int>(dist / a.road_radius);
  }
  __syncthreads();
  if (tid == 0) {
    eoff[0] = NC;
    for (int q = 0; q < nedge; ++q) eoff[q + 1] += eoff[q];
    if (eoff[nedge] > a.wcap) flags_s |= kMapOverflow;
  }
  __syncthreads();
  if (flags_s & kMapOverflow) {
    if (tid == 0) {
      a.ntg[b] = 0;
      a.nraw[b] = 0;
      a.status[b] = flags_s;
    }
    return;
  }
  const int W = eoff[nedge];
  if (tid < NC) wp[tid] = city[tid];
  for (int q = 0; q < nedge; ++q) {
    const double2 p1 = city[elist[q].x], p2 = city[elist[q].y];
    const double dist = edist[q];
    const double sx = (p2.x - p1.x) / dist, sy = (p2.y - p1.y) / dist;
    const int n = eoff[q + 1] - eoff[q];
    for (int k = tid; k < n; k += kMapThreads) {
      const double kk = static_cast<double>(k);
      wp[eoff[q] + k] = make_double2(p1.x + (sx * kk) * a.road_radius, p1.y + (sy * kk) * a.road_radius);
    }
  }
  __syncthreads();
  // 4. lattice points near a road: sqrt(min_w |p - w|^2) <= near_radius, i.e. (sqrt and
  // its rounding being monotone) some waypoint w with sqrt(|p - w|^2) <= near_radius
  const double nr = a.near_radius, n2lo = nr * nr * (1.0 - 0x1p-50), n2hi = nr * nr * (1.0 + 0x1p-50);
  auto near = [&](double2 p, double2 q) {  // the squared distance decides unless at the edge
    const double dx = p.x - q.x, dy = p.y - q.y, s = dx * dx + dy * dy;
    return s <= n2lo || (s <= n2hi && sqrt(s) <= nr);
  };
  if (a.G > 0) {
    // waypoints counting-sorted into cells of side gh > near_radius, so every waypoint
    // near p lies in the 3 x 3 cells around p's cell (the margin, gh - near_radius =
    // near_radius * 2^-20, dwarfs the rounding of the cell coordinates)
    const int G = a.G;
    auto gcell = [&](double v, double o) {
      const double f = (v - o) / a.gh;
      return f >= 0.0 ? (f < (double)G ? (int)f : G - 1) : 0;  // NaN: 0 (never near anything)
    };
    for (int c = tid; c < G * G; c += kMapThreads) cend[c] = 0;
    __syncthreads();
    for (int w = tid; w < W; w += kMapThreads) atomicAdd(&cend[gcell(wp[w].x, a.gx0) * G + gcell(wp[w].y, a.gy0)], 1);
    __syncthreads();
    const int per = (G * G + kMapThreads - 1) / kMapThreads;
    const int c0 = min(G * G, tid * per), c1 = min(G * G, c0 + per);
    int run = 0;
    for (int c = c0; c < c1; ++c) run += cend[c];
    int wtot;
    run = block_exscan(run, wsum, &wtot);
    for (int c = c0; c < c1; ++c) {  // each cell's start; the scatter below leaves its end
      const int n = cend[c];
      cend[c] = run;
      run += n;
    }
    __syncthreads();
    for (int w = tid; w < W; w += kMapThreads)
      widx[atomicAdd(&cend[gcell(wp[w].x, a.gx0) * G + gcell(wp[w].y, a.gy0)], 1)] = w;
    __syncthreads();
    for (int l = tid; l < L; l += kMapThreads) {
      const double2 p = a.lat[l];
      const int ci = gcell(p.x, a.gx0), cj = gcell(p.y, a.gy0);
      bool found = false;
      for (int i = max(ci - 1, 0); i <= min(ci + 1, G - 1) && !found; ++i)
        for (int j = max(cj - 1, 0); j <= min(cj + 1, G - 1) && !found; ++j) {
          const int c = i * G + j, k1 = cend[c];
          for (int k = c > 0 ? cend[c - 1] : 0; k < k1 && !found; ++k) found = near(p, wp[widx[k]]);
        }
      cidx[l] = found ? 1 : 0;
    }
  } else {
    for (int l = tid; l < L; l += kMapThreads) {  // every waypoint (LDS broadcasts)
      const double2 p = a.lat[l];
      bool found = false;
      for (int w = 0; w < W && !found; ++w) found = near(p, wp[w]);
      cidx[l] = found ? 1 : 0;
    }
  }
  __syncthreads();
  // 5a. number the near points in lattice order (contiguous chunks per thread)
  const int chunk = (L + kMapThreads - 1) / kMapThreads;
  const int l0 = min(L, tid * chunk), l1 = min(L, l0 + chunk);
  int local = 0;
  for (int l = l0; l < l1; ++l) local += cidx[l];
  int t0;
  int pos = block_exscan(local, wsum, &t0);
  for (int l = l0; l < l1; ++l) {
    if (cidx[l]) {
      parent[pos] = pos;
      cnt[pos] = 0;
      cidx[l] = pos++;
    } else {
      cidx[l] = -1;
    }
  }
  __syncthreads();
  // 5b. links to the points of the (2K+1)^2 cells around each point
  const int K = a.K, NJ = a.NJ;
  for (int l = tid; l < L; l += kMapThreads) {
    const int u = cidx[l];
    if (u < 0) continue;
    const int g = a.lat_cell[l], gi = g / NJ, gj = g - gi * NJ;
    const double2 p = a.lat[l];
    for (int di = -K; di <= K; ++di) {
      const int ni = gi + di;
      if (ni < 0 || ni >= a.NI) continue;
      for (int dj = -K; dj <= K; ++dj) {
        const int nj = gj + dj;
        if (nj < 0 || nj >= NJ) continue;
        const int l2 = a.cell[ni * NJ + nj];
        if (l2 < 0) continue;
        const int v = cidx[l2];
        if (v <= u) continue;  // each pair once
        const double2 q = a.lat[l2];
        const double dx = p.x - q.x, dy = p.y - q.y;
        const double r = sqrt(dx * dx + dy * dy);
        if (r > 0.0 && r <= a.link_radius) uf_unite(parent, u, v);
      }
    }
  }
  __syncthreads();
  // 5c. every node to its root, component sizes
  for (int u = tid; u < t0; u += kMapThreads) {
    const int r = uf_find(parent, u);
    parent[u] = r;
    atomicAdd(&cnt[r], 1);
  }
  __syncthreads();
  // 5d. the largest component, ties to the lowest root
  unsigned long long key = 0ull;
  for (int u = tid; u < t0; u += kMapThreads)
    if (parent[u] == u) {
      const unsigned long long k2 = (static_cast<unsigned long long>(cnt[u]) << 32) | (0xFFFFFFFFull - u);
      key = k2 > key ? k2 : key;
    }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(key, d, 64);
    key = o > key ? o : key;
  }
  if ((tid & 63) == 0) atomicMax(&best_s, key);
  __syncthreads();
  const unsigned long long best = best_s;
  const int T = static_cast<int>(best >> 32);
  const int root = static_cast<int>(0xFFFFFFFFull - (best & 0xFFFFFFFFull));
  int fl = flags_s;
  if (T > a.Tmax) fl |= kMapTooMany;
  if (T < a.R) fl |= kMapTooFew;
  if (fl & (kMapTooMany | kMapTooFew)) {
    if (tid == 0) {
      a.ntg[b] = 0;
      a.nraw[b] = T;
      a.status[b] = fl;
    }
    return;
  }
  // 6. the component's points in lattice order
  local = 0;
  for (int l = l0; l < l1; ++l) local += (cidx[l] >= 0 && parent[cidx[l]] == root) ? 1 : 0;
  int tot;
  pos = block_exscan(local, wsum, &tot);
  double2* out = reinterpret_cast<double2*>(a.tgt) + (size_t)b * a.Tmax;
  for (int l = l0; l < l1; ++l)
    if (cidx[l] >= 0 && parent[cidx[l]] == root) out[pos++] = a.lat[l];
  if (tid == 0) {
    a.ntg[b] = T;
    a.nraw[b] = T;
    a.status[b] = fl;
  }
}

}  // namespace

size_t cov_map_lds_bytes(int L, int wcap, int G) {
  return (size_t)wcap * 16 + (size_t)L * 12 + (G > 0 ? (size_t)G * G * 4 + (size_t)wcap * 4 : 0);
}

hipError_t launch_cov_map_cities(const CovMapArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(cov_map_cities_kernel, dim3(a.n_sel), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_cov_map(const CovMapArgs& a, hipStream_t s) {
  const size_t lds = cov_map_lds_bytes(a.L, a.wcap, a.G);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cov_map_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cov_map_kernel, dim3(a.n_sel), dim3(kMapThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace gf
