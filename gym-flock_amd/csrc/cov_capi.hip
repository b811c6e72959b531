// C-ABI of the Coverage-v0 engine (include/gymflock.h, cov_* functions).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "coverage_internal.h"
#include "device_alloc.h"
#include "gymflock.h"

namespace gf {
int set_error(int code, const std::string& msg);
}

namespace {

int cfail(int code, const std::string& m) { return gf::set_error(code, m); }

#define CV_HIP(expr)                                                                 \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) return cfail(GF_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
int calloc_dev(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) return GF_OK;
  hipError_t e = gf::device_alloc(reinterpret_cast<void**>(p), n * sizeof(T));
  if (e != hipSuccess) return cfail(GF_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMemset(*p, 0, n * sizeof(T));
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("hipMemset: ") + hipGetErrorString(e));
  // hipMemset may still be running on the null stream, which the handle's non-blocking
  // stream does not order against: finish it before any kernel writes the buffer
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("hipDeviceSynchronize: ") + hipGetErrorString(e));
  return GF_OK;
}

}  // namespace

struct cov_handle {
  cov_config cfg{};
  hipStream_t stream = nullptr;
  // Split steps as in fe_handle: envs [0, ceil(B/2)) step on `stream`, the rest on
  // `stream2`; each half depends only on its own previous step, every other call first
  // makes `stream` wait for `stream2`.
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_s2 = nullptr, ev_main = nullptr;
  // launches per step (cov_set_streams): 0 = auto, the greedy steps (COV_ACTIONS_GREEDY)
  // split in two, every other step one launch; 1; 2
  int nsplit = 0;
  bool s2_pending = false, main_dirty = true;
  bool other_work = true;  // non-step work since the last step: next step is one launch
  hipEvent_t tw[2] = {nullptr, nullptr};
  int64_t tw_steps = 0;
  gf::CovArgs a{};
  int32_t* ntg = nullptr;
  double* tgt = nullptr;
  int32_t* actions = nullptr;
  int32_t* start = nullptr;
  uint8_t* visited0 = nullptr;
  int32_t* envsel = nullptr;
  int* err = nullptr;
  std::vector<int> ntg_host;
  bool has_graph = false, has_state = false;
  // greedy expert (allocated on first use)
  uint16_t* tm_cost = nullptr;
  uint8_t* tm_cost8 = nullptr;   // uint8 copy of the cost rows (envs that fit), greedy step
  uint8_t* tm_wide = nullptr;    // (B) 1: the env's matrix needed uint16 entries
  std::vector<uint8_t> tm_wide_host;
  int16_t* tm_prevT = nullptr;
  uint16_t* tm_glist = nullptr;  // greedy lists (B,Tmax,gstride), Tmax <= kGreedyListMaxT
  uint16_t* tm_glen = nullptr;   // (B,Tmax)
  int gstride = 0;
  uint8_t* tm_flags = nullptr;
  uint8_t* needs_random = nullptr;
  int32_t* tm_envsel = nullptr;
  uint32_t* tm_sched = nullptr;
  int32_t* tm_lev = nullptr;  // (B, 4 * Tmax + 2): the schedule levels' slot offsets
  int32_t* tm_nslots = nullptr;
  int32_t* tm_nlev = nullptr;
  uint8_t* tm_overflow = nullptr;
  std::vector<int> n_motion_host;
  std::vector<char> tm_valid;
  bool tm_ready = false;           // every env's time matrix (and greedy lists) is current
  int64_t tm_wide_envs = 0;  // envs whose matrix needed uint16 entries (diagnostics)
  // wire formats: scratch for host-bound outputs, graph-tuple offsets
  unsigned char* scratch = nullptr;
  size_t scratch_bytes = 0;
  int64_t* goff = nullptr;
  // step-kernel timing (cov_kernel_timing): HIP events around every stride-th launch
  bool timing = false;
  int timing_stride = 1;
  int64_t timing_count = 0;
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  int32_t* herr = nullptr;  // cov_step_host: page-locked per-env copies of the error word
  // cov_step_host: the launch's completion flag (done_flag.h): device counter, page-locked
  // word, its mapped address
  int32_t* fin_cnt = nullptr;
  int32_t* fin_host = nullptr;
  int32_t* fin_dev = nullptr;
  int32_t fin_seq = 0;
  // COV_GREEDY_RNG: every env's np_random stream (cov_set_rng; allocated on first use)
  uint32_t* mt_key = nullptr;  // (B,624)
  int32_t* mt_pos = nullptr;   // (B)
  // cov_generate_maps (allocated on first use): each env's map stream (the reference's
  // global np.random), its cities, the kernel's per-env outputs, and the lattice of the
  // last map configuration (the same for every env)
  uint32_t* map_key = nullptr;   // (B,624)
  int32_t* map_pos = nullptr;    // (B)
  bool map_seeded = false;
  double* map_cities = nullptr;  // (B, kMapMaxCities, 2)
  int32_t* map_nraw = nullptr;   // (B)
  int32_t* map_status = nullptr; // (B)
  double2* lat = nullptr;        // (L)
  int32_t* lat_cell = nullptr;   // (L)
  int32_t* lat_grid = nullptr;   // (NI * NJ)
  int lat_L = 0, lat_NI = 0, lat_NJ = 0;
  double lat_key[5] = {0, 0, 0, 0, 0};  // x_min, x_max, y_min, y_max, spacing of `lat`
};

namespace {

int join_s2(cov_handle* h) {
  if (h->s2_pending) {
    CV_HIP(hipEventRecord(h->ev_s2, h->stream2));
    CV_HIP(hipStreamWaitEvent(h->stream, h->ev_s2, 0));
    h->s2_pending = false;
  }
  return GF_OK;
}

// Every call but cov_step: the device, `stream` after all outstanding work, and what
// it enqueues ordered before the next second-half step.
int use(cov_handle* h) {
  CV_HIP(hipSetDevice(h->cfg.device));
  if (int rc = join_s2(h)) return rc;
  h->main_dirty = true;
  h->other_work = true;
  return GF_OK;
}

void cov_release(cov_handle* h) {
  if (!h) return;
  hipSetDevice(h->cfg.device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->stream2) hipStreamSynchronize(h->stream2);
  gf::CovArgs& a = h->a;
  void* bufs[] = {h->ntg, h->tgt, a.nbr, a.cnt, a.n_motion, a.xr, a.cur, a.visited, a.nvisited,
                  a.step_counter, a.dirty, h->actions, a.reward, a.done, a.nodes, a.edges, a.senders,
                  a.receivers, a.obs_step, a.axy, a.nrec, h->err, h->start, h->visited0, h->envsel, h->tm_cost, h->tm_cost8, h->tm_wide, h->tm_prevT, h->tm_glist, h->tm_glen,
                  h->tm_flags, h->needs_random, h->tm_envsel, h->tm_sched, h->tm_lev, h->tm_nslots, h->tm_nlev, h->tm_overflow, h->scratch,
                  h->goff, h->mt_key, h->mt_pos, h->map_key, h->map_pos, h->map_cities, h->map_nraw,
                  h->map_status, h->lat, h->lat_cell, h->lat_grid};
  for (void* p : bufs)
    if (p) hipFree(p);
  for (hipEvent_t e : h->ev) hipEventDestroy(e);
  if (h->herr) hipHostFree(h->herr);
  if (h->fin_cnt) hipFree(h->fin_cnt);
  if (h->fin_host) hipHostFree(h->fin_host);
  for (hipEvent_t e : {h->ev_s2, h->ev_main, h->tw[0], h->tw[1]})
    if (e) hipEventDestroy(e);
  if (h->stream) hipStreamDestroy(h->stream);
  if (h->stream2) hipStreamDestroy(h->stream2);
  delete h;
}

// Read and clear the device error bits; translate to a status.
int check_err(cov_handle* h) {
  int err = 0;
  CV_HIP(hipMemcpyAsync(&err, h->err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  if (!err) return GF_OK;
  CV_HIP(hipMemsetAsync(h->err, 0, sizeof(int), h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  std::string m;
  if (err & 1) m += "a target has more than 4 motion-graph neighbours (coverage.py:257 assert); ";
  if (err & 2) m += "motion edges + 8*n_robots exceed 4*max_nodes (\"Increase MAX_EDGES\", coverage.py:288); ";
  if (err & 4) m += "action outside [0, 4) (coverage.py:189 index); ";
  if (err & 8) m += "greedy next hop is not among the robot's action targets (IndexError at coverage.py:869); ";
  return cfail(GF_EINVAL, m);
}

int copy_out(cov_handle* h, void* dst, const void* src, size_t bytes) {
  if (!dst) return GF_OK;
  CV_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  return GF_OK;
}

// Time matrices of every env whose graph changed since they were last built.
int ensure_time_matrix(cov_handle* h) {
  const int B = h->cfg.n_envs, Tm = h->a.Tmax;
  const int kcap = h->cfg.horizon > -1 ? h->cfg.horizon + 1 : Tm + 1;
  const int nchunk = (Tm + 63) / 64;
  const int sched_stride = 4 * Tm * 16 + 16;  // motion edges <= 4 per target, batches <= 16, + prefetch slack
  if (!h->tm_cost) {
    int rc;
    if ((rc = calloc_dev(&h->tm_cost, (size_t)B * Tm * Tm)) || (rc = calloc_dev(&h->tm_prevT, (size_t)B * Tm * Tm)) ||
        (rc = calloc_dev(&h->tm_flags, (size_t)B * nchunk * kcap)) ||
        (rc = calloc_dev(&h->needs_random, (size_t)B * h->cfg.n_robots)) || (rc = calloc_dev(&h->tm_envsel, (size_t)B)) ||
        (rc = calloc_dev(&h->tm_sched, (size_t)B * sched_stride)) || (rc = calloc_dev(&h->tm_nslots, (size_t)B)) ||
        (rc = calloc_dev(&h->tm_lev, (size_t)B * (4 * Tm + 2))) ||
        (rc = calloc_dev(&h->tm_nlev, (size_t)B)) || (rc = calloc_dev(&h->tm_overflow, (size_t)B)) ||
        (rc = calloc_dev(&h->tm_cost8, (size_t)B * Tm * Tm)) || (rc = calloc_dev(&h->tm_wide, (size_t)B)))
      return rc;
    if (Tm <= gf::kGreedyListMaxT) {  // rows padded to 16 bytes (greedy_from_list's loads)
      h->gstride = (Tm + gf::kGreedyListPad - 1) & ~(gf::kGreedyListPad - 1);
      if ((rc = calloc_dev(&h->tm_glist, (size_t)B * Tm * h->gstride)) || (rc = calloc_dev(&h->tm_glen, (size_t)B * Tm)))
        return rc;
    }
    h->tm_wide_host.assign(B, 0);
  }
  std::vector<int32_t> sel;
  int t_lds = 0, e_max = 0;
  for (int b = 0; b < B; ++b) {
    if (h->tm_valid[b]) continue;
    sel.push_back(b);
    t_lds = std::max(t_lds, h->ntg_host[b]);
    e_max = std::max(e_max, h->n_motion_host[b]);
  }
  if (sel.empty()) {
    h->tm_ready = true;
    return GF_OK;
  }
  if (gf::cov_time_matrix_lds_bytes(t_lds, false) > 160 * 1024 ||
      gf::cov_tm_schedule_lds_bytes(t_lds, e_max) > 160 * 1024)
    return cfail(GF_EINVAL, "time matrix: (n_targets + 1) * 64 bytes exceed the 160 KB LDS of a CU");
  gf::CovTmArgs t{};
  t.R = h->a.R;
  t.M = h->a.M;
  t.Tmax = Tm;
  t.horizon = h->cfg.horizon;
  t.kcap = kcap;
  t.nchunk = nchunk;
  t.t_lds = t_lds;
  t.envs = h->tm_envsel;
  t.ntg = h->ntg;
  t.n_motion = h->a.n_motion;
  t.senders = h->a.senders;
  t.receivers = h->a.receivers;
  t.flags = h->tm_flags;
  t.cost = h->tm_cost;
  t.cost8 = h->tm_cost8;
  t.prevT = h->tm_prevT;
  t.sched = h->tm_sched;
  t.nslots = h->tm_nslots;
  t.nlev = h->tm_nlev;
  t.overflow = h->tm_overflow;
  t.sched_stride = sched_stride;
  t.lev_off = h->tm_lev;
  t.lev_stride = 4 * Tm + 2;  // levels <= motion edges <= 4 per target, + the end offset
  CV_HIP(hipMemcpyAsync(h->tm_envsel, sel.data(), sel.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
  hipError_t e = gf::launch_cov_tm_schedule(t, (int)sel.size(), e_max, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_tm_schedule_kernel: ") + hipGetErrorString(e));
  // uint8 entries first (twice the waves per CU); envs it cannot bound get uint16
  e = gf::launch_cov_time_matrix(t, (int)sel.size(), false, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_time_matrix_kernel: ") + hipGetErrorString(e));
  std::vector<uint8_t> ovf(B);
  CV_HIP(hipMemcpyAsync(ovf.data(), h->tm_overflow, B, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  std::vector<int32_t> wide;
  int t_wide = 0;
  for (int b : sel)
    if (ovf[b]) {
      wide.push_back(b);
      t_wide = std::max(t_wide, h->ntg_host[b]);
    }
  if (!wide.empty()) {
    if (gf::cov_time_matrix_lds_bytes(t_wide, true) > 160 * 1024)
      return cfail(GF_EINVAL, "time matrix: hop counts above 254 need (n_targets + 1) * 128 bytes of LDS (> 160 KB)");
    CV_HIP(hipMemsetAsync(h->tm_overflow, 0, B, h->stream));
    CV_HIP(hipMemcpyAsync(h->tm_envsel, wide.data(), wide.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
    t.t_lds = t_wide;
    e = gf::launch_cov_time_matrix(t, (int)wide.size(), true, h->stream);
    if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_time_matrix_kernel: ") + hipGetErrorString(e));
    CV_HIP(hipStreamSynchronize(h->stream));
  }
  h->tm_wide_envs += (int64_t)wide.size();
  for (int b : sel) h->tm_wide_host[b] = 0;
  for (int b : wide) h->tm_wide_host[b] = 1;
  CV_HIP(hipMemcpyAsync(h->tm_wide, h->tm_wide_host.data(), B, hipMemcpyHostToDevice, h->stream));
  if (h->tm_glist) {  // every selected env's greedy lists, from its final matrix
    t.wide = h->tm_wide;
    t.nbr = h->a.nbr;
    t.cnt = h->a.cnt;
    t.glist = h->tm_glist;
    t.glen = h->tm_glen;
    t.gstride = h->gstride;
    CV_HIP(hipMemcpyAsync(h->tm_envsel, sel.data(), sel.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
    e = gf::launch_cov_greedy_lists(t, (int)sel.size(), h->stream);
    if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_greedy_list_kernel: ") + hipGetErrorString(e));
  }
  CV_HIP(hipStreamSynchronize(h->stream));
  for (int b : sel) h->tm_valid[b] = 1;
  h->tm_ready = true;
  return GF_OK;
}

// Device scratch of at least `bytes` (grown on demand, reused across calls).
int scratch(cov_handle* h, size_t bytes, unsigned char** out) {
  if (bytes > h->scratch_bytes) {
    if (h->scratch) CV_HIP(hipFree(h->scratch));
    h->scratch = nullptr;
    h->scratch_bytes = 0;
    if (hipMalloc(reinterpret_cast<void**>(&h->scratch), bytes) != hipSuccess)
      return cfail(GF_ENOMEM, "hipMalloc of wire-format scratch failed");
    h->scratch_bytes = bytes;
  }
  *out = h->scratch;
  return GF_OK;
}

// Edge counts of the unpack_obs tuple and their exclusive offsets.
void graph_sizes(const cov_handle* h, bool mask_all, std::vector<int32_t>& ne, std::vector<int64_t>& off) {
  const int B = h->cfg.n_envs, R = h->cfg.n_robots, M = h->cfg.max_nodes;
  ne.assign(B, 0);
  off.assign(B + 1, 0);
  for (int b = 0; b < B; ++b) {
    ne[b] = (mask_all || b == 0) ? h->n_motion_host[b] + 8 * R : 4 * M;
    off[b + 1] = off[b] + ne[b];
  }
}

// Python's float floor division (numpy floor_divide on float64), for generate_lattice's
// `//` (make_map.py:40, :45-46).
double py_floordiv(double a, double b) {
  double mod = std::fmod(a, b);
  double div = (a - mod) / b;
  if (mod != 0.0 && ((b < 0) != (mod < 0))) div -= 1.0;
  if (div == 0.0) return std::copysign(0.0, a / b);
  double fl = std::floor(div);
  if (div - fl > 0.5) fl += 1.0;
  return fl;
}

int check_map_config(const cov_map_config* mc) {
  if (!mc) return cfail(GF_EINVAL, "null map configuration");
  if (!(mc->x_max > mc->x_min) || !(mc->y_max > mc->y_min)) return cfail(GF_EINVAL, "map: empty arena");
  if (!(mc->lattice_spacing > 0) || !(mc->world_radius > 0) || !(mc->road_radius > 0) || !(mc->near_radius > 0) ||
      !(mc->link_radius > 0))
    return cfail(GF_EINVAL, "map: spacing and radii must be positive");
  if (mc->n_cities < 3 || mc->n_cities > gf::kMapMaxCities) return cfail(GF_EINVAL, "map: n_cities must be in [3, 32]");
  return GF_OK;
}

// generate_lattice (make_map.py:30-67) with the square lattice vectors (-s, 0), (0, -s)
// (coverage.py:125-128): the points in its order as [y, x], and each point's cell
// i * NJ + j in the (arange(-nx, nx), arange(-ny, nx)) grid it sheared.
void build_lattice(const cov_map_config* mc, std::vector<double>& xy, std::vector<int32_t>& cell, int* NI, int* NJ) {
  const double s = mc->lattice_spacing;
  const double w = mc->x_max - mc->x_min, hgt = mc->y_max - mc->y_min;
  const double cx = py_floordiv(w, 2.0), cy = py_floordiv(hgt, 2.0);
  const double nx = py_floordiv(w, s), ny = py_floordiv(hgt, s);
  const int ni = static_cast<int>(std::ceil(nx - -nx)), nj = static_cast<int>(std::ceil(nx - -ny));  // np.arange lengths
  xy.clear();
  cell.clear();
  for (int i = 0; i < ni; ++i) {
    const double xs = -nx + i;
    for (int j = 0; j < nj; ++j) {
      const double ys = -ny + j;
      const double xl = -s * xs + 0.0 * ys, yl = 0.0 * xs + -s * ys;
      if (xl < w / 2.0 && xl > -w / 2.0 && yl < hgt / 2.0 && yl > -hgt / 2.0) {
        xy.push_back(yl + (cy + mc->y_min));
        xy.push_back(xl + (cx + mc->x_min));
        cell.push_back(i * nj + j);
      }
    }
  }
  *NI = ni;
  *NJ = nj;
}

// The lattice of mc on the device (rebuilt when the arena or spacing changes).
int ensure_lattice(cov_handle* h, const cov_map_config* mc) {
  const double key[5] = {mc->x_min, mc->x_max, mc->y_min, mc->y_max, mc->lattice_spacing};
  if (h->lat && std::memcmp(key, h->lat_key, sizeof(key)) == 0) return GF_OK;
  std::vector<double> xy;
  std::vector<int32_t> cell;
  int NI = 0, NJ = 0;
  build_lattice(mc, xy, cell, &NI, &NJ);
  const int L = static_cast<int>(cell.size());
  if (L < 1) return cfail(GF_EINVAL, "map: the lattice has no point in the arena");
  if ((size_t)NI * NJ > (size_t)1 << 26) return cfail(GF_EINVAL, "map: lattice grid too large");
  for (void* p : {static_cast<void*>(h->lat), static_cast<void*>(h->lat_cell), static_cast<void*>(h->lat_grid)})
    if (p) CV_HIP(hipFree(p));
  h->lat = nullptr;
  h->lat_cell = h->lat_grid = nullptr;
  std::vector<int32_t> grid((size_t)NI * NJ, -1);
  for (int l = 0; l < L; ++l) grid[cell[l]] = l;
  int rc;
  if ((rc = calloc_dev(&h->lat, (size_t)L)) || (rc = calloc_dev(&h->lat_cell, (size_t)L)) ||
      (rc = calloc_dev(&h->lat_grid, (size_t)NI * NJ)))
    return rc;
  CV_HIP(hipMemcpy(h->lat, xy.data(), (size_t)L * 16, hipMemcpyHostToDevice));
  CV_HIP(hipMemcpy(h->lat_cell, cell.data(), (size_t)L * 4, hipMemcpyHostToDevice));
  CV_HIP(hipMemcpy(h->lat_grid, grid.data(), grid.size() * 4, hipMemcpyHostToDevice));
  h->lat_L = L;
  h->lat_NI = NI;
  h->lat_NJ = NJ;
  std::memcpy(h->lat_key, key, sizeof(key));
  return GF_OK;
}

int put(cov_handle* h, void* dst, const void* src, size_t bytes, bool dev_dst, bool dev_src) {
  if (!dst || !bytes) return GF_OK;
  const hipMemcpyKind k = dev_dst ? (dev_src ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                                  : (dev_src ? hipMemcpyDeviceToHost : hipMemcpyHostToHost);
  CV_HIP(hipMemcpyAsync(dst, src, bytes, k, h->stream));
  return GF_OK;
}

}  // namespace

extern "C" {

int cov_create(const cov_config* cfg, cov_handle** out) {
  if (!cfg || !out) return cfail(GF_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->n_robots < 1 || cfg->n_envs < 1 || cfg->max_nodes <= cfg->n_robots)
    return cfail(GF_EINVAL, "need n_robots >= 1, n_envs >= 1, max_nodes > n_robots");
  if (cfg->n_robots > 4096) return cfail(GF_EINVAL, "n_robots > 4096 not supported");
  if (!(cfg->res > 0) || !(cfg->motion_radius > 0)) return cfail(GF_EINVAL, "bad res/motion_radius");
  if (cfg->horizon < -1) return cfail(GF_EINVAL, "horizon must be >= -1");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return cfail(GF_EHIP, "no HIP device available (libgymflock needs an MI355X)");
  if (cfg->device < 0 || cfg->device >= ndev) return cfail(GF_EINVAL, "device ordinal out of range");
  cov_handle* h = new cov_handle();
  h->cfg = *cfg;
  const size_t B = cfg->n_envs, R = cfg->n_robots, M = cfg->max_nodes, Tm = M - R, E = 4 * M;
  gf::CovArgs& a = h->a;
  a.B = (int)B;
  a.R = (int)R;
  a.M = (int)M;
  a.Tmax = (int)Tm;
  a.episode_length = cfg->episode_length;
  a.res = cfg->res;
  a.motion_radius = cfg->motion_radius;
  int rc = GF_OK;
  if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_s2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_main, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&h->tw[0]) != hipSuccess || hipEventCreate(&h->tw[1]) != hipSuccess) {
    cov_release(h);
    return cfail(GF_EHIP, "stream create failed");
  }
  if ((rc = calloc_dev(&h->ntg, B)) || (rc = calloc_dev(&h->tgt, B * Tm * 2)) || (rc = calloc_dev(&a.nbr, B * Tm * 4)) ||
      (rc = calloc_dev(&a.cnt, B * Tm)) || (rc = calloc_dev(&a.n_motion, B)) || (rc = calloc_dev(&a.xr, B * R * 2)) ||
      (rc = calloc_dev(&a.cur, B * R)) || (rc = calloc_dev(&a.visited, B * Tm)) || (rc = calloc_dev(&a.nvisited, B)) ||
      (rc = calloc_dev(&a.step_counter, B)) || (rc = calloc_dev(&a.dirty, B)) || (rc = calloc_dev(&h->actions, B * R)) ||
      (rc = calloc_dev(&a.reward, B)) || (rc = calloc_dev(&a.done, B)) || (rc = calloc_dev(&a.nodes, B * M * 3)) ||
      (rc = calloc_dev(&a.edges, B * E)) || (rc = calloc_dev(&a.senders, B * E)) || (rc = calloc_dev(&a.receivers, B * E)) ||
      (rc = calloc_dev(&a.obs_step, B)) || (rc = calloc_dev(&a.axy, B * Tm * 8)) || (rc = calloc_dev(&a.nrec, B * Tm * 16)) || (rc = calloc_dev(&h->err, 1)) || (rc = calloc_dev(&h->start, B * R)) ||
      (rc = calloc_dev(&h->visited0, B * Tm)) || (rc = calloc_dev(&h->envsel, B))) {
    cov_release(h);
    return rc;
  }
  a.tgt = h->tgt;
  a.ntg = h->ntg;
  a.err = h->err;
  h->ntg_host.assign(B, 0);
  h->n_motion_host.assign(B, 0);
  h->tm_valid.assign(B, 0);
  *out = h;
  return GF_OK;
}

int cov_destroy(cov_handle* h) {
  cov_release(h);
  return GF_OK;
}

int cov_set_targets(cov_handle* h, int env, int n_targets, const double* targets) {
  if (!h || !targets) return cfail(GF_EINVAL, "null argument");
  const int B = h->cfg.n_envs, Tm = h->a.Tmax;
  if (env >= B) return cfail(GF_EINVAL, "env index out of range");
  if (n_targets < 1 || n_targets > Tm)
    return cfail(GF_EINVAL, "n_targets must be in [1, max_nodes - n_robots] (PAD_NODES, coverage.py:540-543)");
  if (n_targets < h->cfg.n_robots) return cfail(GF_EINVAL, "fewer targets than robots (reset draws distinct starts)");
  if (int rc = use(h)) return rc;
  const int b0 = env < 0 ? 0 : env, b1 = env < 0 ? B : env + 1;
  std::vector<int32_t> sel;
  for (int b = b0; b < b1; ++b) {
    CV_HIP(hipMemcpyAsync(h->tgt + (size_t)b * Tm * 2, targets, (size_t)n_targets * 2 * sizeof(double),
                          hipMemcpyHostToDevice, h->stream));
    h->ntg_host[b] = n_targets;
    sel.push_back(b);
  }
  CV_HIP(hipMemcpyAsync(h->ntg, h->ntg_host.data(), B * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
  CV_HIP(hipMemcpyAsync(h->envsel, sel.data(), sel.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
  hipError_t e = gf::launch_cov_graph(h->a, h->envsel, (int)sel.size(), h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_graph_kernel: ") + hipGetErrorString(e));
  if (int rc = check_err(h)) return rc;
  CV_HIP(hipMemcpy(h->n_motion_host.data(), h->a.n_motion, B * sizeof(int32_t), hipMemcpyDeviceToHost));
  for (int b = b0; b < b1; ++b) h->tm_valid[b] = 0;
  h->tm_ready = false;
  h->has_graph = true;
  for (int b = 0; b < B; ++b) h->has_graph = h->has_graph && h->ntg_host[b] > 0;
  return GF_OK;
}

int cov_map_lattice(const cov_map_config* mc, double* xy, int32_t* n) {
  if (!n) return cfail(GF_EINVAL, "null count");
  if (int rc = check_map_config(mc)) return rc;
  std::vector<double> pts;
  std::vector<int32_t> cell;
  int NI = 0, NJ = 0;
  build_lattice(mc, pts, cell, &NI, &NJ);
  const int32_t cap = *n;
  *n = static_cast<int32_t>(cell.size());
  if (!xy) return GF_OK;
  if (cap < *n) return cfail(GF_EINVAL, "lattice: the output holds fewer points than the lattice has");
  std::memcpy(xy, pts.data(), pts.size() * sizeof(double));
  return GF_OK;
}

int cov_generate_maps(cov_handle* h, const cov_map_config* mc, int env, uint64_t map_seed, const double* cities,
                      int flags, int32_t* n_targets_out, int32_t* status_out, double* cities_out) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (int rc = check_map_config(mc)) return rc;
  if (flags & ~(COV_MAP_SEED | COV_MAP_CITIES)) return cfail(GF_EINVAL, "flags: COV_MAP_SEED | COV_MAP_CITIES");
  const bool given = flags & COV_MAP_CITIES;
  if (given && !cities) return cfail(GF_EINVAL, "COV_MAP_CITIES needs the cities");
  const int B = h->cfg.n_envs, NC = mc->n_cities;
  if (env >= B) return cfail(GF_EINVAL, "env index out of range");
  if (!given && (flags & COV_MAP_SEED) && map_seed + (uint64_t)B > 0x100000000ull)
    return cfail(GF_EINVAL, "map_seed + n_envs must fit in 32 bits (np.random.seed)");
  if (!given && !(flags & COV_MAP_SEED) && !h->map_seeded)
    return cfail(GF_ESTATE, "the envs' map streams were never seeded (COV_MAP_SEED)");
  if (int rc = use(h)) return rc;
  int rc;
  if (!h->map_cities) {
    if ((rc = calloc_dev(&h->map_key, (size_t)B * gf::kMtN)) || (rc = calloc_dev(&h->map_pos, (size_t)B)) ||
        (rc = calloc_dev(&h->map_cities, (size_t)B * gf::kMapMaxCities * 2)) || (rc = calloc_dev(&h->map_nraw, (size_t)B)) ||
        (rc = calloc_dev(&h->map_status, (size_t)B)))
      return rc;
  }
  if ((rc = ensure_lattice(h, mc))) return rc;
  // waypoints: the cities plus at most int(dist / road_radius) per Delaunay edge (at most
  // 3 NC - 6 of them, none longer than the cities' square's diagonal), within the LDS left
  const double diag = 2.0 * std::sqrt(2.0) * mc->world_radius;
  const double wbound = NC + (3.0 * NC - 6.0) * (std::floor(diag / mc->road_radius) + 1.0);
  const size_t lds_max = 150 * 1024, lds_lat = (size_t)h->lat_L * 12;
  if (lds_lat + 64 * 16 > lds_max) return cfail(GF_EINVAL, "map: lattice too large for the LDS");
  // the waypoint grid of the near-road test: cells of side near_radius (1 + 2^-20) over the
  // cities' square and the arena, one cell of margin; without room for it (or for an odd
  // configuration), every lattice point scans every waypoint
  const double gh = mc->near_radius * (1.0 + 0x1p-20);
  const double gx0 = std::min(mc->x_min, -mc->world_radius) - gh, gy0 = std::min(mc->y_min, -mc->world_radius) - gh;
  const double gspan = std::max(std::max(mc->x_max, mc->world_radius) + gh - gx0, std::max(mc->y_max, mc->world_radius) + gh - gy0);
  int G = (gh > 0.0 && std::isfinite(gspan / gh) && gspan / gh < 256.0) ? static_cast<int>(std::ceil(gspan / gh)) : 0;
  const double wcap_scan = std::min<double>(wbound, (double)((lds_max - lds_lat) / 16));
  const double wfit_g = G > 0 ? ((double)lds_max - (double)lds_lat - 4.0 * G * G) / 20.0 : 0.0;
  if (wfit_g < wcap_scan) G = 0;  // the grid would cost waypoint capacity
  const int wcap = static_cast<int>(wcap_scan);
  const int b0 = env < 0 ? 0 : env, b1 = env < 0 ? B : env + 1, nsel = b1 - b0;
  std::vector<int32_t> sel;
  for (int b = b0; b < b1; ++b) sel.push_back(b);
  CV_HIP(hipMemcpyAsync(h->envsel, sel.data(), sel.size() * 4, hipMemcpyHostToDevice, h->stream));
  gf::CovMapArgs m{};
  m.n_sel = nsel;
  m.envs = h->envsel;
  m.R = h->a.R;
  m.Tmax = h->a.Tmax;
  m.NC = NC;
  m.lo = -mc->world_radius;
  m.range = mc->world_radius - -mc->world_radius;  // uniform(low, high): high - low
  m.road_radius = mc->road_radius;
  m.near_radius = mc->near_radius;
  m.link_radius = mc->link_radius;
  m.L = h->lat_L;
  m.lat = h->lat;
  m.lat_cell = h->lat_cell;
  m.cell = h->lat_grid;
  m.NI = h->lat_NI;
  m.NJ = h->lat_NJ;
  m.K = static_cast<int>(std::floor(mc->link_radius / mc->lattice_spacing)) + 1;
  m.wcap = wcap;
  m.G = G;
  m.gx0 = gx0;
  m.gy0 = gy0;
  m.gh = gh;
  m.cities = h->map_cities;
  m.mt_key = h->map_key;
  m.mt_pos = h->map_pos;
  m.seed0 = static_cast<uint32_t>(map_seed);
  m.seed = (flags & COV_MAP_SEED) ? 1 : 0;
  m.tgt = h->tgt;
  m.ntg = h->ntg;
  m.nraw = h->map_nraw;
  m.status = h->map_status;
  hipError_t e = hipSuccess;
  if (given) {
    CV_HIP(hipMemcpy2DAsync(h->map_cities + (size_t)b0 * gf::kMapMaxCities * 2, gf::kMapMaxCities * 16, cities,
                            (size_t)NC * 16, (size_t)NC * 16, nsel, hipMemcpyHostToDevice, h->stream));
  } else {
    e = gf::launch_cov_map_cities(m, h->stream);
    if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_map_cities_kernel: ") + hipGetErrorString(e));
    if (flags & COV_MAP_SEED) h->map_seeded = true;
  }
  e = gf::launch_cov_map(m, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_map_kernel: ") + hipGetErrorString(e));
  e = gf::launch_cov_graph(h->a, h->envsel, nsel, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_graph_kernel: ") + hipGetErrorString(e));
  std::vector<int32_t> nraw(nsel), st(nsel), ntg(B);
  CV_HIP(hipMemcpyAsync(nraw.data(), h->map_nraw + b0, nsel * 4, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipMemcpyAsync(st.data(), h->map_status + b0, nsel * 4, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipMemcpyAsync(ntg.data(), h->ntg, B * 4, hipMemcpyDeviceToHost, h->stream));
  if (cities_out)
    CV_HIP(hipMemcpy2DAsync(cities_out, (size_t)NC * 16, h->map_cities + (size_t)b0 * gf::kMapMaxCities * 2,
                            gf::kMapMaxCities * 16, (size_t)NC * 16, nsel, hipMemcpyDeviceToHost, h->stream));
  if (int rc2 = check_err(h)) return rc2;  // synchronises; motion-graph errors (degree > 4, edges)
  CV_HIP(hipMemcpy(h->n_motion_host.data(), h->a.n_motion, B * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::string bad;
  for (int k = 0; k < nsel; ++k) {
    const int b = b0 + k;
    h->ntg_host[b] = ntg[b];
    h->tm_valid[b] = 0;
    if (n_targets_out) n_targets_out[k] = nraw[k];
    if (status_out) status_out[k] = st[k];
    if (bad.empty() && (st[k] & (gf::kMapTooMany | gf::kMapTooFew | gf::kMapOverflow))) {
      bad = "env " + std::to_string(b) + ": ";
      if (st[k] & gf::kMapTooMany)
        bad += "the map has " + std::to_string(nraw[k]) + " targets, more than max_nodes - n_robots = " +
               std::to_string(h->a.Tmax) + " (the reference's padded observation cannot hold them)";
      else if (st[k] & gf::kMapTooFew)
        bad += "the map has " + std::to_string(nraw[k]) + " targets, fewer than the robots";
      else
        bad += "more road waypoints than the map kernel holds";
    }
  }
  h->tm_ready = false;
  h->has_graph = true;
  for (int b = 0; b < B; ++b) h->has_graph = h->has_graph && h->ntg_host[b] > 0;
  if (!bad.empty()) return cfail(GF_EINVAL, "cov_generate_maps: " + bad);
  return GF_OK;
}

int cov_get_targets(cov_handle* h, int env, double* targets) {
  if (!h || !targets || env < 0 || env >= h->cfg.n_envs) return cfail(GF_EINVAL, "bad argument");
  if (h->ntg_host[env] < 1) return cfail(GF_ESTATE, "the env has no target map");
  if (int rc = use(h)) return rc;
  CV_HIP(hipMemcpyAsync(targets, h->tgt + (size_t)env * h->a.Tmax * 2, (size_t)h->ntg_host[env] * 16,
                        hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_reset(cov_handle* h, const int32_t* start, const uint8_t* visited) {
  if (!h || !start || !visited) return cfail(GF_EINVAL, "null argument");
  if (!h->has_graph) return cfail(GF_ESTATE, "set the target graph of every env first (cov_set_targets)");
  const size_t B = h->cfg.n_envs, R = h->cfg.n_robots, Tm = h->a.Tmax;
  for (size_t b = 0; b < B; ++b)
    for (size_t i = 0; i < R; ++i)
      if (start[b * R + i] < 0 || start[b * R + i] >= h->ntg_host[b]) return cfail(GF_EINVAL, "start target out of range");
  if (int rc = use(h)) return rc;
  CV_HIP(hipMemcpyAsync(h->start, start, B * R * 4, hipMemcpyHostToDevice, h->stream));
  CV_HIP(hipMemcpyAsync(h->visited0, visited, B * Tm, hipMemcpyHostToDevice, h->stream));
  hipError_t e = gf::launch_cov_reset(h->a, h->start, h->visited0, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_reset_kernel: ") + hipGetErrorString(e));
  gf::CovArgs a = h->a;
  a.actions = nullptr;
  e = gf::launch_cov_step(a, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_kernel: ") + hipGetErrorString(e));
  CV_HIP(hipStreamSynchronize(h->stream));
  h->has_state = true;
  return GF_OK;
}

int cov_reset_seeded(cov_handle* h, uint64_t seed, double frac_active, int32_t* start_out, uint8_t* visited_out) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (!h->has_graph) return cfail(GF_ESTATE, "set the target graph of every env first (cov_set_targets)");
  const size_t B = h->cfg.n_envs, R = h->cfg.n_robots, Tm = h->a.Tmax;
  if (seed + B > 0x100000000ull) return cfail(GF_EINVAL, "seed + n_envs must fit in 32 bits (RandomState seeds)");
  if (!(frac_active >= 0.0 && frac_active <= 1.0)) return cfail(GF_EINVAL, "frac_active must be in [0, 1]");
  if ((size_t)gf::kMtN * 4 + Tm * 5 > 65536)  // the draw kernel's LDS: key, permutation, flags
    return cfail(GF_EINVAL, "max_nodes - n_robots too large for the device reset draws (draw on the host)");
  if (int rc = use(h)) return rc;
  if (!h->mt_key) {
    int rc;
    if ((rc = calloc_dev(&h->mt_key, B * gf::kMtN)) || (rc = calloc_dev(&h->mt_pos, B))) return rc;
  }
  gf::CovArgs a = h->a;
  a.mt_key = h->mt_key;
  a.mt_pos = h->mt_pos;
  hipError_t e = gf::launch_cov_seed_reset(a, static_cast<uint32_t>(seed), frac_active, h->start, h->visited0, h->stream);
  if (e == hipSuccess) e = gf::launch_cov_reset(h->a, h->start, h->visited0, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_reset_seeded: ") + hipGetErrorString(e));
  a = h->a;
  a.actions = nullptr;
  e = gf::launch_cov_step(a, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_kernel: ") + hipGetErrorString(e));
  if (start_out) CV_HIP(hipMemcpyAsync(start_out, h->start, B * R * 4, hipMemcpyDeviceToHost, h->stream));
  if (visited_out) CV_HIP(hipMemcpyAsync(visited_out, h->visited0, B * Tm, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  h->has_state = true;
  return GF_OK;
}

int cov_set_actions(cov_handle* h, const int32_t* actions) {
  if (!h || !actions) return cfail(GF_EINVAL, "null argument");
  if (int rc = use(h)) return rc;
  CV_HIP(hipMemcpyAsync(h->actions, actions, (size_t)h->cfg.n_envs * h->cfg.n_robots * 4, hipMemcpyHostToDevice,
                        h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_set_rng(cov_handle* h, const uint32_t* keys, const int32_t* pos) {
  if (!h || !keys || !pos) return cfail(GF_EINVAL, "null argument");
  const size_t B = h->cfg.n_envs;
  if (h->cfg.n_robots > gf::kMtN)
    return cfail(GF_EINVAL, "device np_random draws need n_robots <= 624 (one key regeneration per step)");
  for (size_t b = 0; b < B; ++b)
    if (pos[b] < 0 || pos[b] > gf::kMtN) return cfail(GF_EINVAL, "stream position outside [0, 624]");
  if (int rc = use(h)) return rc;
  if (!h->mt_key) {
    int rc;
    if ((rc = calloc_dev(&h->mt_key, B * gf::kMtN)) || (rc = calloc_dev(&h->mt_pos, B))) return rc;
  }
  CV_HIP(hipMemcpyAsync(h->mt_key, keys, B * gf::kMtN * 4, hipMemcpyHostToDevice, h->stream));
  CV_HIP(hipMemcpyAsync(h->mt_pos, pos, B * 4, hipMemcpyHostToDevice, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_get_rng(cov_handle* h, uint32_t* keys, int32_t* pos) {
  if (!h || !keys || !pos) return cfail(GF_EINVAL, "null argument");
  if (!h->mt_key) return cfail(GF_ESTATE, "no np_random streams on the device (cov_set_rng)");
  if (int rc = use(h)) return rc;
  const size_t B = h->cfg.n_envs;
  CV_HIP(hipMemcpyAsync(keys, h->mt_key, B * gf::kMtN * 4, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipMemcpyAsync(pos, h->mt_pos, B * 4, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

// n_steps fused greedy expert steps with the device fallback draws in one launch; equal to
// n_steps calls of cov_step(h, NULL, COV_ACTIONS_GREEDY | COV_GREEDY_RNG).
int cov_step_expert(cov_handle* h, int n_steps, double* rewards, uint8_t* done) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  if (n_steps < 1) return cfail(GF_EINVAL, "n_steps must be at least 1");
  if (!h->mt_key) return cfail(GF_ESTATE, "set the envs' np_random streams first (cov_set_rng or cov_reset_seeded)");
  if (h->cfg.n_robots > gf::kMtN) return cfail(GF_EINVAL, "n_robots <= 624 (one key regeneration per step)");
  if (int rc = use(h)) return rc;
  if (!h->tm_ready || !h->tm_glist)
    if (int rc = ensure_time_matrix(h)) return rc;
  if (!h->tm_glist) return cfail(GF_EINVAL, "the fused expert needs max_nodes - n_robots <= 1024 (the greedy lists)");
  if (int rc = join_s2(h)) return rc;
  gf::CovArgsM m{};
  m.a = h->a;
  m.a.actions = nullptr;
  m.a.glist = h->tm_glist;
  m.a.glen = h->tm_glen;
  m.a.gstride = h->gstride;
  m.a.gcost = h->tm_cost;
  m.a.gprev = h->tm_prevT;
  m.a.gactions = h->actions;
  m.a.needs_random = h->needs_random;
  m.a.mt_key = h->mt_key;
  m.a.mt_pos = h->mt_pos;
  m.k_steps = n_steps;
  const size_t B = h->cfg.n_envs, n = (size_t)n_steps * B;
  unsigned char* buf = nullptr;
  if (rewards || done) {
    if (int rc = scratch(h, n * 9, &buf)) return rc;
    m.reward_k = reinterpret_cast<double*>(buf);
    m.done_k = buf + n * 8;
  }
  hipError_t e = gf::launch_cov_step_multi(m, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_multi_kernel: ") + hipGetErrorString(e));
  h->main_dirty = true;
  h->other_work = true;
  if (!buf) return GF_OK;
  if (int rc = copy_out(h, rewards, m.reward_k, n * 8)) return rc;
  if (int rc = copy_out(h, done, m.done_k, n)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  return check_err(h);
}

int cov_step(cov_handle* h, const int32_t* actions, int flags) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  CV_HIP(hipSetDevice(h->cfg.device));
  gf::CovArgs a = h->a;
  if ((flags & COV_GREEDY_RNG) && !(flags & COV_ACTIONS_GREEDY))
    return cfail(GF_EINVAL, "COV_GREEDY_RNG needs COV_ACTIONS_GREEDY");
  if ((flags & COV_GREEDY_RNG) && !h->mt_key)
    return cfail(GF_ESTATE, "COV_GREEDY_RNG: set the envs' np_random streams first (cov_set_rng)");
  if ((flags & COV_GREEDY_RNG) && h->cfg.n_robots > gf::kMtN)
    return cfail(GF_EINVAL, "COV_GREEDY_RNG needs n_robots <= 624 (one key regeneration per step)");
  if (flags & COV_ACTIONS_GREEDY) {
    // controller(greedy=True) in the step's own launch, from the greedy lists
    if (!h->tm_ready || !h->tm_glist) {
      if (int rc = use(h)) return rc;
      if (int rc = ensure_time_matrix(h)) return rc;
    }
    if (!h->tm_glist) {  // Tmax > kGreedyListMaxT: the row-scan greedy kernel, then the step
      if (flags & COV_GREEDY_RNG)
        return cfail(GF_EINVAL, "COV_GREEDY_RNG needs max_nodes - n_robots <= 1024 (the greedy lists)");
      if (int rc = cov_controller_greedy(h, nullptr, nullptr, nullptr)) return rc;
      return cov_step(h, nullptr, COV_ACTIONS_RESIDENT);
    }
    a.actions = nullptr;
    a.glist = h->tm_glist;
    a.glen = h->tm_glen;
    a.gstride = h->gstride;
    a.gcost = h->tm_cost;
    a.gprev = h->tm_prevT;
    a.gactions = h->actions;
    a.needs_random = h->needs_random;
    if (flags & COV_GREEDY_RNG) {
      a.mt_key = h->mt_key;
      a.mt_pos = h->mt_pos;
    }
  } else if (flags & COV_ACTIONS_DEVICE) {
    if (!actions) return cfail(GF_EINVAL, "null action pointer");
    a.actions = actions;
  } else if (flags & COV_ACTIONS_RESIDENT) {
    a.actions = h->actions;
  } else {
    if (!actions) return cfail(GF_EINVAL, "null action pointer");
    const size_t n = (size_t)h->cfg.n_envs * h->cfg.n_robots;
    for (size_t k = 0; k < n; ++k)
      if (actions[k] < 0 || actions[k] >= 4) return cfail(GF_EINVAL, "action outside [0, 4) (coverage.py:189 index)");
    if (int rc = join_s2(h)) return rc;  // the previous second half may still read h->actions
    CV_HIP(hipMemcpyAsync(h->actions, actions, n * 4, hipMemcpyHostToDevice, h->stream));
    h->main_dirty = h->other_work = true;
    a.actions = h->actions;
  }
  const bool split = (h->nsplit == 2 || (h->nsplit == 0 && (flags & COV_ACTIONS_GREEDY))) && a.B >= 2 && !h->other_work;
  h->other_work = false;
  if (split) {
    if (h->main_dirty) {
      CV_HIP(hipEventRecord(h->ev_main, h->stream));
      CV_HIP(hipStreamWaitEvent(h->stream2, h->ev_main, 0));
      h->main_dirty = false;
    }
    gf::CovArgs a1 = a;
    a.B = (a.B + 1) / 2;
    a1.env0 = a.B;
    a1.B = h->a.B - a.B;
    hipError_t e = gf::launch_cov_step(a, h->stream);
    if (e == hipSuccess) e = gf::launch_cov_step(a1, h->stream2);
    if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_kernel: ") + hipGetErrorString(e));
    h->s2_pending = true;
    if (h->timing) h->tw_steps++;
    if (!(flags & (COV_ACTIONS_DEVICE | COV_ACTIONS_RESIDENT | COV_ACTIONS_GREEDY)))
      CV_HIP(hipStreamSynchronize(h->stream));
    return GF_OK;
  }
  if (int rc = join_s2(h)) return rc;
  h->main_dirty = true;
  if (h->timing && h->nsplit != 1) h->tw_steps++;  // the window counts every step
  const bool sample = h->timing && h->nsplit == 1 && (h->timing_count++ % h->timing_stride) == 0;
  if (sample) {
    if (h->ev_used + 2 > h->ev.size()) {
      for (int k = 0; k < 64; ++k) {
        hipEvent_t ev;
        CV_HIP(hipEventCreate(&ev));
        h->ev.push_back(ev);
      }
    }
    CV_HIP(hipEventRecord(h->ev[h->ev_used], h->stream));
  }
  hipError_t e = gf::launch_cov_step(a, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_kernel: ") + hipGetErrorString(e));
  if (sample) {
    CV_HIP(hipEventRecord(h->ev[h->ev_used + 1], h->stream));
    h->ev_used += 2;
  }
  if (!(flags & (COV_ACTIONS_DEVICE | COV_ACTIONS_RESIDENT | COV_ACTIONS_GREEDY)))
    CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

}  // extern "C"

namespace {
// The device address of page-locked host memory, or nullptr (pageable; its failed
// lookup's error is cleared so later launch checks do not see it).
template <class T>
T* cov_mapped(T* p) {
  if (!p) return nullptr;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return static_cast<T*>(d);
}
}  // namespace

extern "C" {

int cov_step_host(cov_handle* h, const int32_t* actions, float* nodes, float* edges, int32_t* senders,
                  int32_t* receivers, int64_t* step, double* reward, uint8_t* done, int32_t* closest,
                  int32_t* next_actions, uint8_t* needs_random, int flags) {
  if (!h || !actions) return cfail(GF_EINVAL, "null argument");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  if (flags & ~COV_NEXT_GREEDY) return cfail(GF_EINVAL, "flags: 0 or COV_NEXT_GREEDY");
  const bool ng = flags & COV_NEXT_GREEDY;
  if (!ng && (next_actions || needs_random)) return cfail(GF_EINVAL, "next_actions / needs_random need COV_NEXT_GREEDY");
  const size_t B = h->cfg.n_envs, R = h->cfg.n_robots, M = h->cfg.max_nodes, E = 4 * M, n = B * R;
  for (size_t k = 0; k < n; ++k)
    if (actions[k] < 0 || actions[k] >= 4) return cfail(GF_EINVAL, "action outside [0, 4) (coverage.py:189 index)");
  // one launch on the handle's stream after everything outstanding on both streams
  if (int rc = use(h)) return rc;
  gf::CovArgs a = h->a;
  if (ng) {
    if (!h->tm_ready || !h->tm_glist)
      if (int rc = ensure_time_matrix(h)) return rc;
    if (!h->tm_glist)
      return cfail(GF_EINVAL, "COV_NEXT_GREEDY needs max_nodes - n_robots <= 1024 (the per-node greedy lists)");
    a.next_greedy = 1;
    a.glist = h->tm_glist;
    a.glen = h->tm_glen;
    a.gstride = h->gstride;
    a.gcost = h->tm_cost;
    a.gprev = h->tm_prevT;
    a.gactions = h->actions;  // the next expert actions stay resident as well
    a.needs_random = h->needs_random;
  }
  // page-locked destinations are written by the step's own workgroups through their
  // mapped addresses; any other one gets a copy after the launch
  a.h_nodes = cov_mapped(nodes);
  a.h_edges = cov_mapped(edges);
  a.h_senders = cov_mapped(senders);
  a.h_receivers = cov_mapped(receivers);
  a.h_step = cov_mapped(step);
  a.h_reward = cov_mapped(reward);
  a.h_done = cov_mapped(done);
  a.h_closest = cov_mapped(closest);
  a.h_next = cov_mapped(next_actions);
  a.h_nrand = cov_mapped(needs_random);
  // the device error word of each env as its workgroup ends, in page-locked scratch
  if (!h->herr) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(B, 16) * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return cfail(GF_ENOMEM, "hipHostMalloc (error words)");
    h->herr = static_cast<int32_t*>(p);
  }
  std::memset(h->herr, 0, B * sizeof(int32_t));
  a.h_err = cov_mapped(h->herr);
  // every destination page-locked and the actions inline: the launch is the call's only
  // device work, and the host waits for the kernel's own completion flag (done_flag.h)
  const bool fin = n * 4 <= (size_t)gf::kCovUInlineBytes && (!nodes || a.h_nodes) && (!edges || a.h_edges) &&
                   (!senders || a.h_senders) && (!receivers || a.h_receivers) && (!step || a.h_step) &&
                   (!reward || a.h_reward) && (!done || a.h_done) && (!closest || a.h_closest) &&
                   (!next_actions || a.h_next) && (!needs_random || a.h_nrand);
  if (fin) {
    if (!h->fin_cnt) {
      if (int rc = calloc_dev(&h->fin_cnt, 1)) return rc;
      void* p = nullptr;
      if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return cfail(GF_ENOMEM, "hipHostMalloc (completion flag)");
      h->fin_host = static_cast<int32_t*>(p);
      *h->fin_host = 0;
      h->fin_dev = cov_mapped(h->fin_host);
      if (!h->fin_dev) return cfail(GF_EHIP, "completion flag: no mapped address");
    }
    a.fin.cnt = h->fin_cnt;
    a.fin.host = h->fin_dev;
    h->fin_seq = (h->fin_seq & 0x3fffffff) + 1;  // never 0 (the word's initial value), no overflow
    a.fin.seq = h->fin_seq;
  }
  hipError_t e;
  if (n * 4 <= (size_t)gf::kCovUInlineBytes) {
    e = gf::launch_cov_step_uin(a, actions, h->stream);  // actions in the kernel arguments
  } else {
    CV_HIP(hipMemcpyAsync(h->actions, actions, n * 4, hipMemcpyHostToDevice, h->stream));
    a.actions = h->actions;
    e = gf::launch_cov_step(a, h->stream);
  }
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_kernel: ") + hipGetErrorString(e));
  const gf::CovArgs& d = h->a;
  if (nodes && !a.h_nodes) CV_HIP(hipMemcpyAsync(nodes, d.nodes, B * M * 3 * 4, hipMemcpyDeviceToHost, h->stream));
  if (edges && !a.h_edges) CV_HIP(hipMemcpyAsync(edges, d.edges, B * E * 4, hipMemcpyDeviceToHost, h->stream));
  if (senders && !a.h_senders) CV_HIP(hipMemcpyAsync(senders, d.senders, B * E * 4, hipMemcpyDeviceToHost, h->stream));
  if (receivers && !a.h_receivers)
    CV_HIP(hipMemcpyAsync(receivers, d.receivers, B * E * 4, hipMemcpyDeviceToHost, h->stream));
  if (step && !a.h_step) CV_HIP(hipMemcpyAsync(step, d.obs_step, B * 8, hipMemcpyDeviceToHost, h->stream));
  if (reward && !a.h_reward) CV_HIP(hipMemcpyAsync(reward, d.reward, B * 8, hipMemcpyDeviceToHost, h->stream));
  if (done && !a.h_done) CV_HIP(hipMemcpyAsync(done, d.done, B, hipMemcpyDeviceToHost, h->stream));
  if (closest && !a.h_closest) CV_HIP(hipMemcpyAsync(closest, d.cur, n * 4, hipMemcpyDeviceToHost, h->stream));
  if (next_actions && !a.h_next) CV_HIP(hipMemcpyAsync(next_actions, h->actions, n * 4, hipMemcpyDeviceToHost, h->stream));
  if (needs_random && !a.h_nrand)
    CV_HIP(hipMemcpyAsync(needs_random, h->needs_random, n, hipMemcpyDeviceToHost, h->stream));
  if (fin) {
    const hipError_t q = gf::wait_done(h->fin_host, h->fin_seq, h->stream);
    if (q == hipErrorUnknown) return cfail(GF_EHIP, "cov_step_host: the step finished without its completion flag");
    if (q != hipSuccess) return cfail(GF_EHIP, std::string("cov_step_host: ") + hipGetErrorString(q));
  } else {
    // spin on the stream: a drop-in step is latency-bound (a blocking wait's wake-up
    // costs a sizeable part of it)
    for (;;) {
      const hipError_t q = hipStreamQuery(h->stream);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return cfail(GF_EHIP, std::string("cov_step_host: ") + hipGetErrorString(q));
    }
  }
  int err = 0;
  for (size_t b = 0; b < B; ++b) err |= h->herr[b];
  if (err) return check_err(h);  // reads, clears and reports the device error word
  return GF_OK;
}

int cov_kernel_timing(cov_handle* h, int enable, double* avg_ms, int64_t* launches) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (int rc = use(h)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  if (enable >= 1) {  // start: time every enable-th step launch
    h->ev_used = 0;
    h->timing = true;
    h->timing_stride = enable;
    h->timing_count = 0;
    h->tw_steps = 0;  // split steps: one window, device time per step
    CV_HIP(hipEventRecord(h->tw[0], h->stream));
    h->other_work = false;  // both streams idle: the first timed step splits like the rest
    return GF_OK;
  }
  if (h->tw_steps > 0) {
    CV_HIP(hipEventRecord(h->tw[1], h->stream));
    CV_HIP(hipEventSynchronize(h->tw[1]));
    float ms = 0;
    CV_HIP(hipEventElapsedTime(&ms, h->tw[0], h->tw[1]));
    if (avg_ms) *avg_ms = ms / h->tw_steps;
    if (launches) *launches = h->tw_steps;
    if (enable == 0) h->timing = false;
    else {
      h->tw_steps = 0;
      CV_HIP(hipEventRecord(h->tw[0], h->stream));
    }
    return GF_OK;
  }
  double tot = 0;
  for (size_t k = 0; k + 1 < h->ev_used; k += 2) {
    float ms = 0;
    CV_HIP(hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1]));
    tot += ms;
  }
  const int64_t n = (int64_t)(h->ev_used / 2);
  if (avg_ms) *avg_ms = n ? tot / n : 0.0;
  if (launches) *launches = n;
  if (enable == 0) h->timing = false;
  return GF_OK;
}

int cov_set_robot_positions(cov_handle* h, int env, const double* xr) {
  if (!h || !xr || env < 0 || env >= h->cfg.n_envs) return cfail(GF_EINVAL, "bad argument");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  if (int rc = use(h)) return rc;
  const size_t R = h->cfg.n_robots;
  const uint8_t one = 1;
  CV_HIP(hipMemcpyAsync(h->a.xr + env * R * 2, xr, R * 2 * sizeof(double), hipMemcpyHostToDevice, h->stream));
  CV_HIP(hipMemcpyAsync(h->a.dirty + env, &one, 1, hipMemcpyHostToDevice, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_get_obs(cov_handle* h, int env, float* nodes, float* edges, int32_t* senders, int32_t* receivers,
                int64_t* step) {
  if (!h || env < 0 || env >= h->cfg.n_envs) return cfail(GF_EINVAL, "bad argument");
  // before the first reset the arrays hold the graph's static part (the motion edges the
  // env's nearby-starts draw walks, coverage.py:655-673); the robots' part follows reset
  if (!h->has_state && !h->has_graph) return cfail(GF_ESTATE, "set the targets (cov_set_targets) or reset first");
  if (int rc = use(h)) return rc;
  const size_t M = h->cfg.max_nodes, E = 4 * M;
  const gf::CovArgs& a = h->a;
  if (int rc = copy_out(h, nodes, a.nodes + env * M * 3, M * 3 * 4)) return rc;
  if (int rc = copy_out(h, edges, a.edges + env * E, E * 4)) return rc;
  if (int rc = copy_out(h, senders, a.senders + env * E, E * 4)) return rc;
  if (int rc = copy_out(h, receivers, a.receivers + env * E, E * 4)) return rc;
  if (int rc = copy_out(h, step, a.obs_step + env, 8)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  return check_err(h);
}

int cov_get_rewards(cov_handle* h, double* reward, uint8_t* done) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (int rc = use(h)) return rc;
  const size_t B = h->cfg.n_envs;
  if (int rc = copy_out(h, reward, h->a.reward, B * 8)) return rc;
  if (int rc = copy_out(h, done, h->a.done, B)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  return check_err(h);
}

int cov_get_robots(cov_handle* h, int env, double* xr, int32_t* nodes) {
  if (!h || env < 0 || env >= h->cfg.n_envs) return cfail(GF_EINVAL, "bad argument");
  if (int rc = use(h)) return rc;
  const size_t R = h->cfg.n_robots;
  if (int rc = copy_out(h, xr, h->a.xr + env * R * 2, R * 16)) return rc;
  if (int rc = copy_out(h, nodes, h->a.cur + env * R, R * 4)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_get_visited(cov_handle* h, int env, uint8_t* visited) {
  if (!h || !visited || env < 0 || env >= h->cfg.n_envs) return cfail(GF_EINVAL, "bad argument");
  if (int rc = use(h)) return rc;
  const size_t Tm = h->a.Tmax;
  if (int rc = copy_out(h, visited, h->a.visited + env * Tm, Tm)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_get_n_motion(cov_handle* h, int32_t* n_motion) {
  if (!h || !n_motion) return cfail(GF_EINVAL, "null argument");
  if (int rc = use(h)) return rc;
  if (int rc = copy_out(h, n_motion, h->a.n_motion, (size_t)h->cfg.n_envs * 4)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_controller_greedy(cov_handle* h, int32_t* actions, uint8_t* needs_random, int64_t* n_random) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  if (int rc = use(h)) return rc;
  if (int rc = ensure_time_matrix(h)) return rc;
  gf::CovGreedyArgs g{};
  const gf::CovArgs& a = h->a;
  g.B = a.B;
  g.R = a.R;
  g.Tmax = a.Tmax;
  g.ntg = h->ntg;
  g.tgt = h->tgt;
  g.xr = a.xr;
  g.dirty = a.dirty;
  g.cur = a.cur;
  g.cost = h->tm_cost;
  g.cost8 = h->tm_cost8;
  g.wide = h->tm_wide;
  g.prevT = h->tm_prevT;
  g.visited = a.visited;
  g.nvisited = a.nvisited;
  g.nbr = a.nbr;
  g.cnt = a.cnt;
  g.actions = h->actions;
  g.needs_random = h->needs_random;
  g.err = h->err;
  g.glist = h->tm_glist;
  g.glen = h->tm_glen;
  g.gstride = h->gstride;
  hipError_t e = gf::launch_cov_greedy(g, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_greedy_kernel: ") + hipGetErrorString(e));
  if (!actions && !needs_random && !n_random) return GF_OK;
  const size_t n = (size_t)a.B * a.R;
  std::vector<uint8_t> mask;
  uint8_t* rnd = needs_random;
  if (n_random && !rnd) {
    mask.resize(n);
    rnd = mask.data();
  }
  if (int rc = copy_out(h, actions, h->actions, n * 4)) return rc;
  if (int rc = copy_out(h, rnd, h->needs_random, n)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  if (n_random) {
    int64_t cnt = 0;
    for (size_t k = 0; k < n; ++k) cnt += rnd[k] ? 1 : 0;
    *n_random = cnt;
  }
  return check_err(h);
}

int cov_get_actions(cov_handle* h, int32_t* actions, uint8_t* needs_random) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (int rc = use(h)) return rc;
  const size_t n = (size_t)h->cfg.n_envs * h->cfg.n_robots;
  if (int rc = copy_out(h, actions, h->actions, n * 4)) return rc;
  if (needs_random) {
    if (h->needs_random) {
      if (int rc = copy_out(h, needs_random, h->needs_random, n)) return rc;
    } else {
      std::memset(needs_random, 0, n);
    }
  }
  CV_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int cov_get_time_matrix(cov_handle* h, int env, int32_t* cost, int32_t* prev) {
  if (!h || env < 0 || env >= h->cfg.n_envs) return cfail(GF_EINVAL, "bad argument");
  if (!h->has_graph) return cfail(GF_ESTATE, "set the target graph first (cov_set_targets)");
  if (int rc = use(h)) return rc;
  if (int rc = ensure_time_matrix(h)) return rc;
  const size_t Tm = h->a.Tmax, T = h->ntg_host[env];
  std::vector<uint16_t> c(Tm * Tm);
  std::vector<int16_t> p(Tm * Tm);
  CV_HIP(hipMemcpyAsync(c.data(), h->tm_cost + env * Tm * Tm, Tm * Tm * 2, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipMemcpyAsync(p.data(), h->tm_prevT + env * Tm * Tm, Tm * Tm * 2, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  for (size_t i = 0; i < T; ++i)
    for (size_t j = 0; j < T; ++j) {
      if (cost) cost[i * T + j] = c[i * Tm + j] == 0xFFFF ? 1000 : c[i * Tm + j];
      if (prev) prev[i * T + j] = p[j * Tm + i];  // graph_previous[i, j] lives at prevT[j][i]
    }
  return GF_OK;
}

int cov_get_flat_obs(cov_handle* h, void* dst, int flags) {
  if (!h || !dst) return cfail(GF_EINVAL, "null argument");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  if (int rc = use(h)) return rc;
  const bool f32 = flags & COV_FLAT_F32;
  const size_t bytes = (size_t)h->cfg.n_envs * (15 * (size_t)h->cfg.max_nodes + 1) * (f32 ? 4 : 8);
  void* out = dst;
  if (!(flags & COV_OUT_DEVICE)) {
    unsigned char* sc = nullptr;
    if (int rc = scratch(h, bytes, &sc)) return rc;
    out = sc;
  }
  hipError_t e = gf::launch_cov_flat_obs(h->a, out, f32, h->stream);
  if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_flat_obs_kernel: ") + hipGetErrorString(e));
  if (flags & COV_OUT_DEVICE) return GF_OK;  // stream-ordered; cov_sync before reading
  CV_HIP(hipMemcpyAsync(dst, out, bytes, hipMemcpyDeviceToHost, h->stream));
  CV_HIP(hipStreamSynchronize(h->stream));
  return check_err(h);
}

int cov_graphs_tuple_sizes(cov_handle* h, int32_t* n_edge, int64_t* total_edges, int flags) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (!h->has_graph) return cfail(GF_ESTATE, "set the target graph first (cov_set_targets)");
  std::vector<int32_t> ne;
  std::vector<int64_t> off;
  graph_sizes(h, flags & COV_MASK_ALL, ne, off);
  if (n_edge) std::memcpy(n_edge, ne.data(), ne.size() * sizeof(int32_t));
  if (total_edges) *total_edges = off.back();
  return GF_OK;
}

int cov_get_graphs_tuple(cov_handle* h, int32_t* n_node, float* nodes, int32_t* n_edge, float* edges,
                         int32_t* senders, int32_t* receivers, float* globs, int flags) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (!h->has_state) return cfail(GF_ESTATE, "reset first (cov_reset)");
  if ((edges != nullptr) != (senders != nullptr) || (edges != nullptr) != (receivers != nullptr))
    return cfail(GF_EINVAL, "edges, senders and receivers go together (all or none)");
  if (int rc = use(h)) return rc;
  const bool dev = flags & COV_OUT_DEVICE;
  const int B = h->cfg.n_envs, M = h->cfg.max_nodes;
  std::vector<int32_t> ne;
  std::vector<int64_t> off;
  graph_sizes(h, flags & COV_MASK_ALL, ne, off);
  const int64_t total = off.back();
  if (!h->goff)
    if (hipMalloc(reinterpret_cast<void**>(&h->goff), (B + 1) * sizeof(int64_t)) != hipSuccess)
      return cfail(GF_ENOMEM, "hipMalloc of graph offsets failed");
  CV_HIP(hipMemcpyAsync(h->goff, off.data(), (B + 1) * sizeof(int64_t), hipMemcpyHostToDevice, h->stream));
  if (edges) {
    float* e_out = edges;
    int32_t *s_out = senders, *r_out = receivers;
    if (!dev) {
      unsigned char* sc = nullptr;
      if (int rc = scratch(h, (size_t)total * 12, &sc)) return rc;
      e_out = reinterpret_cast<float*>(sc);
      s_out = reinterpret_cast<int32_t*>(sc + (size_t)total * 4);
      r_out = reinterpret_cast<int32_t*>(sc + (size_t)total * 8);
    }
    hipError_t e = gf::launch_cov_graphs(h->a, h->goff, flags & COV_MASK_ALL, e_out, s_out, r_out, h->stream);
    if (e != hipSuccess) return cfail(GF_EHIP, std::string("cov_graphs_kernel: ") + hipGetErrorString(e));
    if (!dev) {
      if (int rc = put(h, edges, e_out, (size_t)total * 4, false, true)) return rc;
      if (int rc = put(h, senders, s_out, (size_t)total * 4, false, true)) return rc;
      if (int rc = put(h, receivers, r_out, (size_t)total * 4, false, true)) return rc;
    }
  }
  if (int rc = put(h, nodes, h->a.nodes, (size_t)B * M * 3 * sizeof(float), dev, true)) return rc;
  std::vector<int32_t> nn(B, M);
  if (int rc = put(h, n_node, nn.data(), B * sizeof(int32_t), dev, false)) return rc;
  if (int rc = put(h, n_edge, ne.data(), B * sizeof(int32_t), dev, false)) return rc;
  std::vector<float> gl(B);
  if (globs) {
    std::vector<int64_t> st(B);
    CV_HIP(hipMemcpyAsync(st.data(), h->a.obs_step, B * sizeof(int64_t), hipMemcpyDeviceToHost, h->stream));
    CV_HIP(hipStreamSynchronize(h->stream));
    for (int b = 0; b < B; ++b) gl[b] = static_cast<float>(st[b]);
    if (int rc = put(h, globs, gl.data(), B * sizeof(float), dev, false)) return rc;
  }
  CV_HIP(hipStreamSynchronize(h->stream));  // host temporaries above
  return check_err(h);
}

int cov_set_streams(cov_handle* h, int n) {
  if (!h || n < 0 || n > 2) return cfail(GF_EINVAL, "n must be 0 (auto), 1 or 2");
  if (int rc = use(h)) return rc;
  h->nsplit = n;
  return GF_OK;
}

int cov_sync(cov_handle* h) {
  if (!h) return cfail(GF_EINVAL, "null handle");
  if (int rc = use(h)) return rc;
  CV_HIP(hipStreamSynchronize(h->stream));
  // both streams idle: the next step may split. main_dirty stays set (use_dev): reads of
  // the outputs a zero-copy consumer enqueues on `stream` after this call come before
  // the next step's second half
  h->other_work = false;
  return check_err(h);
}

}  // extern "C"
