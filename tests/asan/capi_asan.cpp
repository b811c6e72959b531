// Host AddressSanitizer driver for the C-ABI (include/gymflock.h). Built by
// tests/asan/Makefile with the host side of every translation unit instrumented
// (-Xarch_host -fsanitize=address; device code is not instrumented: GPU ASan is not
// available on this pool). Without a GPU it runs every argument-validation and
// no-device path; with one (MI355X box) it also runs a short FlockingRelative /
// Flocking-v0 / Coverage / graph-helper session through the borrowed-host-pointer
// entry points, so that ASan sees every host buffer the library reads or writes.
// Exit code 0 = all checks passed and ASan reported nothing (it aborts otherwise).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>

#include "gymflock.h"

static int failures = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "FAIL %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, \
                   #cond, fe_last_error());                                      \
      ++failures;                                                                \
    }                                                                            \
  } while (0)

static fe_config flock_cfg(int n, int b, int k) {
  fe_config c{};
  c.n_agents = n;
  c.n_envs = b;
  c.comm_radius = 0.9;
  c.dt = 0.01;
  c.action_scalar = 10.0;
  c.mean_pooling = 1;
  c.centralized = 1;
  c.n_neighbors = k;
  c.device = 0;
  return c;
}

static void validation_paths() {
  CHECK(fe_abi_version() >= 1);
  fe_handle* h = reinterpret_cast<fe_handle*>(0x1);
  CHECK(fe_create(nullptr, &h) != 0);
  CHECK(h == reinterpret_cast<fe_handle*>(0x1));  // untouched on a null config
  fe_config c = flock_cfg(0, 1, 0);
  CHECK(fe_create(&c, &h) != 0 && h == nullptr);
  c = flock_cfg(16, 0, 0);
  CHECK(fe_create(&c, &h) != 0);
  c = flock_cfg(16, 1, 9);  // k not in the supported set
  CHECK(fe_create(&c, &h) != 0);
  c = flock_cfg(4, 1, 7);  // k > n_agents
  CHECK(fe_create(&c, &h) != 0);
  c = flock_cfg(16, 1, 0);
  c.comm_radius = 0.0;
  CHECK(fe_create(&c, &h) != 0);
  CHECK(std::strlen(fe_last_error()) > 0);
  // null handles on every entry point that takes one
  CHECK(fe_destroy(nullptr) == 0);
  CHECK(fe_step(nullptr, nullptr, 0) != 0);
  CHECK(fe_sync(nullptr) != 0);
  CHECK(fe_get_rewards(nullptr, nullptr) != 0);
  CHECK(fe_get_state(nullptr, nullptr) != 0);
  CHECK(fe_set_state(nullptr, nullptr) != 0);
  CHECK(fe_controller(nullptr, 1, nullptr) != 0);
  CHECK(fe_get_knn(nullptr, 0, nullptr, nullptr) != 0);
  cov_handle* ch = nullptr;
  CHECK(cov_create(nullptr, &ch) != 0);
  cov_config cc{};
  cc.n_robots = 0;
  cc.n_envs = 1;
  cc.max_nodes = 100;
  cc.episode_length = 75;
  cc.res = 5.5;
  cc.motion_radius = 6.6;
  CHECK(cov_create(&cc, &ch) != 0);
  CHECK(cov_destroy(nullptr) == 0);
  CHECK(gu_create(0, nullptr) != 0);
  // round-5 entry points: null handles fail, the host-only query fills what it is given
  CHECK(fe_set_params(nullptr, nullptr) != 0);
  CHECK(fe_step_host(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0) != 0);
  CHECK(fe_step_host_knn_ctrl(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0) != 0);
  CHECK(cov_set_rng(nullptr, nullptr, nullptr) != 0);
  CHECK(cov_get_rng(nullptr, nullptr, nullptr) != 0);
  CHECK(cov_step_host(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                      nullptr, nullptr, 0) != 0);
  int32_t rt = -1, drv = -1, nccl = -1;
  char hp[512], rp[512];
  CHECK(fe_runtime_info(nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0) == 0);
  CHECK(fe_runtime_info(&rt, &drv, &nccl, hp, sizeof hp, rp, sizeof rp) == 0 && rt > 0 && nccl > 0);
  // round-6 map entry points: the host-only lattice query, null handles and configs
  cov_map_config mc{};
  int32_t nl = 0;
  CHECK(cov_map_lattice(nullptr, nullptr, &nl) != 0);
  CHECK(cov_map_lattice(&mc, nullptr, &nl) != 0);  // zero spacing
  mc.x_min = mc.y_min = -20.0;
  mc.x_max = mc.y_max = 20.0;
  mc.lattice_spacing = 5.5;
  mc.world_radius = 20.0;
  mc.road_radius = mc.link_radius = 6.6;
  mc.near_radius = 6.6 / 1.4;
  mc.n_cities = 12;
  CHECK(cov_map_lattice(&mc, nullptr, &nl) == 0 && nl > 0);
  std::vector<double> lat((size_t)nl * 2);
  CHECK(cov_map_lattice(&mc, lat.data(), &nl) == 0);
  CHECK(cov_generate_maps(nullptr, &mc, -1, 0, nullptr, COV_MAP_SEED, nullptr, nullptr, nullptr) != 0);
  CHECK(cov_get_targets(nullptr, 0, lat.data()) != 0);
}

static bool have_device() {
  fe_config c = flock_cfg(16, 1, 0);
  fe_handle* h = nullptr;
  const int rc = fe_create(&c, &h);
  if (rc == 0) {
    fe_destroy(h);
    return true;
  }
  // the no-device path must fail loudly, not crash
  CHECK(std::strstr(fe_last_error(), "device") != nullptr || std::strstr(fe_last_error(), "HIP") != nullptr);
  return false;
}

static void flocking_session() {
  const int N = 96, B = 3, K = 7;
  fe_config c = flock_cfg(N, B, K);
  fe_handle* h = nullptr;
  CHECK(fe_create(&c, &h) == 0);
  if (!h) return;
  CHECK(fe_reset_synthetic(h, 11, 5.0) == 0);
  std::vector<double> x((size_t)B * N * 4);
  CHECK(fe_get_state(h, x.data()) == 0);
  std::vector<float> u((size_t)B * N * 2);
  for (size_t i = 0; i < u.size(); ++i) u[i] = static_cast<float>((i % 17) / 8.5 - 1.0);
  for (int s = 0; s < 4; ++s) CHECK(fe_step(h, u.data(), FE_WITH_KNN) == 0);
  CHECK(fe_set_actions(h, u.data(), 0) == 0);
  for (int s = 0; s < 4; ++s) CHECK(fe_step(h, nullptr, FE_U_RESIDENT | FE_WITH_KNN) == 0);
  CHECK(fe_step(h, nullptr, FE_U_RESIDENT | FE_WITH_CONTROLLER) == 0);
  CHECK(fe_step(h, nullptr, FE_U_EXPERT | FE_WITH_CONTROLLER) == 0);
  std::vector<double> ctl((size_t)B * N * 2);
  CHECK(fe_controller(h, 1, ctl.data()) == 0);
  std::vector<float> sv((size_t)N * 6), net((size_t)N * N);
  std::vector<double> rew(B), vd(N), md(N), ctrl_env((size_t)N * 2);
  std::vector<int32_t> idx((size_t)B * N * K), deg(N);
  std::vector<float> obs((size_t)B * N * 4 * K);
  for (int e = 0; e < B; ++e) {
    CHECK(fe_get_state_values(h, e, sv.data()) == 0);
    CHECK(fe_get_network(h, e, net.data()) == 0);
    CHECK(fe_get_network_rows(h, e, N - 5, 5, net.data()) == 0);
    CHECK(fe_get_controls(h, e, ctrl_env.data()) == 0);
    CHECK(fe_get_stats_ex(h, e, vd.data(), md.data(), deg.data()) == 0);
  }
  CHECK(fe_get_rewards(h, rew.data()) == 0);
  CHECK(fe_get_knn(h, -1, idx.data(), obs.data()) == 0);
  for (int32_t j : idx) CHECK(j >= 0 && j < N);
  CHECK(fe_get_state_values(h, B, sv.data()) != 0);  // env out of range
  CHECK(fe_get_network_rows(h, 0, N - 2, 5, net.data()) != 0);
  std::vector<uint64_t> bits((size_t)N * ((N + 63) / 64));
  CHECK(fe_step(h, nullptr, FE_U_RESIDENT | FE_PACKED_NETWORK) == 0);
  CHECK(fe_get_network_packed(h, 1, bits.data(), deg.data()) == 0);
  fe_variant v{};
  v.n_frozen = 2;
  v.n_vel_zero = 2;
  v.u_scale = 10.0;
  v.x_scale = 1.0;
  CHECK(fe_set_variant(h, &v) == 0);
  CHECK(fe_step(h, u.data(), FE_WITH_CONTROLLER) == 0);
  std::vector<double> dts(B, 0.01);
  CHECK(fe_set_dt(h, dts.data()) == 0);
  CHECK(fe_step(h, u.data(), 0) == 0);
  CHECK(fe_set_state_env(h, 1, x.data()) == 0);
  CHECK(fe_get_state_env(h, 2, x.data()) == 0);
  fe_buffers bufs{};
  CHECK(fe_device_buffers(h, &bufs) == 0 && bufs.x != nullptr);
  CHECK(fe_sync(h) == 0);
  CHECK(fe_destroy(h) == 0);
  // the one-call drop-in step of one env: pageable destinations (copies after the launch,
  // the stream waited for) and page-locked ones (written by the kernel, its completion
  // flag waited for), with the fused controller and the 7 nearest; then a parameter change
  c = flock_cfg(N, 1, K);
  CHECK(fe_create(&c, &h) == 0);
  if (!h) return;
  CHECK(fe_reset_synthetic(h, 12, 5.0) == 0);
  std::vector<float> sv1((size_t)N * 6), net1((size_t)N * N), kobs((size_t)N * 4 * K);
  std::vector<double> r1(1), c1((size_t)N * 2);
  std::vector<int32_t> kidx((size_t)N * K);
  CHECK(fe_step_host(h, u.data(), sv1.data(), net1.data(), r1.data(), c1.data(), 0) == 0);
  CHECK(fe_step_host_knn_ctrl(h, u.data(), sv1.data(), net1.data(), r1.data(), c1.data(), kidx.data(), kobs.data(),
                              0) == 0);
  void* pin = nullptr;
  const size_t nsv = (size_t)N * 6 * 4, nnet = (size_t)N * N * 4, nk = (size_t)N * K * 4;
  const size_t bytes = nsv + nnet + 8 + (size_t)N * 16 + nk + 4 * nk;
  CHECK(fe_host_alloc(bytes, &pin) == 0);
  if (pin) {
    unsigned char* b = static_cast<unsigned char*>(pin);
    float* psv = reinterpret_cast<float*>(b);
    float* pnet = reinterpret_cast<float*>(b + nsv);
    double* pr = reinterpret_cast<double*>(b + nsv + nnet);
    double* pc = reinterpret_cast<double*>(b + nsv + nnet + 8);
    int32_t* pidx = reinterpret_cast<int32_t*>(b + nsv + nnet + 8 + (size_t)N * 16);
    float* pobs = reinterpret_cast<float*>(b + nsv + nnet + 8 + (size_t)N * 16 + nk);
    for (int s = 0; s < 3; ++s) {
      CHECK(fe_step_host(h, u.data(), psv, pnet, pr, pc, 0) == 0);
      CHECK(fe_step_host_knn_ctrl(h, u.data(), psv, pnet, pr, pc, pidx, pobs, 0) == 0);
    }
    for (int i = 0; i < N * K; ++i) CHECK(pidx[i] >= 0 && pidx[i] < N);
    fe_config c2 = c;
    c2.comm_radius = 1.2;
    c2.centralized = 0;
    CHECK(fe_set_params(h, &c2) == 0);
    CHECK(fe_step_host(h, u.data(), psv, pnet, pr, pc, 0) == 0);
    CHECK(fe_host_free(pin) == 0);
  }
  CHECK(fe_destroy(h) == 0);
}

static void coverage_session() {
  const int R = 6, B = 2, M = 200;
  cov_config cc{};
  cc.n_robots = R;
  cc.n_envs = B;
  cc.max_nodes = M;
  cc.episode_length = 75;
  cc.res = 5.5;
  cc.motion_radius = 6.6;
  cc.device = 0;
  cc.horizon = -1;
  cov_handle* h = nullptr;
  CHECK(cov_create(&cc, &h) == 0);
  if (!h) return;
  // a 10 x 8 lattice of targets, spacing res
  const int T = 80;
  std::vector<double> tg((size_t)T * 2);
  for (int i = 0; i < T; ++i) {
    tg[2 * i] = 5.5 * (i % 10);
    tg[2 * i + 1] = 5.5 * (i / 10);
  }
  CHECK(cov_set_targets(h, -1, T, tg.data()) == 0);
  std::vector<int32_t> start((size_t)B * R);
  for (int i = 0; i < B * R; ++i) start[i] = (7 * i) % T;
  std::vector<uint8_t> visited((size_t)B * (M - R), 0);  // [B][max_nodes - R]
  CHECK(cov_reset(h, start.data(), visited.data()) == 0);
  std::vector<int32_t> act((size_t)B * R);
  std::vector<uint8_t> rnd((size_t)B * R);
  int64_t nrnd = 0;
  for (int s = 0; s < 6; ++s) {
    CHECK(cov_controller_greedy(h, act.data(), rnd.data(), &nrnd) == 0);
    for (int i = 0; i < B * R; ++i)
      if (rnd[i]) act[i] = i % 4;
    CHECK(cov_step(h, act.data(), 0) == 0);
  }
  std::vector<float> nodes((size_t)M * 3), edges((size_t)4 * M);
  std::vector<int32_t> snd((size_t)4 * M), rcv((size_t)4 * M), rn(R);
  int64_t step = 0;
  CHECK(cov_get_obs(h, 1, nodes.data(), edges.data(), snd.data(), rcv.data(), &step) == 0);
  std::vector<double> rew(B), xr((size_t)R * 2);
  std::vector<uint8_t> done(B), vis(M - R);  // cov_get_visited: max_nodes - R entries
  CHECK(cov_get_rewards(h, rew.data(), done.data()) == 0);
  CHECK(cov_get_robots(h, 0, xr.data(), rn.data()) == 0);
  CHECK(cov_get_visited(h, 0, vis.data()) == 0);
  std::vector<int32_t> cost((size_t)T * T), prev((size_t)T * T);
  CHECK(cov_get_time_matrix(h, 0, cost.data(), prev.data()) == 0);
  CHECK(cov_get_obs(h, B, nodes.data(), edges.data(), snd.data(), rcv.data(), &step) != 0);
  // the fused greedy step drawing the fallbacks from device np_random streams
  std::vector<uint32_t> keys((size_t)B * 624);
  std::vector<int32_t> pos(B, 624);
  for (size_t i = 0; i < keys.size(); ++i) keys[i] = static_cast<uint32_t>(i * 2654435761u);
  CHECK(cov_step(h, nullptr, COV_ACTIONS_GREEDY | COV_GREEDY_RNG) != 0);  // streams not set
  CHECK(cov_set_rng(h, keys.data(), pos.data()) == 0);
  for (int s = 0; s < 4; ++s) CHECK(cov_step(h, nullptr, COV_ACTIONS_GREEDY | COV_GREEDY_RNG) == 0);
  // the same expert steps in one launch, every step's rewards and done flags to the host
  std::vector<double> rk((size_t)5 * B);
  std::vector<uint8_t> dk((size_t)5 * B);
  CHECK(cov_step_expert(h, 5, rk.data(), dk.data()) == 0);
  CHECK(cov_step_expert(h, 3, nullptr, nullptr) == 0);
  CHECK(cov_step_expert(h, 0, nullptr, nullptr) != 0);
  CHECK(cov_step_expert(nullptr, 1, nullptr, nullptr) != 0);
  CHECK(cov_get_rng(h, keys.data(), pos.data()) == 0);
  for (int b = 0; b < B; ++b) CHECK(pos[b] >= 0 && pos[b] <= 624);
  // the one-call drop-in step: pageable destinations, then page-locked ones
  std::vector<float> bn((size_t)B * M * 3), be((size_t)B * 4 * M);
  std::vector<int32_t> bs((size_t)B * 4 * M), br((size_t)B * 4 * M), bc((size_t)B * R), bnx((size_t)B * R);
  std::vector<int64_t> bst(B);
  std::vector<double> brw(B);
  std::vector<uint8_t> bd(B), bnr((size_t)B * R);
  for (int i = 0; i < B * R; ++i) act[i] = i % 4;
  CHECK(cov_step_host(h, act.data(), bn.data(), be.data(), bs.data(), br.data(), bst.data(), brw.data(), bd.data(),
                      bc.data(), bnx.data(), bnr.data(), COV_NEXT_GREEDY) == 0);
  void* pin = nullptr;
  const size_t nb = (size_t)B * M * 3 * 4 + 3 * (size_t)B * 4 * M * 4 + 64 + (size_t)B * R * 9;
  CHECK(fe_host_alloc(nb + 64, &pin) == 0);
  if (pin) {
    unsigned char* p = static_cast<unsigned char*>(pin);
    float* pn = reinterpret_cast<float*>(p);
    float* pe = pn + (size_t)B * M * 3;
    int32_t* ps = reinterpret_cast<int32_t*>(pe + (size_t)B * 4 * M);
    int32_t* pr = ps + (size_t)B * 4 * M;
    int64_t* pst = reinterpret_cast<int64_t*>(pr + (size_t)B * 4 * M);
    double* prw = reinterpret_cast<double*>(pst + B);
    int32_t* pc = reinterpret_cast<int32_t*>(prw + B);
    int32_t* pnx = pc + (size_t)B * R;
    uint8_t* pd = reinterpret_cast<uint8_t*>(pnx + (size_t)B * R);
    uint8_t* pnr = pd + B;
    for (int s = 0; s < 3; ++s)
      CHECK(cov_step_host(h, act.data(), pn, pe, ps, pr, pst, prw, pd, pc, pnx, pnr, COV_NEXT_GREEDY) == 0);
    for (int i = 0; i < B * R; ++i) CHECK(pnx[i] >= 0 && pnx[i] < 4);
    CHECK(fe_host_free(pin) == 0);
  }
  CHECK(cov_sync(h) == 0);
  CHECK(cov_destroy(h) == 0);
}

// Per-episode maps: the lattice query, seeded and continued device streams, given cities,
// the targets read back, a map too big for its handle, then a step on the new maps.
static void map_session() {
  cov_map_config mc{};
  mc.x_min = mc.y_min = -120.0;
  mc.x_max = mc.y_max = 120.0;
  mc.lattice_spacing = 5.5;
  mc.world_radius = 120.0;
  mc.road_radius = mc.link_radius = 6.6;
  mc.near_radius = 6.6 / 1.4;
  mc.n_cities = 12;
  int32_t nl = 0;
  CHECK(cov_map_lattice(&mc, nullptr, &nl) == 0 && nl > 0);
  std::vector<double> lat((size_t)nl * 2);
  int32_t short_n = 3;
  CHECK(cov_map_lattice(&mc, lat.data(), &short_n) != 0 && short_n == nl);  // capacity short
  CHECK(cov_map_lattice(&mc, lat.data(), &nl) == 0);
  const int R = 6, B = 2;
  cov_config cc{};
  cc.n_robots = R;
  cc.n_envs = B;
  cc.max_nodes = 1000;
  cc.episode_length = 75;
  cc.res = 5.5;
  cc.motion_radius = 6.6;
  cc.device = 0;
  cc.horizon = -1;
  cov_handle* h = nullptr;
  CHECK(cov_create(&cc, &h) == 0);
  if (!h) return;
  std::vector<int32_t> nt(B), st(B);
  std::vector<double> cities((size_t)B * 12 * 2);
  CHECK(cov_generate_maps(h, &mc, -1, 8, nullptr, COV_MAP_SEED, nt.data(), st.data(), cities.data()) == 0);
  for (int b = 0; b < B; ++b) CHECK(nt[b] > R && nt[b] <= 1000 - R);
  CHECK(cov_generate_maps(h, &mc, 1, 0, nullptr, 0, nt.data(), st.data(), nullptr) == 0);  // stream continues
  CHECK(cov_generate_maps(h, &mc, 0, 0, cities.data(), COV_MAP_CITIES, nt.data(), st.data(), nullptr) == 0);
  std::vector<double> tg((size_t)nt[0] * 2);
  CHECK(cov_get_targets(h, 0, tg.data()) == 0);
  CHECK(cov_get_targets(h, B, tg.data()) != 0);
  mc.n_cities = 33;  // more than the kernel holds
  CHECK(cov_generate_maps(h, &mc, -1, 8, nullptr, COV_MAP_SEED, nt.data(), st.data(), nullptr) != 0);
  CHECK(cov_destroy(h) == 0);
  // the same maps cannot fit a handle of 200 nodes: GF_EINVAL with the sizes reported
  cc.max_nodes = 200;
  mc.n_cities = 12;
  CHECK(cov_create(&cc, &h) == 0);
  if (!h) return;
  CHECK(cov_generate_maps(h, &mc, -1, 8, nullptr, COV_MAP_SEED, nt.data(), st.data(), nullptr) != 0);
  CHECK((st[0] & COV_MAP_TOO_MANY) != 0);
  CHECK(std::strlen(fe_last_error()) > 0);
  CHECK(cov_destroy(h) == 0);
}

static void graph_session() {
  gu_graph* g = nullptr;
  CHECK(gu_create(0, &g) == 0);
  if (!g) return;
  const int n = 40;
  std::vector<double> p((size_t)n * 2);
  for (int i = 0; i < n; ++i) {
    p[2 * i] = 0.37 * i;
    p[2 * i + 1] = 0.11 * (i % 7);
  }
  int64_t ne = 0;
  CHECK(gu_radius_edges(g, p.data(), n, nullptr, n, 1.0, 0, &ne) == 0 && ne > 0);
  CHECK(gu_radius_edges(g, p.data(), -1, nullptr, n, 1.0, 0, &ne) != 0);
  std::vector<int32_t> s(ne > 0 ? ne : 1), r(ne > 0 ? ne : 1);
  std::vector<double> d(ne > 0 ? ne : 1), diff(ne > 0 ? 2 * ne : 2);
  CHECK(gu_get_edges(g, s.data(), r.data(), d.data(), diff.data()) == 0);
  CHECK(gu_destroy(g) == 0);
}

int main() {
  validation_paths();
  if (have_device()) {
    std::printf("device present: running the GPU sessions\n");
    flocking_session();
    coverage_session();
    map_session();
    graph_session();
  } else {
    std::printf("no device: validation and no-device paths only\n");
  }
  if (failures) std::fprintf(stderr, "%d check(s) failed\n", failures);
  else std::printf("capi_asan: ok\n");
  std::fflush(stdout);
  std::fflush(stderr);
  // skip static destructors: ASan's device-allocator hook (ROCm) fails a CHECK when its
  // quarantine recycles a block after the HIP runtime has unloaded at exit
  _exit(failures ? 1 : 0);
}
