/*
 * gymflock.h — C-ABI of libgymflock.so, the MI355X (gfx950) env-step engine for
 * gym-flock's FlockingRelative-v0 / Flocking-v0 hot path.
 *
 * The reference (katetolstaya/gym-flock) has no FFI: its boundary is the Python
 * gym.Env method surface. Each entry point below replaces one
 * NumPy code region of that surface; the citation after each declaration names it
 * (paths relative to the reference root). The Python binding that sits on top of
 * this ABI (gym-flock_amd/gym_flock/_native.py, ctypes) mirrors the reference's
 * reset()/step()/controller()/get_stats() methods; INTEGRATION.md shows it.
 *
 * Conventions
 *  - Every function returns int: GF_OK (0) or a GF_E* code; the message of the
 *    last failure on the calling thread is fe_last_error().
 *  - Arrays are row-major, C-contiguous. Shapes use B = n_envs, N = n_agents.
 *  - Host pointers are borrowed for the duration of the call. The library owns
 *    all device memory; fe_device_buffers() exposes it for zero-copy consumers.
 *  - One handle per host thread. A step's two half-batch launches run on the
 *    handle's stream and a second one (fe_set_streams); every other call orders the
 *    handle's stream after both first, and getters synchronise it before copying out.
 *    Zero-copy consumers of fe_buffers.stream call fe_join() after fe_step.
 *  - Agent state is float64 (B,N,4) = [px, py, vx, vy] because the reference
 *    integrates in float64 (flocking_relative.py:157); observations are float32.
 */
#ifndef GYMFLOCK_H
#define GYMFLOCK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GF_ABI_VERSION 1

enum gf_status {
  GF_OK = 0,
  GF_EINVAL = 1,   /* bad argument (shape, pointer, flag)                      */
  GF_EHIP = 2,     /* HIP runtime error (no device, launch failure, ...)       */
  GF_ENOMEM = 3,   /* device allocation failed                                  */
  GF_ESTATE = 4,   /* call out of order (e.g. step before set_state)            */
  GF_ECOMM = 5     /* RCCL error                                                */
};

/* fe_step / fe_compute_helpers flags */
#define FE_WITH_CONTROLLER 0x01 /* also run controller() on the post-step state   */
#define FE_U_DEVICE        0x02 /* u is a device pointer (else host)              */
#define FE_U_F64           0x04 /* u is float64 (else float32); selects the NumPy
                                   dtype-dependent arithmetic of :96-105          */
#define FE_U_EXPERT        0x08 /* u := controller output of the previous call
                                   (closed loop, float64; u argument ignored)     */
#define FE_WITH_KNN        0x10 /* Flocking-v0 k-nearest observation              */
#define FE_NO_NETWORK      0x20 /* skip the dense (N,N) state_network write       */
#define FE_NO_STATE_VALUES 0x40 /* skip the (N,6) state_values write              */
#define FE_U_RESIDENT      0x80 /* u := the handle's action buffer as last set by
                                   fe_set_actions (already in HBM; u ignored)     */
#define FE_OUT_MAPPED        0x1 /* fe_get_outputs: destinations that are page-locked
                                   (fe_host_alloc) are written by one device copy
                                   kernel through their mapped addresses instead of
                                   one DMA copy each; others still take a copy     */
#define FE_PACKED_NETWORK 0x100 /* also write the adjacency as bits (B,N,ceil(N/64))
                                   uint64 + degree (B,N) int32, the packed output
                                   mode; with FE_NO_NETWORK the
                                   dense (N,N) write is skipped: 32x fewer bytes  */

typedef struct fe_config {
  int32_t n_agents;      /* N  (flocking_relative.py:38; params_from_cfg :74)      */
  int32_t n_envs;        /* B  independent envs batched on this device            */
  double comm_radius;    /* 0.9  (:39)                                            */
  double dt;             /* 0.01 (:40)                                            */
  double action_scalar;  /* 10.0 (:64)                                            */
  int32_t mean_pooling;  /* 1 (:27): network = adj / deg, else adj                */
  int32_t centralized;   /* 1 (:28): controller sums over all agents              */
  int32_t n_neighbors;   /* k of Flocking-v0 (flocking.py:9, 7); 0 = no kNN buffers */
  int32_t device;        /* HIP device ordinal                                    */
} fe_config;

typedef struct fe_handle fe_handle;

/* Flocking variants on the same step. Defaults reproduce
 * FlockingRelative-v0; the registered variants set (reference files under
 * gym_flock/envs/flocking/):
 *   FlockingLeader-v0      u_scale 1, n_frozen 2               (flocking_leader.py:13-15, :21-33)
 *   FlockingObstacle-v0    u_scale 1, n_frozen 4, n_vel_zero 4 (flocking_obstacle.py:19-21, :34-49, :75-80)
 *   FlockingStochastic-v0  u_scale 6, u_clip 0.5, x_scale 6, ctrl_clip 0.5, per-step dt
 *                          (flocking_stoch.py:9-12, :14-36, :39-46; dt via fe_set_dt)
 *   FlockingTwoFlocks-v0   defaults (only its reset differs, host side)        */
typedef struct fe_variant {
  int32_t n_frozen;      /* agents [0,n) ignore actions: their mask is 0 (leaders, obstacles) */
  int32_t n_vel_zero;    /* pairs touching agents [0,n) have zero velocity difference          */
  double u_scale;        /* the step's action multiplier (10 = cfg action_scalar by default);
                            the controller still divides by cfg action_scalar (:211)          */
  double u_clip;         /* clip actions to +-u_clip before scaling; <= 0: none               */
  double x_scale;        /* state multiplied before and divided after the update; 1: none     */
  double ctrl_clip;      /* controller output clip after the /action_scalar; <= 0: none       */
} fe_variant;

/* Device pointers owned by the handle (valid until fe_destroy). Ping-pong
 * buffers are reported as their CURRENT slot (the one the next getter reads).
 * state_values and network are NULL while the last observation went to host arrays
 * only (fe_step_host / fe_step_host_knn*: the device copies are stale then). */
typedef struct fe_buffers {
  double* x;             /* (B,N,4) float64 current state                        */
  float* state_values;   /* (B,N,6) float32                                      */
  float* network;        /* (B,N,N) float32                                      */
  double* controls;      /* (B,N,2) float64 last controller() output             */
  double* rewards;       /* (B)     float64                                      */
  int32_t* knn_idx;      /* (B,N,k) int32 or NULL                                */
  float* knn_obs;        /* (B,N,4k) float32 or NULL                             */
  void* stream;          /* hipStream_t of the handle                            */
  uint64_t* adj_bits;    /* (B,N,ceil(N/64)) packed adjacency or NULL (FE_PACKED_NETWORK) */
  int32_t* degree;       /* (B,N) neighbour counts or NULL (FE_PACKED_NETWORK)   */
} fe_buffers;

/* Lifecycle ---------------------------------------------------------------- */
int fe_create(const fe_config* cfg, fe_handle** out);      /* FlockingRelativeEnv.__init__ :20-66 */
int fe_destroy(fe_handle* h);                               /* close() :303 */
int fe_get_config(const fe_handle* h, fe_config* out);
/* Change comm_radius, dt, action_scalar, mean_pooling and centralized for the following
 * launches, keeping the state (the reference reads these attributes at call time, e.g.
 * self.centralized in controller() :200-201). n_agents, n_envs, n_neighbors and device
 * must equal the handle's (GF_EINVAL otherwise). A change of comm_radius, centralized or
 * action_scalar drops the last controller output (it was computed under the old values):
 * FE_U_EXPERT and fe_get_controls then need a new fe_controller / FE_WITH_CONTROLLER. */
int fe_set_params(fe_handle* h, const fe_config* cfg);

/* State ---------------------------------------------------------------------- */
int fe_set_state(fe_handle* h, const double* x);            /* env.x = ... (:189) */
int fe_set_state_env(fe_handle* h, int env, const double* x);  /* one env's (N,4) */
/* Synthetic init (reset()'s distribution without the rejection loop,
 * :164-175): env b is drawn from MT19937 seeded with seed + b in NumPy
 * RandomState's order (length, angle, bias, vx, vy), with r_max = sqrt(N). The
 * uniforms are NumPy's bit for bit; cos/sin come from the C library, so positions
 * may differ from NumPy's in the last ulp. */
int fe_reset_synthetic(fe_handle* h, uint64_t seed, double v_max);
int fe_get_state(fe_handle* h, double* x);                  /* env.x (B,N,4) */
int fe_get_state_env(fe_handle* h, int env, double* x);     /* one env's (N,4) */

/* Hot path ------------------------------------------------------------------- */
/* Upload (B,N,2) actions (float32, or float64 if f64) into the handle's resident
 * action buffer, used by fe_step(..., FE_U_RESIDENT). */
int fe_set_actions(fe_handle* h, const void* u, int f64);
/* compute_helpers() on the current state (:111-134); used by reset() (:191). */
int fe_compute_helpers(fe_handle* h, int flags);
/* step(u) (:91-109): dynamics (:96-105) + compute_helpers + instant_cost (:145-147),
 * optionally fused controller() (:194-226) and Flocking-v0 kNN (flocking.py:20-25).
 * u: (B,N,2) float32 or float64 (FE_U_F64), host or device (FE_U_DEVICE). Async. */
int fe_step(fe_handle* h, const void* u, int flags);
/* The drop-in env's step(u) (:91-109) as one launch and one wait, for small batches
 * where latency, not bandwidth, counts (FlockingRelativeEnv.step, N ~ 100-1000, B = 1).
 * u: (B,N,2) host actions, float32 or float64 (FE_U_F64). One env of at most one tile
 * (N <= 512) whose actions fit 3 KiB (N <= 384 in float32, 192 in float64) passes them in
 * the kernel arguments; otherwise page-locked ones (fe_host_alloc) are read by the kernel
 * in place, others copied first. Either way u may be reused on return. u == NULL: no dynamics,
 * compute_helpers (:111-134) on the current state (reset's observation). Outputs, any of
 * them NULL (not computed): state_values (B,N,6) f32, network (B,N,N) f32, rewards (B)
 * f64 and controls (B,N,2) f64 = controller() (:194-212) of the resulting state (fused,
 * FE_WITH_CONTROLLER implied). Page-locked destinations are written by the kernel
 * through their mapped addresses; others by a copy after it. Returns when all are in
 * place. Observations written to host arrays are not kept on the device (the device
 * getters then return GF_ESTATE); rewards also go to the ring (fe_get_rewards, metrics
 * path). flags: FE_U_F64, FE_WITH_CONTROLLER. */
int fe_step_host(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                 double* controls, int flags);
/* Flocking-v0's drop-in step(u) (flocking.py:12-25 over flocking_relative.py:91-109) as
 * one call and one wait: fe_step_host (no controller) plus the new state's k nearest
 * neighbours (the selection fused into the step, or the kNN kernel), written to knn_idx
 * (B,N,K) int32 and knn_obs (B,N,4K) float32 (either may be NULL, not both): page-locked
 * destinations through their mapped addresses (both page-locked: the step and its rim
 * kNN write the rows there directly; otherwise one copy kernel or copies). Needs
 * n_neighbors > 0. Afterwards fe_get_knn returns the same rows (recomputed on the device
 * when they were written straight to the host). */
int fe_step_host_knn(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                     int32_t* knn_idx, float* knn_obs, int flags);
/* Flocking-v0's drop-in expert loop, `u = env.controller(); env.step(u)` (controller()
 * inherited from flocking_relative.py:194-212 by flocking.py:5, step flocking.py:12-14):
 * fe_step_host_knn plus controls (B,N,2) f64 = controller() of the resulting state, fused
 * into the same launch (controls may be NULL: then as fe_step_host_knn). */
int fe_step_host_knn_ctrl(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                          double* controls, int32_t* knn_idx, float* knn_obs, int flags);
/* controller(centralized) (:194-212) on the current state; centralized < 0 means the
 * config default. Writes (B,N,2) float64 to u_out (host) if non-NULL. */
int fe_controller(fe_handle* h, int centralized, double* u_out);
/* get_stats() (:136-143) on the current state: vel_diffs (N) and min_dists (N). */
int fe_get_stats(fe_handle* h, int env, double* vel_diffs, double* min_dists);
/* get_stats plus each agent's degree (r2 < comm_radius^2): reset()'s acceptance test
 * (:177-184) on the device. Any output pointer may be NULL. */
int fe_get_stats_ex(fe_handle* h, int env, double* vel_diffs, double* min_dists, int32_t* degree);
/* Per-env summaries of get_stats for the metrics path: dst (B,2) = np.mean(vel_diffs),
 * np.mean(min_dists) of every env's current state (flocking_relative.py:136-143), taken
 * on the device (a fixed summation tree: deterministic, ulps from NumPy's order). */
int fe_stats_summary(fe_handle* h, double* dst);

/* Outputs (host copies; env < 0 copies all B envs) ---------------------------- */
int fe_get_state_values(fe_handle* h, int env, float* dst);  /* (N,6) :128-129 */
int fe_get_network(fe_handle* h, int env, float* dst);       /* (N,N) :131-134 */
int fe_get_network_rows(fe_handle* h, int env, int row0, int nrows, float* dst);
/* Packed output of the last FE_PACKED_NETWORK step: bit j%64 of word j/64 of row i is
 * adj(i,j) (r2 < comm_radius^2, :117); the network is adj/max(degree,1) (:120-122).
 * env < 0: all envs. Either pointer may be NULL. */
int fe_get_network_packed(fe_handle* h, int env, uint64_t* bits, int32_t* degree);
int fe_get_controls(fe_handle* h, int env, double* dst);     /* (N,2) :210-211 */
int fe_get_rewards(fe_handle* h, double* dst);
/* The step's host outputs in one call with one stream sync (the drop-in env's
 * (state_values, network), reward tuple of step(), flocking_relative.py:109): any of
 * state_values (N,6) / network (N,N) of `env` (env < 0: all envs) and rewards (B) may be
 * NULL. flags: 0, or FE_OUT_MAPPED (page-locked destinations written by one copy
 * kernel: one launch instead of up to three DMA copies, each of which costs ~12-15 us of
 * latency at drop-in sizes). Returns after the data is in the destinations. */
int fe_get_outputs(fe_handle* h, int env, float* state_values, float* network, double* rewards, int flags);
/* Page-locked host memory for output arrays (the drop-in env hands such buffers to the
 * caller as fresh arrays and recycles them once released). */
int fe_host_alloc(size_t bytes, void** out);
int fe_host_free(void* p);               /* (B)   :145-147 */
int fe_get_knn(fe_handle* h, int env, int32_t* idx, float* obs); /* (N,k), (N,4k) */
int fe_device_buffers(fe_handle* h, fe_buffers* out);
int fe_sync(fe_handle* h);
/* Select a flocking variant for every later step / controller call (NULL: back to
 * FlockingRelative). */
int fe_set_variant(fe_handle* h, const fe_variant* v);
/* Per-env dt[B] for the following steps (FlockingStochastic-v0 draws one per step,
 * flocking_stoch.py:24); NULL reverts to cfg dt. */
int fe_set_dt(fe_handle* h, const double* dt);

/* Multi-GPU metrics path (RCCL over xGMI) ---------------------- */
/* The env batch is sharded contiguously over ranks (one process per GPU); the
 * step path has no exchange. Only per-env rewards (and, optionally, get_stats
 * summaries) are all-gathered, on a side stream, so the collective never sits on the
 * step critical path. Shards may differ in size (shard.py's shard_range gives the first
 * B % world ranks one env more): every gathered block is padded to the largest shard,
 * max_envs, and rank r's entries past its own n_envs are zero. Every wait for a
 * collective is bounded by the init timeout: a rank that never joins or stops
 * responding makes the others' calls return GF_ECOMM (the communicator is then aborted
 * and the handle keeps stepping) instead of hanging. All ranks make the same sequence
 * of metrics calls after the same number of steps. */
int fe_comm_unique_id(uint8_t id[128]);
/* Creates the communicator (non-blocking RCCL init, polled) and all-gathers every
 * rank's n_envs (fe_comm_shard_sizes). Bounded by timeout_s (fe_comm_init: 300 s). */
int fe_comm_init(fe_handle* h, int nranks, int rank, const uint8_t id[128]);
int fe_comm_init_timeout(fe_handle* h, int nranks, int rank, const uint8_t id[128], double timeout_s);
/* The rule fe_comm_init applies to the exchanged sizes: GF_OK when every n_envs[r]
 * (r < nranks) is >= 1, else GF_ECOMM naming them. Host-only (no device). */
int fe_check_shard_sizes(int nranks, const int32_t* n_envs);
/* The communicator as RCCL sees it: ncclCommCount, ncclCommUserRank, the HIP device
 * ordinal it runs on (ncclCommCuDevice) and that device's PCI bus id (bus_id_len bytes,
 * hipDeviceGetPCIBusId). Any output pointer may be NULL. */
int fe_comm_info(fe_handle* h, int32_t* count, int32_t* user_rank, int32_t* device, char* bus_id, int bus_id_len);
/* Every rank's n_envs (sizes[nranks]) and the largest, the gathers' padded width. */
int fe_comm_shard_sizes(fe_handle* h, int32_t* sizes, int32_t* max_envs);
/* Enqueue (side stream, after the latest step) an all-gather of the per-env rewards of
 * every step since the previous reward all-gather (or since fe_comm_init), each step
 * exactly once, at any interval up to 64 steps. GF_ESTATE if no step was taken since,
 * or if more than 64 were (the oldest were overwritten: the call then skips them all). */
int fe_allgather_rewards(fe_handle* h);
/* Wait (bounded) for the latest reward all-gather; dst gets (nranks, steps, max_envs)
 * rewards, rank-major, steps = fe_gathered_steps(h) (oldest first). */
int fe_get_gathered_rewards(fe_handle* h, double* dst);
int fe_gathered_steps(fe_handle* h);
/* Enqueue (side stream) an all-gather of every rank's fe_stats_summary of the current
 * state: the optional get_stats aggregates of SURVEY.md §8e. The summaries are taken
 * on the handle's stream after both step halves (a join, so the next step is one launch,
 * unlike the reward all-gather); call it per episode or logging interval, not per step.
 * fe_get_gathered_stats waits (bounded) for it; dst gets (nranks, max_envs, 2),
 * rank-major. */
int fe_allgather_stats(fe_handle* h);
int fe_get_gathered_stats(fe_handle* h, double* dst);
/* Destroys the communicator and the metrics path's buffers; fe_comm_init may follow. A
 * side stream that does not drain within the collective timeout is aborted instead. */
int fe_comm_destroy(fe_handle* h);
/* Tests only: close = 1 enqueues on the collectives' side stream a one-wave kernel that
 * spins (s_sleep) until close = 0 is called or max_seconds pass, standing in for a
 * collective whose peer stopped responding; close = 0 releases it. Needs fe_comm_init. */
int fe_debug_comm_gate(fe_handle* h, int close, double max_seconds);
/* Tests only: what the metrics path saw, out[12]: [0] ring-slot reuse checks that found
 * a gather's staging copy still listed, [1] whether that copy had stored its completion
 * word at the last one (1) or not (0), [2] its bounded wait's status (-1: no wait), [3]
 * the communicator's async state at that wait's first poll, [4] staging copies listed
 * after the last reward gather, [5] whether its copy was complete right after the
 * gather was enqueued, [6] hipStreamQuery of the side stream right after the last gate
 * launch, [7] polls of the last bounded wait, [8] the gate kernel has started (1), [9]
 * how it ended (0 running, 1 opened, 2 timed out), [10] a communicator is live, [11]
 * staging copies listed now. */
int fe_debug_comm_state(fe_handle* h, int32_t* out);
/* The HIP runtime and RCCL this library is bound to in this process (a process that
 * loaded another copy of either first, e.g. PyTorch's bundled ones, binds that copy):
 * hipRuntimeGetVersion, hipDriverGetVersion (0 without a driver), ncclGetVersion, and the
 * paths of the shared objects those entry points resolved to (dladdr). Host-only; any
 * pointer may be NULL. */
int fe_runtime_info(int32_t* hip_runtime_version, int32_t* hip_driver_version, int32_t* rccl_version, char* hip_path,
                    int hip_path_len, char* rccl_path, int rccl_path_len);

/* ============================ Coverage-v0 ==================================== */
/* gym_flock/envs/spatial/coverage.py. B envs of n_robots robots moving on a per-env
 * target graph (at most max_nodes - n_robots targets). Node indices are global as in
 * the reference: robots 0..R-1, targets R..R+T-1. */
typedef struct cov_config {
  int32_t n_robots;        /* R (coverage.py:83, N_ROBOTS=6; config 4 uses 200)        */
  int32_t n_envs;          /* B                                                         */
  int32_t max_nodes;       /* padded node count (MAX_NODES :55; config 4 uses 1000)     */
  int32_t episode_length;  /* 75 (EPISODE_LENGTH :64)                                   */
  double res;              /* lattice spacing, edge-feature scale (DELTA 5.5, :80)       */
  double motion_radius;    /* res * 1.2 (:136)                                          */
  int32_t device;
  int32_t horizon;         /* greedy expert: relaxation sweeps - 1 (HORIZON=10, :66);
                              -1 = until converged                                       */
} cov_config;

typedef struct cov_handle cov_handle;

#define COV_ACTIONS_DEVICE   0x1 /* actions is a device pointer                          */
#define COV_ACTIONS_RESIDENT 0x2 /* use the actions last given to cov_set_actions        */
#define COV_ACTIONS_GREEDY   0x20 /* the step's actions are controller(greedy=True)'s (:800-872),
                                    computed in the same launch from per-node greedy lists
                                    built with the time matrix; robots the reference hands to
                                    np_random.choice(4) take action 0 (needs_random flags them),
                                    or with COV_GREEDY_RNG draw it on the device. The actions
                                    taken stay resident (COV_ACTIONS_RESIDENT). */
#define COV_GREEDY_RNG       0x80 /* with COV_ACTIONS_GREEDY: each fallback robot takes
                                    np_random.choice(4) (:861-864) from its env's stream (set
                                    by cov_set_rng), in robot order, bit-exact with numpy's
                                    legacy RandomState; the stream advances on the device */

int cov_create(const cov_config* cfg, cov_handle** out);        /* CoverageEnv.__init__ :83 */
int cov_destroy(cov_handle* h);
/* Targets of one env (env < 0: every env) and its motion graph + static observation
 * (_initialize_graph :529-594, utils._get_graph_edges :8-24), built on the device. */
int cov_set_targets(cov_handle* h, int env, int n_targets, const double* targets);

/* Per-episode target maps, _generate_targets (coverage.py:516-527) as every reset() calls
 * it (:378-397), with generate_lattice (make_map.py:30-67) and generate_geometric_roads
 * (make_map.py:207-231). The reference's values: arena (-120, 120, -120, 120) (XMAX/YMAX
 * :75-76), lattice_spacing DELTA = 5.5 (:61, the lattice vectors :125-128), 12 cities,
 * world_radius x_max, road_radius and link_radius motion_radius (= res * 1.2), near_radius
 * motion_radius / 1.4. */
typedef struct cov_map_config {
  double x_min, x_max, y_min, y_max; /* the arena: generate_lattice's free_region           */
  double lattice_spacing;            /* square lattice vectors (-s, 0), (0, -s)             */
  double world_radius;               /* cities U(-r, r)^2 (make_map.py:208)                 */
  double road_radius;                /* waypoint spacing along each Delaunay road (:228-229) */
  double near_radius;                /* lattice points within it of a waypoint (:521)       */
  double link_radius;                /* the target graph's radius (:523-524)                */
  int32_t n_cities;                  /* 12 (:518); at most 32                               */
} cov_map_config;
#define COV_MAP_SEED   0x1 /* seed env b's map stream as np.random.seed(map_seed + b) first;
                              otherwise the streams continue from the previous maps, as the
                              reference's global np.random does from one reset to the next */
#define COV_MAP_CITIES 0x2 /* the cities are given (host (n_sel, n_cities, 2), the drop-in
                              env draws them from np.random itself); no stream is used      */
/* status_out bits (per env) */
#define COV_MAP_NEAR_DEGENERATE 0x1 /* an orientation or incircle sign of the cities fell
                                       inside its rounding bound: Qhull decides such sets by
                                       its own precision handling (parity unpinned)         */
#define COV_MAP_TOO_MANY        0x2 /* more targets than max_nodes - n_robots              */
#define COV_MAP_TOO_FEW         0x4 /* fewer targets than robots                           */
#define COV_MAP_OVERFLOW        0x8 /* more waypoints than the kernel holds                */
/* New maps on the device for env `env` (env < 0: every env): the cities (drawn on the
 * device from each env's stream, numpy's legacy uniform, or given), their Delaunay roads,
 * the lattice points near them and the largest connected component of their radius
 * graph; then the motion graph and static observation as cov_set_targets builds them.
 * n_targets_out, status_out (n_sel) and cities_out (n_sel, n_cities, 2) may be NULL. A
 * map that cannot be used (TOO_MANY / TOO_FEW / OVERFLOW) fails the call with GF_EINVAL,
 * that env left without a graph; NEAR_DEGENERATE maps are used and reported. */
int cov_generate_maps(cov_handle* h, const cov_map_config* mc, int env, uint64_t map_seed, const double* cities,
                      int flags, int32_t* n_targets_out, int32_t* status_out, double* cities_out);
/* The targets (n_targets, 2) of env `env`'s current map. */
int cov_get_targets(cov_handle* h, int env, double* targets);
/* Host only (no device): generate_lattice's points (make_map.py:30-67) for mc, [y, x]
 * columns in its order, into xy (capacity *n points; *n receives the count, also when
 * the capacity is short, which fails with GF_EINVAL). xy may be NULL to query *n. */
int cov_map_lattice(const cov_map_config* mc, double* xy, int32_t* n);

/* reset() after its random draws (:405-424): start[B][R] target-local start nodes,
 * visited[B][max_nodes-R] (1 = visited); computes reset's observation (:424). */
int cov_reset(cov_handle* h, const int32_t* start, const uint8_t* visited);
/* reset() with its random draws on the device (:405-424): env b as a reference env whose
 * np_random was seeded seed + b, RandomState(seed + b)'s choice(arange(T), R,
 * replace=False) for the start targets and choice(arange(T) + R, int(T * frac_active),
 * replace=False) for the unvisited ones, bit-exact; the envs' streams then continue on the
 * device for COV_GREEDY_RNG (as after cov_set_rng). start_out (B,R) and visited_out
 * (B, max_nodes - R) may be NULL; otherwise they receive the draws, in cov_reset's layout. */
int cov_reset_seeded(cov_handle* h, uint64_t seed, double frac_active, int32_t* start_out, uint8_t* visited_out);
/* step(action) (:174-204, :234-364): actions[B][R] in [0,4). */
int cov_step(cov_handle* h, const int32_t* actions, int flags);
/* n_steps fused greedy expert steps (COV_ACTIONS_GREEDY | COV_GREEDY_RNG: controller(greedy=
 * True)'s actions and the reference's np_random.choice(4) fallback draws, coverage.py:800-872,
 * then step, :174-364) in ONE launch, each env's workgroup stepping its env n_steps times:
 * the same result as n_steps calls of cov_step(h, NULL, COV_ACTIONS_GREEDY | COV_GREEDY_RNG)
 * (expert rollouts: the reference's demonstrations). Needs the envs' streams on the device
 * (cov_set_rng / cov_reset_seeded), n_robots <= 624 and max_nodes - n_robots <= 1024.
 * rewards / done (both may be NULL; then the call returns without waiting): (n_steps, B) host
 * arrays of every step's reward and done flag; the last step's are also cov_get_rewards'. */
int cov_step_expert(cov_handle* h, int n_steps, double* rewards, uint8_t* done);
int cov_set_actions(cov_handle* h, const int32_t* actions);
/* Every env's np_random stream for COV_GREEDY_RNG steps, in the layout of numpy's
 * RandomState.get_state() (MT19937): keys[B][624] the key words, pos[B] in [0, 624] the
 * position. Needs n_robots <= 624. cov_get_rng reads them back (after the steps that
 * drew from them), to continue the stream on the host with RandomState.set_state. */
int cov_set_rng(cov_handle* h, const uint32_t* keys, const int32_t* pos);
int cov_get_rng(cov_handle* h, uint32_t* keys, int32_t* pos);
/* The drop-in env's step(action) (coverage.py:174-204 with _get_obs_reward :234-364) as
 * one launch and one wait, the reference driver's loop (test.py:43-74): actions[B][R] in
 * [0,4) (B*R <= 512: passed in the kernel arguments), then the whole observation of every
 * env, step counter, reward, done flag and each robot's node after the step (the next
 * step's last_loc, closest_targets :427-432) written to the given host arrays: nodes
 * (B,M,3) f32, edges (B,4M) f32, senders / receivers (B,4M) i32, step (B) i64, reward (B)
 * f64, done (B) u8, closest (B,R) i32. Page-locked destinations (fe_host_alloc) are
 * written by the step's own workgroups through their mapped addresses, others by copies
 * after it; any pointer may be NULL. flags: COV_NEXT_GREEDY also computes, in the same
 * launch, controller(greedy=True)'s actions of the resulting state (:800-872) into
 * next_actions (B,R) i32 and needs_random (B,R) u8 (robots the reference hands to
 * np_random.choice(4), action 0 here), which also stay resident (COV_ACTIONS_RESIDENT);
 * it builds the time matrices first if the graph changed. */
#define COV_NEXT_GREEDY 0x40
int cov_step_host(cov_handle* h, const int32_t* actions, float* nodes, float* edges, int32_t* senders,
                  int32_t* receivers, int64_t* step, double* reward, uint8_t* done, int32_t* closest,
                  int32_t* next_actions, uint8_t* needs_random, int flags);
/* Place one env's robots anywhere (x[:R] = ...); closest targets are recomputed. */
int cov_set_robot_positions(cov_handle* h, int env, const double* xr);
/* Observation of one env (:353): nodes (M,3) f32, edges (4M) f32, senders/receivers
 * (4M) i32, step; any pointer may be NULL. */
int cov_get_obs(cov_handle* h, int env, float* nodes, float* edges, int32_t* senders, int32_t* receivers,
                int64_t* step);
int cov_get_rewards(cov_handle* h, double* reward, uint8_t* done);   /* (B), (B) */
int cov_get_robots(cov_handle* h, int env, double* xr, int32_t* nodes); /* closest_targets :427 */
int cov_get_visited(cov_handle* h, int env, uint8_t* visited); /* (max_nodes - R): reset()'s layout */
int cov_get_n_motion(cov_handle* h, int32_t* n_motion);
/* Launches per cov_step. n = 0 (the default): fused greedy steps (COV_ACTIONS_GREEDY) go
 * out as two half-batch launches on two streams (as fe_set_streams), every other step as
 * one launch, which the device, not the host, bounds (scripts/cov_launch_probe.py); n = 2
 * splits every step, n = 1 none. Every other call, cov_sync included, first orders the
 * handle's stream after both. */
int cov_sync(cov_handle* h);
int cov_set_streams(cov_handle* h, int n);
/* Greedy expert, controller(greedy=True) :800-872. On first use after cov_set_targets
 * it builds each env's time matrix (construct_time_matrix :621-653) on the device;
 * then every robot heads for its nearest unvisited target via the predecessor matrix.
 * The actions stay resident for cov_step(.., COV_ACTIONS_RESIDENT). Robots the
 * reference hands to np_random.choice(4) (target out of reach, :839-844 and :863-864)
 * get action 0 and needs_random = 1: draw those on the host in robot order and upload
 * the patched array with cov_set_actions. actions[B][R], needs_random[B][R] and
 * n_random may be NULL; with all three NULL the call does not synchronise. */
int cov_controller_greedy(cov_handle* h, int32_t* actions, uint8_t* needs_random, int64_t* n_random);
/* The resident actions (B,R) (the last cov_set_actions, cov_controller_greedy or
 * COV_ACTIONS_GREEDY step) and the needs_random flags (B,R) of the last greedy call;
 * either pointer may be NULL. */
int cov_get_actions(cov_handle* h, int32_t* actions, uint8_t* needs_random);
/* One env's graph_cost (inf -> MAX_COST=1000, as :651) and graph_previous, each
 * (T,T) row-major, T = that env's target count; builds the matrix if needed. */
int cov_get_time_matrix(cov_handle* h, int env, int32_t* cost, int32_t* prev);

/* Observation wire formats for graph trainers. */
#define COV_OUT_DEVICE 0x4 /* output pointers are device memory (else host)             */
#define COV_FLAT_F32   0x8 /* flat rows as float32 (the wrapper's Box dtype), else float64 */
#define COV_MASK_ALL   0x10 /* graph tuple: drop every graph's padded edges, not only graph
                               0's as the reference's unpack_obs does (see below)         */
/* Every env's observation flattened like gym's FlattenDictWrapper over keys
 * ['nodes','edges','senders','receivers','step'] (coverage.py:90, test.py:33):
 * dst (B, 15*max_nodes + 1), float64 (np.concatenate's promotion) or float32. */
int cov_get_flat_obs(cov_handle* h, void* dst, int flags);
/* unpack_obs (coverage.py:689-741) of the batch without TensorFlow: n_edge[B] and the
 * total edge count of the tuple cov_get_graphs_tuple writes. The reference masks edges
 * after offsetting senders by the graph's first node, so only graph 0 drops its padding
 * (COV_MASK_ALL drops all). */
int cov_graphs_tuple_sizes(cov_handle* h, int32_t* n_edge, int64_t* total_edges, int flags);
/* n_node[B] (= max_nodes), nodes (B*max_nodes, 3) f32, n_edge[B], edges (total, 1) f32,
 * senders/receivers (total) i32 offset by b*max_nodes, globs (B, 1) f32 (step). Any
 * pointer may be NULL; with COV_OUT_DEVICE all are device pointers. */
int cov_get_graphs_tuple(cov_handle* h, int32_t* n_node, float* nodes, int32_t* n_edge, float* edges,
                         int32_t* senders, int32_t* receivers, float* globs, int flags);

/* Graph helpers of gym_flock/envs/spatial/utils.py ------
 * A context owns device scratch and the last edge list. Positions are host float64
 * (n, 2) arrays; pos2 == NULL means pos2 = pos1 (the reference's pos2=None), with the
 * diagonal as the self pair. Edges come out in np.nonzero's row-major order. */
typedef struct gu_graph gu_graph;
int gu_create(int device, gu_graph** out);
int gu_destroy(gu_graph* g);
/* _get_graph_edges(rad, pos1, pos2=None, self_loops=False), utils.py:8-24: pairs with
 * r = |pos1[i] - pos2[j]| != 0 and not r > rad. *n_edges = their count. */
int gu_radius_edges(gu_graph* g, const double* pos1, int32_t n1, const double* pos2, int32_t n2, double rad,
                    int self_loops, int64_t* n_edges);
/* _get_k_edges(k, pos1, pos2=None, self_loops=False, allow_nearest=False),
 * utils.py:60-88: per row the k smallest r (allow_nearest), or the k+1 smallest minus
 * the row's argmin. Equal distances at the k-th boundary go to the lower column (numpy
 * leaves that choice to its selection algorithm). GF_EINVAL where np.argpartition
 * raises (kth >= row length). */
int gu_k_edges(gu_graph* g, int32_t k, const double* pos1, int32_t n1, const double* pos2, int32_t n2,
               int self_loops, int allow_nearest, int64_t* n_edges);
/* The last result: senders/receivers (E) i32, r (E) f64, diff (2E) f64 = every edge's
 * dx, then every dy (the reference's np.hstack of the two difference columns). Any
 * pointer may be NULL. */
int gu_get_edges(gu_graph* g, int32_t* senders, int32_t* receivers, double* r, double* diff);
/* _nodes_within_radius(rad, pos1, pos2), utils.py:27-39: valid[j] = 1 when the column
 * sum of r (r > rad zeroed) over pos1 is > 0. */
int gu_nodes_within_radius(gu_graph* g, const double* pos1, int32_t n1, const double* pos2, int32_t n2, double rad,
                           uint8_t* valid);

/* Diagnostics ---------------------------------------------------------------- */
const char* fe_last_error(void);
int fe_abi_version(void);
/* Average device time (ms) of the step kernel, measured with HIP events on the
 * handle's stream (bench roofline). enable >= 1 starts timing every enable-th launch
 * (events keep a sampled launch from overlapping its neighbours); 0 reads and stops;
 * -1 reads and keeps timing. With split steps (fe_set_streams, 2 by default) the
 * result is the device time of the whole window since enable divided by the steps in
 * it, and `launches` counts steps (each two concurrent half-batch launches). */
int fe_kernel_timing(fe_handle* h, int enable, double* avg_ms, int64_t* launches);
/* Launches per step: 2 (default) sends envs
 * [0, ceil(B/2)) to the handle's stream and the rest to a second stream; each half
 * depends only on its own previous step, so one launch's ramp and tail overlap the
 * other's body. Every other call first orders the handle's stream after both halves,
 * so getters and fe_sync see whole steps. A step follows as one launch when other
 * work was enqueued on the handle since the previous step. */
int fe_set_streams(fe_handle* h, int n);
/* Order the handle's stream after all of its outstanding work (enqueue only, no host
 * wait): for zero-copy consumers that enqueue on fe_buffers.stream after fe_step. */
int fe_join(fe_handle* h);
/* The same for cov_step_kernel on a Coverage handle. */
int cov_kernel_timing(cov_handle* h, int enable, double* avg_ms, int64_t* launches);
/* Diagnostics for roofline work: what = 0/1 times `reps` launches of a float4
 * plain/non-temporal fill of the network buffer (the write-bandwidth ceiling).
 * what = 0x10000 | bits (16 bits) sets ablation switches on later step launches
 * (0x10000 clears) in the diagnostic build only (make diag, -DGF_DIAG); the product
 * library returns GF_EINVAL for it and never reads an environment variable. */
int fe_diag(fe_handle* h, int what, int reps, double* avg_ms);

#ifdef __cplusplus
}
#endif
#endif /* GYMFLOCK_H */
