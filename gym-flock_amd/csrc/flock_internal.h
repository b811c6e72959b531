// Internal interface between the C-ABI (capi.hip) and the kernels (flock_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "done_flag.h"

namespace gf {

// Ablation switches (StepArgs / KnnArgs .diag, timing experiments that give wrong
// outputs) exist only in the diagnostic build (make diag: -DGF_DIAG); the product build
// compiles every such branch out.
// -DGF_CT_ABLATE=<mask>: the same switches as compile-time constants, for register
// studies (scripts/vgpr_phases.sh: each phase compiled out, -Rpass-analysis per build).
#if defined(GF_CT_ABLATE)
#define GF_ABLATE(args, bits) ((static_cast<unsigned long long>(GF_CT_ABLATE) & (bits)) != 0)
#elif defined(GF_DIAG)
#define GF_ABLATE(args, bits) (((args).diag & (bits)) != 0)
#else
#define GF_ABLATE(args, bits) false
#endif

constexpr int kThreads = 256;   // 4 wave64s per workgroup
constexpr int kTileMax = 1024;      // max agents per LDS tile (32 KiB of float64 state)
constexpr int kTileDefault = 512;   // default tile (measured best, see step_tile)
constexpr size_t kStepLdsPlainFloor = 24 * 1024;  // plain step: 6 workgroups per CU, not 7
constexpr int kKnnLdsMax = 4096;    // kNN stages the env's positions in LDS up to this N
constexpr int kKnnGridCells = 2048; // kNN: cells of the per-env uniform grid (at most)
constexpr int kInlineRimU = 4;      // fused kNN inline rim scan: columns in flight per lane
constexpr int kStoreTab = 16;      // network rows: float4 table entries per wave (one per nibble)
constexpr int kStepInlineRim = 2;  // fused kNN: unranked rows a wave ranks itself (more: rim kernel)
constexpr int kStepExactKnnMax = 128;  // fused kNN: envs up to this size are ranked exactly in
                                       // the step (KX: one tile in LDS, no rim kernel)
constexpr int kStepExactKnnMaxOneEnv = 192;  // the same for a handle of one env (the drop-in
                                             // step: its tile then holds the whole env); beyond
                                             // it the per-row scan costs more than the rim
                                             // kernel it saves (profiles/r05/ab_dropin_exact_one_env.txt)
constexpr int kKnnRimGrid = 256;     // rim kNN: workgroups walking the flagged blocks
constexpr int kKnnRimHalfGrid = kKnnRimGrid / 2;  // the same per half-batch launch
constexpr int kKnnFewSlow = 16;     // kNN: up to this many rows to scan per workgroup are
                                    // scanned wave-cooperatively from L2, more through the grid
// kNN LDS: positions (16 B per agent), the grid's cell offsets, agent indices by cell
constexpr size_t knn_lds_bytes(int N) {
  return (size_t)N * 16 + (size_t)(kKnnGridCells + 1) * 4 + (((size_t)N * 2 + 15) / 16) * 16;
}

// One batched hot-path launch. Pointers are device pointers; all per-env arrays
// are [B][N][...] contiguous.
struct StepArgs {
  const double* x_in;     // (B,N,4) state before the step
  double* x_out;          // (B,N,4) state after the step (DYN only)
  const void* u;          // (B,N,2) float or double actions (DYN only)
  float* state_values;    // (B,N,6) or nullptr
  float* network;         // (B,N,N) or nullptr
  double* ctrl_out;       // (B,N,2) or nullptr (CTRL only)
  double* reward;         // (B) or nullptr
  double* reward2;        // (B) or nullptr: a second copy (fe_step_host's page-locked array)
  double dt, action_scalar, cr, cr2;
  float dt_f, as_f;
  int N, B;
  int R;                  // rows per workgroup (power of two, 4..64)
  int T;                  // agents per LDS tile (multiple of 64)
  int bpe;                // workgroups per env = ceil(N / R)
  int mean_pooling, centralized;
  int prefetch;           // tiled step issues each tile's loads one tile ahead (T <= 512)
  int store_fast;         // network rows by the fast bit-extract loop (N % 1024 == 0)
  int u_inline;           // u is a host pointer: its B*N actions travel in the kernel arguments
                          // (StepArgsU; one env of one tile, <= kUInlineBytes)
  int diag;               // ablation switches, read only by the diagnostic build (GF_ABLATE):
                          // 2 skip feature pass,
                          // 4 non-temporal network stores, 8 skip pass 1 (bits are left
                          // unwritten: timing only), 16 skip tile loads (timing only),
                          // 64 / 128 generic / fast network store loop (A/B), 256 no
                          // per-row outputs, 512 no reward, 1024 constant network rows
                          // (timing only), 8192 plain XCD remap for the plain step (A/B)
  // Flocking variants (flocking_leader/obstacle/stoch.py). variant == 0 keeps the
  // FlockingRelative path untouched; otherwise the fields below apply (tiled kernel).
  int variant;
  int n_frozen;           // agents [0,n) ignore actions (their mask is 0)
  int n_vel_zero;         // pairs touching agents [0,n) have zero velocity difference
  double u_scale;         // the step's action multiplier (action_scalar is the controller's)
  double u_clip;          // clip actions to +-u_clip before scaling; <= 0: none
  double x_scale;         // state multiplied before / divided after the update
  double ctrl_clip;       // controller output clip; <= 0: none
  float us_f, uc_f;       // float32 copies of u_scale, u_clip
  const double* dt_env;   // (B) per-env dt of this step, or nullptr (dt)
  uint64_t* adj_bits;     // (B,N,Wn) packed adjacency or nullptr
  int32_t* degree_out;    // (B,N) degrees or nullptr
  // Flocking-v0 k-nearest selection fused into the feature pass (kStepFusedK neighbours):
  // rows the step can rank exactly get idx + obs; the others get idx[row*K] = -1 and
  // are finished by flock_knn_kernel in rim mode. Key of a ranked pair:
  // (min(floor(r2 * knn_qscale / Tr), knn_qmax) << knn_jbits) | j (see the kernel).
  int32_t* knn_idx;       // (B,N,K) or nullptr: no fused selection
  float* knn_obs;         // (B,N,4K)
  float* knn_r2;          // (B,N) k-th nearest r2 of the state two steps back (0: none),
                          // replaced by this state's for the rows ranked here
  uint8_t* knn_rimflag;   // (B, ceil(N/256)): set for each 256-row block holding a row
                          // left to the rim kNN (its workgroups read only this byte)
  double knn_qscale;      // 2^qbits
  unsigned knn_qmax;      // 2^qbits - 2
  double knn_qmaxd;       // the same as a double (compared with r2 * scale)
  int knn_jbits;          // bits of the agent index (qbits = 32 - jbits)
  int knn_exact;          // the handle's fused selection is exact in the step (step_knn_exact)
  DoneFlag fin;           // drop-in launch: the grid's completion flag (done_flag.h)
};

// The drop-in step's actions passed in the kernel arguments (fe_step_host, one env of up
// to kUInlineBytes of actions: 384 agents in float32, 192 in float64)
constexpr int kUInlineBytes = 3072;
struct StepArgsU {
  StepArgs a;
  alignas(16) unsigned char u[kUInlineBytes];
};

constexpr int kStepFusedK = 7;  // Flocking-v0's n_neighbors (flocking.py:9)

struct KnnArgs {
  const double* x;        // (B,N,4) current state
  int32_t* idx;           // (B,N,K)
  float* obs;             // (B,N,4K)
  int N, B, K;
  const uint64_t* adj_bits;  // (B,N,Wn) adjacency of x from the step, or nullptr
  const int32_t* degree;     // (B,N) with adj_bits
  int rim;                   // only rows the fused step left unranked (idx[row*K] < 0)
  float* r2k;                // (B,N) or nullptr: each ranked row's k-th nearest r2
  uint8_t* rimflag;          // rim mode: (B, ceil(N/256)) blocks the step marked (cleared here)
  int grid_cap;              // rim mode: workgroups (0: kKnnRimGrid)
  int diag;                  // ablation (fe_diag bits << 12, apart from the step's): 0x4000 no ranking on the neighbour path, 0x8000 no neighbour path,
                             // 0x1000 grid built but no search, 0x2000 no grid / scan, 0x0800 no outputs
  DoneFlag fin;              // drop-in launch: the grid's completion flag (done_flag.h)
};

struct StatsArgs {
  const double* x;        // (B,N,4)
  double* vel_diffs;      // (B,N)
  double* min_dists;      // (B,N)
  int32_t* degree;        // (B,N) neighbours with r2 < comm_radius^2
  double cr2;
  int N, B;
};

// Launch-geometry helpers shared by host and tests.
int step_rows_per_block(int N);
int step_tile(int N);
size_t step_lds_bytes(int N, int R, int T, bool ctrl, bool knn);

hipError_t launch_step(const StepArgs& a, bool dyn, bool u_f64, bool ctrl, hipStream_t s);

// Whether a step of this geometry can carry the fused k-nearest selection (K ==
// kStepFusedK, no variant, no tile prefetch, at least K word-slices per row).
bool step_fused_knn_ok(int N, int R, int K, bool variant, bool prefetch);
// Whether the fused selection of a handle of B envs of N agents (tile T) ranks every row
// exactly in the step (the KX instantiation: one tile, N <= kStepExactKnnMax, or one env of
// up to kStepExactKnnMaxOneEnv agents): no rim kernel follows.
bool step_knn_exact(int N, int T, int B);
hipError_t launch_knn(const KnnArgs& a, hipStream_t s);
hipError_t launch_stats(const StatsArgs& a, hipStream_t s);
// per env: mean vel_diffs, mean min_dists of launch_stats' outputs -> out (B,2)
hipError_t launch_stats_summary(const StatsArgs& a, double* out, hipStream_t s);
// Diagnostic: stream `bytes` of float4 stores into p (nt = non-temporal), the
// write-bandwidth ceiling of the network buffer on this device.
hipError_t launch_fill(void* p, size_t bytes, bool nt, hipStream_t s);

}  // namespace gf
