// Internal interface of the Coverage-v0 kernels (coverage_kernels.hip) for the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gf {

// Device buffers of a batch of B Coverage envs with R robots and room for M nodes
// (robots + targets), i.e. at most Tmax = M - R targets per env.
struct CovArgs {
  int B, R, M, Tmax, episode_length;
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
  int* err;               // device error bits: 1 degree > 4, 2 edges overflow, 4 bad action
};

size_t cov_step_lds_bytes(int R, int M);
hipError_t launch_cov_graph(const CovArgs& a, const int32_t* envs, int n, hipStream_t s);
hipError_t launch_cov_reset(const CovArgs& a, const int32_t* start, const uint8_t* visited0, hipStream_t s);
hipError_t launch_cov_step(const CovArgs& a, hipStream_t s);

}  // namespace gf
