// Completion flag of a drop-in launch (fe_step_host*, cov_step_host), which writes every
// output straight into page-locked host memory: the launch's last workgroup to finish
// stores a sequence number into a page-locked host word with a system-scope release,
// after every workgroup has made its own results visible system-wide, and the host polls
// that word instead of the stream. The stream's completion reaches a polling host ~8 us
// after the kernel's last store (scripts/flagprobe.hip: 21.2 us per launch round trip
// waiting for the stream, 13.1 us waiting for the flag).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>

namespace gf {

struct DoneFlag {
  int32_t* cnt;   // device word, 0 between launches: workgroups finished
  int32_t* host;  // mapped address of the page-locked word, or nullptr: no flag
  int32_t seq;    // value stored when the whole grid is done
  int32_t fence;  // host == nullptr: still make this launch's results visible system-wide
                  // before it ends (a later launch of the same call carries the flag)
};

// Every thread of every workgroup calls it as its last action (uniform branch).
__device__ __forceinline__ void signal_done(const DoneFlag& f) {
  if (!f.host && !f.fence) return;
  __threadfence_system();  // this thread's results, system-wide, before the count
  if (!f.host) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nb = static_cast<int>(gridDim.x * gridDim.y * gridDim.z);
    const int old = __hip_atomic_fetch_add(f.cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old == nb - 1) {
      __hip_atomic_store(f.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
      __hip_atomic_store(f.host, f.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Host: wait for the flag to read seq. Every ~50 us the stream is queried for a launch
// error; a stream that completed without the flag is an error too (hipErrorUnknown).
inline hipError_t wait_done(const int32_t* flag, int32_t seq, hipStream_t s) {
  using clk = std::chrono::steady_clock;
  auto next = clk::now() + std::chrono::microseconds(50);
  for (unsigned k = 1;; ++k) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return hipSuccess;
    if ((k & 63) == 0 && clk::now() >= next) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq ? hipSuccess : hipErrorUnknown;
      if (q != hipErrorNotReady) return q;
      next = clk::now() + std::chrono::microseconds(50);
    }
  }
}

}  // namespace gf
