// Launch-to-host round trip of a one-workgroup kernel (the drop-in step's shape): how the
// host learns that the kernel is done.
//   query: launch, then poll hipStreamQuery until the stream is idle (the library's wait)
//   flag:  launch, then poll a page-locked word the kernel's last wave stores with system
//          scope release after its results (the kernel announces itself)
//   flag+query: the flag, then the stream's completion (how much later the CP signals)
// hipcc -O3 --offload-arch=gfx950 scripts/flagprobe.hip -o /tmp/flagprobe && /tmp/flagprobe
#include <hip/hip_runtime.h>

#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__global__ __launch_bounds__(256) void work(float* out, float* hout, int n, int* hflag, int seq) {
  // a little work and a host-bound result, like the drop-in step's outputs
  for (int k = threadIdx.x; k < n; k += 256) {
    const float v = out[k] * 1.0001f + 1.0f;
    out[k] = v;
    hout[k] = v;
  }
  if (hflag) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();
      __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

int main() {
  const int n = 100 * 106;  // ~ a 100-agent env's outputs (state values + network)
  float* d;
  float* h;
  float* hd;
  int* flag;
  int* flagd;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemset(d, 0, n * 4));
  CK(hipHostMalloc(reinterpret_cast<void**>(&h), n * 4, hipHostMallocMapped));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), h, 0));
  CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocMapped));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&flagd), flag, 0));
  *flag = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());
  using clk = std::chrono::steady_clock;
  const int iters = 3000;
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      int seq = 0;
      double lag = 0.0;
      const auto t0 = clk::now();
      for (int it = 0; it < iters; ++it) {
        ++seq;
        hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, d, hd, n, mode ? flagd : nullptr, seq);
        if (mode == 0) {
          while (hipStreamQuery(s) == hipErrorNotReady) {
          }
        } else {
          const auto w0 = clk::now();
          while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
            if (std::chrono::duration<double>(clk::now() - w0).count() > 2.0) {
              std::fprintf(stderr, "flag never arrived\n");
              return 1;
            }
          }
          if (mode == 2) {
            const auto f = clk::now();
            while (hipStreamQuery(s) == hipErrorNotReady) {
            }
            lag += std::chrono::duration<double>(clk::now() - f).count();
          }
        }
      }
      CK(hipStreamSynchronize(s));
      const double us = 1e6 * std::chrono::duration<double>(clk::now() - t0).count() / iters;
      std::printf("%-11s rep %d: %.2f us per launch round trip%s", mode == 0 ? "query" : mode == 1 ? "flag" : "flag+query",
                  rep, us, mode == 2 ? "" : "\n");
      if (mode == 2) std::printf(" (completion %.2f us after the flag)\n", 1e6 * lag / iters);
    }
  }
  // host cost of an enqueue alone: back-to-back launches, one wait at the end
  for (int rep = 0; rep < 2; ++rep) {
    const auto t0 = clk::now();
    for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, d, hd, 64, nullptr, 0);
    const double enq = 1e6 * std::chrono::duration<double>(clk::now() - t0).count() / iters;
    CK(hipStreamSynchronize(s));
    const double all = 1e6 * std::chrono::duration<double>(clk::now() - t0).count() / iters;
    std::printf("enqueue     rep %d: %.2f us host per launch, %.2f us per launch with the drain\n", rep, enq, all);
  }
  // two streams: one thread enqueueing to both alternately, then two threads, one per stream
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = clk::now();
    for (int it = 0; it < iters; ++it) {
      hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, d, hd, 64, nullptr, 0);
      hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s2, d + 64, hd + 64, 64, nullptr, 0);
    }
    const double one = 1e6 * std::chrono::duration<double>(clk::now() - t0).count() / iters;
    CK(hipDeviceSynchronize());
    t0 = clk::now();
    std::thread other([&] {
      for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s2, d + 64, hd + 64, 64, nullptr, 0);
    });
    for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, d, hd, 64, nullptr, 0);
    other.join();
    const double two = 1e6 * std::chrono::duration<double>(clk::now() - t0).count() / iters;
    CK(hipDeviceSynchronize());
    std::printf("2 streams   rep %d: %.2f us host per launch pair from one thread, %.2f us from two threads\n", rep,
                one, two);
  }
  return 0;
}
