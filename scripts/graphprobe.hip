// Host cost of issuing a two-half step (diagnostic only): two kernels on two streams per
// iteration, (a) as two hipLaunchKernelGGL calls, (b) as one hipGraphLaunch of a captured
// fork/join graph holding both, (c) as two hipExtLaunchKernelGGL calls. Prints the host
// time to enqueue an iteration and the wall time per iteration, for kernels whose
// workgroups spin 0 or 3 us.
// Build: hipcc -O3 --offload-arch=gfx950 graphprobe.hip -o /tmp/graphprobe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int NP>
struct Big {  // kernel arguments of 8 NP + 8 bytes (NP = 32: about the Coverage step's)
  void* p[NP];
  int spin;
};

template <int NP>
__global__ void touch(Big<NP> a) {
  if (threadIdx.x == 0) {
    long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < a.spin) {
    }
    static_cast<int*>(a.p[0])[blockIdx.x] = blockIdx.x;
  }
}

using clk = std::chrono::steady_clock;

template <int NP>
void sweep(int* p, hipStream_t s1, hipStream_t s2, int spin) {
  Big<NP> a{};
  a.p[0] = p;
  a.spin = spin;
  const int K = 2000, G = 256;
  auto issue = [&] {
    hipLaunchKernelGGL(touch<NP>, dim3(G), dim3(256), 0, s1, a);
    hipLaunchKernelGGL(touch<NP>, dim3(G), dim3(256), 0, s2, a);
  };
  for (int k = 0; k < 50; ++k) issue();
  CK(hipDeviceSynchronize());
  auto t0 = clk::now();
  for (int k = 0; k < K; ++k) issue();
  auto t1 = clk::now();
  CK(hipDeviceSynchronize());
  auto t2 = clk::now();
  printf("args %4d B  spin %3d  2 x hipLaunchKernel: enqueue %6.2f us/iter  wall %6.2f us/iter\n", (int)sizeof(a), spin,
         std::chrono::duration<double, std::micro>(t1 - t0).count() / K,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / K);
  fflush(stdout);
}

// two launches per iteration through each C launch API, arguments of 264 bytes
void api_sweep(int* p, hipStream_t s1, hipStream_t s2, int spin) {
  Big<32> a{};
  a.p[0] = p;
  a.spin = spin;
  hipFunction_t f;
  CK(hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&touch<32>)));
  void* args[] = {&a};
  const int K = 2000, G = 256;
  for (int mode = 0; mode < 3; ++mode) {
    auto issue = [&] {
      for (hipStream_t s : {s1, s2}) {
        if (mode == 0)
          hipLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, s, a);
        else if (mode == 1)
          CK(hipLaunchKernel(reinterpret_cast<const void*>(&touch<32>), dim3(G), dim3(256), args, 0, s));
        else
          CK(hipModuleLaunchKernel(f, G, 1, 1, 256, 1, 1, 0, s, args, nullptr));
      }
    };
    for (int k = 0; k < 50; ++k) issue();
    CK(hipDeviceSynchronize());
    auto t0 = clk::now();
    for (int k = 0; k < K; ++k) issue();
    auto t1 = clk::now();
    CK(hipDeviceSynchronize());
    auto t2 = clk::now();
    printf("spin %3d  %-28s enqueue %6.2f us/iter  wall %6.2f us/iter\n", spin,
           mode == 0 ? "2 x hipLaunchKernelGGL" : mode == 1 ? "2 x hipLaunchKernel" : "2 x hipModuleLaunchKernel",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / K,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / K);
    fflush(stdout);
  }
}

int main() {
  int* p;
  CK(hipMalloc(&p, 1 << 20));
  hipStream_t s1, s2, cs;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  for (int rep = 0; rep < 3; ++rep)
    for (int spin : {0, 100}) api_sweep(p, s1, s2, spin);
  if (getenv("API_ONLY")) return 0;
  for (int rep = 0; rep < 2; ++rep)
    for (int spin : {0, 100}) {
      sweep<32>(p, s1, s2, spin);
      sweep<1>(p, s1, s2, spin);
      sweep<15>(p, s1, s2, spin);
      sweep<7>(p, s1, s2, spin);
      sweep<32>(p, s1, s2, spin);
      sweep<1>(p, s1, s2, spin);
    }
  const int K = 2000, G = 256;
  for (int spin : {0, 300}) {
    Big<32> a{};
    a.p[0] = p;
    a.spin = spin;
    // (a) two launches per iteration
    for (int mode = 0; mode < 3; ++mode) {
      hipGraphExec_t ge = nullptr;
      if (mode == 1) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        CK(hipEventRecord(fork, cs));
        CK(hipStreamWaitEvent(s2, fork, 0));
        hipLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, cs, a);
        hipLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, s2, a);
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(cs, join, 0));
        CK(hipStreamEndCapture(cs, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      }
      auto issue = [&] {
        if (mode == 0) {
          hipLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, s1, a);
          hipLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, s2, a);
        } else if (mode == 1) {
          CK(hipGraphLaunch(ge, cs));
        } else {
          hipExtLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, s1, nullptr, nullptr, 0, a);
          hipExtLaunchKernelGGL(touch<32>, dim3(G), dim3(256), 0, s2, nullptr, nullptr, 0, a);
        }
      };
      for (int k = 0; k < 50; ++k) issue();
      CK(hipDeviceSynchronize());
      auto t0 = clk::now();
      for (int k = 0; k < K; ++k) issue();
      auto t1 = clk::now();
      CK(hipDeviceSynchronize());
      auto t2 = clk::now();
      const double enq = std::chrono::duration<double, std::micro>(t1 - t0).count() / K;
      const double wall = std::chrono::duration<double, std::micro>(t2 - t0).count() / K;
      printf("spin %3d  %-22s enqueue %6.2f us/iter  wall %6.2f us/iter\n", spin,
             mode == 0 ? "2 x hipLaunchKernel" : mode == 1 ? "1 x hipGraphLaunch" : "2 x hipExtLaunchKernel", enq,
             wall);
      fflush(stdout);
    }
  }
  return 0;
}
