// Back-to-back launch period on one stream (diagnostic only): K launches of a kernel that
// does nothing but (optionally) store one word per workgroup, for several grid / block
// shapes, on one stream and alternating between two streams; prints us per launch.
// Build: hipcc -O3 --offload-arch=gfx950 launchgap.hip -o /tmp/launchgap
#include <hip/hip_runtime.h>

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

__global__ void touch(int* p, int spin) {
  if (threadIdx.x == 0) {
    long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
    }
    p[blockIdx.x] = blockIdx.x;
  }
}

float period(int grid, int block, int nstreams, int spin, hipStream_t* s, int* p) {
  const int K = 2000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int k = 0; k < 50; ++k) hipLaunchKernelGGL(touch, dim3(grid), dim3(block), 0, s[k % nstreams], p, spin);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, s[0]));
  for (int k = 1; k < nstreams; ++k) CK(hipStreamWaitEvent(s[k], e0, 0));
  for (int k = 0; k < K; ++k) hipLaunchKernelGGL(touch, dim3(grid), dim3(block), 0, s[k % nstreams], p, spin);
  hipEvent_t ej[4];
  for (int k = 1; k < nstreams; ++k) {
    CK(hipEventCreate(&ej[k]));
    CK(hipEventRecord(ej[k], s[k]));
    CK(hipStreamWaitEvent(s[0], ej[k], 0));
  }
  CK(hipEventRecord(e1, s[0]));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3f * ms / K;
}

int main() {
  int* p;
  CK(hipMalloc(&p, 1 << 20));
  hipStream_t s[4];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  for (int spin : {0, 200, 500}) {  // 100 MHz ticks: 0, 2, 5 us per workgroup
    for (int grid : {1, 256, 512}) {
      for (int block : {64, 256}) {
        printf("spin %3d  grid %4d  block %3d:  1 stream %6.2f us/launch  2 streams %6.2f  4 streams %6.2f\n", spin,
               grid, block, period(grid, block, 1, spin, s, p), period(grid, block, 2, spin, s, p),
               period(grid, block, 4, spin, s, p));
        fflush(stdout);
      }
    }
  }
  return 0;
}
