// Store-pattern probe for config 5's dense network write (diagnostic only): 32 envs x
// 8192 rows x 8192 float32 = 8 GiB as 16-byte lane stores, in row blocks of R rows (wave
// w writes rows [w R/4, (w+1) R/4)), XCD-grouped like the step kernel; the dynamic LDS
// size sets the resident workgroups per CU. Prints us per 8 GiB and TB/s.
// Build: hipcc -O3 --offload-arch=gfx950 storebench8k.hip -o /tmp/storebench8k
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));
#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int N = 8192, B = 32, Q = N / 4;

__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int xcd = bid & 7, q = G >> 3, r = G & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <int R, bool NT>
__global__ __launch_bounds__(256) void blocks(f4v* net) {
  extern __shared__ unsigned char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  if (lane == 0 && wid == 0) lds[0] = 1;
  const size_t row0 = (size_t)L * R;
  for (int m = 0; m < R / 4; ++m) {
    f4v* rowp = net + (row0 + wid * (R / 4) + m) * Q;
    const float iv = 1.0f / (float)(m + 1);
    for (int q = lane; q < Q; q += 64) {
      const unsigned h = (unsigned)q * 2654435761u;
      const f4v v{(h & 1u) ? iv : 0.f, (h & 2u) ? iv : 0.f, (h & 4u) ? iv : 0.f, (h & 8u) ? iv : 0.f};
      if (NT) __builtin_nontemporal_store(v, &rowp[q]); else rowp[q] = v;
    }
  }
}

template <int R, bool NT>
float run(f4v* net, int lds) {
  const int grid = B * N / R;
  CK(hipFuncSetAttribute((const void*)&blocks<R, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((blocks<R, NT>), dim3(grid), dim3(256), lds, 0, net);
  CK(hipEventRecord(e0, 0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((blocks<R, NT>), dim3(grid), dim3(256), lds, 0, net);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3f * ms / reps;
}

int main() {
  f4v* net;
  const size_t bytes = (size_t)B * N * N * 4;
  CK(hipMalloc(&net, bytes));
  const int ldss[] = {37376, 26624, 20480, 16384, 1024};  // 4, 6, 7, 8, >8 per CU
  for (int l : ldss) {
    float t16 = run<16, false>(net, l), t8 = run<8, false>(net, l), t32 = run<32, false>(net, l);
    float t16n = run<16, true>(net, l);
    printf("lds %6d B: R=16 %8.1f us (%.2f TB/s)  R=8 %8.1f  R=32 %8.1f  R=16 nt %8.1f\n", l, t16,
           bytes / (t16 * 1e-6) / 1e12, t8, t32, t16n);
  }
  CK(hipFree(net));
  return 0;
}
