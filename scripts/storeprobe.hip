// Store-order probe for the dense network write (diagnostic only). Same row-block shape
// as storebench8k.hip (R rows per workgroup, wave w writes rows [w R/4, (w+1) R/4), 16-byte
// lane stores, XCD-grouped), with the column order of each row varied:
//   order 0: columns from 0 (the step kernel's order)
//   order 1: each row starts at a per-workgroup rotated 1 KiB column block and wraps
//   order 2: column-block-major over the wave's rows (all its rows' block c, then c + 1)
//   order 3: rotated start per row (row index * 5 blocks)
// and a plain grid-stride linear fill as the reference. Sizes: 32 x 8192^2 (8 GiB,
// config 5), 4 x 8192^2 (1 GiB, config-5 rows), 256 x 1024^2 (1 GiB, config 2).
// Build: hipcc -O3 --offload-arch=gfx950 storeprobe.hip -o /tmp/storeprobe
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

__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int xcd = bid & 7, q = G >> 3, r = G & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ f4v val(int q, float iv) {
  const unsigned h = (unsigned)q * 2654435761u;
  return f4v{(h & 1u) ? iv : 0.f, (h & 2u) ? iv : 0.f, (h & 4u) ? iv : 0.f, (h & 8u) ? iv : 0.f};
}

template <int R, int ORDER>
__global__ __launch_bounds__(256) void blocks(f4v* net, int Q) {
  extern __shared__ unsigned char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  if (lane == 0 && wid == 0) lds[0] = 1;
  const size_t row0 = (size_t)L * R + wid * (R / 4);
  const int nb = Q / 64;  // 1 KiB column blocks per row
  if (ORDER == 2) {
    for (int c = 0; c < nb; ++c)
      for (int m = 0; m < R / 4; ++m) {
        f4v* rowp = net + (row0 + m) * Q;
        rowp[c * 64 + lane] = val(c * 64 + lane, 1.0f / (float)(m + 1));
      }
    return;
  }
  for (int m = 0; m < R / 4; ++m) {
    f4v* rowp = net + (row0 + m) * Q;
    const float iv = 1.0f / (float)(m + 1);
    const int s = ORDER == 1 ? (L * 7) % nb : ORDER == 3 ? (int)(((row0 + m) * 5) % nb) : 0;
    for (int k = 0; k < nb; ++k) {
      int c = s + k;
      if (c >= nb) c -= nb;
      const int q = c * 64 + lane;
      rowp[q] = val(q, iv);
    }
  }
}

__global__ __launch_bounds__(256) void linear(f4v* p, size_t n4) {
  for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n4; k += (size_t)gridDim.x * 256)
    p[k] = val((int)k, 0.5f);
}

template <int R, int ORDER>
float run(f4v* net, int rows, int Q, int lds) {
  const int grid = rows / R;
  CK(hipFuncSetAttribute((const void*)&blocks<R, ORDER>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((blocks<R, ORDER>), dim3(grid), dim3(256), lds, 0, net, Q);
  CK(hipEventRecord(e0, 0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((blocks<R, ORDER>), dim3(grid), dim3(256), lds, 0, net, Q);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3f * ms / reps;
}

float run_linear(f4v* p, size_t bytes, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(linear, dim3(grid), dim3(256), 0, 0, p, bytes / 16);
  CK(hipEventRecord(e0, 0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(linear, dim3(grid), dim3(256), 0, 0, p, bytes / 16);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3f * ms / reps;
}

template <int R>
void shape(const char* name, f4v* net, int rows, int N, int lds) {
  const int Q = N / 4;
  const double bytes = (double)rows * N * 4;
  const float t0 = run<R, 0>(net, rows, Q, lds), t1 = run<R, 1>(net, rows, Q, lds);
  const float t2 = run<R, 2>(net, rows, Q, lds), t3 = run<R, 3>(net, rows, Q, lds);
  printf("%-22s R=%2d lds %6d: cols-from-0 %8.1f us (%.2f TB/s)  wg-rotated %8.1f (%.2f)  block-major %8.1f (%.2f)  row-rotated %8.1f (%.2f)\n",
         name, R, lds, t0, bytes / (t0 * 1e-6) / 1e12, t1, bytes / (t1 * 1e-6) / 1e12, t2,
         bytes / (t2 * 1e-6) / 1e12, t3, bytes / (t3 * 1e-6) / 1e12);
  fflush(stdout);
}

int main(int argc, char** argv) {
  f4v* net;
  const size_t big = (size_t)32 * 8192 * 8192 * 4;
  if (argc > 1 && argv[1][0] == 'c') {  // physically contiguous allocation
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&net), big, hipDeviceMallocContiguous));
    printf("allocation: hipExtMallocWithFlags(hipDeviceMallocContiguous)\n");
    if (argc > 2) {  // config-5 shapes only
      shape<16>("8GiB N=8192 (cfg5)", net, 32 * 8192, 8192, 37376);
      CK(hipFree(net));
      return 0;
    }
  } else {
    CK(hipMalloc(&net, big));
    printf("allocation: hipMalloc\n");
    if (argc > 2) {
      shape<16>("8GiB N=8192 (cfg5)", net, 32 * 8192, 8192, 37376);
      CK(hipFree(net));
      return 0;
    }
  }
  for (int g : {2048, 8192, 32768}) {
    const float t8 = run_linear(net, big, g), t1 = run_linear(net, big / 8, g);
    printf("linear grid %5d: 8 GiB %8.1f us (%.2f TB/s)  1 GiB %8.1f us (%.2f TB/s)\n", g, t8,
           big / (t8 * 1e-6) / 1e12, t1, big / 8 / (t1 * 1e-6) / 1e12);
  }
  fflush(stdout);
  shape<16>("8GiB N=8192 (cfg5)", net, 32 * 8192, 8192, 37376);
  shape<8>("8GiB N=8192 (cfg5)", net, 32 * 8192, 8192, 37376);
  shape<16>("1GiB N=8192", net, 4 * 8192, 8192, 37376);
  shape<16>("1GiB N=1024 (cfg2)", net, 256 * 1024, 1024, 24576);
  shape<16>("8GiB N=1024", net, 2048 * 1024, 1024, 24576);
  CK(hipFree(net));
  return 0;
}
