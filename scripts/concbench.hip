// Fused vs split-and-concurrent (diagnostic only): does a compute phase placed in
// front of each workgroup's network stores cost the store stream more than the same
// compute run as its own kernel beside a store-only kernel on a second stream?
// 8192 workgroups x 128 KiB of stores (the step kernel's 32-row blocks, XCD grouped),
// a synthetic VALU-heavy compute phase of ITERS rounds per workgroup.
// Build: hipcc -O3 --offload-arch=gfx950 concbench.hip -o build/concbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);     \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int N = 1024, B = 256, R = 32, BPE = N / R, Q = N / 4;

__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int xcd = bid & 7, q = G >> 3, r = G & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// VALU-heavy phase: 8 independent fma chains, ITERS rounds, a little LDS traffic
__device__ __forceinline__ float compute_phase(int iters, float seed, float* lds) {
  float c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = seed + k;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = c[k] * 0.999f + 0.001f;
    if ((it & 15) == 0) {
      lds[threadIdx.x] = c[it & 7];
      __syncthreads();
      c[0] += lds[(threadIdx.x + 64) & 255];
    }
  }
  return ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
}

__device__ __forceinline__ void store_block(f4v* net, int L, float iv) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = L / BPE, rb = L % BPE;
  for (int m = 0; m < R / 4; ++m) {
    const int row = rb * R + wid * (R / 4) + m;
    f4v* rowp = net + ((size_t)b * N + row) * Q;
#pragma unroll
    for (int q = lane; q < Q; q += 64) {
      const unsigned h = (unsigned)q * 2654435761u;
      rowp[q] = f4v{(h & 1u) ? iv : 0.f, (h & 2u) ? iv : 0.f, (h & 4u) ? iv : 0.f, (h & 8u) ? iv : 0.f};
    }
  }
}

// compute only (writes one float per thread)
__global__ __launch_bounds__(256) void comp(const float* src, float* out, int iters) {
  extern __shared__ float lds[];
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const float s = src[(L * 256 + threadIdx.x) & 0xFFFF];
  out[(size_t)L * 256 + threadIdx.x] = compute_phase(iters, s, lds);
}

// store only: one dependent load (the 4 KiB of bits a real expand kernel reads), stores
__global__ __launch_bounds__(256) void expand(f4v* net, const float* src) {
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const float iv = src[(L * 256 + threadIdx.x) & 0xFFFF] + 0.25f;
  store_block(net, L, iv);
}

// fused: load, compute, stores
__global__ __launch_bounds__(256) void fused(f4v* net, const float* src, float* out, int iters) {
  extern __shared__ float lds[];
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const float s = src[(L * 256 + threadIdx.x) & 0xFFFF];
  const float v = compute_phase(iters, s, lds);
  store_block(net, L, 0.25f + (v == 12345.f ? 1.f : 0.f));
  out[(size_t)L * 256 + threadIdx.x] = v;
}

int main() {
  const size_t bytes = (size_t)B * N * N * 4;
  const int G = B * BPE;
  f4v* net;
  float *src, *out;
  CK(hipMalloc(&net, bytes));
  CK(hipMalloc(&src, 65536 * 4));
  CK(hipMalloc(&out, (size_t)G * 256 * 4));
  CK(hipMemset(src, 0, 65536 * 4));
  CK(hipMemset(net, 0, bytes));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1, ea, eb;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));
  const size_t lds = 26 * 1024;  // 6 workgroups per CU, like the step kernel
  auto timeit = [&](const char* name, auto body) {
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      body();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sa));
      CK(hipStreamWaitEvent(sb, e0, 0));
      for (int r = 0; r < 10; ++r) body();
      CK(hipEventRecord(eb, sb));
      CK(hipStreamWaitEvent(sa, eb, 0));
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms / 10 < best) best = ms / 10;
    }
    printf("%-40s %8.1f us per step\n", name, best * 1e3);
  };
  for (int iters : {0, 200, 400, 800}) {
    char nm[96];
    snprintf(nm, sizeof nm, "compute only, iters %d", iters);
    timeit(nm, [&]() { comp<<<G, 256, lds, sa>>>(src, out, iters); });
    snprintf(nm, sizeof nm, "fused, iters %d", iters);
    timeit(nm, [&]() { fused<<<G, 256, lds, sa>>>(net, src, out, iters); });
    snprintf(nm, sizeof nm, "compute || expand (2 streams), iters %d", iters);
    timeit(nm, [&]() {
      comp<<<G, 256, lds, sa>>>(src, out, iters);
      expand<<<G, 256, 0, sb>>>(net, src);
    });
    snprintf(nm, sizeof nm, "compute then expand (1 stream), iters %d", iters);
    timeit(nm, [&]() {
      comp<<<G, 256, lds, sa>>>(src, out, iters);
      expand<<<G, 256, 0, sa>>>(net, src);
    });
  }
  timeit("expand only", [&]() { expand<<<G, 256, 0, sb>>>(net, src); });
  return 0;
}
