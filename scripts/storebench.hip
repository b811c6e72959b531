// Store-pattern sweep for the step kernel's dense network write (diagnostic only).
// 256 envs x 1024 rows x 1024 float32 = 1 GiB, written as 16-byte lane stores.
// Every variant writes the same bytes; only which workgroup/wave writes which row, in
// what order, and how many workgroups are resident per CU, change.
// Build: hipcc -O3 --offload-arch=gfx950 storebench.hip -o /tmp/storebench
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

constexpr int N = 1024, B = 256, R = 32, BPE = N / R;  // rows, envs, rows per block
constexpr int Q = N / 4;                                 // float4 per row

__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int xcd = bid & 7, q = G >> 3, r = G & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <bool NT>
__device__ __forceinline__ void st(f4v* p, f4v v) {
  if (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

// one row (4 KiB) by one wave: 4 x 1 KiB instructions
template <bool NT>
__device__ __forceinline__ void row_store(f4v* rowp, int lane, float iv) {
#pragma unroll
  for (int q = lane; q < Q; q += 64) {
    const unsigned m = (unsigned)q * 2654435761u;
    st<NT>(&rowp[q], f4v{(m & 1u) ? iv : 0.f, (m & 2u) ? iv : 0.f, (m & 4u) ? iv : 0.f, (m & 8u) ? iv : 0.f});
  }
}

// MODE 0: current kernel (contiguous 32-row block, wave w rows [8w, 8w+8), remapped)
// MODE 1: block rb of an env owns rows rb + 32k (strided across the env's blocks)
// MODE 2: current, plain blockIdx order (no XCD remap)
// MODE 3: strided, no remap
// MODE 4: current but wave w rows w, w+4, ... (interleaved waves)
template <int MODE, bool NT>
__global__ __launch_bounds__(256) void blocks(f4v* net) {
  extern __shared__ unsigned char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = (MODE == 2 || MODE == 3) ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int b = L / BPE, rb = L % BPE;
  if (lane == 0 && wid == 0) lds[0] = 1;  // occupancy set by the dynamic LDS size
  for (int m = 0; m < R / 4; ++m) {
    const int k = (MODE == 4) ? wid + 4 * m : wid * (R / 4) + m;
    const int row = (MODE == 1 || MODE == 3) ? rb + BPE * k : rb * R + k;
    row_store<NT>(net + ((size_t)b * N + row) * Q, lane, 0.25f);
  }
}

// persistent: G workgroups loop over the 8192 (env, row block) units, in unit order
// u = blockIdx + G*t (a unit is the current 32-row contiguous block); WAVEROW: each
// wave sweeps its own rows
template <bool NT>
__global__ __launch_bounds__(256) void persistent(f4v* net) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int u = blockIdx.x; u < B * BPE; u += gridDim.x) {
    const int b = u / BPE, rb = u % BPE;
    for (int m = 0; m < R / 4; ++m) {
      const int row = rb * R + wid * (R / 4) + m;
      row_store<NT>(net + ((size_t)b * N + row) * Q, lane, 0.25f);
    }
  }
}

// persistent, XCD-aware: the workgroups of XCD x (blockIdx % 8 == x under round-robin
// dispatch) walk the contiguous unit range [x*U/8, (x+1)*U/8) in order, each taking
// every (G/8)-th unit
template <bool NT>
__global__ __launch_bounds__(256) void persistent_xcd(f4v* net) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int U = B * BPE, per_xcd = U / 8, gx = gridDim.x / 8;
  const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
  for (int t = k; t < per_xcd; t += gx) {
    const int u = x * per_xcd + t;
    const int b = u / BPE, rb = u % BPE;
    for (int m = 0; m < R / 4; ++m) {
      const int row = rb * R + wid * (R / 4) + m;
      row_store<NT>(net + ((size_t)b * N + row) * Q, lane, 0.25f);
    }
  }
}

// one-shot grid (current mapping) with a dependent global round trip and a spin of
// DELAY cycles before the stores: the latency a step-kernel workgroup spends first
template <int DELAY>
__global__ __launch_bounds__(256) void delayed(f4v* net, const float* src) {
  extern __shared__ unsigned char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int b = L / BPE, rb = L % BPE;
  float iv = src[(L * 64 + threadIdx.x) & 0xFFFF] + 0.25f;  // a load the stores depend on
  if (DELAY) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < DELAY) __builtin_amdgcn_s_sleep(1);
  }
  if (lane == 0 && wid == 0) lds[0] = 1;
  for (int m = 0; m < R / 4; ++m) {
    const int row = rb * R + wid * (R / 4) + m;
    row_store<false>(net + ((size_t)b * N + row) * Q, lane, iv);
  }
}

// env-resident pipelined shape: G workgroups (XCD-remapped), SPE per env; slice s of
// env e writes its env's 32-row blocks s, s+SPE, ... (STRIDED) or a contiguous run
template <bool STRIDED>
__global__ __launch_bounds__(256) void resident(f4v* net, int spe) {
  extern __shared__ unsigned char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int e = L / spe, sl = L % spe;
  if (lane == 0 && wid == 0) lds[0] = 1;
  const int per = (BPE + spe - 1) / spe;
  for (int t = 0; t < per; ++t) {
    const int rb = STRIDED ? sl + spe * t : sl * per + t;
    if (rb >= BPE || (!STRIDED && t >= per)) break;
    for (int m = 0; m < R / 4; ++m) {
      const int row = rb * R + wid * (R / 4) + m;
      row_store<false>(net + ((size_t)e * N + row) * Q, lane, 0.25f);
    }
  }
}

// grid-stride fill of the whole buffer (reference point)
template <bool NT>
__global__ __launch_bounds__(256) void fill(f4v* p, size_t n4) {
  for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n4; k += (size_t)gridDim.x * 256) {
    const unsigned m = (unsigned)k * 2654435761u;
    st<NT>(&p[k], f4v{(m & 1u) ? 0.25f : 0.f, (m & 2u) ? 0.25f : 0.f, (m & 4u) ? 0.25f : 0.f, 0.f});
  }
}

int main() {
  const size_t bytes = (size_t)B * N * N * 4, n4 = bytes / 16;
  f4v* a;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int G = B * BPE;
  struct V {
    const char* name;
    int kind;
  };
  auto run = [&](const char* name, auto launch) {
    float best = 1e9, sum = 0;
    for (int rep = 0; rep < 3; ++rep) {
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 10;
      sum += ms;
      if (ms < best) best = ms;
    }
    printf("%-34s best %7.1f us  avg %7.1f us  %6.0f GB/s\n", name, best * 1e3, sum / 3 * 1e3,
           bytes / (best * 1e-3) / 1e9);
  };
  for (int lds : {26 * 1024}) {
    char nm[96];
#define RUNB(MODE, NT, label)                                                             \
  snprintf(nm, sizeof nm, "%s lds%dK", label, lds / 1024);                                \
  run(nm, [&]() { blocks<MODE, NT><<<G, 256, lds>>>(a); });
    RUNB(0, false, "current");
    RUNB(0, true, "current nt");
    RUNB(1, false, "strided rows");
    RUNB(1, true, "strided rows nt");
    RUNB(2, false, "current no-remap");
    RUNB(3, false, "strided no-remap");
    RUNB(4, false, "interleaved waves");
  }
  for (int g : {1024}) {
    char nm[96];
    snprintf(nm, sizeof nm, "persistent G=%d", g);
    run(nm, [&]() { persistent<false><<<g, 256>>>(a); });
    snprintf(nm, sizeof nm, "persistent nt G=%d", g);
    run(nm, [&]() { persistent<true><<<g, 256>>>(a); });
  }
  for (int g : {1024, 1536, 2048}) {
    char nm[96];
    snprintf(nm, sizeof nm, "persistent xcd G=%d", g);
    run(nm, [&]() { persistent_xcd<false><<<g, 256>>>(a); });
  }
  for (int spe : {2, 3, 4}) {
    for (int lds : {40 * 1024, 60 * 1024}) {
      char nm[96];
      const int g = B * spe;
      snprintf(nm, sizeof nm, "resident strided spe%d lds%dK", spe, lds / 1024);
      run(nm, [&]() { resident<true><<<g, 256, lds>>>(a, spe); });
      snprintf(nm, sizeof nm, "resident contig spe%d lds%dK", spe, lds / 1024);
      run(nm, [&]() { resident<false><<<g, 256, lds>>>(a, spe); });
    }
  }
  float* src;
  CK(hipMalloc(&src, 65536 * 4));
  CK(hipMemset(src, 0, 65536 * 4));
  for (int lds : {26 * 1024, 20 * 1024}) {
    char nm[96];
#define RUND(D)                                                                \
  snprintf(nm, sizeof nm, "delayed %d cyc lds%dK", D, lds / 1024);             \
  run(nm, [&]() { delayed<D><<<G, 256, lds>>>(a, src); });
    RUND(0) RUND(10000)
  }
  for (int g : {1024, 4096, 16384}) {
    char nm[96];
    snprintf(nm, sizeof nm, "fill G=%d", g);
    run(nm, [&]() { fill<false><<<g, 256>>>(a, n4); });
    snprintf(nm, sizeof nm, "fill nt G=%d", g);
    run(nm, [&]() { fill<true><<<g, 256>>>(a, n4); });
  }
  return 0;
}
