// Write/read/copy bandwidth ceilings on MI355X for the network-buffer shape
// (contiguous float32, 16 B per lane). Diagnostic only: the roofline context for the
// step kernel's dense network write. Build: hipcc -O3 --offload-arch=gfx950 membw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

// mode: 0 plain grid-stride, 1 nt grid-stride, 2 plain unroll4 (4 KiB per wave per iter),
// 3 nt unroll4, 4 block-contiguous chunks (each block owns a contiguous range)
template <int MODE>
__global__ __launch_bounds__(256) void fill(f4v* p, size_t n4) {
  const f4v v{1.0f, 0.0f, 0.5f, 0.0f};
  if (MODE <= 1) {
    for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n4; k += (size_t)gridDim.x * 256) {
      if (MODE == 1) __builtin_nontemporal_store(v, &p[k]); else p[k] = v;
    }
  } else if (MODE <= 3) {
    const size_t stride = (size_t)gridDim.x * 1024;
    for (size_t k = blockIdx.x * 1024ull + threadIdx.x; k < n4; k += stride) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t q = k + u * 256;
        if (q < n4) {
          if (MODE == 3) __builtin_nontemporal_store(v, &p[q]); else p[q] = v;
        }
      }
    }
  } else {
    const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const size_t b = blockIdx.x * per, e = b + per < n4 ? b + per : n4;
    for (size_t k = b + threadIdx.x; k < e; k += 256) p[k] = v;
  }
}

// The step kernel's network-store shape: block b owns rows [64b, 64b+64) of N=1024 floats
// (one contiguous 256 KiB range); wave w writes rows w, w+4, ... as 4 x 1 KiB
// instructions per row. DELAY: cycles of s_sleep before storing (startup latency).
template <int DELAY, bool NT>
__global__ __launch_bounds__(256) void fill_rows(f4v* p, size_t n4) {
  if (DELAY) {
    for (int k = 0; k < DELAY / 64; ++k) __builtin_amdgcn_s_sleep(1);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const f4v v{1.0f, 0.0f, 0.5f, 0.0f};
  f4v* base = p + (size_t)blockIdx.x * 64 * 256;
  for (int r = wid; r < 64; r += 4)
    for (int q = lane; q < 256; q += 64) {
      if (NT) __builtin_nontemporal_store(v, &base[r * 256 + q]); else base[r * 256 + q] = v;
    }
}

// The tiled step kernel's shape (32 rows x N=1024 per block, 8192 blocks per GiB) with
// one of its side costs added, to find what slows its store stream:
// V=0 plain, 1 +26 KB LDS (occupancy), 2 +40 KB L2-resident reads per block (the env
// tile), 3 +scattered per-row small writes (state_values / x), 4 values built from LDS
// bits, 5 = 2+3+4.
template <int V>
__global__ __launch_bounds__(256) void rows32(f4v* p, const f4v* src, float* small, size_t n4) {
  extern __shared__ unsigned char lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f4v acc{0, 0, 0, 0};
  if (V == 2 || V == 5) {  // 40 KB per block, the same 40 KB for each group of 32 blocks
    const f4v* s = src + (size_t)(blockIdx.x / 32) * 2560;
    for (int k = threadIdx.x; k < 2560; k += 256) acc += s[k];
  }
  unsigned long long* bits = reinterpret_cast<unsigned long long*>(lds);
  if (V == 4 || V == 5) {
    for (int k = threadIdx.x; k < 32 * 16; k += 256) bits[k] = 0x9249249249249249ull * (k + 1);
    __syncthreads();
  }
  if (V == 1) {
    lds[threadIdx.x] = 1;
    __syncthreads();
  }
  f4v* base = p + (size_t)blockIdx.x * 32 * 256;
  const float iv = 0.25f + acc.x;
  for (int r = wid; r < 32; r += 4)
    for (int q = lane; q < 256; q += 64) {
      f4v v{iv, 0.0f, iv, 0.0f};
      if (V == 4 || V == 5) {
        const unsigned nib = (unsigned)(bits[r * 16 + (q >> 4)] >> ((q & 15) << 2)) & 0xFu;
        v = f4v{(nib & 1u) ? iv : 0.f, (nib & 2u) ? iv : 0.f, (nib & 4u) ? iv : 0.f, (nib & 8u) ? iv : 0.f};
      }
      base[r * 256 + q] = v;
    }
  if (V == 3 || V == 5) {  // 6 floats + 4 doubles per row, one lane per row
    const int S = 8, fr = threadIdx.x / S, fs = threadIdx.x % S;
    if (fs == 0) {
      const size_t g = (size_t)blockIdx.x * 32 + fr;
      for (int k = 0; k < 6; ++k) small[g * 6 + k] = iv;
      double* x = reinterpret_cast<double*>(small + (size_t)gridDim.x * 32 * 6);
      for (int k = 0; k < 4; ++k) x[g * 4 + k] = iv;
    }
  }
}

__global__ __launch_bounds__(256) void readk(const f4v* p, size_t n4, float* out) {
  f4v acc{0, 0, 0, 0};
  for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n4; k += (size_t)gridDim.x * 256) acc += p[k];
  if (acc.x == 12345.f) out[0] = acc.y;
}

__global__ __launch_bounds__(256) void copyk(const f4v* a, f4v* b, size_t n4) {
  for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n4; k += (size_t)gridDim.x * 256) b[k] = a[k];
}

int main(int argc, char** argv) {
  const size_t MB = 1 << 20;
  std::vector<size_t> sizes = {128 * MB, 512 * MB, 1024 * MB, 4096 * MB};
  const int grids[] = {1024, 4096, 16384};
  f4v *a = nullptr, *b = nullptr;
  float* o = nullptr;
  if (argc > 1 && argv[1][0] == 'v') {  // side-cost variants of the 32-row store shape
    const size_t bytes = 1024 * MB, n4 = bytes / 16;
    const int g = (int)(bytes / (32 * 1024 * 4));
    f4v* src;
    float* small;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&src, (size_t)(g / 32 + 1) * 2560 * 16));
    CK(hipMemset(src, 0, (size_t)(g / 32 + 1) * 2560 * 16));
    CK(hipMalloc(&small, (size_t)g * 32 * (24 + 32)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep)
      for (int v = 0; v < 6; ++v) {
        auto launch = [&]() {
          switch (v) {
            case 0: rows32<0><<<g, 256, 0>>>(a, src, small, n4); break;
            case 1: rows32<1><<<g, 256, 26 * 1024>>>(a, src, small, n4); break;
            case 2: rows32<2><<<g, 256, 0>>>(a, src, small, n4); break;
            case 3: rows32<3><<<g, 256, 0>>>(a, src, small, n4); break;
            case 4: rows32<4><<<g, 256, 4096>>>(a, src, small, n4); break;
            case 5: rows32<5><<<g, 256, 4096>>>(a, src, small, n4); break;
          }
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        static const char* names[] = {"plain", "+26KB LDS", "+40KB L2 reads", "+small writes", "+LDS bits",
                                      "+reads+small+bits"};
        printf("rows32 %-18s %8.1f us %7.0f GB/s\n", names[v], ms / 10 * 1e3, bytes / (ms / 10 * 1e-3) / 1e9);
      }
    return 0;
  }
  if (argc > 1) {  // rows mode: the step kernel's store shape at 1 GiB, 16384 blocks
    const size_t bytes = 1024 * MB, n4 = bytes / 16;
    const int g = (int)(bytes / (64 * 1024 * 4));
    CK(hipMalloc(&a, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 8; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: fill_rows<0, false><<<g, 256>>>(a, n4); break;
          case 1: fill_rows<0, true><<<g, 256>>>(a, n4); break;
          case 2: fill_rows<2048, false><<<g, 256>>>(a, n4); break;
          case 3: fill_rows<8192, false><<<g, 256>>>(a, n4); break;
          case 4: fill_rows<16384, false><<<g, 256>>>(a, n4); break;
          case 5: fill_rows<32768, false><<<g, 256>>>(a, n4); break;
          case 6: fill<4><<<4096, 256>>>(a, n4); break;
          case 7: fill<4><<<g, 256>>>(a, n4); break;
        }
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      static const char* names[] = {"rows", "rows_nt", "rows+2k cyc", "rows+8k cyc", "rows+16k cyc",
                                    "rows+32k cyc", "chunk g4096", "chunk g16384"};
      printf("1 GiB %-14s %8.1f us %7.0f GB/s\n", names[mode], ms / 10 * 1e3, bytes / (ms / 10 * 1e-3) / 1e9);
    }
    return 0;
  }
  CK(hipMalloc(&a, 4096 * MB));
  CK(hipMalloc(&b, 4096 * MB));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 0, 4096 * MB));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t bytes : sizes) {
    const size_t n4 = bytes / 16;
    const int reps = bytes >= 1024 * MB ? 10 : 40;
    for (int g : grids) {
      for (int mode = 0; mode < 7; ++mode) {
        auto launch = [&]() {
          switch (mode) {
            case 0: fill<0><<<g, 256>>>(a, n4); break;
            case 1: fill<1><<<g, 256>>>(a, n4); break;
            case 2: fill<2><<<g, 256>>>(a, n4); break;
            case 3: fill<3><<<g, 256>>>(a, n4); break;
            case 4: fill<4><<<g, 256>>>(a, n4); break;
            case 5: readk<<<g, 256>>>(a, n4, o); break;
            case 6: copyk<<<g, 256>>>(a, b, n4); break;
          }
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double t = ms / reps * 1e-3;
        const double moved = mode == 6 ? 2.0 * bytes : (double)bytes;
        static const char* names[] = {"fill", "fill_nt", "fill_u4", "fill_u4_nt", "fill_chunk", "read", "copy(r+w)"};
        printf("%5zu MiB grid %5d %-11s %8.1f us %7.0f GB/s\n", bytes / MB, g, names[mode], t * 1e6, moved / t / 1e9);
      }
    }
  }
  return 0;
}
