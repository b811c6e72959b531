// Occupancy probe (diagnostic): how many 256-thread workgroups with a given dynamic
// LDS size run at once on one CU of this device. Each workgroup sleeps ~20 us and
// records its start/end time and HW_ID/XCC_ID; the host counts the peak overlap per CU.
// Build: hipcc -O3 --offload-arch=gfx950 occprobe.hip -o build/occprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned long long* out) {
  extern __shared__ unsigned char lds[];
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    lds[0] = 1;
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(10);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 3 + 0] = t0;
    out[blockIdx.x * 3 + 1] = t1;
    out[blockIdx.x * 3 + 2] = ((unsigned long long)xcc << 32) | hw;
  }
  __syncthreads();
}

int main() {
  const int G = 256 * 12;
  unsigned long long* d;
  hipMalloc(&d, G * 3 * 8);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  std::vector<unsigned long long> h(G * 3);
  for (int kb : {0, 16, 20, 24, 26, 27, 28, 30, 31, 32, 33, 40, 48, 53, 54, 64, 80}) {
    hipLaunchKernelGGL(probe, dim3(G), dim3(256), kb * 1024, 0, d);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, G * 3 * 8, hipMemcpyDeviceToHost);
    std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;
    for (int b = 0; b < G; ++b) {
      const unsigned long long id = h[b * 3 + 2] & 0xF0000FF00ull;  // xcc, se/sh/cu
      const unsigned long long key = (h[b * 3 + 2] >> 32 << 16) | ((h[b * 3 + 2] >> 8) & 0xFF);
      (void)id;
      ev[key].push_back({h[b * 3], +1});
      ev[key].push_back({h[b * 3 + 1], -1});
    }
    int peak_min = 1 << 30, peak_max = 0;
    for (auto& kv : ev) {
      auto v = kv.second;
      std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
      int c = 0, p = 0;
      for (auto& e : v) p = std::max(p, c += e.second);
      peak_min = std::min(peak_min, p);
      peak_max = std::max(peak_max, p);
    }
    printf("LDS %3d KiB: CUs seen %zu, peak workgroups per CU min %d max %d\n", kb, ev.size(), peak_min, peak_max);
  }
  return 0;
}
