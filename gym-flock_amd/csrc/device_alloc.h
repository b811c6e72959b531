// Device buffer allocation shared by the C-ABI files (capi.hip, cov_capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace gf {

// Large buffers (the dense network: 1 GiB at config 2, 8 GiB at config 5; the Coverage
// time matrices) are requested physically contiguous: the network store stream of config
// 2 ran 180 -> 165 us per step and config 5's 1.50 -> 1.44 ms in them (bench A/B,
// profiles/r03/ab_contiguous_outputs.txt). If the device cannot provide one, plain
// hipMalloc; the failed request's error is cleared so later launch checks do not see it.
inline hipError_t device_alloc(void** p, size_t bytes) {
  if (bytes >= (size_t(256) << 20) &&
      hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess)
    return hipSuccess;
  (void)hipGetLastError();
  return hipMalloc(p, bytes);
}

}  // namespace gf
