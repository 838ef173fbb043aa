// Wave reductions shared by the reduce (kernels_common.hip) and the analytic cartpole (kernels_cartpole.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace mppi {

// ------------------------------------------------------------------------------------------------
// Wave / block reductions (fixed order -> bitwise deterministic).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}

}  // namespace mppi
