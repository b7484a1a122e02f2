// SB3 VecEnv wrappers the reference stacks on its envs, on the device.
//
// lz_frame_stack: VecFrameStack(venv, n_stack) for a 1-D Box observation space
// (code/lorenz_filter/train.py:113-115 stacks 4 HR observations), restating SB3 2.7.1
// common/vec_env/stacked_observations.py StackedObservations (channels-last):
//   reset:  stacked = 0; stacked[:, -O:] = obs
//   update: stacked = roll(stacked, -O, axis=-1); stacked[done] = 0; stacked[:, -O:] = obs
// One thread per env row (the row is n_stack * O floats, read whole before written).
#include <hip/hip_runtime.h>

#include "lz_internal.h"

namespace lz {

__global__ __launch_bounds__(256) void k_frame_stack(float* __restrict__ st, const float* __restrict__ obs,
                                                    const uint8_t* __restrict__ done, int64_t n,
                                                    int S, int O, int reset) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float* row = st + i * (int64_t)S * O;
  const bool clear = reset || (done && done[i] != 0);
  const int keep = (S - 1) * O;
  for (int j = 0; j < keep; ++j) row[j] = clear ? 0.0f : row[j + O];
  for (int j = 0; j < O; ++j) row[keep + j] = obs[i * O + j];
}

}  // namespace lz

extern "C" lz_status lz_frame_stack(float* stacked, const float* obs, const uint8_t* done,
                                    int64_t n, int32_t n_stack, int32_t obs_dim, int32_t reset,
                                    int32_t device, void* stream) {
  if (!stacked || !obs || (!reset && !done)) return lz::set_error(LZ_ERR_INVALID, "NULL buffer");
  if (n < 0 || n_stack < 1 || obs_dim < 1) return lz::set_error(LZ_ERR_INVALID, "bad shape");
  if (n == 0) return LZ_OK;
  if (hipSetDevice(device) != hipSuccess) return lz::set_error(LZ_ERR_HIP, "hipSetDevice failed");
  hipLaunchKernelGGL(lz::k_frame_stack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), stacked, obs, done, n, n_stack, obs_dim,
                     reset);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lz::set_error(LZ_ERR_HIP, hipGetErrorString(e));
  return LZ_OK;
}
