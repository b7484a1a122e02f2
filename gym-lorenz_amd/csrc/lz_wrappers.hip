// SB3 VecEnv wrappers the reference stacks on its envs, on the device.
//
// lz_frame_stack: VecFrameStack(venv, n_stack) for a 1-D Box observation space
// (code/lorenz_filter/train.py:113-115 stacks 4 HR observations), restating SB3 2.7.1
// common/vec_env/stacked_observations.py StackedObservations (channels-last):
//   reset:  stacked = 0; stacked[:, -O:] = obs
//   update: stacked = roll(stacked, -O, axis=-1); stacked[done] = 0; stacked[:, -O:] = obs
//
// The update is in place and every element of a row moves, so a row must be read whole
// before any of it is written.  k_frame_stack_tile gives each workgroup 256 whole rows:
// the tile's [256, S*O] stack slice and [256, O] obs slice are contiguous in HBM and come
// into LDS as 16-B vectors (every wave instruction covers 1 KiB of consecutive bytes),
// one barrier, then the rolled rows go out the same way -- instead of one lane per row
// walking its 4*S*O-byte row (a wave instruction then touches 64 rows 96 B apart).
// Rows wider than the LDS tile allows (S*O + O > 64 floats) use the per-row kernel.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "lz_internal.h"

namespace lz {

constexpr int kFsRows = 256;     // rows per workgroup
constexpr int kFsMaxWidth = 64;  // S*O + O floats per row that the LDS tile holds

typedef float fs4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_frame_stack_tile(float* __restrict__ st,
                                                          const float* __restrict__ obs,
                                                          const uint8_t* __restrict__ done,
                                                          int64_t n, int S, int O, int reset,
                                                          int vec) {
  extern __shared__ float sm[];
  __shared__ uint8_t s_clr[kFsRows];
  const int SO = S * O, keep = SO - O;
  const int tid = (int)threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kFsRows;
  const int rows = (int)((n - r0) < kFsRows ? (n - r0) : kFsRows);
  float* s_st = sm;                    // [rows][SO]
  float* s_ob = sm + kFsRows * SO;     // [rows][O]
  float* dst = st + r0 * SO;
  const float* ob = obs + r0 * O;
  const int tot = rows * SO, tob = rows * O;
  if (vec) {  // 16-B aligned slices (the host checks the base pointers and S*O, O)
    const fs4* s4 = reinterpret_cast<const fs4*>(dst);
    const fs4* o4 = reinterpret_cast<const fs4*>(ob);
    for (int v = tid; v < tot / 4; v += 256)
      reinterpret_cast<fs4*>(s_st)[v] = __builtin_nontemporal_load(s4 + v);
    for (int v = tid; v < tob / 4; v += 256)
      reinterpret_cast<fs4*>(s_ob)[v] = __builtin_nontemporal_load(o4 + v);
    for (int e = (tob / 4) * 4 + tid; e < tob; e += 256) s_ob[e] = ob[e];
  } else {
    for (int e = tid; e < tot; e += 256) s_st[e] = dst[e];
    for (int e = tid; e < tob; e += 256) s_ob[e] = ob[e];
  }
  if (tid < rows) s_clr[tid] = (uint8_t)(reset || (done && done[r0 + tid] != 0));
  __syncthreads();
  auto val = [&](int e) __attribute__((always_inline)) {
    const int row = e / SO, j = e - row * SO;
    return j < keep ? (s_clr[row] ? 0.0f : s_st[e + O]) : s_ob[row * O + (j - keep)];
  };
  if (vec) {
    for (int v = tid; v < tot / 4; v += 256) {
      const fs4 w = {val(4 * v), val(4 * v + 1), val(4 * v + 2), val(4 * v + 3)};
      __builtin_nontemporal_store(w, reinterpret_cast<fs4*>(dst) + v);
    }
  } else {
    for (int e = tid; e < tot; e += 256) dst[e] = val(e);
  }
}

// one lane per row: rows too wide for the LDS tile
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
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int SO = n_stack * obs_dim;
  // LZ_FRAME_STACK_ROWS=1 forces the per-row kernel (A/B measurements only)
  static const bool force_rows = std::getenv("LZ_FRAME_STACK_ROWS") != nullptr;
  if (SO + obs_dim <= lz::kFsMaxWidth && !force_rows) {
    // 16-B vectors: a tile's stack slice starts at r0 * S*O floats and its obs slice at
    // r0 * O (r0 a multiple of 256), so both are aligned whenever the base pointers are;
    // rows * S*O is a multiple of 4 when S*O is, the obs slice's tail is loaded scalar
    const int v = (reinterpret_cast<uintptr_t>(stacked) % 16 == 0) &&
                  (reinterpret_cast<uintptr_t>(obs) % 16 == 0) && (SO % 4 == 0);
    const size_t lds = (size_t)lz::kFsRows * (SO + obs_dim) * sizeof(float);
    hipLaunchKernelGGL(lz::k_frame_stack_tile, dim3((unsigned)((n + lz::kFsRows - 1) / lz::kFsRows)),
                       dim3(256), lds, s, stacked, obs, done, n, n_stack, obs_dim, reset, v);
  } else {
    hipLaunchKernelGGL(lz::k_frame_stack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, stacked,
                       obs, done, n, n_stack, obs_dim, reset);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lz::set_error(LZ_ERR_HIP, hipGetErrorString(e));
  return LZ_OK;
}
