// RunningMeanStd arithmetic shared by the stand-alone statistics kernels (lz_rms.hip)
// and the VecNormalize epilogue of the step kernel (lz_kernels.hip), so that both
// produce the same bits from the same moments.  Internal, not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

namespace lz {

// stable-baselines3 2.7.1 RunningMeanStd.update_from_moments
// (common/running_mean_std.py) for one dimension, with the batch mean / var derived
// from the (count bc, sum s, sum of squares q) moments.
__device__ __forceinline__ void rms_new(double mean, double var, double c, double bc, double s,
                                        double q, double& new_mean, double& new_var) {
  const double bm = s / bc;
  double bv = q / bc - bm * bm;
  if (bv < 0.0) bv = 0.0;
  const double delta = bm - mean;
  const double tot = c + bc;
  new_mean = mean + delta * bc / tot;
  const double m_a = var * c;
  const double m_b = bv * bc;
  const double m_2 = m_a + m_b + delta * delta * c * bc / tot;
  new_var = m_2 / tot;
}

// VecNormalize._normalize_obs / normalize_reward for one element:
// clip((x - mean if center else x) / sqrt(var + eps), -clip, clip), np.clip semantics
// (NaN propagates).
__device__ __forceinline__ float rms_norm_sd(double v, double mean, double sd, bool center,
                                             double clip) {
  if (center) v = v - mean;
  v = v / sd;
  v = v < -clip ? -clip : (v > clip ? clip : v);
  return (float)v;
}
// sd = sqrt(var + eps), hoisted by callers that normalise many elements of a column
__device__ __forceinline__ float rms_norm(double v, double mean, double var, bool center,
                                          double eps, double clip) {
  return rms_norm_sd(v, mean, sqrt(var + eps), center, clip);
}

// Column totals of lz_step_vecnorm's per-workgroup moment partials (column-major
// [W][n_wg]), in one fixed order shared by every caller -- k_vn_colsum (LZ_VN_DEFER)
// and every workgroup of the normalise pass -- so that they all derive the same bits.
// 256 threads: thread t adds rows t, t + 256, ... of every column in order (coalesced
// loads, W in flight per row step); the [W][256] lane sums go through LDS, where
// thread (c, s) adds the s-th run of 256 / S lane sums of column c in lane order, and
// thread c < W the S run sums in run order.  No cross-lane shuffles (float64 shuffles
// of the butterfly measured slower) and no lane-strided global loads (one cache line
// per lane: measured 4 us per 262k-env step).  red: LZ_VN_RED(W) doubles of LDS.
#define LZ_VN_RED(W) ((W) * 257 + 256)
template <int W>
__device__ __forceinline__ void vn_col_totals(const double* part, int n_wg, double* red,
                                              double* out) {
  constexpr int CS = W <= 16 ? 16 : 32, S = 256 / CS, RUN = 256 / S;
  static_assert(W <= 32, "too many partial columns");
  const int t = (int)threadIdx.x;
  double acc[W];
#pragma unroll
  for (int c = 0; c < W; ++c) acc[c] = 0.0;
  for (int r = t; r < n_wg; r += 256) {
#pragma unroll
    for (int c = 0; c < W; ++c) acc[c] += part[(int64_t)c * n_wg + r];
  }
#pragma unroll
  for (int c = 0; c < W; ++c) red[c * 257 + t] = acc[c];
  __syncthreads();
  double* run = red + W * 257;
  const int c = t % CS, sg = t / CS;
  if (c < W) {
    const double* x = red + c * 257 + sg * RUN;
    double v = x[0];
#pragma unroll
    for (int k = 1; k < RUN; ++k) v += x[k];
    run[sg * CS + c] = v;
  }
  __syncthreads();
  if (t < W) {
    double v = run[t];
#pragma unroll
    for (int k = 1; k < S; ++k) v += run[k * CS + t];
    out[t] = v;
  }
  __syncthreads();
}

}  // namespace lz
