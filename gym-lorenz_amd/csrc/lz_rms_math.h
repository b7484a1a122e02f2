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

}  // namespace lz
