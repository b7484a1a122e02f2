// On-device VecNormalize statistics: stable-baselines3 2.7.1
// RunningMeanStd (common/running_mean_std.py) and the VecNormalize arithmetic
// (common/vec_env/vec_normalize.py) over the env axis of the batched step outputs,
// float64 statistics as in SB3.  The batch moments are (count, sum, sum of squares):
// plain sums, so a multi-GPU run all-reduces them (RCCL, one 2*dim+1 double vector)
// before the update and every rank keeps identical statistics.
//
// Reductions are deterministic: per-workgroup partials in a fixed grid-stride order,
// then one workgroup sums the partials in a fixed tree order -- no float atomics.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "lorenz_env.h"
#include "lz_internal.h"

namespace {

constexpr int kRmsBlock = 256;
constexpr int kRmsMaxBlocks = 1024;
constexpr int kRmsMaxDim = 16;

lz_status rfail(lz_status s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
lz_status rfail(lz_status s, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return lz::set_error(s, buf);  // shared with lz_last_error()
}

template <typename T>
__device__ __forceinline__ double ldx(const void* x, int64_t i) {
  return (double)static_cast<const T*>(x)[i];
}

// per-workgroup partial (sum, sumsq) of each of the D columns, rows grid-strided
template <typename T, int D>
__global__ __launch_bounds__(kRmsBlock) void k_moments_partial(const void* x, int64_t n,
                                                               double* partial) {
  __shared__ double red[kRmsBlock / 64][2 * D];
  double s[D], q[D];
#pragma unroll
  for (int d = 0; d < D; ++d) s[d] = q[d] = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * kRmsBlock + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * kRmsBlock) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const double v = ldx<T>(x, r * D + d);
      s[d] += v;
      q[d] += v * v;
    }
  }
  // wave tree (fixed order), then the 4 waves in order
#pragma unroll
  for (int d = 0; d < D; ++d) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      s[d] += __shfl_down(s[d], off, 64);
      q[d] += __shfl_down(q[d], off, 64);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) { red[wave][d] = s[d]; red[wave][D + d] = q[d]; }
  }
  __syncthreads();
  if (threadIdx.x < 2 * D) {
    double acc = 0.0;
    for (int w = 0; w < kRmsBlock / 64; ++w) acc += red[w][threadIdx.x];
    partial[(int64_t)blockIdx.x * 2 * D + threadIdx.x] = acc;
  }
}

// one workgroup: moments = (n, sum[D], sumsq[D]) from nb partials, fixed order
__global__ __launch_bounds__(kRmsBlock) void k_moments_final(const double* partial, int nb, int D,
                                                             int64_t n, double* moments) {
  __shared__ double red[kRmsBlock];
  for (int c = 0; c < 2 * D; ++c) {
    double acc = 0.0;
    for (int b = threadIdx.x; b < nb; b += kRmsBlock) acc += partial[(int64_t)b * 2 * D + c];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = kRmsBlock / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) moments[1 + c] = red[0];
    __syncthreads();
  }
  if (threadIdx.x == 0) moments[0] = (double)n;
}

// RunningMeanStd.update_from_moments (running_mean_std.py), batch mean / var from the
// (count, sum, sumsq) moments
__global__ void k_rms_update(double* mean, double* var, double* count, const double* moments,
                             int D) {
  const int d = threadIdx.x;  // launched with 64 threads >= D: every lane reaches the barrier
  const double bc = moments[0];
  const double c = *count;
  double new_mean = 0.0, new_var = 0.0;
  const bool act = d < D && bc > 0.0;
  if (act) {
    const double bm = moments[1 + d] / bc;
    double bv = moments[1 + D + d] / bc - bm * bm;
    if (bv < 0.0) bv = 0.0;
    const double delta = bm - mean[d];
    const double tot = c + bc;
    new_mean = mean[d] + delta * bc / tot;
    const double m_a = var[d] * c;
    const double m_b = bv * bc;
    const double m_2 = m_a + m_b + delta * delta * c * bc / tot;
    new_var = m_2 / tot;
  }
  __syncthreads();  // every lane has read *count before lane 0 rewrites it
  if (act) {
    mean[d] = new_mean;
    var[d] = new_var;
    if (d == 0) *count = c + bc;
  }
}

// VecNormalize._normalize_obs / normalize_reward: clip((x - mean) / sqrt(var + eps))
template <typename T>
__global__ void k_rms_normalize(const void* x, int64_t n, int D, const double* mean,
                                const double* var, int center, double eps, double clip, float* y) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * D) return;
  const int d = (int)(e % D);
  double v = ldx<T>(x, e);
  if (center) v = v - mean[d];
  v = v / sqrt(var[d] + eps);
  v = v < -clip ? -clip : (v > clip ? clip : v);  // np.clip (NaN-propagating)
  y[e] = (float)v;
}

// VecNormalize._update_reward / step_wait: returns = returns * gamma + reward, then
// (phase 1) returns[dones] = 0
template <typename T>
__global__ void k_returns(double* ret, const void* rew, const uint8_t* done, int64_t n,
                          double gamma, int phase) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (phase == 0) ret[i] = ret[i] * gamma + ldx<T>(rew, i);
  else if (done[i]) ret[i] = 0.0;
}

}  // namespace

struct lz_rms {
  int dim;
  int device;
  hipStream_t stream;
  double* state;    // mean[dim], var[dim], count
  double* partial;  // [kRmsMaxBlocks][2*dim]
};

#define RMS_HIP(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return rfail(LZ_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

extern "C" {

lz_status lz_rms_create(int32_t dim, int32_t device, double count_init, lz_rms** out) {
  if (!out) return rfail(LZ_ERR_INVALID, "out is NULL");
  *out = nullptr;
  if (dim < 1 || dim > kRmsMaxDim) return rfail(LZ_ERR_INVALID, "dim must be in [1, %d]", kRmsMaxDim);
  int ndev = 0;
  RMS_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return rfail(LZ_ERR_INVALID, "device %d out of range", device);
  RMS_HIP(hipSetDevice(device));
  lz_rms* r = new (std::nothrow) lz_rms();
  if (!r) return rfail(LZ_ERR_OOM, "host allocation failed");
  r->dim = dim;
  r->device = device;
  r->stream = nullptr;
  r->state = nullptr;
  r->partial = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&r->state), (2 * dim + 1) * sizeof(double)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&r->partial),
                (size_t)kRmsMaxBlocks * 2 * dim * sizeof(double)) != hipSuccess) {
    lz_rms_destroy(r);
    return rfail(LZ_ERR_OOM, "device allocation failed");
  }
  // RunningMeanStd.__init__(epsilon=1e-4): mean 0, var 1, count epsilon
  double init[2 * kRmsMaxDim + 1];
  for (int d = 0; d < dim; ++d) { init[d] = 0.0; init[dim + d] = 1.0; }
  init[2 * dim] = count_init;
  if (hipMemcpy(r->state, init, (2 * dim + 1) * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    lz_rms_destroy(r);
    return rfail(LZ_ERR_HIP, "state upload failed");
  }
  *out = r;
  return LZ_OK;
}

lz_status lz_rms_destroy(lz_rms* r) {
  if (!r) return LZ_OK;
  (void)hipSetDevice(r->device);
  if (r->state) (void)hipFree(r->state);
  if (r->partial) (void)hipFree(r->partial);
  delete r;
  return LZ_OK;
}

lz_status lz_rms_set_stream(lz_rms* r, void* stream) {
  if (!r) return rfail(LZ_ERR_INVALID, "rms is NULL");
  r->stream = static_cast<hipStream_t>(stream);
  return LZ_OK;
}

lz_status lz_rms_state(lz_rms* r, double** mean, double** var, double** count) {
  if (!r) return rfail(LZ_ERR_INVALID, "rms is NULL");
  if (mean) *mean = r->state;
  if (var) *var = r->state + r->dim;
  if (count) *count = r->state + 2 * r->dim;
  return LZ_OK;
}

lz_status lz_rms_moments(lz_rms* r, const void* x, int32_t dtype, int64_t n, double* moments_out) {
  if (!r || !moments_out || (!x && n > 0)) return rfail(LZ_ERR_INVALID, "NULL argument");
  if (dtype != LZ_DTYPE_F32 && dtype != LZ_DTYPE_F64) return rfail(LZ_ERR_INVALID, "bad dtype");
  RMS_HIP(hipSetDevice(r->device));
  const int D = r->dim;
  int64_t nb64 = (n + kRmsBlock - 1) / kRmsBlock;
  const int nb = (int)(nb64 < 1 ? 1 : (nb64 > kRmsMaxBlocks ? kRmsMaxBlocks : nb64));
  const bool f64 = dtype == LZ_DTYPE_F64;
#define RMS_LAUNCH_D(DD)                                                                         \
  if (f64)                                                                                       \
    hipLaunchKernelGGL((k_moments_partial<double, DD>), dim3(nb), dim3(kRmsBlock), 0, r->stream, x, \
                       n, r->partial);                                                          \
  else                                                                                           \
    hipLaunchKernelGGL((k_moments_partial<float, DD>), dim3(nb), dim3(kRmsBlock), 0, r->stream, x, \
                       n, r->partial);
  switch (D) {
    case 1: RMS_LAUNCH_D(1) break;
    case 2: RMS_LAUNCH_D(2) break;
    case 3: RMS_LAUNCH_D(3) break;
    case 6: RMS_LAUNCH_D(6) break;
    case 8: RMS_LAUNCH_D(8) break;
    default: return rfail(LZ_ERR_UNSUPPORTED, "moments for dim %d not instantiated", D);
  }
#undef RMS_LAUNCH_D
  RMS_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_moments_final, dim3(1), dim3(kRmsBlock), 0, r->stream, r->partial, nb, D, n,
                     moments_out);
  RMS_HIP(hipGetLastError());
  return LZ_OK;
}

lz_status lz_rms_update(lz_rms* r, const double* moments) {
  if (!r || !moments) return rfail(LZ_ERR_INVALID, "NULL argument");
  RMS_HIP(hipSetDevice(r->device));
  const int D = r->dim;
  hipLaunchKernelGGL(k_rms_update, dim3(1), dim3(64), 0, r->stream, r->state, r->state + D,
                     r->state + 2 * D, moments, D);
  RMS_HIP(hipGetLastError());
  return LZ_OK;
}

lz_status lz_rms_normalize(lz_rms* r, const void* x, int32_t dtype, int64_t n, float* y,
                           int32_t center, double eps, double clip) {
  if (!r || (!x && n > 0) || (!y && n > 0)) return rfail(LZ_ERR_INVALID, "NULL argument");
  if (dtype != LZ_DTYPE_F32 && dtype != LZ_DTYPE_F64) return rfail(LZ_ERR_INVALID, "bad dtype");
  if (n == 0) return LZ_OK;
  RMS_HIP(hipSetDevice(r->device));
  const int D = r->dim;
  const int64_t tot = n * D;
  const dim3 grid((unsigned)((tot + 255) / 256)), block(256);
  if (dtype == LZ_DTYPE_F64)
    hipLaunchKernelGGL(k_rms_normalize<double>, grid, block, 0, r->stream, x, n, D, r->state,
                       r->state + D, center, eps, clip, y);
  else
    hipLaunchKernelGGL(k_rms_normalize<float>, grid, block, 0, r->stream, x, n, D, r->state,
                       r->state + D, center, eps, clip, y);
  RMS_HIP(hipGetLastError());
  return LZ_OK;
}

lz_status lz_returns_update(double* returns, const void* rew, int32_t dtype, const uint8_t* done,
                            int64_t n, double gamma, int32_t phase, int32_t device, void* stream) {
  if (!returns || (phase == 0 && !rew) || (phase == 1 && !done))
    return rfail(LZ_ERR_INVALID, "NULL argument");
  if (n == 0) return LZ_OK;
  RMS_HIP(hipSetDevice(device));
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dtype == LZ_DTYPE_F64)
    hipLaunchKernelGGL(k_returns<double>, grid, block, 0, s, returns, rew, done, n, gamma, phase);
  else
    hipLaunchKernelGGL(k_returns<float>, grid, block, 0, s, returns, rew, done, n, gamma, phase);
  RMS_HIP(hipGetLastError());
  return LZ_OK;
}

}  // extern "C"
