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
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>

#include "lorenz_env.h"
#include "lz_internal.h"
#include "lz_rms_math.h"

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
  if (act)
    lz::rms_new(mean[d], var[d], c, bc, moments[1 + d], moments[1 + D + d], new_mean, new_var);
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
  y[e] = lz::rms_norm(ldx<T>(x, e), mean[d], var[d], center != 0, eps, clip);
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

// lz_vecnorm_apply: the normalised outputs of one VecNormalize.step_wait.  The first
// row_blocks workgroups grid-stride over the row tiles (256 threads owning R
// consecutive env rows each, R * O a multiple of 4, so the obs columns of each element
// are compile-time constants and the rows move as 16-B vectors when aligned): obs rows,
// rewards and the done flags as 0/1 bytes (SB3's bool dones); the remaining workgroups
// grid-stride over the n_done terminal rows.  Inputs are rounded to float32 first:
// SB3's VecNormalize sees DummyVecEnv's float32 buffers.  In training every workgroup
// first reduces the step's moment partials (vn_col_totals: one fixed order, the same
// bits in every workgroup and in the LZ_VN_DEFER reduction) -- the first tile's loads
// are issued before that, so the reduction runs while they are in flight.
struct VnApplyArgs {
  int64_t n;
  const void* obs;
  const void* rew;
  const void* term;
  const uint8_t* done;
  const int32_t* n_done;
  const int32_t* counter;  // the step's done cursor (nullptr: read n_done)
  int32_t* n_done_out;     // published from *counter by block 0 (nullable)
  double* os;        // obs_rms mean[O], var[O], count
  double* rs;        // ret_rms mean, var, count
  lz::VnUpdate upd;  // statistics updates folded into this pass (upd.part or upd.tot)
  double eps, clip_obs, clip_rew;
  float* obs_n;
  float* rew_n;
  float* term_n;
  uint8_t* dones;
  int64_t row_tiles;
  int norm_obs, norm_rew, vec, row_blocks;
};

typedef float f4a __attribute__((ext_vector_type(4)));

// kRed: this instance reduces the partials (fused path); the others carry no
// reduction code (its accumulators would raise every instance's VGPR count)
template <typename T, int O, bool kRed>
__global__ __launch_bounds__(256) void k_vn_apply(VnApplyArgs p) {
  constexpr int R = (O % 4 == 0) ? 1 : (O % 2 == 0 ? 2 : 4);
  constexpr int E = R * O;
  constexpr int W = 2 * (O + 1);
  constexpr bool kF32 = std::is_same<T, float>::value;
  const int t = (int)threadIdx.x;
  const bool rows = (int)blockIdx.x < p.row_blocks;
  const T* obs = static_cast<const T*>(p.obs);
  const T* rew = static_cast<const T*>(p.rew);
  auto tile_full = [&](int64_t tl) { return (tl + 1) * 256 * R <= p.n; };  // uniform
  // the first tile's raw obs (16-B vectors, read once: non-temporal), rewards, dones
  f4a q[E / 4];
  float rw[R];
  uint8_t dn[R];
  auto load_obs = [&](int64_t tl) {
    const f4a* src = reinterpret_cast<const f4a*>(obs + tl * 256 * E);
#pragma unroll
    for (int k = 0; k < E / 4; ++k) q[k] = __builtin_nontemporal_load(src + t + 256 * k);
  };
  auto load_rd = [&](int64_t tl) {  // a full tile's rewards / done bytes
    const int64_t r0 = (tl * 256 + t) * R;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      rw[k] = (float)rew[r0 + k];
      dn[k] = p.dones ? p.done[r0 + k] : 0;
    }
  };
  if (p.n_done_out && blockIdx.x == 0 && t == 0) *p.n_done_out = *p.counter;
  int64_t tile = blockIdx.x;
  // (the split path has nothing to overlap: no prefetch, fewer live registers)
  const bool pre = kRed && kF32 && rows && p.vec && tile < p.row_tiles && tile_full(tile);
  if (pre) {
    load_obs(tile);
    load_rd(tile);
  }

  double mean[O], sd[O], rsd;
  if (p.upd.part || p.upd.tot) {
    // RunningMeanStd.update_from_moments for every obs column (lanes 0..O-1) and the
    // returns (lane 64), from the step's column totals and the pre-step snapshot, then
    // broadcast through LDS
    __shared__ double s_red[kRed ? LZ_VN_RED(W) : 1];
    __shared__ double s_tot[W];
    __shared__ double s_st[2 * O + 1];
    if constexpr (kRed) {
      lz::vn_col_totals<W>(p.upd.part, p.upd.n_wg, s_red, s_tot);
    } else {
      if (t < W) s_tot[t] = p.upd.tot[t];
      __syncthreads();
    }
    const double* old = p.upd.old;
    const double bc = p.upd.batch;
    if (t < O) {
      double nm = old[t], nv = old[O + t];
      if (p.upd.upd_obs)
        lz::rms_new(old[t], old[O + t], old[2 * O], bc, s_tot[t], s_tot[O + 1 + t], nm, nv);
      s_st[t] = nm;
      s_st[O + t] = sqrt(nv + p.eps);
      if (blockIdx.x == 0 && p.upd.upd_obs) {
        p.os[t] = nm;
        p.os[O + t] = nv;
        if (t == 0) p.os[2 * O] = old[2 * O] + bc;
      }
    }
    if (t == 64) {
      const double* r = old + 2 * O + 1;
      double nm, nv;
      lz::rms_new(r[0], r[1], r[2], bc, s_tot[O], s_tot[2 * O + 1], nm, nv);
      s_st[2 * O] = sqrt(nv + p.eps);
      if (blockIdx.x == 0) {
        p.rs[0] = nm;
        p.rs[1] = nv;
        p.rs[2] = r[2] + bc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < O; ++d) {
      mean[d] = s_st[d];
      sd[d] = s_st[O + d];
    }
    rsd = s_st[2 * O];
  } else {
#pragma unroll
    for (int d = 0; d < O; ++d) {
      mean[d] = p.os[d];
      sd[d] = sqrt(p.os[O + d] + p.eps);
    }
    rsd = sqrt(p.rs[1] + p.eps);
  }
  if (rows) {
    __shared__ f4a lds[256 * E / 4];
    // split path: one tile per workgroup (the grid covers them), no loop
    const int64_t tile_end = kRed ? p.row_tiles : (tile < p.row_tiles ? tile + 1 : tile);
    for (; tile < tile_end; tile += p.row_blocks) {
      const int64_t r0 = (tile * 256 + t) * R;
      float x[E], y[E];
      const bool pref = pre && tile == (int64_t)blockIdx.x;  // loaded before the statistics
      bool rd = pref;                                        // rw / dn loaded
      if (kF32 && p.vec && tile_full(tile)) {
        // the workgroup's [256 R, O] slice moves as contiguous float4s through LDS
        if (!pref) load_obs(tile);
        __syncthreads();  // the previous tile's stores have read lds
#pragma unroll
        for (int k = 0; k < E / 4; ++k) lds[t + 256 * k] = q[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < E / 4; ++k) {
          const f4a v = lds[t * (E / 4) + k];
          x[4 * k] = v[0]; x[4 * k + 1] = v[1]; x[4 * k + 2] = v[2]; x[4 * k + 3] = v[3];
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
          y[e] = p.norm_obs ? lz::rms_norm_sd((double)x[e], mean[e % O], sd[e % O], true, p.clip_obs)
                            : x[e];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < E / 4; ++k)
          lds[t * (E / 4) + k] = (f4a){y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]};
        __syncthreads();
        f4a* dst = reinterpret_cast<f4a*>(p.obs_n + tile * 256 * E);
#pragma unroll
        for (int k = 0; k < E / 4; ++k)  // normalised obs: written once (non-temporal)
          __builtin_nontemporal_store(lds[t + 256 * k], dst + t + 256 * k);
      } else {  // the last, partial tile (or unaligned / float64 inputs): no barriers
        if (r0 >= p.n) continue;
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = (r0 + e / O < p.n) ? (float)obs[r0 * O + e] : 0.0f;
#pragma unroll
        for (int e = 0; e < E; ++e)
          y[e] = p.norm_obs ? lz::rms_norm_sd((double)x[e], mean[e % O], sd[e % O], true, p.clip_obs)
                            : x[e];
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (r0 + e / O < p.n) p.obs_n[r0 * O + e] = y[e];
#pragma unroll
        for (int k = 0; k < R; ++k) {
          if (r0 + k < p.n) {
            rw[k] = (float)rew[r0 + k];
            dn[k] = p.dones ? p.done[r0 + k] : 0;
          }
        }
        rd = true;
      }
      if (!rd) load_rd(tile);  // after the obs stores, as few registers live as possible
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if (r0 + k >= p.n) break;
        p.rew_n[r0 + k] =
            p.norm_rew ? lz::rms_norm_sd((double)rw[k], 0.0, rsd, false, p.clip_rew) : rw[k];
        if (p.dones) p.dones[r0 + k] = dn[k] != 0;
      }
    }
    return;
  }
  if (p.term == nullptr) return;
  const T* term = static_cast<const T*>(p.term);
  const int64_t m = p.counter ? *p.counter : *p.n_done;
  const int64_t stride = (int64_t)(gridDim.x - p.row_blocks) * 256;
  for (int64_t j = (int64_t)(blockIdx.x - p.row_blocks) * 256 + t; j < m; j += stride) {
#pragma unroll
    for (int d = 0; d < O; ++d) {
      const float x = (float)term[j * O + d];
      p.term_n[j * O + d] =
          p.norm_obs ? lz::rms_norm_sd((double)x, mean[d], sd[d], true, p.clip_obs) : x;
    }
  }
}

// The split path's normalise pass (n above the fused limit): one row tile per
// workgroup, the statistics from the totals k_vn_colsum left, no prefetch -- the
// round-1 kernel, kept as is because its lower register count (56 VGPRs against 76 for
// the fused kernel's non-reducing instance) fits the whole 1M-env grid in one round.
template <typename T, int O>
__global__ __launch_bounds__(256) void k_vn_apply_split(VnApplyArgs p) {
  constexpr int R = (O % 4 == 0) ? 1 : (O % 2 == 0 ? 2 : 4);
  constexpr int E = R * O;
  double mean[O], sd[O], rsd;
  if (p.upd.tot) {
    // RunningMeanStd.update_from_moments for every obs column (lanes 0..O-1) and the
    // returns (lane 64), from the pre-step snapshot -- so no workgroup reads statistics
    // that workgroup 0 is rewriting -- then broadcast through LDS
    __shared__ double s_st[2 * O + 1];
    const int t = (int)threadIdx.x;
    const double* old = p.upd.old;
    const double bc = p.upd.batch;
    if (t < O) {
      double nm = old[t], nv = old[O + t];
      if (p.upd.upd_obs)
        lz::rms_new(old[t], old[O + t], old[2 * O], bc, p.upd.tot[t], p.upd.tot[O + 1 + t], nm, nv);
      s_st[t] = nm;
      s_st[O + t] = sqrt(nv + p.eps);
      if (blockIdx.x == 0 && p.upd.upd_obs) {
        p.os[t] = nm;
        p.os[O + t] = nv;
        if (t == 0) p.os[2 * O] = old[2 * O] + bc;
      }
    }
    if (t == 64) {
      const double* r = old + 2 * O + 1;
      double nm, nv;
      lz::rms_new(r[0], r[1], r[2], bc, p.upd.tot[O], p.upd.tot[2 * O + 1], nm, nv);
      s_st[2 * O] = sqrt(nv + p.eps);
      if (blockIdx.x == 0) {
        p.rs[0] = nm;
        p.rs[1] = nv;
        p.rs[2] = r[2] + bc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < O; ++d) {
      mean[d] = s_st[d];
      sd[d] = s_st[O + d];
    }
    rsd = s_st[2 * O];
  } else {
#pragma unroll
    for (int d = 0; d < O; ++d) {
      mean[d] = p.os[d];
      sd[d] = sqrt(p.os[O + d] + p.eps);
    }
    rsd = sqrt(p.rs[1] + p.eps);
  }
  const T* obs = static_cast<const T*>(p.obs);
  if ((int)blockIdx.x < p.row_blocks) {
    const int64_t r0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * R;
    if (r0 >= p.n) return;  // only in the last (partial, barrier-free) tile
    const bool tile_full = ((int64_t)blockIdx.x + 1) * 256 * R <= p.n;  // uniform
    float x[E], y[E];
    if (std::is_same<T, float>::value && p.vec && tile_full) {
      // the workgroup's [256 R, O] slice moves as contiguous float4s through LDS
      __shared__ f4a tile[256 * E / 4];
      const f4a* src = reinterpret_cast<const f4a*>(obs + (int64_t)blockIdx.x * 256 * E);
#pragma unroll
      for (int k = 0; k < E / 4; ++k)  // raw obs: read once (non-temporal)
        tile[threadIdx.x + 256 * k] = __builtin_nontemporal_load(src + threadIdx.x + 256 * k);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < E / 4; ++k) {
        const f4a q = tile[threadIdx.x * (E / 4) + k];
        x[4 * k] = q[0]; x[4 * k + 1] = q[1]; x[4 * k + 2] = q[2]; x[4 * k + 3] = q[3];
      }
#pragma unroll
      for (int e = 0; e < E; ++e)
        y[e] = p.norm_obs ? lz::rms_norm_sd((double)x[e], mean[e % O], sd[e % O], true, p.clip_obs)
                          : x[e];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < E / 4; ++k)
        tile[threadIdx.x * (E / 4) + k] = (f4a){y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]};
      __syncthreads();
      f4a* dst = reinterpret_cast<f4a*>(p.obs_n + (int64_t)blockIdx.x * 256 * E);
#pragma unroll
      for (int k = 0; k < E / 4; ++k)  // normalised obs: written once (non-temporal)
        __builtin_nontemporal_store(tile[threadIdx.x + 256 * k], dst + threadIdx.x + 256 * k);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) x[e] = (r0 + e / O < p.n) ? (float)obs[r0 * O + e] : 0.0f;
#pragma unroll
      for (int e = 0; e < E; ++e)
        y[e] = p.norm_obs ? lz::rms_norm_sd((double)x[e], mean[e % O], sd[e % O], true, p.clip_obs)
                          : x[e];
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (r0 + e / O < p.n) p.obs_n[r0 * O + e] = y[e];
    }
    const T* rew = static_cast<const T*>(p.rew);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (r0 + k >= p.n) break;
      const float r = (float)rew[r0 + k];
      p.rew_n[r0 + k] = p.norm_rew ? lz::rms_norm_sd((double)r, 0.0, rsd, false, p.clip_rew) : r;
      if (p.dones) p.dones[r0 + k] = p.done[r0 + k] != 0;
    }
    return;
  }
  if (p.term == nullptr) return;
  const T* term = static_cast<const T*>(p.term);
  const int64_t m = *p.n_done;
  const int64_t stride = (int64_t)(gridDim.x - p.row_blocks) * 256;
  for (int64_t j = (int64_t)(blockIdx.x - p.row_blocks) * 256 + threadIdx.x; j < m; j += stride) {
#pragma unroll
    for (int d = 0; d < O; ++d) {
      const float x = (float)term[j * O + d];
      p.term_n[j * O + d] =
          p.norm_obs ? lz::rms_norm_sd((double)x, mean[d], sd[d], true, p.clip_obs) : x;
    }
  }
}

// SB3-exact VecNormalize (lz_internal.h PStepArgs): the statistics update of one step
// from the float64 tile moments, one workgroup per obs dim d (sums column d, squares
// column O + d): thread t sums tiles t, t + 256, ... from 0.0 in order, then the LDS
// tree s[t] += s[t + m], m = 128 .. 1.  snap holds the statistics the step normalised
// with (S_k); S_{k+1} goes to state (read-only snap: no race between the workgroups),
// or with moments != nullptr the batch moments (n, sums, sums of squares) for an
// all-reduce + k_rms_update instead.
__global__ __launch_bounds__(256) void k_vn_tile_update(const double* tiles, int64_t ntiles, int O,
                                                        double batch, const double* snap,
                                                        double* state, double* moments) {
  __shared__ double red[2][256];
  const int d = (int)blockIdx.x, t = (int)threadIdx.x;
  const double* cs = tiles + (int64_t)d * ntiles;
  const double* cq = tiles + (int64_t)(O + d) * ntiles;
  double a = 0.0, b = 0.0;
  // the same in-order sums, with 16 rows of loads issued before their adds (the plain
  // loop left one load in flight per add: 12 us at 8,192 tiles)
  int64_t r = t;
  for (; r + 15 * 256 < ntiles; r += 16 * 256) {
    double va[16], vb[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      va[u] = cs[r + u * 256];
      vb[u] = cq[r + u * 256];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      a += va[u];
      b += vb[u];
    }
  }
  for (; r < ntiles; r += 256) {
    a += cs[r];
    b += cq[r];
  }
  red[0][t] = a;
  red[1][t] = b;
  __syncthreads();
  for (int m = 128; m >= 1; m >>= 1) {
    if (t < m) {
      red[0][t] += red[0][t + m];
      red[1][t] += red[1][t + m];
    }
    __syncthreads();
  }
  if (t == 0) {
    if (moments) {
      moments[1 + d] = red[0][0];
      moments[1 + O + d] = red[1][0];
      if (d == 0) moments[0] = batch;
    } else {
      double nm, nv;
      lz::rms_new(snap[d], snap[O + d], snap[2 * O], batch, red[0][0], red[1][0], nm, nv);
      state[d] = nm;
      state[O + d] = nv;
      if (d == 0) state[2 * O] = snap[2 * O] + batch;
    }
  }
}

// The tile moments of an obs array x [n, O] float32 in k_policy_step_f32's order (one
// wave per tile of 32 envs, half 0 sums, half 1 squares, 32-lane butterfly) -- the
// reset() update of the SB3-exact collect; block 0 snapshots the statistics.
__global__ __launch_bounds__(256) void k_obs_tile_moments(const float* x, int64_t n, int O,
                                                          double* tiles, const double* state,
                                                          double* snap) {
  const int lane = (int)threadIdx.x & 63, h = lane >> 5, slot = lane & 31;
  if (blockIdx.x == 0 && (int)threadIdx.x < 2 * O + 1) snap[threadIdx.x] = state[threadIdx.x];
  const int64_t ntiles = (n + lz::kVnTile - 1) / lz::kVnTile;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); tile < ntiles;
       tile += (int64_t)gridDim.x * 4) {
    const int64_t i = tile * lz::kVnTile + slot;
    for (int j = 0; j < O; ++j) {
      const double v = i < n ? (double)x[i * O + j] : 0.0;
      double m = h ? v * v : v;
#pragma unroll
      for (int q = 16; q >= 1; q >>= 1) m += __shfl_xor(m, q, 64);
      if (slot == 0) tiles[(int64_t)(h * O + j) * ntiles + tile] = m;
    }
  }
}

}  // namespace

struct lz_rms {
  int dim;
  int device;
  hipStream_t stream;
  double* state;    // mean[dim], var[dim], count
  double* partial;  // [kRmsMaxBlocks][2*dim]
  double* tiles;    // lz_rms_update_obs: [2*dim][ntiles] tile moments + [2*dim+1] snapshot
  int64_t tiles_n;  // doubles allocated
};

#define RMS_HIP(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return rfail(LZ_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

namespace lz {

int rms_dim(const lz_rms* r) { return r->dim; }
int rms_device(const lz_rms* r) { return r->device; }
double* rms_state(lz_rms* r) { return r->state; }

int launch_rms_update(lz_rms* r, const double* moments, void* stream) {
  const int D = r->dim;
  hipLaunchKernelGGL(k_rms_update, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     r->state, r->state + D, r->state + 2 * D, moments, D);
  return (int)hipGetLastError();
}

// row workgroups of the normalise pass: 512 (two per CU), LZ_VN_APPLY_BLOCKS for A/B
static int vn_apply_blocks() {
  static const int b = [] {
    const char* e = std::getenv("LZ_VN_APPLY_BLOCKS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 512;
  }();
  return b;
}

int launch_vn_apply(int f64, int O, int64_t n, const void* obs, const void* rew,
                    const uint8_t* done, const void* term, const int32_t* n_done,
                    double* obs_state, double* ret_state, int norm_obs, int norm_rew,
                    double eps, double clip_obs, double clip_rew, float* obs_n, float* rew_n,
                    uint8_t* dones, float* term_n, const VnUpdate& upd, const int32_t* counter,
                    int32_t* n_done_out, void* stream) {
  if (n == 0) return 0;
  const int R = (O % 4 == 0) ? 1 : (O % 2 == 0 ? 2 : 4);
  VnApplyArgs p;
  p.n = n;
  p.obs = obs;
  p.rew = rew;
  p.term = term;
  p.done = done;
  p.n_done = n_done;
  p.counter = counter;
  p.n_done_out = n_done_out;
  p.os = obs_state;
  p.rs = ret_state;
  p.upd = upd;
  p.eps = eps;
  p.clip_obs = clip_obs;
  p.clip_rew = clip_rew;
  p.obs_n = obs_n;
  p.rew_n = rew_n;
  p.term_n = term_n;
  p.dones = dones;
  p.norm_obs = norm_obs;
  p.norm_rew = norm_rew;
  p.vec = !f64 && ((uintptr_t)obs % 16 == 0) && ((uintptr_t)obs_n % 16 == 0);
  p.row_tiles = (n + 256 * R - 1) / (256 * R);
  // fused: at most vn_apply_blocks() row workgroups (each reduces the partials once);
  // otherwise one per row tile
  const int64_t cap = upd.part ? vn_apply_blocks() : p.row_tiles;
  p.row_blocks = (int)(p.row_tiles < cap ? p.row_tiles : cap);
  const int tb = term ? (p.row_blocks < 64 ? p.row_blocks : 64) : 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)(p.row_blocks + tb)), block(256);
  // 1: reduce the partials here (fused); 0: publish the done count, no reduction (not
  // training); 2: the split path's round-1 kernel (totals from k_vn_colsum, which also
  // published the done count)
  const int kind = upd.part ? 1 : counter ? 0 : 2;
#define LZ_VN_APPLY(T, O_)                                                                        \
  if (kind == 1) hipLaunchKernelGGL((k_vn_apply<T, O_, true>), grid, block, 0, s, p);             \
  else if (kind == 0) hipLaunchKernelGGL((k_vn_apply<T, O_, false>), grid, block, 0, s, p);       \
  else hipLaunchKernelGGL((k_vn_apply_split<T, O_>), grid, block, 0, s, p);
  switch (O * 2 + (f64 ? 1 : 0)) {
    case 12: LZ_VN_APPLY(float, 6) break;
    case 13: LZ_VN_APPLY(double, 6) break;
    case 16: LZ_VN_APPLY(float, 8) break;
    case 17: LZ_VN_APPLY(double, 8) break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LZ_VN_APPLY
  return (int)hipGetLastError();
}

int launch_vn_tile_update(const double* tiles, int64_t ntiles, int O, double batch,
                          const double* snap, double* state, double* moments, void* stream) {
  hipLaunchKernelGGL(k_vn_tile_update, dim3((unsigned)O), dim3(256), 0, static_cast<hipStream_t>(stream),
                     tiles, ntiles, O, batch, snap, state, moments);
  return (int)hipGetLastError();
}

int launch_obs_tile_moments(const float* x, int64_t n, int O, double* tiles, const double* state,
                            double* snap, void* stream) {
  const int64_t ntiles = (n + kVnTile - 1) / kVnTile;
  const int64_t g = (ntiles + 3) / 4;
  const unsigned grid = (unsigned)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
  hipLaunchKernelGGL(k_obs_tile_moments, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), x,
                     n, O, tiles, state, snap);
  return (int)hipGetLastError();
}

}  // namespace lz

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
  r->tiles = nullptr;
  r->tiles_n = 0;
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
  if (r->tiles) (void)hipFree(r->tiles);
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

lz_status lz_rms_update_obs(lz_rms* r, const float* x, int64_t n, double* moments_out) {
  if (!r || (!x && n > 0)) return rfail(LZ_ERR_INVALID, "NULL argument");
  if (n <= 0) return rfail(LZ_ERR_INVALID, "n must be >= 1");
  RMS_HIP(hipSetDevice(r->device));
  const int D = r->dim;
  if (D > lz::kVnMaxObs) return rfail(LZ_ERR_UNSUPPORTED, "lz_rms_update_obs: dim > %d", lz::kVnMaxObs);
  const int64_t ntiles = (n + lz::kVnTile - 1) / lz::kVnTile;
  const int64_t need = 2 * D * ntiles + 2 * D + 1;
  if (r->tiles_n < need) {
    if (r->tiles) RMS_HIP(hipFree(r->tiles));
    r->tiles = nullptr;
    r->tiles_n = 0;
    if (hipMalloc(reinterpret_cast<void**>(&r->tiles), (size_t)need * sizeof(double)) != hipSuccess)
      return rfail(LZ_ERR_OOM, "lz_rms_update_obs: tile scratch (%lld doubles)", (long long)need);
    r->tiles_n = need;
  }
  double* snap = r->tiles + 2 * D * ntiles;
  RMS_HIP((hipError_t)lz::launch_obs_tile_moments(x, n, D, r->tiles, r->state, snap, r->stream));
  RMS_HIP((hipError_t)lz::launch_vn_tile_update(r->tiles, ntiles, D, (double)n, snap, r->state,
                                                moments_out, r->stream));
  return LZ_OK;
}

}  // extern "C"
