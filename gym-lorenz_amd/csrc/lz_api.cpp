// C-ABI of libgym_lorenz_amd.so: handle lifetime, validation, device buffers and
// launch plumbing around the kernels in lz_kernels.hip.  See include/lorenz_env.h.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <mutex>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "lorenz_env.h"
#include "lz_internal.h"

using lz::KArgs;

namespace {

thread_local std::string g_err;

lz_status fail(lz_status s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
lz_status fail(lz_status s, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(LZ_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

struct SysDesc {
  int state_dim, action_dim, obs_dim, init_dim, n_planes;
  int step_plane;
};

SysDesc describe(int system) {
  switch (system) {
    case LZ_SYS_LORENZ3: return {3, 3, 6, 3, 4, LZ_L3_STEP};
    case LZ_SYS_LORENZ4: return {8, 3, 8, 8, 9, LZ_L4_STEP};
    case LZ_SYS_PMSM: return {6, 2, 6, 6, 11, LZ_PMSM_STEP};
    case LZ_SYS_T1: return {3, 2, 6, 3, 4, LZ_T1_STEP};
    case LZ_SYS_T2: return {8, 3, 8, 8, 9, LZ_T2_STEP};
    case LZ_SYS_TP: return {6, 2, 6, 6, 7, LZ_TP_STEP};
    case LZ_SYS_SC: return {3, 2, 6, 3, 4, LZ_SC_STEP};
    default: return {6, 2, 6, 7, 10, LZ_HR_STEP};
  }
}

// element size of plane p (T planes, f32 planes, i32 planes)
int plane_elem(int system, int f64, int p) {
  const SysDesc d = describe(system);
  if (p < 0 || p >= d.n_planes) return 0;
  if (p == d.step_plane) return 4;
  const int t = f64 ? 8 : 4;
  switch (system) {
    case LZ_SYS_PMSM: return 4;                   // float32 / int32 throughout
    case LZ_SYS_HR: return p <= LZ_HR_SIGMA ? t : 4;  // filtered_action is float32
    default: return t;
  }
}

}  // namespace

namespace lz {
lz_status set_error(lz_status s, const char* msg) {
  g_err = msg;
  return s;
}
}  // namespace lz

struct lz_handle {
  lz_config cfg;
  SysDesc desc;
  int f64;
  hipStream_t stream;
  void* planes[lz::kMaxPlanes];
  int32_t* counters;  // [2] compact-list cursors, ping-pong by call parity
  uint64_t* ticks;    // [2] device-resident call counter (RNG counter), ping-pong
  float* bc;          // PMSM bias-correction pairs [bc_len][2]
  int32_t bc_len;
  int parity;         // which slot of counters/ticks the next launch reads
  int count_steps;
  int32_t max_steps;
  bool was_reset;
  int num_cus;         // compute units of the device (policy rollout grid)
  double* pol_part;    // policy rollout obs-moment partials (lazily allocated)
  int64_t pol_part_n;  // doubles allocated
  // lz_policy_step_f32 (SB3-exact VecNormalize): tile moments [2 O][ntiles] + the
  // statistics snapshot [2 O + 1], the raw terminal-obs carry [N, O], the collect's
  // compact-list cursor (+ one spare int), all lazily allocated
  double* ps_tiles;
  float* ps_term;
  int32_t* ps_cursor;
  int32_t ps_next_k;   // the step lz_policy_step_f32 expects next (-1: none, start at 0)
  uint64_t ps_gen;     // gen right after its previous step
  uint8_t* vn_ws;      // lz_step_vecnorm moment partials (lazily allocated)
  int vn_pending;      // lz_step_vecnorm left totals for lz_vecnorm_apply's updates
  int32_t* vn_nd_out;  // lz_step_vecnorm's n_done_out, published by lz_vecnorm_apply
  int32_t* vn_counter; // ... from this done cursor (the step's)
  uint64_t gen;        // launches on the handle (every parity flip)
  uint64_t vn_gen;     // gen right after the lz_step_vecnorm that set vn_pending / vn_nd_out
  uint8_t* hs_pin;     // lz_step_host: mapped host staging (actions | noise || obs | rew | done)
  uint8_t* hs_dev;     // lz_step_host: its device address
  size_t hs_in, hs_out;  // bytes of the input / output parts
  // lz_resident_step: mailbox in mapped coherent host memory (cmd | resp | act | noise
  // || obs | rew | done || published state planes) and its device address
  uint8_t* rs_pin;
  uint8_t* rs_dev;
  bool rs_member;       // registered with its device's resident server
  bool rs_active;       // ... whose launch may be running
  bool rs_pub_valid;    // the published planes are this launch's (a request was served)
  int rs_use_noise;     // serving injected noise
  int64_t rs_seq;       // number of the last request served (after the reply)
  int64_t rs_posted;    // number of the last request posted
  uint64_t rs_line[lz::kRsLineWords];  // the granules of its request line as last posted
  int rs_slot;          // its request line in the server (= its wave)
  // one env: the reply arrives as tagged granules (lz_internal.h ResBox::reply); the data
  // words of the last accepted reply (the published state for lz_resident_read_state)
  uint32_t rs_rep[lz::kRsReplyWords];
};

// Stop the resident step server serving the handle (if it runs) and wait for it: every
// other call on the handle starts with this, so the server's register-held state is
// back in the planes and the handle's stream ordering is the plain one again.
// (rs_member changes only in calls on this handle; rs_active -- another thread's
// lz_resident_step may relaunch the server with this handle -- is read under the lock)
#define RESIDENT_QUIESCE(h)                           \
  do {                                                \
    if ((h)->rs_member) {                             \
      const lz_status q_ = resident_quiesce(h);       \
      if (q_ != LZ_OK) return q_;                     \
    }                                                 \
  } while (0)

extern "C" {

static lz_status resident_quiesce(lz_handle* h);
static void resident_leave(lz_handle* h);

int32_t lz_abi_version(void) { return LZ_ABI_VERSION; }

const char* lz_last_error(void) { return g_err.c_str(); }

lz_status lz_config_init(lz_config* cfg, int32_t system) {
  if (!cfg) return fail(LZ_ERR_INVALID, "cfg is NULL");
  std::memset(cfg, 0, sizeof *cfg);
  cfg->system = system;
  cfg->dtype = LZ_DTYPE_F32;
  cfg->num_envs = 1;
  cfg->t_done_step = -1;
  double* p = cfg->params;
  switch (system) {
    case LZ_SYS_LORENZ3:  // dynamic.py:31-33 (u, i, o), :73-75 (0.01), :11-12 (+-500)
      p[0] = 10; p[1] = 28; p[2] = 8.0 / 3; p[3] = 0.01; p[4] = 500; p[5] = 10;  // T_end :86
      break;
    case LZ_SYS_LORENZ4:  // lorenz_env_transient.py:270-273, :327-330 (0.001), :255-256, :369
      p[0] = 10; p[1] = 8.0 / 3; p[2] = 28; p[3] = 0.001; p[4] = 2; p[5] = 5;
      break;
    case LZ_SYS_PMSM:  // lorenz_env_try_pmsm.py:12-14, :20-23, :39, :50, :113, :174
      p[0] = 5.46; p[1] = 20.0; p[2] = 0.001; p[3] = 50; p[4] = 0.001; p[5] = 0.9;
      p[6] = 0.999; p[7] = 1e-8; p[8] = 5.0; p[9] = 2000; p[10] = 1000;
      cfg->alpha = 0.5f;  // :9
      break;
    case LZ_SYS_HR:  // lorenz_env_try.py:32-36, :40, :174
      p[0] = 1.0; p[1] = 3.0; p[2] = 1.0; p[3] = 5.0; p[4] = 0.006; p[5] = 4.0; p[6] = 3.2;
      p[7] = -1.6; p[8] = 0.001; p[9] = 50.0; p[10] = 20.0; p[11] = 0.95; p[12] = 70.0;
      break;
    case LZ_SYS_T1:  // lorenz_env_transient1.py:21-22 (clip), :38-39 (a, b), :84 (0.01), :100
      p[0] = 5.46; p[1] = 20; p[3] = 0.01; p[4] = 10; p[5] = 10;
      break;
    case LZ_SYS_T2:  // lorenz_env_transient2.py:118-119, :133-137, :193 (0.001), :211 (100),
                     // :192 (0.01), :235
      p[0] = 30; p[1] = 1; p[2] = 36; p[3] = 0.001; p[4] = 2; p[5] = 5; p[6] = 0.5;
      p[7] = 0.003; p[8] = 100; p[9] = 0.01;
      break;
    case LZ_SYS_TP:  // lorenz_env_transient_pmsm.py:22-23, :40-41, :91 (20), :97, :129, :86
      p[0] = 5.46; p[1] = 20; p[2] = 20; p[3] = 0.01; p[4] = 2; p[5] = 5; p[6] = 3;
      cfg->flags = LZ_FLAG_ADD_NOISE;
      break;
    case LZ_SYS_SC:  // lorenz_singlecontrol.py:100-101, :117-118, :121, :147, :154, :169
      p[0] = 5.46; p[1] = 20; p[3] = 0.01; p[4] = 100; p[5] = 1000; p[6] = 3;
      p[7] = 25; p[8] = 1; p[9] = -1;
      cfg->flags = LZ_FLAG_ADD_NOISE;
      break;
    default:
      return fail(LZ_ERR_INVALID, "unknown system %d", system);
  }
  return LZ_OK;
}

lz_status lz_create(const lz_config* cfg_in, lz_handle** out) {
  if (!cfg_in || !out) return fail(LZ_ERR_INVALID, "cfg/out is NULL");
  *out = nullptr;
  lz_config cfg = *cfg_in;
  if (cfg.system < LZ_SYS_LORENZ3 || cfg.system > LZ_SYS_SC)
    return fail(LZ_ERR_INVALID, "unknown system %d", cfg.system);
  if (cfg.dtype != LZ_DTYPE_F32 && cfg.dtype != LZ_DTYPE_F64)
    return fail(LZ_ERR_INVALID, "unknown dtype %d", cfg.dtype);
  if (cfg.system == LZ_SYS_PMSM && cfg.dtype != LZ_DTYPE_F32)
    return fail(LZ_ERR_UNSUPPORTED, "PMSM is float32 only (the reference computes it in float32)");
  if (cfg.num_envs <= 0 || cfg.num_envs > (int64_t)INT32_MAX)
    return fail(LZ_ERR_INVALID, "num_envs must be in [1, 2^31-1], got %lld", (long long)cfg.num_envs);
  if (cfg.global_env_offset < 0 || cfg.global_env_offset + cfg.num_envs > (int64_t(1) << 40))
    return fail(LZ_ERR_INVALID, "global env ids must lie in [0, 2^40)");
  if (cfg.max_episode_steps < 0) return fail(LZ_ERR_INVALID, "max_episode_steps < 0");
  if (cfg.integrator != LZ_INT_EULER && cfg.integrator != LZ_INT_RK4)
    return fail(LZ_ERR_INVALID, "unknown integrator %d", cfg.integrator);
  if (cfg.integrator == LZ_INT_RK4 && cfg.system != LZ_SYS_LORENZ3 && cfg.system != LZ_SYS_LORENZ4 &&
      cfg.system != LZ_SYS_HR)
    return fail(LZ_ERR_UNSUPPORTED, "the RK4 integrator mode is LORENZ3 / LORENZ4 only (HR is RK4 already)");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (cfg.device < 0 || cfg.device >= ndev)
    return fail(LZ_ERR_INVALID, "device %d out of range (%d devices)", cfg.device, ndev);
  HIP_TRY(hipSetDevice(cfg.device));

  lz_handle* h = new (std::nothrow) lz_handle();
  if (!h) return fail(LZ_ERR_OOM, "host allocation failed");
  std::memset(h->planes, 0, sizeof h->planes);
  h->counters = nullptr;
  h->bc = nullptr;
  h->desc = describe(cfg.system);
  h->f64 = cfg.dtype == LZ_DTYPE_F64;
  h->stream = nullptr;
  h->ticks = nullptr;
  h->parity = 0;
  h->was_reset = false;
  h->pol_part = nullptr;
  h->pol_part_n = 0;
  h->num_cus = 0;
  if (hipDeviceGetAttribute(&h->num_cus, hipDeviceAttributeMultiprocessorCount, cfg.device) !=
          hipSuccess ||
      h->num_cus <= 0)
    h->num_cus = 256;

  // The reference's float accumulator 't += dt; done = t == T' (dynamic.py:85-89,
  // lorenz_env_transient.py:364,369): replay it on the host in double, exactly as
  // Python does, and record the step at which it fires (-1: never -- the case for the
  // reference constants).
  cfg.t_done_step = -1;
  if (cfg.system != LZ_SYS_PMSM && cfg.system != LZ_SYS_HR) {  // dt = p[3], T = p[5]
    const double dt = cfg.params[3], tend = cfg.params[5];
    double t = 0.0;
    for (int32_t k = 1; k <= 100000000; ++k) {
      t = t + dt;
      if (t == tend) { cfg.t_done_step = k; break; }
      if (t > tend) break;
    }
  }
  int32_t limit = cfg.max_episode_steps;
  if (cfg.system == LZ_SYS_PMSM) {  // own truncation current_step >= max_steps (:179)
    const int32_t own = (int32_t)cfg.params[9];
    if (own > 0 && (limit == 0 || own < limit)) limit = own;
  }
  h->max_steps = limit;
  h->count_steps = (limit > 0 || cfg.t_done_step >= 0) ? 1 : 0;
  h->cfg = cfg;

  const int64_t n = cfg.num_envs;
  for (int p = 0; p < h->desc.n_planes; ++p) {
    const int es = plane_elem(cfg.system, h->f64, p);
    if (hipMalloc(&h->planes[p], (size_t)n * es) != hipSuccess) {
      lz_destroy(h);
      return fail(LZ_ERR_OOM, "hipMalloc of state plane %d (%lld x %d B) failed", p, (long long)n, es);
    }
    if (hipMemset(h->planes[p], 0, (size_t)n * es) != hipSuccess) {
      lz_destroy(h);
      return fail(LZ_ERR_HIP, "hipMemset of state plane %d failed", p);
    }
  }
  if (hipMalloc(reinterpret_cast<void**>(&h->counters), 2 * sizeof(int32_t)) != hipSuccess ||
      hipMemset(h->counters, 0, 2 * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->ticks), 2 * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(h->ticks, 0, 2 * sizeof(uint64_t)) != hipSuccess) {
    lz_destroy(h);
    return fail(LZ_ERR_OOM, "counter allocation failed");
  }
  h->bc_len = 0;
  if (cfg.system == LZ_SYS_PMSM) {
    // (float)(1 - beta**k) exactly as the reference's python-float expression
    // (lorenz_env_try_pmsm.py:130-131): computed here with the same libm pow()
    // CPython uses, tabulated until both saturate at 1.0f for good.
    const double b1 = cfg.params[5], b2 = cfg.params[6];
    std::vector<float> t1, t2;
    int32_t k = 0, run = 0;
    while (true) {
      const float v1 = (float)(1.0 - std::pow(b1, (double)k));
      const float v2 = (float)(1.0 - std::pow(b2, (double)k));
      t1.push_back(v1);
      t2.push_back(v2);
      run = (v1 == 1.0f && v2 == 1.0f) ? run + 1 : 0;
      ++k;
      if (run >= 64 || k >= (1 << 22)) break;
    }
    h->bc_len = (int32_t)t1.size();
    if (hipMalloc(reinterpret_cast<void**>(&h->bc), 2 * t1.size() * sizeof(float)) != hipSuccess) {
      lz_destroy(h);
      return fail(LZ_ERR_OOM, "bias table allocation failed");
    }
    // interleaved pairs [k] = {1 - beta1**k, 1 - beta2**k}: one scalar load per step
    std::vector<float> tb(2 * t1.size());
    for (size_t j = 0; j < t1.size(); ++j) {
      tb[2 * j] = t1[j];
      tb[2 * j + 1] = t2[j];
    }
    if (hipMemcpy(h->bc, tb.data(), tb.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
      lz_destroy(h);
      return fail(LZ_ERR_HIP, "bias table upload failed");
    }
  }
  *out = h;
  return LZ_OK;
}

lz_status lz_destroy(lz_handle* h) {
  if (!h) return LZ_OK;
  (void)hipSetDevice(h->cfg.device);
  if (h->rs_member) resident_leave(h);
  if (h->rs_pin) (void)hipHostFree(h->rs_pin);
  for (int p = 0; p < lz::kMaxPlanes; ++p)
    if (h->planes[p]) (void)hipFree(h->planes[p]);
  if (h->counters) (void)hipFree(h->counters);
  if (h->ticks) (void)hipFree(h->ticks);
  if (h->bc) (void)hipFree(h->bc);
  if (h->pol_part) (void)hipFree(h->pol_part);
  if (h->ps_tiles) (void)hipFree(h->ps_tiles);
  if (h->ps_term) (void)hipFree(h->ps_term);
  if (h->ps_cursor) (void)hipFree(h->ps_cursor);
  if (h->vn_ws) (void)hipFree(h->vn_ws);
  if (h->hs_pin) (void)hipHostFree(h->hs_pin);  // hs_dev is its mapped device address
  delete h;
  return LZ_OK;
}

lz_status lz_io_sizes_for(const lz_config* cfg, int32_t K, int64_t cap, lz_io_sizes* out) {
  if (!cfg || !out) return fail(LZ_ERR_INVALID, "config/out is NULL");
  if (cfg->system < LZ_SYS_LORENZ3 || cfg->system > LZ_SYS_SC) return fail(LZ_ERR_INVALID, "unknown system");
  if (cfg->num_envs < 1 || K < 0 || cap < 0) return fail(LZ_ERR_INVALID, "num_envs >= 1, K >= 0, cap >= 0");
  const SysDesc d = describe(cfg->system);
  const int64_t n = cfg->num_envs, steps = K > 0 ? K : 1;
  const int64_t t = (cfg->dtype == LZ_DTYPE_F64 && cfg->system != LZ_SYS_PMSM) ? 8 : 4;
  const bool needs_act = cfg->system != LZ_SYS_LORENZ4 && cfg->system != LZ_SYS_SC;
  std::memset(out, 0, sizeof *out);
  out->actions = needs_act ? steps * n * d.action_dim * 4 : 0;
  out->noise = K > 0 ? 0 : n * 3 * 8;
  out->obs = steps * n * d.obs_dim * t;
  out->rew = steps * n * t;
  out->done = steps * n;
  out->done_idx = K > 0 ? cap * 8 : n * 4;
  out->terminal_obs = (K > 0 ? cap : n) * d.obs_dim * t;
  out->n_done = 4;
  return LZ_OK;
}

lz_status lz_get_info(const lz_handle* h, lz_info* info) {
  if (!h || !info) return fail(LZ_ERR_INVALID, "handle/info is NULL");
  std::memset(info, 0, sizeof *info);
  const SysDesc& d = h->desc;
  info->state_dim = d.state_dim;
  info->action_dim = d.action_dim;
  info->obs_dim = d.obs_dim;
  info->init_dim = d.init_dim;
  info->n_planes = d.n_planes;
  info->counts_steps = h->count_steps;
  // algorithmic HBM bytes per env per lz_step (what roofline.achieved counts):
  // sio = state planes read + written, io = actions + obs + reward + done
  const int t = h->f64 ? 8 : 4;
  int sio = 0, io = 0;
  switch (h->cfg.system) {
    case LZ_SYS_LORENZ3: sio = 2 * 3 * t; io = 3 * 4 + 6 * t + t + 1; break;  // 24 + 41 (f32)
    case LZ_SYS_LORENZ4: sio = 2 * 8 * t; io = 8 * t + t + 1; break;          // 64 + 37, no act
    case LZ_SYS_PMSM:  // s1,s2 + lambda,m,v + adam_step + current_step
      sio = 2 * (6 * 4 + 3 * 4 + 4 + 4); io = 2 * 4 + 6 * 4 + 4 + 1; break;   // 88 + 37
    case LZ_SYS_HR:
      sio = 2 * 6 * t;
      if (h->cfg.flags & LZ_FLAG_ADD_NOISE) sio += t;        // sigma read
      if (h->cfg.flags & LZ_FLAG_ADD_FILTER) sio += 2 * 2 * 4;  // filtered_action
      io = 2 * 4 + 6 * t + t + 1;
      break;
    case LZ_SYS_T1: sio = 2 * 3 * t; io = 2 * 4 + 6 * t + t + 1; break;
    case LZ_SYS_T2: sio = 2 * 8 * t; io = 3 * 4 + 8 * t + t + 1; break;
    case LZ_SYS_TP: sio = 2 * 6 * t; io = 2 * 4 + 6 * t + t + 1; break;
    case LZ_SYS_SC: sio = 2 * 3 * t; io = 6 * t + t + 1; break;  // no action
  }
  if (h->count_steps && h->cfg.system != LZ_SYS_PMSM) sio += 8;
  const int b = sio + io;
  info->state_io_bytes = sio;
  info->bytes_per_env_step = b;
  return LZ_OK;
}

lz_status lz_get_config(const lz_handle* h, lz_config* cfg) {
  if (!h || !cfg) return fail(LZ_ERR_INVALID, "handle/cfg is NULL");
  *cfg = h->cfg;
  return LZ_OK;
}

lz_status lz_set_stream(lz_handle* h, void* stream) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  h->stream = static_cast<hipStream_t>(stream);
  return LZ_OK;
}

lz_status lz_set_seed(lz_handle* h, uint64_t seed) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  h->cfg.seed = seed;
  // rewind the RNG call counter (both ping-pong slots; stream-ordered after any
  // launch already queued): seed(s) + reset() is then reproducible
  HIP_TRY(hipSetDevice(h->cfg.device));
  HIP_TRY(hipMemsetAsync(h->ticks, 0, 2 * sizeof(uint64_t), h->stream));
  return LZ_OK;
}

lz_status lz_sync(lz_handle* h) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  HIP_TRY(hipSetDevice(h->cfg.device));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return LZ_OK;
}

// the launchers' system argument: the system, + kSysRK4 for the RK4 integrator mode
static int sys_key(const lz_handle* h) {
  const int s = h->cfg.system;
  return (h->cfg.integrator == LZ_INT_RK4 && (s == LZ_SYS_LORENZ3 || s == LZ_SYS_LORENZ4)) ? s + lz::kSysRK4
                                                                                            : s;
}

static void fill_common(const lz_handle* h, KArgs& a) {
  std::memset(&a, 0, sizeof a);
  for (int p = 0; p < lz::kMaxPlanes; ++p) a.pl[p] = h->planes[p];
  a.n = h->cfg.num_envs;
  a.gid0 = h->cfg.global_env_offset;
  a.seed = h->cfg.seed;
  a.tick_in = h->ticks + h->parity;
  a.tick_out = h->ticks + (1 - h->parity);
  a.tick_adv = 1;
  a.bc = h->bc;
  a.bc_len = h->bc_len;
  a.max_steps = h->max_steps;
  a.t_done_step = h->cfg.t_done_step;
  a.count_steps = h->count_steps;
  a.flags = h->cfg.flags;
  a.alpha = h->cfg.alpha;
  a.variant = h->cfg.reserved[0];
  a.num_cus = h->num_cus;
  for (int j = 0; j < LZ_MAX_PARAMS; ++j) a.prm[j] = h->cfg.params[j];
  a.counter = h->counters + h->parity;
  a.counter_next = h->counters + (1 - h->parity);
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

lz_status lz_reset(lz_handle* h, const uint8_t* mask, const void* init, void* obs_out) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  HIP_TRY(hipSetDevice(h->cfg.device));
  KArgs a;
  fill_common(h, a);
  a.mask = mask;
  a.init = init;
  a.obs = obs_out;
  const int e = lz::launch_reset(sys_key(h), h->f64, a, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "reset launch: %s", hipGetErrorString((hipError_t)e));
  h->parity ^= 1;
  ++h->gen;
  h->was_reset = true;
  return LZ_OK;
}

lz_status lz_step(lz_handle* h, const void* actions, const double* noise, void* obs_out,
                  void* rew_out, uint8_t* done_out, int32_t* done_idx_out, void* terminal_obs_out,
                  int32_t* n_done_out) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_step before the first lz_reset");
  // LORENZ4 ignores its action, SC takes none
  const bool needs_act = h->cfg.system != LZ_SYS_LORENZ4 && h->cfg.system != LZ_SYS_SC;
  if ((needs_act && !actions) || !obs_out || !rew_out || !done_out)
    return fail(LZ_ERR_INVALID, "actions/obs_out/rew_out/done_out must be non-NULL");
  if ((done_idx_out == nullptr) != (terminal_obs_out == nullptr))
    return fail(LZ_ERR_INVALID, "done_idx_out and terminal_obs_out go together");
  HIP_TRY(hipSetDevice(h->cfg.device));
  KArgs a;
  fill_common(h, a);
  a.act = actions;
  a.noise = noise;
  a.obs = obs_out;
  a.rew = rew_out;
  a.done = done_out;
  a.done_idx32 = done_idx_out;
  a.term_obs = terminal_obs_out;
  // full 256-env blocks start at 256*A*4 / 256*O*sizeof(T) byte offsets: only the
  // base pointers need 16-B alignment (ragged tail blocks take the scalar path)
  a.vec_ok = (!needs_act || aligned16(actions)) && aligned16(obs_out);
  const int e = lz::launch_step(sys_key(h), h->f64, a, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "step launch: %s", hipGetErrorString((hipError_t)e));
  if (n_done_out)
    HIP_TRY(hipMemcpyAsync(n_done_out, a.counter, sizeof(int32_t), hipMemcpyDeviceToDevice, h->stream));
  h->parity ^= 1;
  ++h->gen;
  return LZ_OK;
}

static size_t align16(size_t b) { return (b + 15) & ~(size_t)15; }

lz_status lz_step_host(lz_handle* h, const float* actions, const double* noise, void* obs_out,
                       void* rew_out, uint8_t* done_out) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_step_host before the first lz_reset");
  const bool needs_act = h->cfg.system != LZ_SYS_LORENZ4 && h->cfg.system != LZ_SYS_SC;
  if ((needs_act && !actions) || !obs_out || !rew_out || !done_out)
    return fail(LZ_ERR_INVALID, "actions/obs_out/rew_out/done_out must be non-NULL");
  HIP_TRY(hipSetDevice(h->cfg.device));
  const int64_t n = h->cfg.num_envs;
  const size_t es = h->f64 ? 8 : 4;
  const size_t b_act = (size_t)n * h->desc.action_dim * 4, b_nz = (size_t)n * 3 * 8;
  const size_t b_obs = (size_t)n * h->desc.obs_dim * es, b_rew = (size_t)n * es;
  const size_t o_nz = align16(b_act), in = align16(o_nz + b_nz);
  const size_t o_rew = align16(b_obs), o_done = align16(o_rew + b_rew), out = o_done + (size_t)n;
  if (!h->hs_pin) {
    // host memory mapped into the device's address space: the step kernel reads the
    // actions and writes its outputs over PCIe, no copy launches
    if (hipHostMalloc(reinterpret_cast<void**>(&h->hs_pin), in + out,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(LZ_ERR_OOM, "lz_step_host: mapped staging (%zu B)", in + out);
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, h->hs_pin, 0) != hipSuccess || !dp)
      return fail(LZ_ERR_HIP, "lz_step_host: no device address for the mapped staging");
    h->hs_dev = static_cast<uint8_t*>(dp);
    h->hs_in = in;
    h->hs_out = out;
  }
  if (needs_act) std::memcpy(h->hs_pin, actions, b_act);
  if (noise) std::memcpy(h->hs_pin + o_nz, noise, b_nz);
  uint8_t* d_out = h->hs_dev + in;
  const lz_status st = lz_step(h, needs_act ? h->hs_dev : nullptr,
                               noise ? reinterpret_cast<const double*>(h->hs_dev + o_nz) : nullptr,
                               d_out, d_out + o_rew, d_out + o_done, nullptr, nullptr, nullptr);
  if (st != LZ_OK) return st;
  HIP_TRY(hipStreamSynchronize(h->stream));  // (a hipStreamQuery spin measured no faster)
  std::memcpy(obs_out, h->hs_pin + in, b_obs);
  std::memcpy(rew_out, h->hs_pin + in + o_rew, b_rew);
  std::memcpy(done_out, h->hs_pin + in + o_done, (size_t)n);
  return LZ_OK;
}

// ---- resident step server (lz_resident_step; lz_internal.h ResBox / ResMember)
// mailbox layout (bytes): resp int64 @128 (own cache line; the request itself goes to the
// server's request line of the handle), actions float32 [n, A] @256 and noise double
// [n, 3] @kRsNoise (the mailbox path: inputs that do not fit in the line), then obs |
// reward | done @kRsOut, then the published state planes (plane p at rs_pub_off + p *
// kRsPubStride(n))
constexpr size_t kRsResp = 128, kRsAct = 256;
constexpr size_t kRsNoise = kRsAct + 64 * 4 * 4, kRsOut = kRsNoise + 64 * 3 * 8;
constexpr int kRsMaxEnvs = 64;

static size_t rs_rew_off(const lz_handle* h) {
  return kRsOut + align16((size_t)h->cfg.num_envs * h->desc.obs_dim * (h->f64 ? 8 : 4));
}
static size_t rs_done_off(const lz_handle* h) {
  return rs_rew_off(h) + align16((size_t)h->cfg.num_envs * (h->f64 ? 8 : 4));
}
static size_t rs_pub_stride(const lz_handle* h) { return align16((size_t)h->cfg.num_envs * 8); }
static size_t rs_pub_off(const lz_handle* h) { return rs_done_off(h) + align16((size_t)h->cfg.num_envs); }
static size_t rs_reply_off(const lz_handle* h) {
  return (rs_pub_off(h) + (size_t)h->desc.n_planes * rs_pub_stride(h) + 63) & ~(size_t)63;
}
static size_t rs_bytes(const lz_handle* h) { return rs_reply_off(h) + lz::kRsReplyWords * 8; }

// Word layout of a one-env handle's tagged reply (ResBox::rep_*): the 8-byte items first
// (float64 planes, then float64 obs and reward), then the 4-byte ones (float32 / int32
// planes, float32 obs and reward), then the done byte as a word.  Returns the word count.
struct RsReplyLayout {
  int32_t obs, rew, done, pub[lz::kMaxPlanes];
};
static int rs_reply_layout(const lz_handle* h, RsReplyLayout& L) {
  int c = 0;
  const int O = h->desc.obs_dim;
  for (int p = 0; p < lz::kMaxPlanes; ++p) L.pub[p] = -1;
  for (int pass = 8; pass >= 4; pass -= 4) {
    for (int p = 0; p < h->desc.n_planes; ++p)
      if (plane_elem(h->cfg.system, h->f64, p) == pass) {
        L.pub[p] = c;
        c += pass / 4;
      }
    if ((h->f64 ? 8 : 4) == pass) {
      L.obs = c;
      c += O * pass / 4;
      L.rew = c;
      c += pass / 4;
    }
  }
  L.done = c++;
  return c;
}
// Every system today fits (worst case 12 float64 planes + 8 float64 obs + reward + done =
// 43 words); a layout that would not fit the reply's kRsReplyWords granules (the host's
// rwords[] and ResShared::rep) takes the mailbox path instead of overflowing them.
static_assert(lz::kMaxPlanes * 2 + 2 * lz::kVnMaxObs + 3 <= lz::kRsReplyWords,
              "the tagged reply of a one-env handle must fit kRsReplyWords granules");
static bool rs_reply_mode(const lz_handle* h) {
  if (h->cfg.num_envs != 1) return false;
  RsReplyLayout L;
  return rs_reply_layout(h, L) <= lz::kRsReplyWords;
}

static volatile int64_t* rs_word(const lz_handle* h, size_t off) {
  return reinterpret_cast<volatile int64_t*>(h->rs_pin + off);
}

// One server per device: the registered handles, the stream (one hardware queue) its
// launch polls on, the member table it reads.  g_rs_mu guards every field and the
// membership; calls on different handles may come from different threads.
constexpr int kRsMaxDevices = 64;
struct RsServer {
  bool init;
  bool active;           // a launch may be running
  int n;
  lz_handle* members[lz::kRsMaxHandles];
  hipStream_t stream;
  hipEvent_t ev;
  lz::ResMember* table_host;  // pinned staging of the member table
  lz::ResMember* table_dev;
  uint64_t* lines;       // the request lines: 64 B per member (lz_internal.h ResBox;
                         // mapped, coherent host memory, 1 KiB)
  const uint64_t* lines_dev;
  int khz;               // wall-clock rate (ticks per ms)
};

// The idle exit in wall-clock ticks, read from LZ_RESIDENT_IDLE_US at every launch (so a
// process can change it between launches): short by default -- a device-wide synchronize
// (torch.cuda.synchronize()) waits for the idle exit, and a caller that leaves > 1 ms
// between steps pays one relaunch (~20 us)
static uint64_t rs_idle_ticks(const RsServer& sv) {
  const char* e = std::getenv("LZ_RESIDENT_IDLE_US");
  const double us = e ? std::atof(e) : 1000.0;
  return (uint64_t)((us > 0 ? us : 1000.0) * sv.khz / 1000.0);
}
constexpr size_t kRsLinesBytes = 16 * lz::kRsLineWords * sizeof(uint64_t);
static_assert(lz::kRsMaxHandles <= 16, "one request line per member in 1 KiB");
constexpr uint64_t kRsStop = ~0ull;  // granule 0 of any line: every wave leaves

static int rs_act_words(const lz_handle* h) {
  const bool needs_act = h->cfg.system != LZ_SYS_LORENZ4 && h->cfg.system != LZ_SYS_SC;
  return needs_act ? h->desc.action_dim : 0;
}
// data words of a request that travels inside its line (1 env: its actions, then its 3
// float64 noise values as lo / hi halves), or -1 (the mailbox path)
static int rs_inline_words(const lz_handle* h, int use_noise) {
  if (h->cfg.num_envs != 1) return -1;
  const int w = rs_act_words(h) + (use_noise ? 6 : 0);
  return w <= lz::kRsLineWords ? w : -1;
}
static uint64_t rs_granule(int64_t seq, uint32_t data) {
  return ((uint64_t)((uint32_t)seq & lz::kRsTagMask) << 32) | data;
}
// the handle's request line into its slot: every granule one aligned 8-B store (the
// poller validates tags, so the order does not matter; granule 0 last)
static void rs_write_line(RsServer& sv, const lz_handle* h) {
  uint64_t* line = sv.lines + (size_t)h->rs_slot * lz::kRsLineWords;
  for (int g = lz::kRsLineWords - 1; g >= 0; --g) __atomic_store_n(&line[g], h->rs_line[g], __ATOMIC_RELEASE);
}

static std::mutex g_rs_mu;  // trivially destructible
static RsServer g_rs[kRsMaxDevices];

static RsServer& rs_server(const lz_handle* h) { return g_rs[h->cfg.device]; }

static lz_status rs_server_init(RsServer& sv, int device) {
  if (sv.init) return LZ_OK;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
  lz::ResMember* th = nullptr;
  lz::ResMember* td = nullptr;
  uint64_t* lines = nullptr;
  void* lines_dev = nullptr;
  const size_t tb = sizeof(lz::ResMember) * lz::kRsMaxHandles;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&th), tb) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&td), tb) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&lines), kRsLinesBytes,
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(&lines_dev, lines, 0) != hipSuccess || !lines_dev) {
    if (st) (void)hipStreamDestroy(st);
    if (ev) (void)hipEventDestroy(ev);
    if (th) (void)hipHostFree(th);
    if (td) (void)hipFree(td);
    if (lines) (void)hipHostFree(lines);
    return fail(LZ_ERR_OOM, "resident server setup failed");
  }
  std::memset(lines, 0, kRsLinesBytes);
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
    khz = 100000;
  sv.stream = st;
  sv.ev = ev;
  sv.table_host = th;
  sv.table_dev = td;
  sv.lines = lines;
  sv.lines_dev = static_cast<const uint64_t*>(lines_dev);
  sv.khz = khz;
  sv.n = 0;
  sv.active = false;
  sv.init = true;
  return LZ_OK;
}

// the launch has ended (stop command or idle exit): every member's state is in its
// planes and its tick in the other ping-pong slot
static void rs_server_ended(RsServer& sv) {
  for (int i = 0; i < sv.n; ++i) {
    lz_handle* m = sv.members[i];
    m->rs_active = false;
    m->rs_pub_valid = false;
    m->parity ^= 1;
    ++m->gen;
  }
  sv.active = false;
}

static lz_status rs_server_stop(RsServer& sv) {
  if (!sv.active) return LZ_OK;
  // one line's stop granule makes every wave leave; the granule is restored after
  lz_handle* m0 = sv.members[0];
  __atomic_store_n(&sv.lines[0], kRsStop, __ATOMIC_RELEASE);
  const hipError_t e = hipStreamSynchronize(sv.stream);
  __atomic_store_n(&sv.lines[0], m0->rs_line[0], __ATOMIC_RELEASE);
  rs_server_ended(sv);
  if (e != hipSuccess) return fail(LZ_ERR_HIP, "resident stop: %s", hipGetErrorString(e));
  return LZ_OK;
}

// process exit without lz_destroy: post the stop commands first (an atexit handler
// registered at the first launch runs before the HIP runtime's own exit-time teardown,
// which was registered earlier).  try_lock: a thread that died holding the lock must not
// hang the exit; the servers are then stopped without it.
static void resident_unload() {
  bool locked = false;
  for (int k = 0; k < 100 && !(locked = g_rs_mu.try_lock()); ++k) usleep(100);
  bool any = false;
  for (int d = 0; d < kRsMaxDevices; ++d) {
    RsServer& sv = g_rs[d];
    if (!sv.init || !sv.active || sv.n == 0) continue;
    __atomic_store_n(&sv.lines[0], kRsStop, __ATOMIC_RELEASE);
    any = true;
  }
  if (any) usleep(2000);  // a poll period is ~2 us; the waves exit on sight
  if (locked) g_rs_mu.unlock();
}

static lz_status rs_server_launch(RsServer& sv) {
  for (int i = 0; i < sv.n; ++i) {
    lz_handle* m = sv.members[i];
    lz::ResMember& r = sv.table_host[i];
    std::memset(&r, 0, sizeof r);
    fill_common(m, r.a);
    r.system = sys_key(m);
    r.f64 = m->f64;
    lz::ResBox& box = r.box;
    m->rs_slot = i;
    rs_write_line(sv, m);  // the slot's line holds this member's latest request
    box.inline_words = rs_inline_words(m, m->rs_use_noise);
    box.act_words = rs_act_words(m);
    box.resp = reinterpret_cast<int64_t*>(m->rs_dev + kRsResp);
    box.act = reinterpret_cast<const float*>(m->rs_dev + kRsAct);
    box.noise = reinterpret_cast<const double*>(m->rs_dev + kRsNoise);
    box.obs = m->rs_dev + kRsOut;
    box.rew = m->rs_dev + rs_rew_off(m);
    box.done = m->rs_dev + rs_done_off(m);
    for (int p = 0; p < m->desc.n_planes; ++p) {
      box.pub[p] = m->rs_dev + rs_pub_off(m) + (size_t)p * rs_pub_stride(m);
      box.pub_es[p] = plane_elem(m->cfg.system, m->f64, p);
    }
    box.next = m->rs_seq + 1;  // the requester's pending request, the others' next one
    box.use_noise = m->rs_use_noise;
    for (int p = 0; p < lz::kMaxPlanes; ++p) box.rep_pub[p] = -1;
    if (rs_reply_mode(m)) {
      RsReplyLayout L;
      box.rep_words = rs_reply_layout(m, L);
      box.rep_obs = L.obs;
      box.rep_rew = L.rew;
      box.rep_done = L.done;
      for (int p = 0; p < lz::kMaxPlanes; ++p) box.rep_pub[p] = L.pub[p];
      box.reply = reinterpret_cast<uint64_t*>(m->rs_dev + rs_reply_off(m));
    }
    // after everything already queued on the member's stream (reset, set_state, ...)
    HIP_TRY(hipEventRecord(sv.ev, m->stream));
    HIP_TRY(hipStreamWaitEvent(sv.stream, sv.ev, 0));
  }
  HIP_TRY(hipMemcpyAsync(sv.table_dev, sv.table_host, sizeof(lz::ResMember) * sv.n,
                         hipMemcpyHostToDevice, sv.stream));
  const int e = lz::launch_resident_multi(sv.table_dev, sv.n, sv.lines_dev, rs_idle_ticks(sv), sv.stream);
  if (e != 0) return fail(LZ_ERR_HIP, "resident launch: %s", hipGetErrorString((hipError_t)e));
  sv.active = true;
  for (int i = 0; i < sv.n; ++i) sv.members[i]->rs_active = true;
  static const int registered = std::atexit(resident_unload);
  (void)registered;
  return LZ_OK;
}

static lz_status resident_quiesce(lz_handle* h) {
  std::lock_guard<std::mutex> lk(g_rs_mu);
  if (!h->rs_active) return LZ_OK;
  (void)hipSetDevice(h->cfg.device);
  return rs_server_stop(rs_server(h));
}

// lz_destroy: stop the server if it serves the handle, drop the membership
static void resident_leave(lz_handle* h) {
  std::lock_guard<std::mutex> lk(g_rs_mu);
  RsServer& sv = rs_server(h);
  if (h->rs_active) (void)rs_server_stop(sv);
  for (int i = 0; i < sv.n; ++i)
    if (sv.members[i] == h) {
      sv.members[i] = sv.members[--sv.n];
      sv.members[i]->rs_slot = i;  // (the relaunch rewrites the command line)
      break;
    }
  h->rs_member = false;
}

lz_status lz_resident_step(lz_handle* h, const float* actions, const double* noise, void* obs_out,
                           void* rew_out, uint8_t* done_out) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_resident_step before the first lz_reset");
  const bool needs_act = h->cfg.system != LZ_SYS_LORENZ4 && h->cfg.system != LZ_SYS_SC;
  if ((needs_act && !actions) || !obs_out || !rew_out || !done_out)
    return fail(LZ_ERR_INVALID, "actions/obs_out/rew_out/done_out must be non-NULL");
  const int64_t n = h->cfg.num_envs;
  if (n > kRsMaxEnvs) return fail(LZ_ERR_UNSUPPORTED, "lz_resident_step: at most %d envs", kRsMaxEnvs);
  if (h->cfg.flags & LZ_FLAG_AUTORESET)
    return fail(LZ_ERR_UNSUPPORTED, "lz_resident_step: handles without LZ_FLAG_AUTORESET only");
  HIP_TRY(hipSetDevice(h->cfg.device));
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (h->stream && hipStreamIsCapturing(h->stream, &cap) == hipSuccess &&
      cap != hipStreamCaptureStatusNone)
    return fail(LZ_ERR_STATE, "lz_resident_step: the handle's stream is being captured "
                              "(a synchronous host round trip cannot be captured)");
  const size_t es = h->f64 ? 8 : 4;
  if (!h->rs_pin) {  // built in locals, assigned to the handle once complete
    const size_t bytes = rs_bytes(h);
    uint8_t* pin = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&pin), bytes, hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
      return fail(LZ_ERR_OOM, "lz_resident_step: mailbox (%zu B)", bytes);
    std::memset(pin, 0, bytes);
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, pin, 0) != hipSuccess || !dp) {
      (void)hipHostFree(pin);
      return fail(LZ_ERR_HIP, "lz_resident_step: no device address for the mailbox");
    }
    h->rs_pin = pin;
    h->rs_dev = static_cast<uint8_t*>(dp);
    h->rs_seq = 0;
    h->rs_posted = 0;
  }
  std::unique_lock<std::mutex> lk(g_rs_mu);
  RsServer& sv = rs_server(h);
  {
    const lz_status q = rs_server_init(sv, h->cfg.device);
    if (q != LZ_OK) return q;
  }
  if (!h->rs_member) {
    if (sv.n >= lz::kRsMaxHandles) {
      // more handles than server waves: this one steps by launches (same results)
      lk.unlock();
      return lz_step_host(h, actions, noise, obs_out, rew_out, done_out);
    }
    const lz_status q = rs_server_stop(sv);  // relaunched below with the new member
    if (q != LZ_OK) return q;
    h->rs_slot = sv.n;
    sv.members[sv.n++] = h;
    h->rs_member = true;
  }
  const int use_noise = noise != nullptr;
  if (h->rs_active && use_noise != h->rs_use_noise) {
    const lz_status q = rs_server_stop(sv);
    if (q != LZ_OK) return q;
  }
  h->rs_use_noise = use_noise;
  const int64_t seq = h->rs_seq + 1;
  const int iw = rs_inline_words(h, use_noise);
  uint32_t words[lz::kRsLineWords] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (iw >= 0) {  // the inputs travel in the request line
    const int aw = rs_act_words(h);
    if (aw) std::memcpy(words, actions, (size_t)aw * 4);
    if (noise) std::memcpy(words + aw, noise, 3 * 8);  // little endian: lo, hi halves
  } else {        // the mailbox path: inputs there first, the line's command granule after
    if (needs_act) std::memcpy(h->rs_pin + kRsAct, actions, (size_t)n * h->desc.action_dim * 4);
    if (noise) std::memcpy(h->rs_pin + kRsNoise, noise, (size_t)n * 3 * 8);
  }
  for (int g = 0; g < lz::kRsLineWords; ++g) h->rs_line[g] = rs_granule(seq, words[g]);
  h->rs_posted = seq;
  // (x86 TSO: the mailbox inputs are visible before the granules)
  rs_write_line(sv, h);
  if (!sv.active) {
    const lz_status q = rs_server_launch(sv);
    if (q != LZ_OK) return q;
  }
  volatile int64_t* resp = rs_word(h, kRsResp);
  const bool rep_mode = rs_reply_mode(h);
  RsReplyLayout L;
  const int rw = rep_mode ? rs_reply_layout(h, L) : 0;
  const uint64_t* rep = reinterpret_cast<const uint64_t*>(h->rs_pin + rs_reply_off(h));
  const uint32_t tag = (uint32_t)seq & lz::kRsTagMask;
  uint32_t rwords[lz::kRsReplyWords];
  // the reply is in: the mailbox's resp word, or every tagged granule (each an atomic 8-B
  // read; any granule still from an earlier request fails the check and is read again)
  auto served = [&]() -> bool {
    if (!rep_mode) return __atomic_load_n(const_cast<int64_t*>(resp), __ATOMIC_ACQUIRE) == seq;
    for (int g = rw - 1; g >= 0; --g) {
      const uint64_t v = __atomic_load_n(&rep[g], __ATOMIC_ACQUIRE);
      if ((uint32_t)(v >> 32) != tag) return false;
      rwords[g] = (uint32_t)v;
    }
    return true;
  };
  for (uint32_t spin = 1;; ++spin) {
    if (served()) break;
    if ((spin & 4095u) == 0) {
      // the server may have exited (idle) before it saw this request
      const hipError_t q = hipStreamQuery(sv.stream);
      if (q == hipErrorNotReady) continue;
      if (served()) break;
      rs_server_ended(sv);
      if (q != hipSuccess) return fail(LZ_ERR_HIP, "resident server: %s", hipGetErrorString(q));
      const lz_status r = rs_server_launch(sv);
      if (r != LZ_OK) return r;
    }
    __builtin_ia32_pause();
  }
  h->rs_seq = seq;
  h->rs_pub_valid = true;
  if (rep_mode) {
    std::memcpy(h->rs_rep, rwords, (size_t)rw * 4);
    lk.unlock();
    std::memcpy(obs_out, rwords + L.obs, (size_t)h->desc.obs_dim * es);
    std::memcpy(rew_out, rwords + L.rew, es);
    *done_out = (uint8_t)rwords[L.done];
    return LZ_OK;
  }
  lk.unlock();
  std::memcpy(obs_out, h->rs_pin + kRsOut, (size_t)n * h->desc.obs_dim * es);
  std::memcpy(rew_out, h->rs_pin + rs_rew_off(h), (size_t)n * es);
  std::memcpy(done_out, h->rs_pin + rs_done_off(h), (size_t)n);
  return LZ_OK;
}

lz_status lz_resident_stop(lz_handle* h) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  HIP_TRY(hipSetDevice(h->cfg.device));
  RESIDENT_QUIESCE(h);
  return LZ_OK;
}

lz_status lz_resident_read_state(lz_handle* h, int32_t plane, void* host_dst) {
  if (!h || !host_dst) return fail(LZ_ERR_INVALID, "handle/host_dst is NULL");
  const int es = plane_elem(h->cfg.system, h->f64, plane);
  if (!es) return fail(LZ_ERR_INVALID, "invalid plane %d", plane);
  const size_t bytes = (size_t)h->cfg.num_envs * es;
  {
    std::lock_guard<std::mutex> lk(g_rs_mu);
    if (h->rs_active && h->rs_pub_valid) {  // the server's copy after its last request
      if (rs_reply_mode(h)) {  // ... carried by that request's reply
        RsReplyLayout L;
        rs_reply_layout(h, L);
        std::memcpy(host_dst, h->rs_rep + L.pub[plane], bytes);
      } else {
        std::memcpy(host_dst, h->rs_pin + rs_pub_off(h) + (size_t)plane * rs_pub_stride(h), bytes);
      }
      return LZ_OK;
    }
  }
  RESIDENT_QUIESCE(h);
  HIP_TRY(hipSetDevice(h->cfg.device));
  HIP_TRY(hipMemcpyAsync(host_dst, h->planes[plane], bytes, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return LZ_OK;
}

static lz_status check_vecnorm(const lz_handle* h, const lz_vecnorm* vn) {
  if (!vn || !vn->obs_rms || !vn->ret_rms || !vn->returns)
    return fail(LZ_ERR_INVALID, "vecnorm: obs_rms/ret_rms/returns must be non-NULL");
  if (lz::rms_dim(vn->obs_rms) != h->desc.obs_dim || lz::rms_dim(vn->ret_rms) != 1)
    return fail(LZ_ERR_INVALID, "vecnorm: obs_rms dim %d (obs_dim %d), ret_rms dim %d (1)",
                lz::rms_dim(vn->obs_rms), h->desc.obs_dim, lz::rms_dim(vn->ret_rms));
  if (lz::rms_device(vn->obs_rms) != h->cfg.device || lz::rms_device(vn->ret_rms) != h->cfg.device)
    return fail(LZ_ERR_INVALID, "vecnorm: statistics live on another device");
  if ((vn->flags & LZ_VN_DEFER) && !vn->moments)
    return fail(LZ_ERR_INVALID, "vecnorm: LZ_VN_DEFER needs moments");
  if (h->desc.obs_dim > lz::kVnMaxObs) return fail(LZ_ERR_UNSUPPORTED, "vecnorm: obs too wide");
  return LZ_OK;
}

lz_status lz_step_vecnorm(lz_handle* h, const lz_vecnorm* vn, const void* actions, void* obs_out,
                          void* rew_out, uint8_t* done_out, int32_t* done_idx_out,
                          void* terminal_obs_out, int32_t* n_done_out) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_step_vecnorm before the first lz_reset");
  const lz_status c = check_vecnorm(h, vn);
  if (c != LZ_OK) return c;
  const bool needs_act = h->cfg.system != LZ_SYS_LORENZ4 && h->cfg.system != LZ_SYS_SC;
  if ((needs_act && !actions) || !obs_out || !rew_out || !done_out || !done_idx_out ||
      !terminal_obs_out || !n_done_out)
    return fail(LZ_ERR_INVALID, "actions/obs/rew/done/done_idx/terminal_obs/n_done must be non-NULL");
  HIP_TRY(hipSetDevice(h->cfg.device));
  const int64_t n = h->cfg.num_envs;
  const int64_t n_wg = (n + lz::vn_block(n) - 1) / lz::vn_block(n);
  if (!h->vn_ws) {  // column-major per-workgroup partials, W = 2 (kVnMaxObs + 1) at most,
                    // then the statistics snapshot (sized for the smallest workgroups)
    const int64_t max_wg = (n + lz::kBlock - 1) / lz::kBlock;
    const size_t bytes = (size_t)(max_wg + 3) * 2 * (lz::kVnMaxObs + 1) * sizeof(double);
    if (hipMalloc(reinterpret_cast<void**>(&h->vn_ws), bytes) != hipSuccess)
      return fail(LZ_ERR_OOM, "vecnorm workspace (%zu B)", bytes);
  }
  KArgs a;
  fill_common(h, a);
  a.act = actions;
  a.obs = obs_out;
  a.rew = rew_out;
  a.done = done_out;
  a.done_idx32 = done_idx_out;
  a.term_obs = terminal_obs_out;
  a.vec_ok = (!needs_act || aligned16(actions)) && aligned16(obs_out);
  lz::VArgs v;
  std::memset(&v, 0, sizeof v);
  v.returns = vn->returns;
  v.part = reinterpret_cast<double*>(h->vn_ws);
  v.old = v.part + (size_t)n_wg * 2 * (lz::kVnMaxObs + 1);
  v.tot = v.old + 2 * (lz::kVnMaxObs + 1) + 4;
  v.fused = lz::vn_fused(n);
  v.n_done_out = n_done_out;
  v.obs_state = lz::rms_state(vn->obs_rms);
  v.ret_state = lz::rms_state(vn->ret_rms);
  v.moments = vn->moments;
  v.gamma = vn->gamma;
  v.flags = vn->flags;
  v.n_wg = (int32_t)n_wg;
  const int e = lz::launch_step_vecnorm(sys_key(h), h->f64, a, v, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "step launch: %s", hipGetErrorString((hipError_t)e));
  h->parity ^= 1;
  ++h->gen;
  h->vn_pending = (vn->flags & LZ_VN_TRAINING) && !(vn->flags & LZ_VN_DEFER);
  // without a second launch the done count is published by the paired lz_vecnorm_apply
  const bool second = (vn->flags & LZ_VN_DEFER) || ((vn->flags & LZ_VN_TRAINING) && !v.fused);
  h->vn_nd_out = second ? nullptr : n_done_out;
  h->vn_counter = a.counter;
  h->vn_gen = h->gen;
  return LZ_OK;
}

lz_status lz_vecnorm_apply(lz_handle* h, const lz_vecnorm* vn, const void* obs_raw,
                           const void* rew_raw, const uint8_t* done, float* obs_norm,
                           float* rew_norm, uint8_t* dones_out, const void* terminal_obs_raw,
                           const int32_t* n_done, float* term_norm) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  const lz_status c = check_vecnorm(h, vn);
  if (c != LZ_OK) return c;
  if (!obs_raw || !rew_raw || !obs_norm || !rew_norm)
    return fail(LZ_ERR_INVALID, "obs_raw/rew_raw/obs_norm/rew_norm must be non-NULL");
  if ((done == nullptr) != (dones_out == nullptr))
    return fail(LZ_ERR_INVALID, "done and dones_out go together");
  const bool term = terminal_obs_raw != nullptr || term_norm != nullptr;
  if (term && (!terminal_obs_raw || !term_norm || !n_done))
    return fail(LZ_ERR_INVALID, "terminal_obs_raw, n_done and term_norm go together");
  if ((h->vn_pending || h->vn_nd_out) && h->gen != h->vn_gen) {
    // another launch since lz_step_vecnorm reused its done cursor (and may have
    // overwritten the moment partials): publishing / updating now would be silently wrong
    h->vn_pending = 0;
    h->vn_nd_out = nullptr;
    return fail(LZ_ERR_STATE, "lz_vecnorm_apply must directly follow its lz_step_vecnorm "
                              "(another launch on the handle came in between)");
  }
  HIP_TRY(hipSetDevice(h->cfg.device));
  const int O = h->desc.obs_dim;
  if ((vn->flags & LZ_VN_DEFER) && (vn->flags & LZ_VN_TRAINING)) {
    int e = 0;
    if (vn->flags & LZ_VN_NORM_OBS) e = lz::launch_rms_update(vn->obs_rms, vn->moments, h->stream);
    if (e == 0) e = lz::launch_rms_update(vn->ret_rms, vn->moments + 2 * O + 1, h->stream);
    if (e != 0) return fail(LZ_ERR_HIP, "statistics update: %s", hipGetErrorString((hipError_t)e));
  }
  // the RunningMeanStd updates of the preceding lz_step_vecnorm (training, not
  // deferred) are applied by this normalise pass
  lz::VnUpdate upd{};
  if (h->vn_pending && (vn->flags & LZ_VN_TRAINING) && !(vn->flags & LZ_VN_DEFER)) {
    const int64_t n = h->cfg.num_envs;
    const int64_t n_wg = (n + lz::vn_block(n) - 1) / lz::vn_block(n);
    const double* part = reinterpret_cast<const double*>(h->vn_ws);
    upd.n_wg = (int)n_wg;
    upd.old = part + (size_t)n_wg * 2 * (lz::kVnMaxObs + 1);
    if (lz::vn_fused(n))
      upd.part = part;
    else
      upd.tot = upd.old + 2 * (lz::kVnMaxObs + 1) + 4;
    upd.batch = (double)h->cfg.num_envs;
    upd.upd_obs = (vn->flags & LZ_VN_NORM_OBS) != 0;
  }
  h->vn_pending = 0;
  int32_t* nd_out = h->vn_nd_out;
  const int32_t* counter = nd_out ? h->vn_counter : nullptr;
  h->vn_nd_out = nullptr;
  const int e = lz::launch_vn_apply(
      h->f64, O, h->cfg.num_envs, obs_raw, rew_raw, done, term ? terminal_obs_raw : nullptr,
      term ? n_done : nullptr, lz::rms_state(vn->obs_rms), lz::rms_state(vn->ret_rms),
      (vn->flags & LZ_VN_NORM_OBS) != 0, (vn->flags & LZ_VN_NORM_REWARD) != 0, vn->epsilon,
      vn->clip_obs, vn->clip_reward, obs_norm, rew_norm, dones_out, term ? term_norm : nullptr,
      upd, counter, nd_out, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "normalise launch: %s", hipGetErrorString((hipError_t)e));
  return LZ_OK;
}

lz_status lz_rollout(lz_handle* h, int32_t K, const void* actions, void* obs_out, void* rew_out,
                     uint8_t* done_out, int64_t* done_idx_out, void* terminal_obs_out, int64_t cap,
                     int32_t* n_done_out) {
  if (!h) return fail(LZ_ERR_INVALID, "handle is NULL");
  RESIDENT_QUIESCE(h);
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_rollout before the first lz_reset");
  if (K <= 0) return fail(LZ_ERR_INVALID, "K must be >= 1");
  const bool needs_act = h->cfg.system != LZ_SYS_LORENZ4 && h->cfg.system != LZ_SYS_SC;
  if ((needs_act && !actions) || !obs_out || !rew_out || !done_out)
    return fail(LZ_ERR_INVALID, "actions/obs_out/rew_out/done_out must be non-NULL");
  if ((done_idx_out == nullptr) != (terminal_obs_out == nullptr))
    return fail(LZ_ERR_INVALID, "done_idx_out and terminal_obs_out go together");
  if ((int64_t)K * h->cfg.num_envs > ((int64_t)1 << 40)) return fail(LZ_ERR_INVALID, "K*N too large");
  HIP_TRY(hipSetDevice(h->cfg.device));
  KArgs a;
  fill_common(h, a);
  a.act = actions;
  a.obs = obs_out;
  a.rew = rew_out;
  a.done = done_out;
  a.done_idx64 = done_idx_out;
  a.term_obs = terminal_obs_out;
  a.term_cap = cap;
  a.K = K;
  a.tick_adv = (uint64_t)K;
  a.vec_ok = (!needs_act || aligned16(actions)) && aligned16(obs_out) && (a.n % 4 == 0);
  const int e = lz::launch_rollout(sys_key(h), h->f64, a, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "rollout launch: %s", hipGetErrorString((hipError_t)e));
  if (n_done_out)
    HIP_TRY(hipMemcpyAsync(n_done_out, a.counter, sizeof(int32_t), hipMemcpyDeviceToDevice, h->stream));
  h->parity ^= 1;
  ++h->gen;
  return LZ_OK;
}

// arch: 0 = MlpPolicy (bf16), 1 = attention extractor, 2 = residual + LayerNorm attention
// on VecFrameStack(n_stack) observations, 3 = MlpPolicy in float32, 4 / 5 = arch 1 / 2 in
// float32
static lz_status rollout_policy(lz_handle* h, const lz_policy_rollout_args* r, int arch,
                                int n_stack = 1, const float* stack_in = nullptr,
                                float* stack_out = nullptr) {
  if (!h || !r) return fail(LZ_ERR_INVALID, "handle/args is NULL");
  RESIDENT_QUIESCE(h);
  const bool attn = arch == 1 || arch == 2 || arch == 4 || arch == 5;
  const bool stacked = arch == 2 || arch == 5;
  if (stacked) {
    if (n_stack != 1 && n_stack != 4) return fail(LZ_ERR_UNSUPPORTED, "n_stack must be 1 or 4");
    if (!stack_in || !stack_out) return fail(LZ_ERR_INVALID, "stack_in / stack_out must be non-NULL");
    if (r->obs_norm || r->obs_moments)
      return fail(LZ_ERR_UNSUPPORTED, "the frame-stacked rollout takes no VecNormalize statistics");
    const int sys = h->cfg.system;
    if (sys != LZ_SYS_LORENZ3 && sys != LZ_SYS_PMSM && sys != LZ_SYS_HR)
      return fail(LZ_ERR_UNSUPPORTED, "the frame-stacked rollout runs LORENZ3 / PMSM / HR");
    if (n_stack * h->desc.obs_dim > lz::kLnMaxIn) return fail(LZ_ERR_UNSUPPORTED, "stacked obs > 32 dims");
  }
  if (arch == 4) {
    const int sys = h->cfg.system;
    if (sys != LZ_SYS_LORENZ3 && sys != LZ_SYS_PMSM && sys != LZ_SYS_HR)
      return fail(LZ_ERR_UNSUPPORTED, "the float32 attention rollout runs LORENZ3 / PMSM / HR");
  }
  if ((r->flags & LZ_POLICY_I8X4) && arch < 3)
    return fail(LZ_ERR_UNSUPPORTED, "LZ_POLICY_I8X4 runs the float32 (attention / MlpPolicy) rollouts only");
  if ((r->flags & LZ_POLICY_I8X4) && arch == 3) {
    const int sys = h->cfg.system;
    if (sys != LZ_SYS_LORENZ3 && sys != LZ_SYS_LORENZ4 && sys != LZ_SYS_PMSM && sys != LZ_SYS_HR)
      return fail(LZ_ERR_UNSUPPORTED, "the i8x4 MlpPolicy rollout runs LORENZ3 / LORENZ4 / PMSM / HR");
  }
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_rollout_policy before the first lz_reset");
  if (h->f64) return fail(LZ_ERR_UNSUPPORTED, "the policy rollout runs float32 handles only");
  if (sys_key(h) != h->cfg.system)
    return fail(LZ_ERR_UNSUPPORTED, "the policy rollouts run the reference's Euler integrator only");
  if (r->K <= 0) return fail(LZ_ERR_INVALID, "K must be >= 1");
  if (!r->blob || !r->obs_in || !r->obs_last || !r->obs_buf || !r->act_buf || !r->logp_buf ||
      !r->val_buf || !r->rew_buf || !r->done_buf || !r->last_values)
    return fail(LZ_ERR_INVALID, "blob / obs / rollout buffers must be non-NULL");
  if ((r->done_idx == nullptr) != (r->terminal_obs == nullptr))
    return fail(LZ_ERR_INVALID, "done_idx and terminal_obs go together");
  if ((int64_t)r->K * h->cfg.num_envs > ((int64_t)1 << 40)) return fail(LZ_ERR_INVALID, "K*N too large");
  if (!(r->act_low <= r->act_high)) return fail(LZ_ERR_INVALID, "act_low > act_high");
  HIP_TRY(hipSetDevice(h->cfg.device));
  const int64_t n = h->cfg.num_envs;
  const lz::PolShape sh = arch >= 4   ? lz::attn_f32_policy_shape(n, h->num_cus, arch == 5)
                         : attn      ? lz::attn_policy_shape(n, h->num_cus)
                         : arch == 3 ? lz::f32_policy_shape(n, h->num_cus, h->cfg.reserved[0])
                                     : lz::policy_shape(n, h->cfg.reserved[0], h->num_cus);
  const int W = sh.waves, grid = sh.grid;
  const int O = h->desc.obs_dim;
  const int64_t need = (int64_t)grid * W * 2 * O;
  if (r->obs_moments && h->pol_part_n < need) {
    if (h->pol_part) HIP_TRY(hipFree(h->pol_part));
    h->pol_part = nullptr;
    h->pol_part_n = 0;
    if (hipMalloc(reinterpret_cast<void**>(&h->pol_part), (size_t)need * sizeof(double)) != hipSuccess)
      return fail(LZ_ERR_OOM, "policy moment scratch allocation failed");
    h->pol_part_n = need;
  }
  KArgs a;
  fill_common(h, a);
  a.obs = r->obs_buf;
  a.rew = r->rew_buf;
  a.done = r->done_buf;
  a.done_idx64 = r->done_idx;
  a.term_obs = r->terminal_obs;
  a.term_cap = r->cap;
  a.K = r->K;
  a.tick_adv = (uint64_t)r->K;
  lz::PArgs p;
  std::memset(&p, 0, sizeof p);
  p.blob = static_cast<const uint8_t*>(r->blob);
  p.obs_in = r->obs_in;
  p.obs_last = r->obs_last;
  p.norm = r->obs_norm;
  p.eps = r->norm_eps;
  p.clip = r->clip_obs;
  p.gamma = (float)r->gamma;
  p.act_lo = r->act_low;
  p.act_hi = r->act_high;
  p.pflags = r->flags;
  p.act = r->act_buf;
  p.logp = r->logp_buf;
  p.val = r->val_buf;
  p.last_val = r->last_values;
  p.partials = r->obs_moments ? h->pol_part : nullptr;
  p.stack_in = stack_in;
  p.stack_out = stack_out;
  int e = arch >= 4 ? lz::launch_rollout_policy_attn_f32(h->cfg.system, arch == 5, n_stack, a, p, sh,
                                                        h->stream)
          : arch == 2 ? lz::launch_rollout_policy_attn_ln(h->cfg.system, n_stack, a, p, sh, h->stream)
          : arch == 1 ? lz::launch_rollout_policy_attn(h->cfg.system, a, p, sh, h->stream)
          : arch == 3 ? lz::launch_rollout_policy_f32(h->cfg.system, a, p, sh, h->stream)
                      : lz::launch_rollout_policy(h->cfg.system, a, p, sh, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "policy rollout launch: %s", hipGetErrorString((hipError_t)e));
  if (r->obs_moments) {
    e = lz::launch_policy_moments_final(h->pol_part, grid * W, 2 * O, (double)r->K * (double)n,
                                        r->obs_moments, h->stream);
    if (e != 0) return fail(LZ_ERR_HIP, "moments launch: %s", hipGetErrorString((hipError_t)e));
  }
  if (r->n_done)
    HIP_TRY(hipMemcpyAsync(r->n_done, a.counter, sizeof(int32_t), hipMemcpyDeviceToDevice, h->stream));
  h->parity ^= 1;
  ++h->gen;
  return LZ_OK;
}

lz_status lz_rollout_policy(lz_handle* h, const lz_policy_rollout_args* r) {
  return rollout_policy(h, r, 0);
}

lz_status lz_rollout_policy_f32(lz_handle* h, const lz_policy_rollout_args* r) {
  return rollout_policy(h, r, 3);
}

lz_status lz_rollout_policy_attn(lz_handle* h, const lz_policy_rollout_args* r) {
  return rollout_policy(h, r, 1);
}

// ---- SB3-exact VecNormalize in the float32 rollout (lz_internal.h PStepArgs)
lz_status lz_policy_step_f32(lz_handle* h, const lz_policy_rollout_args* r, int32_t k,
                             double* obs_rms_state, double* moments_out) {
  if (!h || !r) return fail(LZ_ERR_INVALID, "handle/args is NULL");
  RESIDENT_QUIESCE(h);
  if (r->flags & LZ_POLICY_I8X4)
    return fail(LZ_ERR_UNSUPPORTED, "LZ_POLICY_I8X4 runs the float32 rollouts only, not the per-step collect");
  if (!h->was_reset) return fail(LZ_ERR_STATE, "lz_policy_step_f32 before the first lz_reset");
  if (h->f64) return fail(LZ_ERR_UNSUPPORTED, "the policy rollout runs float32 handles only");
  if (sys_key(h) != h->cfg.system)
    return fail(LZ_ERR_UNSUPPORTED, "the policy rollouts run the reference's Euler integrator only");
  if (r->K <= 0) return fail(LZ_ERR_INVALID, "K must be >= 1");
  if (k < 0 || k > r->K) return fail(LZ_ERR_INVALID, "step %d outside [0, K = %d]", k, r->K);
  if (!obs_rms_state) return fail(LZ_ERR_INVALID, "obs_rms_state must be non-NULL");
  if (r->obs_norm && r->obs_norm != obs_rms_state)
    return fail(LZ_ERR_INVALID, "obs_norm must be NULL or obs_rms_state");
  if (r->obs_moments) return fail(LZ_ERR_INVALID, "obs_moments must be NULL (per-step statistics)");
  if (!r->blob || !r->obs_in || !r->obs_last || !r->obs_buf || !r->act_buf || !r->logp_buf ||
      !r->val_buf || !r->rew_buf || !r->done_buf || !r->last_values)
    return fail(LZ_ERR_INVALID, "blob / obs / rollout buffers must be non-NULL");
  if ((r->done_idx == nullptr) != (r->terminal_obs == nullptr))
    return fail(LZ_ERR_INVALID, "done_idx and terminal_obs go together");
  if ((int64_t)r->K * h->cfg.num_envs > ((int64_t)1 << 40)) return fail(LZ_ERR_INVALID, "K*N too large");
  if (!(r->act_low <= r->act_high)) return fail(LZ_ERR_INVALID, "act_low > act_high");
  const int O = h->desc.obs_dim;
  if (O > lz::kVnMaxObs) return fail(LZ_ERR_UNSUPPORTED, "obs too wide");
  HIP_TRY(hipSetDevice(h->cfg.device));
  const int64_t n = h->cfg.num_envs;
  const int64_t ntiles = (n + lz::kVnTile - 1) / lz::kVnTile;
  if (!h->ps_tiles) {
    double* t = nullptr;
    float* term = nullptr;
    int32_t* cur = nullptr;
    const size_t bt = (size_t)(2 * O * ntiles + 2 * O + 1) * sizeof(double);
    if (hipMalloc(reinterpret_cast<void**>(&t), bt) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&term), (size_t)n * O * sizeof(float)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&cur), 2 * sizeof(int32_t)) != hipSuccess) {
      if (t) (void)hipFree(t);
      if (term) (void)hipFree(term);
      return fail(LZ_ERR_OOM, "lz_policy_step_f32 scratch allocation failed");
    }
    h->ps_tiles = t;
    h->ps_term = term;
    h->ps_cursor = cur;
  }
  // one collect = k = 0 .. K in order with no other launch on the handle in between: the
  // raw terminal-obs carry (ps_term), the collect's done cursor and the RNG tick parity
  // are carried from step to step
  if (k > 0 && (k != h->ps_next_k || h->gen != h->ps_gen)) {
    const int32_t want = h->ps_next_k;
    h->ps_next_k = -1;
    return fail(LZ_ERR_STATE,
                "lz_policy_step_f32: step %d out of order (expected %d, or another launch on the "
                "handle came in between); a collect calls k = 0 .. K in order",
                k, want);
  }
  const bool fin = k == r->K;
  if (k == 0) HIP_TRY(hipMemsetAsync(h->ps_cursor, 0, 2 * sizeof(int32_t), h->stream));
  const lz::PolShape sh = lz::f32_policy_shape(n, h->num_cus, h->cfg.reserved[0]);
  KArgs a;
  fill_common(h, a);
  a.obs = r->obs_buf;
  a.rew = r->rew_buf;
  a.done = r->done_buf;
  a.done_idx64 = r->done_idx;
  a.term_obs = r->terminal_obs;
  a.term_cap = r->cap;
  a.K = r->K;
  a.counter = h->ps_cursor;       // one cursor for the whole collect (zeroed at k = 0)
  // a step launch flips the parity (below): it zeroes the cursor slot the handle's next
  // ordinary launch reads, as every other launch does (fill_common's counter_next)
  lz::PArgs p;
  std::memset(&p, 0, sizeof p);
  p.blob = static_cast<const uint8_t*>(r->blob);
  p.obs_in = r->obs_in;
  p.obs_last = r->obs_last;
  p.norm = obs_rms_state;
  p.eps = r->norm_eps;
  p.clip = r->clip_obs;
  p.gamma = (float)r->gamma;
  p.act_lo = r->act_low;
  p.act_hi = r->act_high;
  p.pflags = r->flags;
  p.act = r->act_buf;
  p.logp = r->logp_buf;
  p.val = r->val_buf;
  p.last_val = r->last_values;
  lz::PStepArgs st;
  std::memset(&st, 0, sizeof st);
  st.k = k;
  st.final_ = fin ? 1 : 0;
  st.ntiles = ntiles;
  st.tiles = fin ? nullptr : h->ps_tiles;
  st.snap = fin ? nullptr : h->ps_tiles + 2 * O * ntiles;
  st.term = h->ps_term;
  st.obs_src = k == 0 ? r->obs_in : r->obs_last;
  int e = lz::launch_policy_step_f32(h->cfg.system, a, p, st, sh, h->stream);
  if (e != 0) return fail(LZ_ERR_HIP, "policy step launch: %s", hipGetErrorString((hipError_t)e));
  if (!fin) {
    h->parity ^= 1;  // the launch advanced the RNG tick by one (ping-pong)
    ++h->gen;
    h->ps_next_k = k + 1;
    h->ps_gen = h->gen;
    e = lz::launch_vn_tile_update(st.tiles, ntiles, O, (double)n, st.snap, obs_rms_state, moments_out,
                                  h->stream);
    if (e != 0) return fail(LZ_ERR_HIP, "statistics update launch: %s", hipGetErrorString((hipError_t)e));
  } else {
    h->ps_next_k = -1;
    if (r->n_done)
      HIP_TRY(hipMemcpyAsync(r->n_done, h->ps_cursor, sizeof(int32_t), hipMemcpyDeviceToDevice, h->stream));
  }
  return LZ_OK;
}

lz_status lz_rollout_policy_f32_vn(lz_handle* h, const lz_policy_rollout_args* r,
                                   double* obs_rms_state) {
  if (!h || !r) return fail(LZ_ERR_INVALID, "handle/args is NULL");
  for (int32_t k = 0; k <= r->K; ++k) {
    const lz_status s = lz_policy_step_f32(h, r, k, obs_rms_state, nullptr);
    if (s != LZ_OK) return s;
  }
  return LZ_OK;
}

lz_status lz_rollout_policy_attn_stack(lz_handle* h, const lz_policy_rollout_args* r,
                                       int32_t n_stack, const float* stack_in, float* stack_out) {
  return rollout_policy(h, r, 2, n_stack, stack_in, stack_out);
}

lz_status lz_rollout_policy_attn_f32(lz_handle* h, const lz_policy_rollout_args* r) {
  return rollout_policy(h, r, 4);
}

lz_status lz_rollout_policy_attn_stack_f32(lz_handle* h, const lz_policy_rollout_args* r,
                                           int32_t n_stack, const float* stack_in, float* stack_out) {
  return rollout_policy(h, r, 5, n_stack, stack_in, stack_out);
}

lz_status lz_get_launch_shape(const lz_handle* h, int32_t call, lz_launch_shape* out) {
  if (!h || !out) return fail(LZ_ERR_INVALID, "handle/out is NULL");
  std::memset(out, 0, sizeof *out);
  const int64_t n = h->cfg.num_envs;
  if (call == LZ_CALL_STEP || call == LZ_CALL_STEP_NOISE || call == LZ_CALL_ROLLOUT) {
    KArgs a;
    fill_common(h, a);
    // lz_step's noise argument (only its presence matters to the launcher): fill_common
    // leaves it NULL, the device-drawn case; LZ_CALL_STEP_NOISE asks for the injected one
    static const double kNoiseTag = 0.0;
    if (call == LZ_CALL_STEP_NOISE) a.noise = &kNoiseTag;
    int32_t o[5] = {0, 0, 0, 0, 0};
    if (lz::env_launch_shape(call == LZ_CALL_ROLLOUT ? 2 : 1, sys_key(h), h->f64, a, o) != 0)
      return fail(LZ_ERR_INVALID, "no launch shape for system %d", h->cfg.system);
    out->kernel = o[0];
    out->envs_per_wave = o[1];
    out->waves = o[2];
    out->grid = o[3];
    out->flags = (uint32_t)o[4];
    out->groups = o[3];
    return LZ_OK;
  }
  lz::PolShape sh;
  switch (call) {
    case LZ_CALL_ROLLOUT_POLICY:
      sh = lz::policy_shape(n, h->cfg.reserved[0], h->num_cus);
      out->kernel = sh.envs_per_wave == 64 ? LZ_KERNEL_POLICY
                    : sh.pair == 2         ? LZ_KERNEL_POLICY_PAIR_PIPE
                    : sh.pair              ? LZ_KERNEL_POLICY_PAIR
                                           : LZ_KERNEL_POLICY;
      break;
    case LZ_CALL_ROLLOUT_POLICY_F32:
      sh = lz::f32_policy_shape(n, h->num_cus, h->cfg.reserved[0]);
      out->kernel = sh.pair == 1 ? LZ_KERNEL_POLICY_SPLIT : LZ_KERNEL_POLICY;
      break;
    case LZ_CALL_POLICY_STEP_F32:
      sh = lz::f32_policy_shape(n, h->num_cus, h->cfg.reserved[0]);
      out->kernel = LZ_KERNEL_POLICY_STEP;
      break;
    case LZ_CALL_ROLLOUT_POLICY_ATTN:
    case LZ_CALL_ROLLOUT_POLICY_ATTN_STACK:
      sh = lz::attn_policy_shape(n, h->num_cus);
      out->kernel = LZ_KERNEL_POLICY_ATTN;
      break;
    case LZ_CALL_ROLLOUT_POLICY_ATTN_F32:
    case LZ_CALL_ROLLOUT_POLICY_ATTN_STACK_F32:
      sh = lz::attn_f32_policy_shape(n, h->num_cus, call == LZ_CALL_ROLLOUT_POLICY_ATTN_STACK_F32);
      out->kernel = LZ_KERNEL_POLICY_ATTN_F32;
      break;
    default:
      return fail(LZ_ERR_INVALID, "unknown call %d", call);
  }
  out->envs_per_wave = sh.envs_per_wave;
  // the split kernel runs 4 tiles per workgroup on 8 waves (actor + critic per tile)
  out->waves = (call == LZ_CALL_ROLLOUT_POLICY_F32 && sh.pair == 1) ? 8 : sh.waves;
  out->grid = sh.grid;
  const int64_t groups = ((n + sh.envs_per_wave - 1) / sh.envs_per_wave + sh.waves - 1) / sh.waves;
  out->groups = (int32_t)groups;
  out->flags = groups > sh.grid ? LZ_SHAPE_GRID_STRIDE : 0u;
  return LZ_OK;
}

int32_t lz_plane_elem_size(const lz_handle* h, int32_t plane) {
  if (!h) return 0;
  return plane_elem(h->cfg.system, h->f64, plane);
}

static lz_status plane_access(lz_handle* h, int32_t plane, void* buf, const int64_t* indices, int64_t count,
                              bool set) {
  if (!h || !buf) return fail(LZ_ERR_INVALID, "handle/%s is NULL", set ? "src" : "dst");
  const int es = plane_elem(h->cfg.system, h->f64, plane);
  if (!es) return fail(LZ_ERR_INVALID, "invalid plane %d", plane);
  if (!indices && count != 0 && count != h->cfg.num_envs)
    return fail(LZ_ERR_INVALID, "whole-plane access (indices NULL) with count %lld != 0 / num_envs",
                (long long)count);
  if (indices && (count < 0 || count > ((int64_t)1 << 40)))
    return fail(LZ_ERR_INVALID, "index count %lld out of range", (long long)count);
  RESIDENT_QUIESCE(h);
  HIP_TRY(hipSetDevice(h->cfg.device));
  if (!indices) {
    const size_t bytes = (size_t)h->cfg.num_envs * es;
    HIP_TRY(set ? hipMemcpyAsync(h->planes[plane], buf, bytes, hipMemcpyDeviceToDevice, h->stream)
                : hipMemcpyAsync(buf, h->planes[plane], bytes, hipMemcpyDeviceToDevice, h->stream));
    return LZ_OK;
  }
  HIP_TRY((hipError_t)lz::launch_plane_index(set, es, h->planes[plane], h->cfg.num_envs, indices, count, buf,
                                             h->stream));
  return LZ_OK;
}

lz_status lz_get_state(lz_handle* h, int32_t plane, void* dst, const int64_t* indices, int64_t count) {
  return plane_access(h, plane, dst, indices, count, false);
}

lz_status lz_set_state(lz_handle* h, int32_t plane, const void* src, const int64_t* indices, int64_t count) {
  return plane_access(h, plane, const_cast<void*>(src), indices, count, true);
}

}  // extern "C"
