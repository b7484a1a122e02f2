// Per-launch floor of a chain of dependent kernels on one stream, the way bench.py
// issues lz_step (a hipGraph of 64 kernel nodes, replayed): (a) an empty kernel of G
// 256-lane workgroups, (b) a non-temporal float4 copy moving the same bytes as one
// LORENZ3 f32 step of N envs (65 B/env: half read, half written), one vector per lane.
// The difference between k_step's time and (a) is the part a faster step body could
// still win; (b) is what pure streaming of that volume costs in the same launch chain.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_empty(int* p) {
  if (p != nullptr && threadIdx.x == 0) p[blockIdx.x] = 0;
}

__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ a, f4* __restrict__ b,
                                              size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

// k_step's I/O with no arithmetic: state planes x,y,z in and out (same buffers every
// step), the [N,3] action slice staged through LDS as float4s, the [N,6] obs slice
// staged out through LDS as float4s, reward and done per lane; action/obs/reward/done
// rotate through a 16-slot ring as in bench.py.  What k_step would cost if its step
// math were free.
__global__ __launch_bounds__(256) void k_io(float* __restrict__ x, float* __restrict__ y,
                                            float* __restrict__ z, const float* __restrict__ act,
                                            float* __restrict__ obs, float* __restrict__ rew,
                                            uint8_t* __restrict__ done) {
  __shared__ __attribute__((aligned(16))) float s_act[256 * 3];
  __shared__ __attribute__((aligned(16))) float s_obs[256 * 6];
  const int t = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 256, i = base + t;
  float a0 = x[i], a1 = y[i], a2 = z[i];
  const f4* ga = reinterpret_cast<const f4*>(act + base * 3);
  if (t < 192) reinterpret_cast<f4*>(s_act)[t] = __builtin_nontemporal_load(ga + t);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  a0 += s_act[3 * t];
  a1 += s_act[3 * t + 1];
  a2 += s_act[3 * t + 2];
  x[i] = a0;
  y[i] = a1;
  z[i] = a2;
  s_obs[6 * t] = a0; s_obs[6 * t + 1] = a1; s_obs[6 * t + 2] = a2;
  s_obs[6 * t + 3] = a2; s_obs[6 * t + 4] = a1; s_obs[6 * t + 5] = a0;
  __builtin_nontemporal_store(a0 + a1, rew + i);
  __builtin_nontemporal_store((uint8_t)(a2 > 1e30f), done + i);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  f4* go = reinterpret_cast<f4*>(obs + base * 6);
  const f4* lo = reinterpret_cast<const f4*>(s_obs);
  __builtin_nontemporal_store(lo[t], go + t);
  if (t < 128) __builtin_nontemporal_store(lo[256 + t], go + 256 + t);
}

static hipStream_t s;

template <class F>
static double us_per_node(F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  const int nodes = 64, reps = 40;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int k = 0; k < nodes; ++k) launch();
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int r = 0; r < 3; ++r) (void)hipGraphLaunch(ge, s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms * 1e3 / (nodes * reps);
}

int main() {
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  const size_t maxb = 70ull << 20, nmax = 1 << 20, R = 16;
  f4 *a, *b;
  if (hipMalloc(&a, maxb) != hipSuccess || hipMalloc(&b, maxb) != hipSuccess) return 1;
  (void)hipMemset(a, 0, maxb);
  (void)hipMemset(b, 0, maxb);
  float *st, *act, *obs, *rew;
  uint8_t* done;
  if (hipMalloc(&st, 3 * nmax * 4) != hipSuccess || hipMalloc(&act, R * nmax * 12) != hipSuccess ||
      hipMalloc(&obs, R * nmax * 24) != hipSuccess || hipMalloc(&rew, R * nmax * 4) != hipSuccess ||
      hipMalloc(&done, R * nmax) != hipSuccess)
    return 1;
  (void)hipMemset(st, 0, 3 * nmax * 4);
  (void)hipMemset(act, 0, R * nmax * 12);
  const long envs[] = {16384, 32768, 65536, 131072, 262144, 1048576};
  for (int rep = 0; rep < 2; ++rep) {
    for (long n : envs) {
      const unsigned groups = (unsigned)(n / 256);
      const double te = us_per_node([&] { hipLaunchKernelGGL(k_empty, dim3(groups), dim3(256), 0, s, nullptr); });
      const size_t vec = (size_t)(n * 65 / 2 + 15) / 16;  // float4s read (= written)
      const double tc = us_per_node([&] {
        hipLaunchKernelGGL(k_copy, dim3((unsigned)((vec + 255) / 256)), dim3(256), 0, s, a, b, vec);
      });
      int k = 0;
      const double ti = us_per_node([&] {
        const size_t sl = (size_t)(k++ % R);
        hipLaunchKernelGGL(k_io, dim3(groups), dim3(256), 0, s, st, st + n, st + 2 * n,
                           act + sl * n * 3, obs + sl * n * 6, rew + sl * n, done + sl * n);
      });
      printf("envs %8ld groups %5u  empty %.3f us/node   copy(65 B/env) %.3f us/node = %.2f TB/s"
             "   k_step-io(ring) %.3f us/node = %.2f TB/s\n",
             n, groups, te, tc, 2.0 * vec * 16 / (tc * 1e-6) / 1e12, ti, 65.0 * n / (ti * 1e-6) / 1e12);
    }
  }
  return 0;
}
