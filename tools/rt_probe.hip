// Host <-> GPU request/reply round trip of the resident drop-in server (lz_resident_step),
// taken apart.  One wave, lane 0 polls a request word in pinned host memory (relaxed
// system-scope loads, as the server's poller); on a new request it writes a reply word
// into pinned host memory, which the host spins on.  Modes (what the reply carries):
//   bare       : the reply word alone, relaxed system-scope store
//   release    : the reply word as a RELEASE system-scope store (the compiler's fence:
//                an L2 writeback, buffer_wbl2, before the store) -- as the server does
//   obs+release: 6 doubles of "observation" (plain stores) + the release reply -- the
//                server's reply exactly
//   obs+wt     : the 6 doubles as relaxed system-scope stores (write-through), a
//                vmcnt(0) wait, then a relaxed reply: ordered without the L2 writeback
//   vram       : (skipped unless the runtime maps fine-grained device memory into the
//                host) the request word in device memory written through the BAR
// Every poll loop has an exit every wave reaches: a stop value, or 200 ms without a new
// request.  Prints one line per mode: the mean and median / p99 of one round trip.
//   hipcc -O3 --offload-arch=gfx950 tools/rt_probe.hip -o tools/rt_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

constexpr uint32_t kStop = 0xffffffffu;

template <int MODE>
__global__ void k_serve(const uint32_t* req, uint32_t* resp, double* obs, uint64_t idle_ticks,
                        uint32_t* served) {
  if (threadIdx.x != 0) return;
  uint32_t seen = 0, n = 0;
  uint64_t last = wall_clock64();
  for (;;) {
    const uint32_t r = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r == kStop) break;
    if (r != seen) {
      seen = r;
      ++n;
      if (MODE == 0) {
        __hip_atomic_store(resp, r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else if (MODE == 1) {
        __hip_atomic_store(resp, r + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else if (MODE == 2) {
        for (int j = 0; j < 6; ++j) obs[j] = (double)r + j;
        __hip_atomic_store(resp, r + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        for (int j = 0; j < 6; ++j)
          __hip_atomic_store(obs + j, (double)r + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(resp, r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      last = wall_clock64();
      continue;
    }
    if (wall_clock64() - last > idle_ticks) break;
  }
  served[0] = n;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

typedef void (*kfn)(const uint32_t*, uint32_t*, double*, uint64_t, uint32_t*);

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  uint32_t* resp = nullptr;
  uint32_t* req = nullptr;
  double* obs = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&resp), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&req), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&obs), 256, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* served = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&served), 16));
  {  // does the runtime map fine-grained device memory into the host?
    void* v = nullptr;
    CK(hipExtMallocWithFlags(&v, 256, hipDeviceMallocFinegrained));
    hipPointerAttribute_t pa{};
    CK(hipPointerGetAttributes(&pa, v));
    std::printf("fine-grained device memory: host pointer %p -> vram mode %s\n", pa.hostPointer,
                pa.hostPointer ? "possible (not run)" : "skipped");
    CK(hipFree(v));
  }
  struct Mode {
    const char* name;
    kfn k;
  };
  const Mode modes[] = {{"bare", k_serve<0>}, {"release", k_serve<1>}, {"obs+release", k_serve<2>},
                        {"obs+wt", k_serve<3>}, {"bare", k_serve<0>}};
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint64_t idle = (uint64_t)khz * 200;  // 200 ms
  for (const Mode& m : modes) {
    __atomic_store_n(req, 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n(resp, 0u, __ATOMIC_SEQ_CST);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(m.k, dim3(1), dim3(64), 0, s, req, resp, obs, idle, served);
    std::vector<double> lat;
    lat.reserve(iters);
    bool lost = false, bad = false;
    const double t0 = now_us();
    for (int i = 1; i <= iters && !lost; ++i) {
      const double a = now_us();
      __atomic_store_n(req, (uint32_t)i, __ATOMIC_SEQ_CST);
      while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != (uint32_t)i + 1) {
        if (now_us() - a > 100000.0) {
          lost = true;
          break;
        }
      }
      if (m.k != k_serve<0> && m.k != k_serve<1> && obs[5] != (double)i + 5) bad = true;
      lat.push_back(now_us() - a);
    }
    const double t1 = now_us();
    __atomic_store_n(req, kStop, __ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(s));
    uint32_t n = 0;
    CK(hipMemcpy(&n, served, 4, hipMemcpyDeviceToHost));
    std::sort(lat.begin(), lat.end());
    std::printf("%-12s %s%s requests %zu served %u  mean %.3f us  median %.3f us  p99 %.3f us\n", m.name,
                lost ? "LOST " : "ok ", bad ? "STALE-OBS" : "", lat.size(), n, (t1 - t0) / (double)lat.size(),
                lat[lat.size() / 2], lat[lat.size() * 99 / 100]);
  }
  {  // host-side per-call costs inside lz_resident_step's steady state
    hipStream_t hs;
    CK(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
    const int R = 200000;
    double t0 = now_us();
    for (int i = 0; i < R; ++i) (void)hipSetDevice(0);
    double t1 = now_us();
    hipStreamCaptureStatus cs;
    for (int i = 0; i < R; ++i) (void)hipStreamIsCapturing(hs, &cs);
    double t2 = now_us();
    for (int i = 0; i < R; ++i) (void)hipStreamQuery(hs);
    double t3 = now_us();
    std::printf("host calls: hipSetDevice %.1f ns, hipStreamIsCapturing %.1f ns, hipStreamQuery %.1f ns\n",
                (t1 - t0) * 1e3 / R, (t2 - t1) * 1e3 / R, (t3 - t2) * 1e3 / R);
    CK(hipStreamDestroy(hs));
  }
  CK(hipStreamDestroy(s));
  return 0;
}
