// Request-line placement for the resident drop-in server (lz_resident_step): where should
// the host write a request so that a polling wave sees it soonest?
//   host : pinned host memory (hipHostMalloc coherent, as lz_api.cpp's request lines):
//          every poll is a PCIe read round trip
//   vram : fine-grained device memory (hipExtMallocWithFlags finegrained) written by the
//          CPU through the BAR; the wave polls local memory.  Variants: with the HDP
//          write-buffer flush register written after the request (hipDeviceAttribute
//          HdpMemFlushCntl), and without.
// One wave, lane 0 polls; the response (the request's sequence number + 1) goes to pinned
// host memory, which the host spins on.  Every poll loop has an exit every wave reaches:
// a stop value, or 200 ms without a new request (so a request the wave never sees ends
// the kernel instead of hanging it).  Prints one line per mode: round trips per second
// and the median / p99 latency of one request -> response.
//   hipcc -O3 --offload-arch=gfx950 tools/vram_poll.hip -o tools/vram_poll
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr uint32_t kStop = 0xffffffffu;

__global__ void k_serve(const uint32_t* req, uint32_t* resp, uint64_t idle_ticks, uint32_t* served) {
  if (threadIdx.x != 0) return;
  uint32_t seen = 0, n = 0;
  uint64_t last = wall_clock64();
  for (;;) {
    const uint32_t r = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r == kStop) break;
    if (r != seen) {
      seen = r;
      ++n;
      __hip_atomic_store(resp, r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      last = wall_clock64();
      continue;
    }
    if (wall_clock64() - last > idle_ticks) break;
  }
  served[0] = n;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  // the attribute's value is a pointer: HIP stores it through the int* as a 64-bit slot
  uint64_t hdp64 = 0;
  if (hipDeviceGetAttribute(reinterpret_cast<int*>(&hdp64), hipDeviceAttributeHdpMemFlushCntl, 0) != hipSuccess)
    hdp64 = 0;
  uint32_t* hdp = reinterpret_cast<uint32_t*>(hdp64);
  std::printf("wall clock %d kHz, HDP flush register %p\n", khz, (void*)hdp);

  uint32_t* resp = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&resp), 256, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* req_host = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&req_host), 256, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* req_vram = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&req_vram), 256, hipDeviceMallocFinegrained));
  uint32_t* served = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&served), 16));
  hipPointerAttribute_t pa{};
  CK(hipPointerGetAttributes(&pa, req_vram));
  std::printf("vram line: device %p host %p type %d\n", pa.devicePointer, pa.hostPointer, (int)pa.type);

  struct Mode {
    const char* name;
    volatile uint32_t* host_view;  // where the CPU writes
    const uint32_t* dev_view;      // where the wave polls
    bool flush;
  };
  std::vector<Mode> modes = {{"host", req_host, req_host, false}};
  // the CPU's view of the fine-grained VRAM line: the same address if the runtime maps it
  // into the host (large BAR), else none -- then the vram modes are skipped
  volatile uint32_t* vh = static_cast<volatile uint32_t*>(pa.hostPointer ? pa.hostPointer : nullptr);
  if (vh) {
    modes.push_back({"vram+hdp", vh, req_vram, hdp != nullptr});
    modes.push_back({"vram", vh, req_vram, false});
  } else {
    std::printf("vram line has no host pointer: vram modes skipped\n");
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint64_t idle = (uint64_t)khz * 200;  // 200 ms
  for (const Mode& m : modes) {
    m.host_view[0] = 0;
    if (m.flush) *reinterpret_cast<volatile uint32_t*>(hdp) = 1;
    __atomic_store_n(resp, 0u, __ATOMIC_SEQ_CST);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_serve, dim3(1), dim3(64), 0, s, m.dev_view, resp, idle, served);
    std::vector<double> lat;
    lat.reserve(iters);
    bool lost = false;
    const double t0 = now_us();
    for (int i = 1; i <= iters && !lost; ++i) {
      const double a = now_us();
      __atomic_store_n(const_cast<uint32_t*>(m.host_view), (uint32_t)i, __ATOMIC_SEQ_CST);
      if (m.flush) *reinterpret_cast<volatile uint32_t*>(hdp) = 1;
      while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != (uint32_t)i + 1) {
        if (now_us() - a > 100000.0) {  // 100 ms: the wave does not see the requests
          lost = true;
          break;
        }
      }
      lat.push_back(now_us() - a);
    }
    const double t1 = now_us();
    m.host_view[0] = kStop;
    if (m.flush) *reinterpret_cast<volatile uint32_t*>(hdp) = 1;
    CK(hipStreamSynchronize(s));  // the wave leaves on the stop value or after 200 ms idle
    uint32_t n = 0;
    CK(hipMemcpy(&n, served, 4, hipMemcpyDeviceToHost));
    std::sort(lat.begin(), lat.end());
    const double med = lat.empty() ? 0 : lat[lat.size() / 2], p99 = lat.empty() ? 0 : lat[lat.size() * 99 / 100];
    std::printf("%-9s %s  requests %zu served %u  %.3f us/round trip  median %.3f us  p99 %.3f us\n", m.name,
                lost ? "LOST" : "ok  ", lat.size(), n, (t1 - t0) / (double)lat.size(), med, p99);
  }
  CK(hipStreamDestroy(s));
  return 0;
}
