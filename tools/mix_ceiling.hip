// Streaming ceiling by read:write mix and per-launch size on this box -- the practical
// roofline of each env kernel, whose traffic is write-heavy (LORENZ3 step 24 B read :
// 41 B written, HR 38 : 62, PMSM 42 : 58 ...): a kernel's HBM fraction of 8 TB/s is
// bounded by the fraction a pure stream of the same mix and size reaches.
//
// R reads + W writes of float4 per lane (one contiguous 16-B vector per lane per
// stream, non-temporal or plain), back-to-back launches over a ring of 16 buffer sets
// (as bench.py's 16-slot rollout ring: no launch re-reads what the previous one wrote),
// HIP events around 20 launches after 4 warm ones.  Prints one JSON line per case.
//   hipcc -O3 --offload-arch=gfx950 tools/mix_ceiling.hip -o tools/mix_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void stv(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

constexpr int kMaxS = 8;
struct Bufs {
  const f4* r[kMaxS];
  f4* w[kMaxS];
};

template <bool NT, int R, int W>
__global__ __launch_bounds__(256) void mix(Bufs b, size_t n, float key) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  f4 v = (f4)key;
#pragma unroll
  for (int r = 0; r < R; ++r) v += ld<NT>(b.r[r] + i);
#pragma unroll
  for (int w = 0; w < W; ++w) stv<NT>(b.w[w] + i, v + (float)w);
  if constexpr (W == 0) {  // read-only: keep the loads alive (never true for zeroed input)
    if (v.x == 1234.5f) b.w[0][i] = v;
  }
}

template <bool NT, int R, int W>
static void run_case(size_t target_bytes) {
  const int S = R + W;
  const size_t n = target_bytes / (16 * (size_t)S);  // float4 per stream
  const int ring = 16;
  std::vector<f4*> mem;
  std::vector<Bufs> sets(ring);
  for (int k = 0; k < ring; ++k) {
    for (int r = 0; r < R; ++r) {
      f4* p;
      if (hipMalloc(&p, n * 16) != hipSuccess) return;
      (void)hipMemset(p, 0, n * 16);
      mem.push_back(p);
      sets[k].r[r] = p;
    }
    for (int w = 0; w < (W ? W : 1); ++w) {
      f4* p;
      if (hipMalloc(&p, n * 16) != hipSuccess) return;
      mem.push_back(p);
      sets[k].w[w] = p;
    }
  }
  const dim3 grid((unsigned)((n + 255) / 256));
  auto launch = [&](int k) { hipLaunchKernelGGL((mix<NT, R, W>), grid, dim3(256), 0, 0, sets[k % ring], n, 0.0f); };
  for (int k = 0; k < 4; ++k) launch(k);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 20;
  (void)hipEventRecord(e0);
  for (int k = 0; k < reps; ++k) launch(k + 4);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double moved = (double)n * 16 * S, us = ms * 1e3 / reps;
  printf("{\"read\": %d, \"write\": %d, \"nt\": %d, \"bytes_per_launch\": %.0f, \"us_per_launch\": %.3f, "
         "\"TBps\": %.4f}\n", R, W, (int)NT, moved, us, moved / (us * 1e-6) / 1e12);
  fflush(stdout);
  for (f4* p : mem) (void)hipFree(p);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

template <int R, int W>
static void both(size_t bytes) {
  run_case<true, R, W>(bytes);
  run_case<false, R, W>(bytes);
}

int main() {
  // per-launch sizes of the bench lines: cfg4 PMSM 262k 33 MB, headline 68 MB, HR 1M
  // 89 MB, PMSM 1M 131 MB, and 1 GiB (no MALL reuse at all)
  const size_t sizes[] = {33u << 20, 68u << 20, 89u << 20, 131u << 20, 1u << 30};
  for (size_t s : sizes) {
    both<1, 0>(s);
    both<0, 1>(s);
    both<1, 1>(s);
    both<2, 3>(s);
    both<3, 5>(s);
    both<1, 2>(s);
    both<3, 2>(s);
  }
  return 0;
}
