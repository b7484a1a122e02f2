// Measured HBM ceiling on this box for streaming traffic, next to bench.py's
// roofline.frac (which is against the 8 TB/s spec): float4 copies (read + write 1:1)
// in several launch shapes / cache hints, and a 2:3 read:write mix (~ LORENZ3's 24 B
// read : 41 B written per env).  Best of each is the practical ceiling.
//   hipcc -O3 --offload-arch=gfx950 tools/copy_ceiling.hip -o tools/copy_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>

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

// one float4 per thread per "unroll" slot, no grid-stride loop
template <bool NT, int U>
__global__ __launch_bounds__(256) void copy_flat(const f4* __restrict__ a, f4* __restrict__ b) {
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NT>(a + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) stv<NT>(b + base + u * 256, v[u]);
}
template <bool NT>
__global__ __launch_bounds__(256) void mix23(const f4* __restrict__ a, f4* __restrict__ b, size_t rows) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  f4 acc = ld<NT>(a + i) + ld<NT>(a + rows + i);
  stv<NT>(b + i, acc);
  stv<NT>(b + rows + i, acc);
  stv<NT>(b + 2 * rows + i, acc);
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  f4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 0, bytes);
  (void)hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](auto launch, double moved) {
    launch();
    (void)hipEventRecord(e0);
    for (int k = 0; k < 10; ++k) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return moved * 10 / (ms * 1e-3) / 1e12;
  };
  for (int rep = 0; rep < 2; ++rep) {
    printf("copy 1:1 plain U1 %.3f TB/s\n", time([&] { hipLaunchKernelGGL((copy_flat<false, 1>), dim3(n / 256), dim3(256), 0, 0, a, b); }, 2.0 * bytes));
    printf("copy 1:1 nt    U1 %.3f TB/s\n", time([&] { hipLaunchKernelGGL((copy_flat<true, 1>), dim3(n / 256), dim3(256), 0, 0, a, b); }, 2.0 * bytes));
    printf("copy 1:1 plain U4 %.3f TB/s\n", time([&] { hipLaunchKernelGGL((copy_flat<false, 4>), dim3(n / 1024), dim3(256), 0, 0, a, b); }, 2.0 * bytes));
    printf("copy 1:1 nt    U4 %.3f TB/s\n", time([&] { hipLaunchKernelGGL((copy_flat<true, 4>), dim3(n / 1024), dim3(256), 0, 0, a, b); }, 2.0 * bytes));
    const size_t rows = n / 4;
    printf("mix 2R:3W plain   %.3f TB/s\n", time([&] { hipLaunchKernelGGL((mix23<false>), dim3(rows / 256), dim3(256), 0, 0, a, b, rows); }, 5.0 * rows * 16));
    printf("mix 2R:3W nt      %.3f TB/s\n", time([&] { hipLaunchKernelGGL((mix23<true>), dim3(rows / 256), dim3(256), 0, 0, a, b, rows); }, 5.0 * rows * 16));
  }
  return 0;
}
