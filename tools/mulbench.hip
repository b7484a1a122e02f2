#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int V>
__global__ void k(uint32_t* out, int iters) {
  uint32_t x = threadIdx.x + blockIdx.x * 977u, z = x * 3u + 1u, y = 5, w = 7, k0 = 1, k1 = 2;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      uint32_t lo0, hi0, lo1, hi1;
      if (V == 0) {
        lo0 = 0xD2511F53u * x; hi0 = __umulhi(0xD2511F53u, x);
        lo1 = 0xCD9E8D57u * z; hi1 = __umulhi(0xCD9E8D57u, z);
      } else {
        uint64_t p0 = (uint64_t)0xD2511F53u * x, p1 = (uint64_t)0xCD9E8D57u * z;
        lo0 = (uint32_t)p0; hi0 = (uint32_t)(p0 >> 32); lo1 = (uint32_t)p1; hi1 = (uint32_t)(p1 >> 32);
      }
      uint32_t nx = hi1 ^ y ^ k0, ny = lo1, nz = hi0 ^ w ^ k1, nw = lo0;
      x = nx; y = ny; z = nz; w = nw; k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ y ^ z ^ w;
}
int main() {
  uint32_t* o; hipMalloc(&o, 4 << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep)
  for (int v = 0; v < 2; ++v) {
    hipEventRecord(a);
    if (v == 0) k<0><<<4096, 256>>>(o, 200); else k<1><<<4096, 256>>>(o, 200);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double blocks = 4096.0 * 256 * 200;
    printf("variant %d: %.3f ms, %.3g philox blocks/s\n", v, ms, blocks / ms * 1e3);
  }
  return 0;
}
