// PMC calibration: streaming kernels with KNOWN byte counts in the access widths the
// env step kernel uses (4-B lane loads/stores of the SoA planes, 16-B vectors of the
// staged act/obs tensors, 1-B done flags).  Run under rocprofv3 --pmc FETCH_SIZE and,
// separately, --pmc WRITE_SIZE; tools/pmc_summary.py divides measured by known bytes.
// MI355X_MICROARCH.md "HBM": FETCH_SIZE reads 1/2 of a 16-B/lane stream on gfx950 and
// other widths are uncalibrated -- this measures them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void copy4(const float* __restrict__ a, float* __restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] * 1.5f;
}
__global__ void copy16(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { float4 v = a[i]; v.x *= 1.5f; b[i] = v; }
}
__global__ void store1(unsigned char* __restrict__ b, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (unsigned char)i;
}

int main() {
  const size_t bytes = (size_t)1 << 30;  // 1 GiB per buffer >> 256 MiB Infinity Cache
  float *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  const size_t n4 = bytes / 4, n16 = bytes / 16;
  for (int r = 0; r < 3; ++r) {
    copy4<<<(unsigned)((n4 + 255) / 256), 256>>>(a, b, n4);
    copy16<<<(unsigned)((n16 + 255) / 256), 256>>>((const float4*)a, (float4*)b, n16);
    store1<<<(unsigned)((bytes + 255) / 256), 256>>>((unsigned char*)b, bytes);
  }
  CK(hipDeviceSynchronize());
  std::printf("known bytes per dispatch: copy4 read %zu write %zu; copy16 read %zu write %zu; "
              "store1 write %zu\n", bytes, bytes, bytes, bytes, bytes);
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
