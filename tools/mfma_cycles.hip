// Issue cost of the two MFMA shapes the attention extractor would choose between
// (VERDICT r05 #4): v_mfma_f32_16x16x4_f32 (today's fc1 / K / V / Q /
// out_proj) vs v_mfma_i32_16x16x64_i8 (the i8x4 digit products).  One wave, CH
// independent accumulator chains, NI back-to-back instructions per chain; cycles from
// s_memtime around the loop.  Build: hipcc --offload-arch=gfx950 -O3 mfma_cycles.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int CH = 8, NI = 512;

__global__ void k_f32(const float* in, float* out, long long* cyc) {
  const int l = threadIdx.x;
  float a = in[l], b = in[64 + l];
  f32x4 c[CH];
  for (int j = 0; j < CH; ++j) c[j] = f32x4{0.f, 0.f, 0.f, (float)j};
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
#pragma unroll
    for (int j = 0; j < CH; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < CH; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s;
  if (l == 0) cyc[0] = t1 - t0;
}

__global__ void k_i8(const int* in, int* out, long long* cyc) {
  const int l = threadIdx.x;
  i32x4 a = {in[l], in[l] ^ 1, in[l] ^ 2, in[l] ^ 3}, b = {in[64 + l], 1, 2, 3};
  i32x4 c[CH];
  for (int j = 0; j < CH; ++j) c[j] = i32x4{0, 0, 0, j};
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
#pragma unroll
    for (int j = 0; j < CH; ++j) c[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c[j], 0, 0, 0);
  }
  int s = 0;
  for (int j = 0; j < CH; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s;
  if (l == 0) cyc[1] = t1 - t0;
}

int main() {
  float* fin;
  float* fout;
  int* iin;
  int* iout;
  long long* cyc;
  hipMalloc(&fin, 512);
  hipMalloc(&fout, 256);
  hipMalloc(&iin, 512);
  hipMalloc(&iout, 256);
  hipMalloc(&cyc, 16);
  hipMemset(fin, 0, 512);
  hipMemset(iin, 0, 512);
  long long h[2] = {0, 0}, best[2] = {1LL << 62, 1LL << 62};
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(k_f32, dim3(1), dim3(64), 0, 0, fin, fout, cyc);
    hipLaunchKernelGGL(k_i8, dim3(1), dim3(64), 0, 0, iin, iout, cyc);
    hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
    for (int k = 0; k < 2; ++k) best[k] = h[k] < best[k] ? h[k] : best[k];
  }
  // s_memtime counts at the shader clock; report cycles per instruction (one wave = one SIMD)
  const double n = (double)CH * NI;
  std::printf("{\"f32_16x16x4_cyc_per_instr\": %.2f, \"i8_16x16x64_cyc_per_instr\": %.2f, "
              "\"chains\": %d, \"per_chain\": %d}\n",
              best[0] / n, best[1] / n, CH, NI);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
