// Host side of the policy C-ABI (include/lorenz_env.h): the packers that turn SB3
// state_dict tensors into the fused rollout kernels' LDS blobs (lz_policy.hip, layouts
// kPol* / kF32* / kAtt* / kLn* / kAF* in lz_internal.h).  Plain C++: no device code, so
// tests/test_sanitizers.py builds it under ASan + UBSan in seconds.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lz_internal.h"

// ------------------------------------------------------------------ host-side C-ABI
namespace {

uint16_t bf16_rne(float f) {  // round to nearest even (= v_cvt_pk_bf16_f32, torch)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// 2 / ln 2 as float: the tanh layers' weights and biases are packed pre-scaled by it
// (bf16(s * W) in float32 arithmetic, s * b), see tanh_scaled
constexpr float kTanhScale = 2.8853900817779268f;

// unit of a 128-wide input feeding k-step kk, element j, lane half h (see file header)
inline int unit_of(int kk, int h, int j) {
  return 32 * (kk >> 1) + 16 * (kk & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}
// output row held by accumulator register g of lane half h within a 32-row tile
inline int row_of(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

void pack_net(uint8_t* net, int O, int rows3, const float* w1, const float* b1, const float* w2,
              const float* b2, const float* w3, const float* b3) {
  using lz::kPolHidden;
  uint16_t* f1 = reinterpret_cast<uint16_t*>(net + lz::kPolW1);
  uint16_t* f2 = reinterpret_cast<uint16_t*>(net + lz::kPolW2);
  uint16_t* f3 = reinterpret_cast<uint16_t*>(net + lz::kPolW3);
  float* c1 = reinterpret_cast<float*>(net + lz::kPolB1);
  float* c2 = reinterpret_cast<float*>(net + lz::kPolB2);
  float* c3 = reinterpret_cast<float*>(net + lz::kPolB3);
  for (int lane = 0; lane < 64; ++lane) {
    const int r = lane & 31, h = lane >> 5;
    for (int j = 0; j < 8; ++j) {
      for (int t = 0; t < 4; ++t) {  // layer 1: A[row r][k = 8h + j], natural k order
        const int k = 8 * h + j;
        f1[(t * 64 + lane) * 8 + j] =
            bf16_rne(k < O ? kTanhScale * w1[(32 * t + r) * O + k] : 0.0f);
      }
      for (int t = 0; t < 4; ++t)
        for (int kk = 0; kk < 8; ++kk)
          f2[((t * 8 + kk) * 64 + lane) * 8 + j] =
              bf16_rne(kTanhScale * w2[(32 * t + r) * kPolHidden + unit_of(kk, h, j)]);
      for (int kk = 0; kk < 8; ++kk)
        f3[(kk * 64 + lane) * 8 + j] =
            bf16_rne(r < rows3 ? w3[r * kPolHidden + unit_of(kk, h, j)] : 0.0f);
    }
  }
  for (int h = 0; h < 2; ++h)
    for (int g = 0; g < 16; ++g) {
      for (int t = 0; t < 4; ++t) {
        c1[(2 * t + h) * 16 + g] = kTanhScale * b1[32 * t + row_of(g, h)];
        c2[(2 * t + h) * 16 + g] = kTanhScale * b2[32 * t + row_of(g, h)];
      }
      c3[h * 16 + g] = row_of(g, h) < rows3 ? b3[row_of(g, h)] : 0.0f;
    }
}

// tanh_tab's coefficients (kF32Tanh in the blob)
const float kTanhTab[72 * 8] = {
    0.0f, 0x1.0000000000000p+0f, 0x1.c0e2b20000000p-22f, -0x1.555bea0000000p-2f, 0x1.06810a0000000p-11f, 0x1.0a051c0000000p-3f, 0.0f, 0.0f,
    0x1.fd59920000000p-4f, 0x1.f815240000000p-1f, -0x1.f574200000000p-4f, -0x1.40a4860000000p-2f, 0x1.51c1e40000000p-4f, 0x1.8de4da0000000p-4f, 0.0f, 0.0f,
    0x1.f597ea0000000p-3f, 0x1.e1499e0000000p-1f, -0x1.d77de40000000p-3f, -0x1.075b220000000p-2f, 0x1.258ef60000000p-3f, 0x1.784c640000000p-5f, 0.0f, 0.0f,
    0x1.6ef53e0000000p-2f, 0x1.be3fb80000000p-1f, -0x1.3fd3c00000000p-2f, -0x1.6e322a0000000p-3f, 0x1.5f12440000000p-3f, -0x1.76ae540000000p-8f, 0.0f, 0.0f,
    0x1.d9353e0000000p-2f, 0x1.92a9460000000p-1f, -0x1.7426460000000p-2f, -0x1.8264340000000p-4f, 0x1.559cc60000000p-3f, -0x1.634c080000000p-5f, 0.0f, 0.0f,
    0x1.1bf47e0000000p-1f, 0x1.6284c20000000p-1f, -0x1.893b040000000p-2f, -0x1.24e9760000000p-6f, 0x1.1c00ce0000000p-3f, -0x1.f82a900000000p-5f, 0.0f, 0.0f,
    0x1.45323e0000000p-1f, 0x1.3173b20000000p-1f, -0x1.8403fc0000000p-2f, 0x1.56a9400000000p-5f, 0x1.977e660000000p-4f, -0x1.00bcee0000000p-4f, 0.0f, 0.0f,
    0x1.6866500000000p-1f, 0x1.02500a0000000p-1f, -0x1.6ba8380000000p-2f, 0x1.4f4f300000000p-4f, 0x1.eb1db60000000p-5f, -0x1.b2d63e0000000p-5f, 0.0f, 0.0f,
    0x1.85efac0000000p-1f, 0x1.ae0dc20000000p-2f, -0x1.4787420000000p-2f, 0x1.a8a1900000000p-4f, 0x1.b57c4e0000000p-6f, -0x1.407aea0000000p-5f, 0.0f, 0.0f,
    0x1.9e5cb60000000p-1f, 0x1.6150040000000p-2f, -0x1.1df01e0000000p-2f, 0x1.c6cada0000000p-4f, 0x1.336ae80000000p-9f, -0x1.9e7f2e0000000p-6f, 0.0f, 0.0f,
    0x1.b2523c0000000p-1f, 0x1.1f25140000000p-2f, -0x1.e729ca0000000p-3f, 0x1.bbd41a0000000p-4f, -0x1.b407840000000p-7f, -0x1.c879220000000p-7f, 0.0f, 0.0f,
    0x1.c278a60000000p-1f, 0x1.cea7460000000p-3f, -0x1.970e820000000p-3f, 0x1.97f8360000000p-4f, -0x1.6603360000000p-6f, -0x1.7519460000000p-8f, 0.0f, 0.0f,
    0x1.cf6f980000000p-1f, 0x1.7216540000000p-3f, -0x1.4efc260000000p-3f, 0x1.67c6940000000p-4f, -0x1.9e1e4a0000000p-6f, -0x1.603d9c0000000p-12f, 0.0f, 0.0f,
    0x1.d9c6fa0000000p-1f, 0x1.265e340000000p-3f, -0x1.1064960000000p-3f, 0x1.33e9b00000000p-4f, -0x1.9ff4a80000000p-6f, 0x1.6a701c0000000p-9f, 0.0f, 0.0f,
    0x1.e1fbfa0000000p-1f, 0x1.d22ca20000000p-4f, -0x1.b6d87e0000000p-4f, 0x1.01bee00000000p-4f, -0x1.8292880000000p-6f, 0x1.1880380000000p-8f, 0.0f, 0.0f,
    0x1.e8789e0000000p-1f, 0x1.6fcfa60000000p-4f, -0x1.5ee8980000000p-4f, 0x1.a85d6c0000000p-5f, -0x1.56176c0000000p-6f, 0x1.38ecea0000000p-8f, 0.0f, 0.0f,
    0x1.ed95060000000p-1f, 0x1.2162c20000000p-4f, -0x1.16f9c80000000p-4f, 0x1.58f26e0000000p-5f, -0x1.24d6160000000p-6f, 0x1.3214000000000p-8f, 0.0f, 0.0f,
    0x1.f1994e0000000p-1f, 0x1.c65b1c0000000p-5f, -0x1.b993580000000p-5f, 0x1.15af780000000p-5f, -0x1.e9aec00000000p-7f, 0x1.16bf740000000p-8f, 0.0f, 0.0f,
    0x1.f4bfd60000000p-1f, 0x1.64108a0000000p-5f, -0x1.5c3d680000000p-5f, 0x1.bbc1f20000000p-6f, -0x1.9277020000000p-7f, 0x1.e5ac020000000p-9f, 0.0f, 0.0f,
    0x1.f737760000000p-1f, 0x1.16a7fc0000000p-5f, -0x1.11e0100000000p-5f, 0x1.608ac80000000p-6f, -0x1.46997e0000000p-7f, 0x1.9ab50e0000000p-9f, 0.0f, 0.0f,
    0x1.f925820000000p-1f, 0x1.b3afe20000000p-6f, -0x1.adda9c0000000p-6f, 0x1.16d5660000000p-6f, -0x1.0683400000000p-7f, 0x1.54263a0000000p-9f, 0.0f, 0.0f,
    0x1.faa7940000000p-1f, 0x1.5452000000000p-6f, -0x1.50c42c0000000p-6f, 0x1.b78e260000000p-7f, -0x1.a2f4000000000p-8f, 0x1.1581420000000p-9f, 0.0f, 0.0f,
    0x1.fbd50a0000000p-1f, 0x1.09a7a60000000p-6f, -0x1.077dd60000000p-6f, 0x1.5988ec0000000p-7f, -0x1.4c77120000000p-8f, 0x1.bfccd00000000p-10f, 0.0f, 0.0f,
    0x1.fcc04c0000000p-1f, 0x1.9e87d00000000p-7f, -0x1.9be6180000000p-7f, 0x1.0f10080000000p-7f, -0x1.06b6a00000000p-8f, 0x1.6650e60000000p-10f, 0.0f, 0.0f,
    0x1.fd77d20000000p-1f, 0x1.434a500000000p-7f, -0x1.41b0c00000000p-7f, 0x1.a8990a0000000p-8f, -0x1.9dd60e0000000p-9f, 0x1.1cecac0000000p-10f, 0.0f, 0.0f,
    0x1.fe06ec0000000p-1f, 0x1.f81bd80000000p-8f, -0x1.f62a160000000p-8f, 0x1.4c220c0000000p-8f, -0x1.451fa40000000p-9f, 0x1.c2fa040000000p-11f, 0.0f, 0.0f,
    0x1.fe767a0000000p-1f, 0x1.88ef660000000p-8f, -0x1.87c1060000000p-8f, 0x1.038d260000000p-8f, -0x1.fddc240000000p-10f, 0x1.639ac00000000p-11f, 0.0f, 0.0f,
    0x1.fecd6c0000000p-1f, 0x1.3238b60000000p-8f, -0x1.3181100000000p-8f, 0x1.955ae60000000p-9f, -0x1.8f2d7a0000000p-10f, 0x1.179dc40000000p-11f, 0.0f, 0.0f,
    0x1.ff112c0000000p-1f, 0x1.dd37d00000000p-9f, -0x1.dc58c00000000p-9f, 0x1.3c587c0000000p-9f, -0x1.3828040000000p-10f, 0x1.b6c8d60000000p-12f, 0.0f, 0.0f,
    0x1.ff45f60000000p-1f, 0x1.73cec00000000p-9f, -0x1.73474a0000000p-9f, 0x1.ed89380000000p-10f, -0x1.e7c4640000000p-11f, 0x1.57b4ac0000000p-12f, 0.0f, 0.0f,
    0x1.ff6f180000000p-1f, 0x1.21a7ae0000000p-9f, -0x1.21556a0000000p-9f, 0x1.80d9700000000p-10f, -0x1.7cd1160000000p-11f, 0x1.0ce2680000000p-12f, 0.0f, 0.0f,
    0x1.ff8f220000000p-1f, 0x1.c347040000000p-10f, -0x1.c2e3180000000p-10f, 0x1.2c03a80000000p-10f, -0x1.2927280000000p-11f, 0x1.a4466a0000000p-13f, 0.0f, 0.0f,
    0x1.ffa8180000000p-1f, 0x1.5f85ac0000000p-10f, -0x1.5f48f80000000p-10f, 0x1.d3a8a20000000p-11f, -0x1.cf8a840000000p-12f, 0x1.4832700000000p-13f, 0.0f, 0.0f,
    0x1.ffbb880000000p-1f, 0x1.11ce6e0000000p-10f, -0x1.11a98a0000000p-10f, 0x1.6c6dd60000000p-11f, -0x1.696d9a0000000p-12f, 0x1.0023620000000p-13f, 0.0f, 0.0f,
    0x1.ffcaac0000000p-1f, 0x1.aa87ce0000000p-11f, -0x1.aa5af40000000p-11f, 0x1.1bf2e20000000p-11f, -0x1.19bcb40000000p-12f, 0x1.8f9f0c0000000p-14f, 0.0f, 0.0f,
    0x1.ffd6780000000p-1f, 0x1.4c36520000000p-11f, -0x1.4c1b0a0000000p-11f, 0x1.ba702e0000000p-12f, -0x1.b725680000000p-13f, 0x1.37a1340000000p-14f, 0.0f, 0.0f,
    0x1.ffdfa80000000p-1f, 0x1.02bec80000000p-11f, -0x1.02ae2c0000000p-11f, 0x1.58aaf00000000p-12f, -0x1.5632180000000p-13f, 0x1.e5df3a0000000p-15f, 0.0f, 0.0f,
    0x1.ffe6ce0000000p-1f, 0x1.930b440000000p-12f, -0x1.92f7060000000p-12f, 0x1.0c7c6a0000000p-12f, -0x1.0a9da60000000p-13f, 0x1.7aad8a0000000p-15f, 0.0f, 0.0f,
    0x1.ffec620000000p-1f, 0x1.39e7820000000p-12f, -0x1.39db2a0000000p-12f, 0x1.a243ee0000000p-13f, -0x1.9f6bf40000000p-14f, 0x1.271a400000000p-15f, 0.0f, 0.0f,
    0x1.fff0b80000000p-1f, 0x1.e8f43c0000000p-13f, -0x1.e8e5260000000p-13f, 0x1.45c9dc0000000p-13f, -0x1.439da40000000p-14f, 0x1.cbe1040000000p-16f, 0.0f, 0.0f,
    0x1.fff41a0000000p-1f, 0x1.7ccec00000000p-13f, -0x1.7cc5840000000p-13f, 0x1.fb80320000000p-14f, -0x1.f829880000000p-15f, 0x1.6640d60000000p-16f, 0.0f, 0.0f,
    0x1.fff6bc0000000p-1f, 0x1.2894480000000p-13f, -0x1.288e9e0000000p-13f, 0x1.8b46180000000p-14f, -0x1.88b4ba0000000p-15f, 0x1.171a0c0000000p-16f, 0.0f, 0.0f,
    0x1.fff8c80000000p-1f, 0x1.cdf5a20000000p-14f, -0x1.cdeea60000000p-14f, 0x1.33dbd40000000p-14f, -0x1.31e0360000000p-15f, 0x1.b2ce400000000p-17f, 0.0f, 0.0f,
    0x1.fffa600000000p-1f, 0x1.67c7600000000p-14f, -0x1.67c30e0000000p-14f, 0x1.df8b600000000p-15f, -0x1.dc79c40000000p-16f, 0x1.52aa580000000p-17f, 0.0f, 0.0f,
    0x1.fffba00000000p-1f, 0x1.1832dc0000000p-14f, -0x1.18302e0000000p-14f, 0x1.757be60000000p-15f, -0x1.731cf80000000p-16f, 0x1.07d4f00000000p-17f, 0.0f, 0.0f,
    0x1.fffc980000000p-1f, 0x1.b470ec0000000p-15f, -0x1.b46d940000000p-15f, 0x1.22e0e40000000p-15f, -0x1.210ba60000000p-16f, 0x1.9b105c0000000p-18f, 0.0f, 0.0f,
    0x1.fffd580000000p-1f, 0x1.53e7140000000p-15f, -0x1.53e4f80000000p-15f, 0x1.c5151c0000000p-16f, -0x1.c239000000000p-17f, 0x1.400d220000000p-18f, 0.0f, 0.0f,
    0x1.fffdee0000000p-1f, 0x1.08b7b60000000p-15f, -0x1.08b6600000000p-15f, 0x1.60de040000000p-16f, -0x1.5ea5540000000p-17f, 0x1.f28c3a0000000p-19f, 0.0f, 0.0f,
    0x1.fffe640000000p-1f, 0x1.9c53760000000p-16f, -0x1.9c51c00000000p-16f, 0x1.12d13a0000000p-16f, -0x1.1118080000000p-17f, 0x1.8454820000000p-19f, 0.0f, 0.0f,
    0x1.fffebe0000000p-1f, 0x1.411ee60000000p-16f, -0x1.411dca0000000p-16f, 0x1.ac0f620000000p-17f, -0x1.a95f840000000p-18f, 0x1.2e64980000000p-19f, 0.0f, 0.0f,
    0x1.ffff060000000p-1f, 0x1.f42dde0000000p-17f, -0x1.f42c680000000p-17f, 0x1.4d60680000000p-17f, -0x1.4b4a280000000p-18f, 0x1.d70dd80000000p-20f, 0.0f, 0.0f,
    0x1.ffff3e0000000p-1f, 0x1.858a640000000p-17f, -0x1.85896a0000000p-17f, 0x1.03a2b60000000p-17f, -0x1.02031a0000000p-18f, 0x1.6ee1380000000p-20f, 0.0f, 0.0f,
    0x1.ffff680000000p-1f, 0x1.2f5ffa0000000p-17f, -0x1.2f5f520000000p-17f, 0x1.9469a00000000p-18f, -0x1.91ea5c0000000p-19f, 0x1.1df0ce0000000p-20f, 0.0f, 0.0f,
    0x1.ffff8a0000000p-1f, 0x1.d889a60000000p-18f, -0x1.d888be0000000p-18f, 0x1.3af4e80000000p-18f, -0x1.38fc400000000p-19f, 0x1.bcf95a0000000p-21f, 0.0f, 0.0f,
    0x1.ffffa40000000p-1f, 0x1.7003540000000p-18f, -0x1.7002b40000000p-18f, 0x1.ea946c0000000p-19f, -0x1.e789c40000000p-20f, 0x1.5ac44a0000000p-21f, 0.0f, 0.0f,
    0x1.ffffb80000000p-1f, 0x1.1e9be60000000p-18f, -0x1.1e9b7c0000000p-18f, 0x1.7e11e00000000p-19f, -0x1.7bcc880000000p-20f, 0x1.0ec8be0000000p-21f, 0.0f, 0.0f,
    0x1.ffffc80000000p-1f, 0x1.be6c3e0000000p-19f, -0x1.be6b9c0000000p-19f, 0x1.298dc20000000p-19f, -0x1.27ba2a0000000p-20f, 0x1.a4eaee0000000p-22f, 0.0f, 0.0f,
    0x1.ffffd40000000p-1f, 0x1.5bacb00000000p-19f, -0x1.5bac320000000p-19f, 0x1.cf76bc0000000p-20f, -0x1.cc7ce60000000p-21f, 0x1.46e1680000000p-22f, 0.0f, 0.0f,
    0x1.ffffde0000000p-1f, 0x1.0ec4f20000000p-19f, -0x1.0ec4900000000p-19f, 0x1.68f1bc0000000p-20f, -0x1.6696900000000p-21f, 0x1.fc8a4a0000000p-23f, 0.0f, 0.0f,
    0x1.ffffe60000000p-1f, 0x1.a5c0340000000p-20f, -0x1.a5bfa80000000p-20f, 0x1.191ab80000000p-20f, -0x1.1742f20000000p-21f, 0x1.8bd10e0000000p-23f, 0.0f, 0.0f,
    0x1.ffffec0000000p-1f, 0x1.4875bc0000000p-20f, -0x1.48755e0000000p-20f, 0x1.b5dbf00000000p-21f, -0x1.b3351a0000000p-22f, 0x1.35f54e0000000p-23f, 0.0f, 0.0f,
    0x1.fffff00000000p-1f, 0x1.ff9c180000000p-21f, -0x1.ff9ba20000000p-21f, 0x1.5503ba0000000p-21f, -0x1.531eac0000000p-22f, 0x1.e539840000000p-24f, 0.0f, 0.0f,
    0x1.fffff40000000p-1f, 0x1.8e712c0000000p-21f, -0x1.8e70b00000000p-21f, 0x1.09921a0000000p-21f, -0x1.07e4e20000000p-22f, 0x1.771bba0000000p-24f, 0.0f, 0.0f,
    0x1.fffff60000000p-1f, 0x1.364e9a0000000p-21f, -0x1.364e0a0000000p-21f, 0x1.9d9b540000000p-22f, -0x1.99fd1a0000000p-23f, 0x1.1c3ce60000000p-24f, 0.0f, 0.0f,
    0x1.fffff80000000p-1f, 0x1.e355b40000000p-22f, -0x1.e3555a0000000p-22f, 0x1.422b420000000p-22f, -0x1.4059560000000p-23f, 0x1.c98be20000000p-25f, 0.0f, 0.0f,
    0x1.fffffa0000000p-1f, 0x1.786be80000000p-22f, -0x1.786bb40000000p-22f, 0x1.f5d4f60000000p-23f, -0x1.f3812a0000000p-24f, 0x1.6887700000000p-25f, 0.0f, 0.0f,
    0x1.fffffc0000000p-1f, 0x1.25284a0000000p-22f, -0x1.2528040000000p-22f, 0x1.86cd8c0000000p-23f, -0x1.8485200000000p-24f, 0x1.1556120000000p-25f, 0.0f, 0.0f,
    0x1.fffffc0000000p-1f, 0x1.c89f580000000p-23f, -0x1.c89f6a0000000p-23f, 0x1.306a580000000p-23f, -0x1.2fd5d00000000p-24f, 0x1.c2272c0000000p-26f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.639e2c0000000p-23f, -0x1.639d480000000p-23f, 0x1.d9f5440000000p-24f, -0x1.d516000000000p-25f, 0x1.40da540000000p-26f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.14f49e0000000p-23f, -0x1.14f4b20000000p-23f, 0x1.7144f40000000p-24f, -0x1.705de60000000p-25f, 0x1.0f59800000000p-26f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.af62e00000000p-24f, -0x1.af60b00000000p-24f, 0x1.1f5d940000000p-24f, -0x1.1a7e740000000p-25f, 0x1.69ea620000000p-27f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.4ff6c80000000p-24f, -0x1.4ff5fe0000000p-24f, 0x1.bfc5e20000000p-25f, -0x1.bb37d80000000p-26f, 0x1.2ea2320000000p-27f, 0.0f, 0.0f,
};

// float32 MlpPolicy net (kF32* layout, see mlp_f32 / lz_internal.h)
void pack_net_f32(uint8_t* net, int O, int rows3, const float* w1, const float* b1, const float* w2,
                  const float* b2, const float* w3, const float* b3) {
  using lz::kPolHidden;
  float* f1 = reinterpret_cast<float*>(net + lz::kF32W1);
  float* f2 = reinterpret_cast<float*>(net + lz::kF32W2);
  float* c1 = reinterpret_cast<float*>(net + lz::kF32B1);
  float* c2 = reinterpret_cast<float*>(net + lz::kF32B2);
  float* hw = reinterpret_cast<float*>(net + lz::kF32H);
  float* hb = reinterpret_cast<float*>(net + lz::kF32HB);
  for (int lane = 0; lane < 64; ++lane) {
    const int r = lane & 31, h = lane >> 5;
    for (int t = 0; t < 4; ++t) {
      for (int s = 0; s < 4; ++s) {  // layer 1: A[row r][k = h] of k-step s = input 2s + h
        const int k = 2 * s + h;
        f1[(t * 64 + lane) * 4 + s] = k < O ? w1[(32 * t + r) * O + k] : 0.0f;
      }
      for (int q = 0; q < 64; ++q)  // layer 2: k-step q = input unit 32 (q >> 4) + row(q & 15, h)
        f2[((t * 16 + q / 4) * 64 + lane) * 4 + q % 4] =
            w2[(32 * t + r) * kPolHidden + 32 * (q >> 4) + row_of(q & 15, h)];
    }
  }
  for (int h = 0; h < 2; ++h)
    for (int g = 0; g < 16; ++g)
      for (int t = 0; t < 4; ++t) {
        c1[(2 * t + h) * 16 + g] = b1[32 * t + row_of(g, h)];
        c2[(2 * t + h) * 16 + g] = b2[32 * t + row_of(g, h)];
        for (int j = 0; j < rows3; ++j)
          hw[(j * 2 + h) * 64 + t * 16 + g] = w3[j * kPolHidden + 32 * t + row_of(g, h)];
      }
  for (int j = 0; j < rows3; ++j) hb[j] = b3[j];
}

// Attention-extractor actor-critic (kAtt* layout, see lz_internal.h / attn_extract).
// log2(e) / sqrt(head_dim 4): the Q projection is stored pre-scaled so that the
// kernel's softmax is exp2(s - max) on q.k directly.
constexpr double kAttQScale = 1.4426950408889634 / 2.0;

// row of a 32-row K|V or Q tile -> in_proj row (-1: zero padding).  A tile row r lands
// in lane half h = (r >> 2) & 1, register g = (r & 3) + 4 (r >> 3): group g >> 2 = r >> 3.
inline int kv_row(int r) {
  const int h = (r >> 2) & 1, grp = r >> 3, d = r & 3;
  return (grp < 2 ? 16 : 32) + 4 * (2 * h + (grp & 1)) + d;  // k heads 2h, 2h+1, then v
}
inline int q_row(int r) {
  const int h = (r >> 2) & 1, grp = r >> 3, d = r & 3;
  return grp < 2 ? 4 * (2 * h + grp) + d : -1;
}

// token dim held by element j of lane half h of a relu8 token fragment
inline int tok_dim(int h, int j) { return (j & 3) + 8 * (j >> 2) + 4 * h; }

// The attention actor-critics.  ln_w == nullptr: code/train.py's extractor (kAtt*
// layout, out_proj folded into post_fc, obs_dim <= 8); otherwise code/lorenz_filter/
// train.py's residual + LayerNorm extractor (kLn* layout, fc1 over <= 32 stacked dims).
void pack_attn(uint8_t* b, const lz_attn_policy* p, const float* ln_w, const float* ln_b) {
  using lz::kPolHidden;
  const bool ln = ln_w != nullptr;
  const int I = p->obs_dim;
  uint16_t* f1 = reinterpret_cast<uint16_t*>(b + (ln ? lz::kLnFc1W : lz::kAttFc1W));
  uint16_t* fkv = reinterpret_cast<uint16_t*>(b + (ln ? lz::kLnKvW : lz::kAttKvW));
  uint16_t* fq = reinterpret_cast<uint16_t*>(b + (ln ? lz::kLnQW : lz::kAttQW));
  uint16_t* fp = reinterpret_cast<uint16_t*>(b + (ln ? lz::kLnPostW : lz::kAttPostW));
  float* c1 = reinterpret_cast<float*>(b + (ln ? lz::kLnFc1B : lz::kAttFc1B));
  float* ckv = reinterpret_cast<float*>(b + (ln ? lz::kLnKvB : lz::kAttKvB));
  float* cq = reinterpret_cast<float*>(b + (ln ? lz::kLnQB : lz::kAttQB));
  float* cp = reinterpret_cast<float*>(b + (ln ? lz::kLnPostB : lz::kAttPostB));
  static_assert(lz::kAttTokens * lz::kAttTokDim == kPolHidden, "token split");
  // post_fc per token i: folded with out_proj (code/train.py, float64)
  //   Wf_i = W_post[:, 16i:16i+16] W_out,  b_f = b_post + sum_i W_post[:, 16i:16i+16] b_out
  // or, after the LayerNorm (lorenz_filter), W_post[:, 16i + tok_dim] itself
  std::vector<double> wf_buf((size_t)lz::kAttTokens * lz::kAttFeat * lz::kAttTokDim);
  auto wf = reinterpret_cast<double (*)[lz::kAttFeat][lz::kAttTokDim]>(wf_buf.data());
  double bfold[lz::kAttFeat];
  for (int f = 0; f < lz::kAttFeat; ++f) {
    double acc = p->post_b[f];
    for (int i = 0; i < lz::kAttTokens; ++i)
      for (int d = 0; d < lz::kAttTokDim; ++d) {
        double w = 0.0;
        if (ln) {
          w = p->post_w[f * kPolHidden + 16 * i + d];
        } else {
          for (int e = 0; e < lz::kAttTokDim; ++e)
            w += (double)p->post_w[f * kPolHidden + 16 * i + e] * (double)p->out_proj_w[e * 16 + d];
        }
        wf[i][f][d] = w;
      }
    if (!ln)
      for (int i = 0; i < lz::kAttTokens; ++i)
        for (int e = 0; e < lz::kAttTokDim; ++e)
          acc += (double)p->post_w[f * kPolHidden + 16 * i + e] * (double)p->out_proj_b[e];
    bfold[f] = acc;
  }
  for (int lane = 0; lane < 64; ++lane) {
    const int r = lane & 31, h = lane >> 5;
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * h + j;       // natural k (obs, head outputs)
      const int td = tok_dim(h, j);  // token dim of a relu8 / LayerNorm fragment
      for (int t = 0; t < 4; ++t) {
        if (ln) {
          for (int s = 0; s < 2; ++s) {
            const int kk = 16 * s + k;  // stacked input dim
            f1[((t * 2 + s) * 64 + lane) * 8 + j] =
                bf16_rne(kk < I ? p->fc1_w[(32 * t + r) * I + kk] : 0.0f);
          }
        } else {
          f1[(t * 64 + lane) * 8 + j] = bf16_rne(k < I ? p->fc1_w[(32 * t + r) * I + k] : 0.0f);
        }
      }
      fkv[lane * 8 + j] = bf16_rne(p->in_proj_w[kv_row(r) * 16 + td]);
      const int qr = q_row(r);
      fq[lane * 8 + j] =
          bf16_rne(qr < 0 ? 0.0f : (float)(kAttQScale * (double)p->in_proj_w[qr * 16 + td]));
      for (int i = 0; i < lz::kAttTokens; ++i)
        for (int T = 0; T < 2; ++T)
          fp[((2 * i + T) * 64 + lane) * 8 + j] =
              bf16_rne((float)wf[i][32 * T + r][ln ? td : k]);
      if (ln) {  // out_proj: rows 0-15 = W_out, natural k (the head outputs)
        uint16_t* fo = reinterpret_cast<uint16_t*>(b + lz::kLnOutW);
        fo[lane * 8 + j] = bf16_rne(r < 16 ? p->out_proj_w[r * 16 + k] : 0.0f);
      }
    }
  }
  for (int h = 0; h < 2; ++h)
    for (int g = 0; g < 16; ++g) {
      const int r = row_of(g, h);
      for (int t = 0; t < 4; ++t) c1[(2 * t + h) * 16 + g] = p->fc1_b[32 * t + r];
      ckv[h * 16 + g] = p->in_proj_b[kv_row(r)];
      cq[h * 16 + g] = q_row(r) < 0 ? 0.0f : (float)(kAttQScale * (double)p->in_proj_b[q_row(r)]);
      for (int T = 0; T < 2; ++T) cp[(2 * T + h) * 16 + g] = (float)bfold[32 * T + r];
      if (ln) {
        float* co = reinterpret_cast<float*>(b + lz::kLnOutB);
        co[h * 16 + g] = r < 16 ? p->out_proj_b[r] : 0.0f;
        if (g < 8) {
          reinterpret_cast<float*>(b + lz::kLnGamma)[h * 8 + g] = ln_w[tok_dim(h, g)];
          reinterpret_cast<float*>(b + lz::kLnBeta)[h * 8 + g] = ln_b[tok_dim(h, g)];
        }
      }
    }
  // the two [128,128] Tanh nets: layer 1 reads the 64 features as 4 k-steps of relu8
  // fragments (feature unit_of(s, h, j)); layers 2 and 3 as in pack_net
  const float* W1[2] = {p->pi_w1, p->vf_w1};
  const float* B1[2] = {p->pi_b1, p->vf_b1};
  const float* W2[2] = {p->pi_w2, p->vf_w2};
  const float* B2[2] = {p->pi_b2, p->vf_b2};
  const float* W3[2] = {p->act_w, p->val_w};
  const float* B3[2] = {p->act_b, p->val_b};
  const int rows3[2] = {p->act_dim, 1};
  for (int n = 0; n < 2; ++n) {
    uint8_t* net = b + (ln ? (n == 0 ? lz::kLnPi : lz::kLnVf) : (n == 0 ? lz::kAttPi : lz::kAttVf));
    uint16_t* g1 = reinterpret_cast<uint16_t*>(net + lz::kAttW1);
    uint16_t* g2 = reinterpret_cast<uint16_t*>(net + lz::kAttW2);
    uint16_t* g3 = reinterpret_cast<uint16_t*>(net + lz::kAttW3);
    float* d1 = reinterpret_cast<float*>(net + lz::kAttB1);
    float* d2 = reinterpret_cast<float*>(net + lz::kAttB2);
    float* d3 = reinterpret_cast<float*>(net + lz::kAttB3);
    for (int lane = 0; lane < 64; ++lane) {
      const int r = lane & 31, h = lane >> 5;
      for (int j = 0; j < 8; ++j) {
        for (int t = 0; t < 4; ++t) {
          for (int s = 0; s < 4; ++s)
            g1[((t * 4 + s) * 64 + lane) * 8 + j] =
                bf16_rne(kTanhScale * W1[n][(32 * t + r) * lz::kAttFeat + unit_of(s, h, j)]);
          for (int kk = 0; kk < 8; ++kk)
            g2[((t * 8 + kk) * 64 + lane) * 8 + j] =
                bf16_rne(kTanhScale * W2[n][(32 * t + r) * kPolHidden + unit_of(kk, h, j)]);
        }
        for (int kk = 0; kk < 8; ++kk)
          g3[(kk * 64 + lane) * 8 + j] =
              bf16_rne(r < rows3[n] ? W3[n][r * kPolHidden + unit_of(kk, h, j)] : 0.0f);
      }
    }
    for (int h = 0; h < 2; ++h)
      for (int g = 0; g < 16; ++g) {
        for (int t = 0; t < 4; ++t) {
          d1[(2 * t + h) * 16 + g] = kTanhScale * B1[n][32 * t + row_of(g, h)];
          d2[(2 * t + h) * 16 + g] = kTanhScale * B2[n][32 * t + row_of(g, h)];
        }
        d3[h * 16 + g] = row_of(g, h) < rows3[n] ? B3[n][row_of(g, h)] : 0.0f;
      }
  }
}

// The attention actor-critics in float32 (kAF* layout, lz_internal.h; 16x16x4 tiles:
// lane (r = lane & 15, G = lane >> 4) holds A[row r][k = G] of every k-step): ln_w ==
// nullptr for code/train.py's extractor, else code/lorenz_filter/train.py's residual +
// LayerNorm variant (fc1 over <= 32 stacked inputs).  Nothing is folded or rescaled
// except Q's exact 1/sqrt(4) = 0.5.
void pack_attn_f32(uint8_t* b, const lz_attn_policy* p, const float* ln_w, const float* ln_b) {
  using lz::kPolHidden;
  const int I = p->obs_dim;
  float* f1 = reinterpret_cast<float*>(b + lz::kAFFc1W);
  float* fk = reinterpret_cast<float*>(b + lz::kAFKW);
  float* fv = reinterpret_cast<float*>(b + lz::kAFVW);
  float* fq = reinterpret_cast<float*>(b + lz::kAFQW);
  float* fo = reinterpret_cast<float*>(b + lz::kAFOW);
  float* fp = reinterpret_cast<float*>(b + lz::kAFPostW);
  for (int lane = 0; lane < 64; ++lane) {
    const int r = lane & 15, G = lane >> 4;
    for (int t = 0; t < lz::kAttTokens; ++t)  // fc1 tile t = token t; k-step s: input 4s + G
      for (int s = 0; s < 8; ++s) {
        const int k = 4 * s + G;
        f1[((t * 2 + s / 4) * 64 + lane) * 4 + s % 4] = k < I ? p->fc1_w[(16 * t + r) * I + k] : 0.0f;
      }
    for (int s = 0; s < 4; ++s) {  // k-step s: token / attention-output dim 4G + s
      const int d = 4 * G + s;
      fk[lane * 4 + s] = p->in_proj_w[(16 + r) * 16 + d];
      fv[lane * 4 + s] = p->in_proj_w[(32 + r) * 16 + d];
      fq[lane * 4 + s] = 0.5f * p->in_proj_w[r * 16 + d];
      fo[lane * 4 + s] = p->out_proj_w[r * 16 + d];
    }
    for (int u = 0; u < 4; ++u)
      for (int i = 0; i < lz::kAttTokens; ++i)
        for (int s = 0; s < 4; ++s)
          fp[((u * 8 + i) * 64 + lane) * 4 + s] = p->post_w[(16 * u + r) * kPolHidden + 16 * i + 4 * G + s];
  }
  float* c1 = reinterpret_cast<float*>(b + lz::kAFFc1B);
  for (int u = 0; u < kPolHidden; ++u) c1[u] = p->fc1_b[u];
  for (int d = 0; d < 16; ++d) {
    reinterpret_cast<float*>(b + lz::kAFKB)[d] = p->in_proj_b[16 + d];
    reinterpret_cast<float*>(b + lz::kAFVB)[d] = p->in_proj_b[32 + d];
    reinterpret_cast<float*>(b + lz::kAFQB)[d] = 0.5f * p->in_proj_b[d];
    reinterpret_cast<float*>(b + lz::kAFOB)[d] = p->out_proj_b[d];
    reinterpret_cast<float*>(b + lz::kAFGam)[d] = ln_w ? ln_w[d] : 1.0f;
    reinterpret_cast<float*>(b + lz::kAFBet)[d] = ln_b ? ln_b[d] : 0.0f;
  }
  for (int f = 0; f < lz::kAttFeat; ++f) reinterpret_cast<float*>(b + lz::kAFPostB)[f] = p->post_b[f];
  const float* W1[2] = {p->pi_w1, p->vf_w1};
  const float* B1[2] = {p->pi_b1, p->vf_b1};
  const float* W2[2] = {p->pi_w2, p->vf_w2};
  const float* B2[2] = {p->pi_b2, p->vf_b2};
  const float* W3[2] = {p->act_w, p->val_w};
  const float* B3[2] = {p->act_b, p->val_b};
  const int rows3[2] = {p->act_dim, 1};
  for (int n = 0; n < 2; ++n) {
    uint8_t* net = b + (n == 0 ? lz::kAFPi : lz::kAFVf);
    float* g1 = reinterpret_cast<float*>(net + lz::kAFN1);
    float* g2 = reinterpret_cast<float*>(net + lz::kAFN2);
    for (int lane = 0; lane < 64; ++lane) {
      const int r = lane & 15, G = lane >> 4;
      for (int t = 0; t < 8; ++t) {
        for (int f = 0; f < 4; ++f)  // layer 1: k-step 4f + s = feature 16f + 4G + s
          for (int s = 0; s < 4; ++s)
            g1[((t * 4 + f) * 64 + lane) * 4 + s] = W1[n][(16 * t + r) * lz::kAttFeat + 16 * f + 4 * G + s];
        for (int q = 0; q < 8; ++q)  // layer 2: k-step 4q + s = unit 16q + 4G + s
          for (int s = 0; s < 4; ++s)
            g2[((t * 8 + q) * 64 + lane) * 4 + s] = W2[n][(16 * t + r) * kPolHidden + 16 * q + 4 * G + s];
      }
    }
    for (int u = 0; u < kPolHidden; ++u) {
      reinterpret_cast<float*>(net + lz::kAFNB1)[u] = B1[n][u];
      reinterpret_cast<float*>(net + lz::kAFNB2)[u] = B2[n][u];
      for (int j = 0; j < rows3[n]; ++j)
        reinterpret_cast<float*>(net + lz::kAFNH)[j * kPolHidden + u] = W3[n][j * kPolHidden + u];
    }
    for (int j = 0; j < rows3[n]; ++j) reinterpret_cast<float*>(net + lz::kAFNHB)[j] = B3[n][j];
  }
}

// The opt-in i8x4 nets (lz_internal.h kAX*): float32 -> V = rint(v 2^q), |V| <= 2^28, as
// four balanced int8 digits (U = V + 0x808080: bytes 0..2 of U ^ 0x80, then U >> 24); q of
// a weight row = 28 - e of its largest |w| = f 2^e.  oracle/lz_oracle.c orc_i8x_* restates
// this independently (tests/test_i8x4_host.py).
int i8x_q(float m) {
  int e = 0;
  (void)std::frexp(m, &e);
  return 28 - e;
}
void i8x_digits(float v, int q, int8_t* d) {
  const int32_t V = (int32_t)std::nearbyint(std::ldexp(v, q));
  const int32_t U = (int32_t)((uint32_t)V + 0x808080u);
  d[0] = (int8_t)((U & 0xff) ^ 0x80);
  d[1] = (int8_t)(((U >> 8) & 0xff) ^ 0x80);
  d[2] = (int8_t)(((U >> 16) & 0xff) ^ 0x80);
  d[3] = (int8_t)(U >> 24);
}
int i8x_row_q(const float* w, int K) {
  float m = 0.0f;
  for (int k = 0; k < K; ++k) m = std::fmax(m, std::fabs(w[k]));
  return i8x_q(m);
}

// pack_attn_f32's blob with the pi / vf nets' two wide layers as digits + row shifts
void pack_attn_i8x4(uint8_t* b, const lz_attn_policy* p, const float* ln_w, const float* ln_b) {
  using lz::kPolHidden;
  pack_attn_f32(b, p, ln_w, ln_b);
  const float* W1[2] = {p->pi_w1, p->vf_w1};
  const float* W2[2] = {p->pi_w2, p->vf_w2};
  {  // post_attention_fc [64, 128]: digits over kAFPostW, row shifts in the pi slot
    int8_t* gp = reinterpret_cast<int8_t*>(b + lz::kAFPostW);
    int16_t* sp = reinterpret_cast<int16_t*>(b + lz::kAFPi + lz::kAXPostSh);
    int qp[lz::kAttFeat];
    for (int f = 0; f < lz::kAttFeat; ++f) {
      qp[f] = i8x_row_q(p->post_w + f * kPolHidden, kPolHidden);
      sp[f] = (int16_t)(24 - qp[f]);
    }
    int8_t d[4];
    for (int lane = 0; lane < 64; ++lane) {
      const int m = lane & 15, G = lane >> 4;
      for (int u = 0; u < 4; ++u)
        for (int kb = 0; kb < 2; ++kb)
          for (int f = 0; f < 4; ++f)
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * u + m;
              i8x_digits(p->post_w[row * kPolHidden + 64 * kb + 16 * f + 4 * G + r], qp[row], d);
              for (int i = 0; i < 4; ++i) gp[(((u * 2 + kb) * 4 + i) * 64 + lane) * 16 + 4 * f + r] = d[i];
            }
    }
  }
  for (int n = 0; n < 2; ++n) {
    uint8_t* net = b + (n == 0 ? lz::kAFPi : lz::kAFVf);
    int8_t* g1 = reinterpret_cast<int8_t*>(net + lz::kAXN1);
    int8_t* g2 = reinterpret_cast<int8_t*>(net + lz::kAXN2);
    int16_t* s1 = reinterpret_cast<int16_t*>(net + lz::kAXSh1);
    int16_t* s2 = reinterpret_cast<int16_t*>(net + lz::kAXSh2);
    int q1[kPolHidden], q2[kPolHidden];
    for (int u = 0; u < kPolHidden; ++u) {
      q1[u] = i8x_row_q(W1[n] + u * lz::kAttFeat, lz::kAttFeat);
      q2[u] = i8x_row_q(W2[n] + u * kPolHidden, kPolHidden);
      s1[u] = (int16_t)(24 - q1[u]);
      s2[u] = (int16_t)(24 - q2[u] - 28);
    }
    int8_t d[4];
    for (int lane = 0; lane < 64; ++lane) {
      const int m = lane & 15, G = lane >> 4;
      for (int t = 0; t < 8; ++t) {
        const int u = 16 * t + m;
        for (int f = 0; f < 4; ++f)
          for (int r = 0; r < 4; ++r) {
            const int j = 4 * f + r;
            i8x_digits(W1[n][u * lz::kAttFeat + 16 * f + 4 * G + r], q1[u], d);
            for (int i = 0; i < 4; ++i) g1[((t * 4 + i) * 64 + lane) * 16 + j] = d[i];
            for (int kb = 0; kb < 2; ++kb) {
              i8x_digits(W2[n][u * kPolHidden + 64 * kb + 16 * f + 4 * G + r], q2[u], d);
              for (int i = 0; i < 4; ++i) g2[(((t * 2 + kb) * 4 + i) * 64 + lane) * 16 + j] = d[i];
            }
          }
      }
    }
  }
}

void pack_gauss(float* ls, int act_dim, const float* log_std) {
  // [log_std(4)][scale(4)][2 scale^2 (4)][log scale (4)]: torch Normal's
  // scale = exp(log_std), var = scale**2 (the kernel divides by 2 * var), log(scale)
  for (int j = 0; j < act_dim; ++j) {
    const float sc = std::exp(log_std[j]);
    ls[j] = log_std[j];
    ls[4 + j] = sc;
    ls[8 + j] = 2.0f * (sc * sc);
    ls[12 + j] = std::log(sc);
  }
}

lz_status pfail(lz_status s, const char* msg) {
  return lz::set_error(s, msg);
}

}  // namespace

extern "C" {

int64_t lz_policy_blob_bytes(void) { return lz::kPolBlobBytes; }

lz_status lz_policy_pack(const lz_mlp_policy* p, void* host_blob, int64_t cap) {
  if (!p || !host_blob) return pfail(LZ_ERR_INVALID, "policy/blob is NULL");
  if (cap < lz::kPolBlobBytes) return pfail(LZ_ERR_INVALID, "blob capacity too small");
  if (p->obs_dim < 1 || p->obs_dim > lz::kPolMaxObs || p->act_dim < 1 || p->act_dim > lz::kPolMaxAct)
    return pfail(LZ_ERR_UNSUPPORTED, "policy supports obs_dim 1..8 and act_dim 1..4");
  const float* req[] = {p->pi_w1, p->pi_b1, p->pi_w2, p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2,
                        p->vf_b2, p->act_w, p->act_b, p->val_w, p->val_b, p->log_std};
  for (const float* q : req)
    if (!q) return pfail(LZ_ERR_INVALID, "a policy weight pointer is NULL");
  uint8_t* b = static_cast<uint8_t*>(host_blob);
  std::memset(b, 0, lz::kPolBlobBytes);
  pack_net(b, p->obs_dim, p->act_dim, p->pi_w1, p->pi_b1, p->pi_w2, p->pi_b2, p->act_w, p->act_b);
  pack_net(b + lz::kPolNet, p->obs_dim, 1, p->vf_w1, p->vf_b1, p->vf_w2, p->vf_b2, p->val_w,
           p->val_b);
  pack_gauss(reinterpret_cast<float*>(b + lz::kPolLogStd), p->act_dim, p->log_std);
  return LZ_OK;
}

lz_status lz_policy_pack_hidden(const lz_mlp_policy* p, int32_t hidden, void* host_blob,
                                int64_t cap) {
  // a [hidden, hidden] net zero-padded to 128 units: a padded unit's pre-activation is
  // exactly 0, tanh(0) = 0, and its zero weights add exact zeros downstream -- the
  // 128-wide kernel computes the narrower net unchanged
  if (!p) return pfail(LZ_ERR_INVALID, "policy is NULL");
  if (hidden == lz::kPolHidden) return lz_policy_pack(p, host_blob, cap);
  if (hidden < 1 || hidden > lz::kPolHidden)
    return pfail(LZ_ERR_UNSUPPORTED, "hidden width must be 1..128");
  if (p->obs_dim < 1 || p->obs_dim > lz::kPolMaxObs || p->act_dim < 1 || p->act_dim > lz::kPolMaxAct)
    return pfail(LZ_ERR_UNSUPPORTED, "policy supports obs_dim 1..8 and act_dim 1..4");
  const float* req[] = {p->pi_w1, p->pi_b1, p->pi_w2, p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2,
                        p->vf_b2, p->act_w, p->act_b, p->val_w, p->val_b, p->log_std};
  for (const float* q : req)
    if (!q) return pfail(LZ_ERR_INVALID, "a policy weight pointer is NULL");
  const int H = lz::kPolHidden, O = p->obs_dim, A = p->act_dim;
  std::vector<float> buf((size_t)2 * (H * O + H + H * H + H) + (size_t)(A + 1) * H, 0.0f);
  float* q = buf.data();
  auto pad = [&](const float* src, int rows, int cols, int prow, int pcol) {
    float* dst = q;
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) dst[r * pcol + c] = src[r * cols + c];
    q += (size_t)prow * pcol;
    return dst;
  };
  lz_mlp_policy w = *p;
  w.pi_w1 = pad(p->pi_w1, hidden, O, H, O);
  w.pi_b1 = pad(p->pi_b1, 1, hidden, 1, H);
  w.pi_w2 = pad(p->pi_w2, hidden, hidden, H, H);
  w.pi_b2 = pad(p->pi_b2, 1, hidden, 1, H);
  w.vf_w1 = pad(p->vf_w1, hidden, O, H, O);
  w.vf_b1 = pad(p->vf_b1, 1, hidden, 1, H);
  w.vf_w2 = pad(p->vf_w2, hidden, hidden, H, H);
  w.vf_b2 = pad(p->vf_b2, 1, hidden, 1, H);
  w.act_w = pad(p->act_w, A, hidden, A, H);
  w.val_w = pad(p->val_w, 1, hidden, 1, H);
  return lz_policy_pack(&w, host_blob, cap);
}

int64_t lz_policy_f32_blob_bytes(void) { return lz::kF32BlobBytes; }

// layer 2 of a packed float32 MlpPolicy net (pack_net_f32) as i8x4 digits + row shifts
static void pack_net_i8x4(uint8_t* net, const float* w2) {
  using lz::kPolHidden;
  int8_t* g2 = reinterpret_cast<int8_t*>(net + lz::kF32W2);
  int16_t* sh = reinterpret_cast<int16_t*>(net + lz::kF32Sh2);
  int q[kPolHidden];
  for (int u = 0; u < kPolHidden; ++u) q[u] = i8x_row_q(w2 + u * kPolHidden, kPolHidden);
  int8_t d[4];
  for (int lane = 0; lane < 64; ++lane) {
    const int m = lane & 31, h = lane >> 5;
    for (int T = 0; T < 4; ++T) {
      const int u = 32 * T + m;
      for (int kb = 0; kb < 4; ++kb)
        for (int j = 0; j < 16; ++j) {
          i8x_digits(w2[u * kPolHidden + 32 * kb + row_of(j, h)], q[u], d);
          for (int i = 0; i < 4; ++i) g2[(((T * 4 + kb) * 4 + i) * 64 + lane) * 16 + j] = d[i];
        }
    }
  }
  for (int T = 0; T < 4; ++T)
    for (int h = 0; h < 2; ++h)
      for (int g = 0; g < 16; ++g) sh[(2 * T + h) * 16 + g] = (int16_t)(24 - q[32 * T + row_of(g, h)] - 28);
}

static lz_status pack_mlp_f32(const lz_mlp_policy* p, int32_t hidden, void* host_blob, int64_t cap, bool i8);

lz_status lz_policy_pack_f32(const lz_mlp_policy* p, int32_t hidden, void* host_blob, int64_t cap) {
  return pack_mlp_f32(p, hidden, host_blob, cap, false);
}

lz_status lz_policy_pack_i8x4(const lz_mlp_policy* p, int32_t hidden, void* host_blob, int64_t cap) {
  return pack_mlp_f32(p, hidden, host_blob, cap, true);
}

static lz_status pack_mlp_f32(const lz_mlp_policy* p, int32_t hidden, void* host_blob, int64_t cap, bool i8) {
  if (!p || !host_blob) return pfail(LZ_ERR_INVALID, "policy/blob is NULL");
  if (cap < lz::kF32BlobBytes) return pfail(LZ_ERR_INVALID, "blob capacity too small");
  if (hidden < 1 || hidden > lz::kPolHidden) return pfail(LZ_ERR_UNSUPPORTED, "hidden width must be 1..128");
  if (p->obs_dim < 1 || p->obs_dim > lz::kPolMaxObs || p->act_dim < 1 || p->act_dim > lz::kPolMaxAct)
    return pfail(LZ_ERR_UNSUPPORTED, "policy supports obs_dim 1..8 and act_dim 1..4");
  const float* req[] = {p->pi_w1, p->pi_b1, p->pi_w2, p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2,
                        p->vf_b2, p->act_w, p->act_b, p->val_w, p->val_b, p->log_std};
  for (const float* q : req)
    if (!q) return pfail(LZ_ERR_INVALID, "a policy weight pointer is NULL");
  // zero-pad a [hidden, hidden] net to the kernel's 128 units (as lz_policy_pack_hidden):
  // a padded unit is tanh(0) = 0 with zero weights, each of its chain steps fma(0, w, acc)
  // returns acc unchanged
  const int H = lz::kPolHidden, O = p->obs_dim, A = p->act_dim;
  std::vector<float> buf((size_t)2 * (H * O + H + H * H + H) + (size_t)(A + 1) * H, 0.0f);
  float* q = buf.data();
  auto pad = [&](const float* src, int rows, int cols, int prow, int pcol) {
    float* dst = q;
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) dst[r * pcol + c] = src[r * cols + c];
    q += (size_t)prow * pcol;
    return dst;
  };
  const float* pw1 = pad(p->pi_w1, hidden, O, H, O);
  const float* pb1 = pad(p->pi_b1, 1, hidden, 1, H);
  const float* pw2 = pad(p->pi_w2, hidden, hidden, H, H);
  const float* pb2 = pad(p->pi_b2, 1, hidden, 1, H);
  const float* vw1 = pad(p->vf_w1, hidden, O, H, O);
  const float* vb1 = pad(p->vf_b1, 1, hidden, 1, H);
  const float* vw2 = pad(p->vf_w2, hidden, hidden, H, H);
  const float* vb2 = pad(p->vf_b2, 1, hidden, 1, H);
  const float* aw = pad(p->act_w, A, hidden, A, H);
  const float* uw = pad(p->val_w, 1, hidden, 1, H);
  uint8_t* b = static_cast<uint8_t*>(host_blob);
  std::memset(b, 0, lz::kF32BlobBytes);
  if (i8) {
    for (const float* w : {pw2, vw2})
      for (int k = 0; k < H * H; ++k)
        if (!std::isfinite(w[k])) return pfail(LZ_ERR_INVALID, "i8x4: layer 2 weights must be finite");
  }
  pack_net_f32(b, O, A, pw1, pb1, pw2, pb2, aw, p->act_b);
  pack_net_f32(b + lz::kF32Net, O, 1, vw1, vb1, vw2, vb2, uw, p->val_b);
  if (i8) {
    pack_net_i8x4(b, pw2);
    pack_net_i8x4(b + lz::kF32Net, vw2);
  }
  pack_gauss(reinterpret_cast<float*>(b + lz::kF32LogStd), A, p->log_std);
  lz::blob_tag(i8 ? LZ_BLOB_MLP_I8X4 : LZ_BLOB_MLP_F32, reinterpret_cast<uint32_t*>(b + lz::kF32Tag));
  // c_j 8^-j: the kernel's Horner runs in u = 8 t (tanh_tab)
  float* tt = reinterpret_cast<float*>(b + lz::kF32Tanh);
  for (int k = 0; k < 72; ++k)
    for (int j = 0; j < 8; ++j) tt[8 * k + j] = std::ldexp(kTanhTab[8 * k + j], -3 * j);
  tt[8 * 72] = 1.0f;  // segment 72: the constant 1 (the rest stays zero)
  return LZ_OK;
}

int64_t lz_attn_policy_blob_bytes(void) { return lz::kAttBlobBytes; }

lz_status lz_attn_policy_pack(const lz_attn_policy* p, void* host_blob, int64_t cap) {
  if (!p || !host_blob) return pfail(LZ_ERR_INVALID, "policy/blob is NULL");
  if (cap < lz::kAttBlobBytes) return pfail(LZ_ERR_INVALID, "blob capacity too small");
  if (p->obs_dim < 1 || p->obs_dim > lz::kPolMaxObs || p->act_dim < 1 || p->act_dim > lz::kPolMaxAct)
    return pfail(LZ_ERR_UNSUPPORTED, "policy supports obs_dim 1..8 and act_dim 1..4");
  const float* req[] = {p->fc1_w, p->fc1_b, p->in_proj_w, p->in_proj_b, p->out_proj_w,
                        p->out_proj_b, p->post_w, p->post_b, p->pi_w1, p->pi_b1, p->pi_w2,
                        p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2, p->vf_b2, p->act_w, p->act_b,
                        p->val_w, p->val_b, p->log_std};
  for (const float* q : req)
    if (!q) return pfail(LZ_ERR_INVALID, "a policy weight pointer is NULL");
  uint8_t* b = static_cast<uint8_t*>(host_blob);
  std::memset(b, 0, lz::kAttBlobBytes);
  pack_attn(b, p, nullptr, nullptr);
  pack_gauss(reinterpret_cast<float*>(b + lz::kAttLogStd), p->act_dim, p->log_std);
  return LZ_OK;
}

int64_t lz_attn_ln_policy_blob_bytes(void) { return lz::kLnBlobBytes; }

lz_status lz_attn_ln_policy_pack(const lz_attn_ln_policy* q, void* host_blob, int64_t cap) {
  if (!q || !host_blob) return pfail(LZ_ERR_INVALID, "policy/blob is NULL");
  if (cap < lz::kLnBlobBytes) return pfail(LZ_ERR_INVALID, "blob capacity too small");
  const lz_attn_policy* p = &q->attn;
  if (p->obs_dim < 1 || p->obs_dim > lz::kLnMaxIn || p->act_dim < 1 || p->act_dim > lz::kPolMaxAct)
    return pfail(LZ_ERR_UNSUPPORTED, "policy supports input dims 1..32 and act_dim 1..4");
  const float* req[] = {p->fc1_w, p->fc1_b, p->in_proj_w, p->in_proj_b, p->out_proj_w,
                        p->out_proj_b, p->post_w, p->post_b, p->pi_w1, p->pi_b1, p->pi_w2,
                        p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2, p->vf_b2, p->act_w, p->act_b,
                        p->val_w, p->val_b, p->log_std, q->ln_w, q->ln_b};
  for (const float* r : req)
    if (!r) return pfail(LZ_ERR_INVALID, "a policy weight pointer is NULL");
  uint8_t* b = static_cast<uint8_t*>(host_blob);
  std::memset(b, 0, lz::kLnBlobBytes);
  pack_attn(b, p, q->ln_w, q->ln_b);
  pack_gauss(reinterpret_cast<float*>(b + lz::kLnLogStd), p->act_dim, p->log_std);
  return LZ_OK;
}

int64_t lz_attn_policy_f32_blob_bytes(void) { return lz::kAFBlobBytes; }

static lz_status pack_attn_f32_checked(const lz_attn_policy* p, const float* ln_w, const float* ln_b,
                                       void* host_blob, int64_t cap, int max_in) {
  if (!p || !host_blob) return pfail(LZ_ERR_INVALID, "policy/blob is NULL");
  if (cap < lz::kAFBlobBytes) return pfail(LZ_ERR_INVALID, "blob capacity too small");
  if (p->obs_dim < 1 || p->obs_dim > max_in || p->act_dim < 1 || p->act_dim > lz::kPolMaxAct)
    return pfail(LZ_ERR_UNSUPPORTED, max_in == lz::kPolMaxObs
                                         ? "policy supports obs_dim 1..8 and act_dim 1..4"
                                         : "policy supports input dims 1..32 and act_dim 1..4");
  const float* req[] = {p->fc1_w, p->fc1_b, p->in_proj_w, p->in_proj_b, p->out_proj_w,
                        p->out_proj_b, p->post_w, p->post_b, p->pi_w1, p->pi_b1, p->pi_w2,
                        p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2, p->vf_b2, p->act_w, p->act_b,
                        p->val_w, p->val_b, p->log_std};
  for (const float* q : req)
    if (!q) return pfail(LZ_ERR_INVALID, "a policy weight pointer is NULL");
  uint8_t* b = static_cast<uint8_t*>(host_blob);
  std::memset(b, 0, lz::kAFBlobBytes);
  pack_attn_f32(b, p, ln_w, ln_b);
  pack_gauss(reinterpret_cast<float*>(b + lz::kAFLogStd), p->act_dim, p->log_std);
  lz::blob_tag(ln_w ? LZ_BLOB_ATTN_LN_F32 : LZ_BLOB_ATTN_F32, reinterpret_cast<uint32_t*>(b + lz::kAFTag));
  float* tt = reinterpret_cast<float*>(b + lz::kAFTanh);
  for (int k = 0; k < 72; ++k)
    for (int j = 0; j < 8; ++j) tt[8 * k + j] = std::ldexp(kTanhTab[8 * k + j], -3 * j);
  tt[8 * 72] = 1.0f;  // segment 72: the constant 1 (the rest stays zero)
  return LZ_OK;
}

lz_status lz_attn_policy_pack_f32(const lz_attn_policy* p, void* host_blob, int64_t cap) {
  return pack_attn_f32_checked(p, nullptr, nullptr, host_blob, cap, lz::kPolMaxObs);
}

static lz_status pack_attn_i8x4_checked(const lz_attn_policy* p, const float* ln_w, const float* ln_b,
                                        void* host_blob, int64_t cap, int max_in) {
  const lz_status st = pack_attn_f32_checked(p, ln_w, ln_b, host_blob, cap, max_in);
  if (st != LZ_OK) return st;
  const float* w[5] = {p->pi_w1, p->vf_w1, p->post_w, p->pi_w2, p->vf_w2};
  for (int j = 0; j < 5; ++j) {
    const int cnt = lz::kPolHidden * (j < 3 ? lz::kAttFeat : lz::kPolHidden);
    for (int k = 0; k < cnt; ++k)
      if (!std::isfinite(w[j][k]))
        return pfail(LZ_ERR_INVALID, "i8x4: the nets' and post_attention_fc's weights must be finite");
  }
  pack_attn_i8x4(static_cast<uint8_t*>(host_blob), p, ln_w, ln_b);
  lz::blob_tag(ln_w ? LZ_BLOB_ATTN_LN_I8X4 : LZ_BLOB_ATTN_I8X4,
               reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(host_blob) + lz::kAFTag));
  return LZ_OK;
}

int32_t lz_policy_blob_format(const void* host_blob, int64_t size) {
  if (!host_blob) return LZ_BLOB_UNKNOWN;
  const uint8_t* b = static_cast<const uint8_t*>(host_blob);
  uint32_t t[4];
  if (size >= lz::kAFBlobBytes) {  // attention families: the tag in the pi slot's spare bytes
    std::memcpy(t, b + lz::kAFTag, 16);
    for (uint32_t f : {LZ_BLOB_ATTN_F32, LZ_BLOB_ATTN_I8X4, LZ_BLOB_ATTN_LN_F32, LZ_BLOB_ATTN_LN_I8X4})
      if (lz::blob_tag_ok(t, f)) return (int32_t)f;
  }
  if (size >= lz::kF32BlobBytes) {
    std::memcpy(t, b + lz::kF32Tag, 16);
    for (uint32_t f : {LZ_BLOB_MLP_F32, LZ_BLOB_MLP_I8X4})
      if (lz::blob_tag_ok(t, f)) return (int32_t)f;
  }
  return LZ_BLOB_UNKNOWN;
}

lz_status lz_attn_policy_pack_i8x4(const lz_attn_policy* p, void* host_blob, int64_t cap) {
  return pack_attn_i8x4_checked(p, nullptr, nullptr, host_blob, cap, lz::kPolMaxObs);
}

lz_status lz_attn_ln_policy_pack_i8x4(const lz_attn_ln_policy* p, void* host_blob, int64_t cap) {
  if (!p) return pfail(LZ_ERR_INVALID, "policy is NULL");
  if (!p->ln_w || !p->ln_b) return pfail(LZ_ERR_INVALID, "layer_norm weight / bias is NULL");
  return pack_attn_i8x4_checked(&p->attn, p->ln_w, p->ln_b, host_blob, cap, lz::kAFMaxIn);
}

lz_status lz_attn_ln_policy_pack_f32(const lz_attn_ln_policy* p, void* host_blob, int64_t cap) {
  if (!p) return pfail(LZ_ERR_INVALID, "policy is NULL");
  if (!p->ln_w || !p->ln_b) return pfail(LZ_ERR_INVALID, "layer_norm weight / bias is NULL");
  return pack_attn_f32_checked(&p->attn, p->ln_w, p->ln_b, host_blob, cap, lz::kAFMaxIn);
}

}  // extern "C"
