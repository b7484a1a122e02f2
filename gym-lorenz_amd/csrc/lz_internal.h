// Internal structures shared by the C-ABI (lz_api.cpp) and the kernels
// (lz_kernels.hip).  Not part of the public ABI.
#pragma once
#include <stdint.h>

#include "lorenz_env.h"

namespace lz {

constexpr int kBlock = 256;   // envs per workgroup (4 waves of 64 lanes)
constexpr int kMaxPlanes = 12;

// Everything a launch needs, passed by value as the kernel argument.
struct KArgs {
  void* pl[kMaxPlanes];      // SoA state planes (see lorenz_env.h plane enums)
  const void* act;           // T [N, A]   (rollout: [K, N, A])
  const double* noise;       // double [N, 3] injected noise or nullptr
  void* obs;                 // T [N, O]   (rollout: [K, N, O])
  void* rew;                 // T [N]      (rollout: [K, N])
  uint8_t* done;             // uint8 [N]  (rollout: [K, N])
  int32_t* done_idx32;       // step: compact env indices (nullable)
  int64_t* done_idx64;       // rollout: compact k*N+env (nullable)
  void* term_obs;            // compact terminal observations (nullable)
  int64_t term_cap;          // rollout capacity of the compact buffers
  int32_t* counter;          // compact-list cursor for this launch
  int32_t* counter_next;     // the other slot, zeroed by this launch for the next
  const float* bc;           // PMSM: {(float)(1 - beta1**k), (float)(1 - beta2**k)}, k < bc_len
  const uint8_t* mask;       // reset: env selection (nullable)
  const void* init;          // reset: injected initial states (nullable)
  int64_t n;                 // envs in this handle
  int64_t gid0;              // global id of env 0 (RNG key)
  uint64_t seed;
  // Call counter (the RNG counter): device-resident so that launches can be captured
  // in a hipGraph and replayed.  Launch reads *tick_in; block 0 lane 0 writes
  // *tick_out = tick + tick_adv (the other slot of a 2-slot ping-pong selected by the
  // host-side call parity).  Rollout step k uses tick + k.
  const uint64_t* tick_in;
  uint64_t* tick_out;
  uint64_t tick_adv;
  int32_t bc_len;
  int32_t max_steps;         // truncation limit (0 = none)
  int32_t t_done_step;       // reference 't == T' step (-1 = never)
  int32_t count_steps;       // maintain the STEP plane
  uint32_t flags;            // LZ_FLAG_*
  int32_t vec_ok;            // act/obs base pointers 16-B aligned
  int32_t K;                 // rollout length
  int32_t variant;           // step-kernel tuning variant (lz_config.reserved[0])
  float alpha;               // PMSM
  int32_t num_cus;           // compute units (k_step_multi's tile count; fills the padding
                             // before prm, so no other kernel's argument offsets move)
  double prm[LZ_MAX_PARAMS];
};

// VecNormalize epilogue of the step kernel (lz_step_vecnorm).  Per-workgroup float64
// partials of the batch moments, column-major [W][n_wg] with W = 2 (O + 1) columns:
// sums of obs column 0..O-1, of the returns, then the sums of squares likewise;
// every workgroup of the normalise pass of lz_vecnorm_apply reduces them (the same
// fixed order, lz_rms_math.h vn_col_totals) and applies the statistics updates; with
// LZ_VN_DEFER k_vn_colsum (the step's only other launch) reduces them into the moments.
// kVnBlock envs per step workgroup on the fused path: 1024, so that a 262,144-env step
// leaves 256 partials per column for every normalise workgroup to read.
constexpr int kVnMaxObs = 8;
constexpr int kVnBlock = 1024;
// Fused path (n <= vn_fuse_max_wg() * kVnBlock envs, 262,144 by default): 1024-env step
// workgroups and the normalise pass reduces the partials itself -- two launches.  Split
// path (larger n): 256-env step workgroups and k_vn_colsum reduces the partials once,
// one workgroup per column -- three launches.  Measured same-box against the round-1
// design (always split): fused +13% at PMSM 262k, but -10% at 393k and 1M.
int vn_fuse_max_wg();        // LZ_VN_FUSE_MAX_WG
bool vn_fused(int64_t n);
int vn_block(int64_t n);     // the step workgroup size for n envs (LZ_VN_BLOCK for A/B)
struct VArgs {
  double* returns;     // [N] VecNormalize.returns
  double* part;        // [W][n_wg]
  double* old;         // [2O+1 obs][3 returns] statistics snapshot (step block 0)
  double* tot;         // [W] column totals (split path: k_vn_colsum -> normalise pass)
  double* obs_state;   // obs_rms mean[O], var[O], count
  double* ret_state;   // ret_rms mean, var, count
  double* moments;     // LZ_VN_DEFER: [2O+1 obs][3 returns] batch moments out
  int32_t* n_done_out; // the step's done count (device)
  double gamma;
  uint32_t flags;      // LZ_VN_*
  int32_t n_wg;
  int32_t fused;       // the normalise pass reduces the partials itself (n_wg small)
};

// Policy-in-the-loop rollout (lz_policy.hip): SB3 ActorCriticPolicy (MlpPolicy,
// net_arch pi=[128,128] vf=[128,128], Tanh, DiagGaussian) packed as bf16 MFMA
// fragments.  Blob layout (bytes) -- produced by lz_policy_pack, read by the kernel:
//   net 0 = policy (mlp_extractor.policy_net + action_net) at 0,
//   net 1 = value (mlp_extractor.value_net + value_net) at kPolNet,
//   log_std float[4] at kPolLogStd.
// Per net: W1 A-fragments [4 out tiles][64 lanes] bf16x8, W2 [4][8 k-steps][64] bf16x8,
// W3 [8 k-steps][64] bf16x8, biases as accumulator initialisers b1/b2 [4][2 halves][16]
// f32 and b3 [2][16] f32 (see lz_policy.hip for the fragment index maps).
constexpr int kPolHidden = 128;
constexpr int kPolW1 = 0;
constexpr int kPolW2 = kPolW1 + 4 * 64 * 16;
constexpr int kPolW3 = kPolW2 + 4 * 8 * 64 * 16;
constexpr int kPolB1 = kPolW3 + 8 * 64 * 16;
constexpr int kPolB2 = kPolB1 + 4 * 2 * 16 * 4;
constexpr int kPolB3 = kPolB2 + 4 * 2 * 16 * 4;
constexpr int kPolNet = kPolB3 + 2 * 16 * 4;       // 46208 B
constexpr int kPolLogStd = 2 * kPolNet;
constexpr int kPolBlobBytes = kPolLogStd + 64;     // 92480 B (resident in LDS)
constexpr int kPolMaxObs = 8, kPolMaxAct = 4;

// The same actor-critic behind code/train.py:52-95's AttentionFeaturesExtractor
// (shared features extractor: fc1 obs->128 ReLU, 8 tokens x 16, 4-head self-attention,
// post_attention_fc 128->64 ReLU; then pi/vf [128,128] Tanh on the 64 features).
// Blob layout (lz_attn_policy_pack; fragment maps in lz_policy.hip):
//   extractor: fc1 A-fragments [4 tiles][64] bf16x8 + bias [4][2][16] f32;
//              K|V projection [64] bf16x8 + bias [2][16]; Q projection (pre-scaled by
//              log2(e)/sqrt(4)) [64] + bias [2][16];
//              out_proj folded into post_attention_fc: per token [8][2 tiles][64] +
//              bias [2][2][16]
//   net 0 (pi) / net 1 (vf): W1 [4 out tiles][4 k-steps][64], W2 [4][8][64], W3 [8][64],
//              b1 / b2 [4][2][16], b3 [2][16]
//   log_std / Normal constants float[16]
constexpr int kAttTokens = 8, kAttTokDim = 16, kAttFeat = 64;
constexpr int kAttFc1W = 0;
constexpr int kAttFc1B = kAttFc1W + 4 * 64 * 16;
constexpr int kAttKvW = kAttFc1B + 4 * 2 * 16 * 4;
constexpr int kAttKvB = kAttKvW + 64 * 16;
constexpr int kAttQW = kAttKvB + 2 * 16 * 4;
constexpr int kAttQB = kAttQW + 64 * 16;
constexpr int kAttPostW = kAttQB + 2 * 16 * 4;
constexpr int kAttPostB = kAttPostW + kAttTokens * 2 * 64 * 16;
constexpr int kAttExt = kAttPostB + 2 * 2 * 16 * 4;  // 23552 B
constexpr int kAttW1 = 0;
constexpr int kAttW2 = kAttW1 + 4 * 4 * 64 * 16;
constexpr int kAttW3 = kAttW2 + 4 * 8 * 64 * 16;
constexpr int kAttB1 = kAttW3 + 8 * 64 * 16;
constexpr int kAttB2 = kAttB1 + 4 * 2 * 16 * 4;
constexpr int kAttB3 = kAttB2 + 4 * 2 * 16 * 4;
constexpr int kAttNet = kAttB3 + 2 * 16 * 4;       // 58496 B
constexpr int kAttPi = kAttExt, kAttVf = kAttExt + kAttNet;
constexpr int kAttLogStd = kAttExt + 2 * kAttNet;
constexpr int kAttBlobBytes = kAttLogStd + 64;     // 140608 B (resident in LDS)

// code/lorenz_filter/train.py:54-103's variant of the extractor: the attention output
// goes through out_proj, a residual connection and LayerNorm(16) per token before
// post_attention_fc (so out_proj cannot be folded), on VecFrameStack(n_stack) inputs of
// up to 32 stacked dims (fc1 K = 2 x 16).  Blob (lz_attn_ln_policy_pack):
//   fc1 [4 tiles][2 k-steps][64] + bias; K|V and Q as kAtt*; out_proj [64] (rows 16-31
//   zero) + bias [2][16]; LayerNorm weight / bias [2 halves][8] f32 each; post_fc
//   [8][2][64] (columns in the token-fragment order) + bias [2][2][16]; nets and
//   log_std as kAtt*.
constexpr int kLnMaxIn = 32, kLnMaxStack = 4;
constexpr int kLnFc1W = 0;
constexpr int kLnFc1B = kLnFc1W + 4 * 2 * 64 * 16;
constexpr int kLnKvW = kLnFc1B + 4 * 2 * 16 * 4;
constexpr int kLnKvB = kLnKvW + 64 * 16;
constexpr int kLnQW = kLnKvB + 2 * 16 * 4;
constexpr int kLnQB = kLnQW + 64 * 16;
constexpr int kLnOutW = kLnQB + 2 * 16 * 4;
constexpr int kLnOutB = kLnOutW + 64 * 16;
constexpr int kLnGamma = kLnOutB + 2 * 16 * 4;
constexpr int kLnBeta = kLnGamma + 16 * 4;
constexpr int kLnPostW = kLnBeta + 16 * 4;
constexpr int kLnPostB = kLnPostW + kAttTokens * 2 * 64 * 16;
constexpr int kLnExt = kLnPostB + 2 * 2 * 16 * 4;   // 28928 B
constexpr int kLnPi = kLnExt, kLnVf = kLnExt + kAttNet;
constexpr int kLnLogStd = kLnExt + 2 * kAttNet;
constexpr int kLnBlobBytes = kLnLogStd + 64;       // 145984 B (resident in LDS)

// The MlpPolicy again at the precision SB3 runs it (float32 operands, float32
// accumulation): f32-input MFMA (v_mfma_f32_32x32x2_f32, bit-for-bit a k-ordered fmaf
// chain) for the two hidden layers, the heads as per-lane fmaf chains, tanh as a
// piecewise polynomial in fmaf -- every result is a fixed sequence of correctly rounded
// operations the C oracle restates exactly.  Blob (lz_policy_pack_f32), per net:
//   W1 [4 out tiles][64 lanes][4 k-steps] f32 (lane (r, h), k-step s: W1[32t + r][2s + h]),
//   W2 [4 out tiles][16 quads][64 lanes][4] f32 (k-step q = 4 quad + e: input unit
//      32 (q >> 4) + row(q & 15, h)), b1 / b2 [4][2 halves][16] f32 as accumulator
//   initialisers, head rows [4][2 halves][64] f32 (element 16t + g: unit 32t + row(g, h)),
//   head bias [4] f32; net 0 = pi (action_net head), net 1 = vf (value_net head);
//   log_std / Normal constants float[16] after both nets, then the tanh coefficient
//   table (lz_policy.hip tanh_tab).
constexpr int kF32W1 = 0;
constexpr int kF32W2 = kF32W1 + 4 * 64 * 4 * 4;
constexpr int kF32B1 = kF32W2 + 4 * 16 * 64 * 4 * 4;
constexpr int kF32B2 = kF32B1 + 4 * 2 * 16 * 4;
constexpr int kF32H = kF32B2 + 4 * 2 * 16 * 4;
constexpr int kF32HB = kF32H + 4 * 2 * 64 * 4;
// opt-in i8x4 (lz_policy_pack_i8x4, LZ_POLICY_I8X4): layer 2's weights at kF32W2 as digits
// ([4 out tiles][4 k-blocks][4 digits][64 lanes][16 B], byte j of lane (m, h) = digit of
// W2[32T + m][32kb + row(j, h)]) and its row shifts 24 - q - 28 here, int16 in the
// accumulator order [4 tiles][2 halves][16] (unused by the float32 kernels)
constexpr int kF32Sh2 = kF32HB + 64;
constexpr int kF32Net = kF32Sh2 + 4 * 2 * 16 * 2;    // 73024 B
constexpr int kF32LogStd = 2 * kF32Net;
// tanh_tab's table: 72 polynomial segments of width 1/8 over [0, 9) and a 73rd, the
// constant 1 (|x| >= 9 clamps into it), 8 floats each
constexpr int kTanhSegs = 73;
constexpr int kF32Tanh = kF32LogStd + 64;
constexpr int kF32BlobBytes = kF32Tanh + kTanhSegs * 32;  // 148448 B (resident in LDS)

// The attention actor-critics at SB3's precision (float32 operands and accumulation;
// lz_attn_policy_pack_f32 / lz_attn_ln_policy_pack_f32 -> k_rollout_policy_attn_f32).
// Every product-sum runs on v_mfma_f32_16x16x4_f32 (a k-ordered fmaf chain: lane group
// G = lane >> 4 supplies k = G of each k-step) with the weights as the A operand: a wave
// holds 16 envs (column c = lane & 15), every 16-unit output tile lands as lane group G,
// register i = unit 4G + i -- token t = fc1 tile t, head G's key / query / value dims
// in lane group G -- and that layout is the next projection's k order (k-step s takes
// register s: input 4G + s), so nothing moves between lanes and each lane group runs
// one head's softmax.  Blob (bytes; "[tile][quad][64 lanes] f32x4" = 4 k-steps per lane
// per 16-B LDS read; biases, LayerNorm affine and head rows in natural order):
//   extractor: fc1 [8 tiles][2 quads][64] (k-step s: input 4s + G, zero past the input
//              width) + bias [128]; keys, values, queries (x 0.5 = 1/sqrt(4), exact),
//              out_proj: [64] f32x4 each (k-step s: token dim 4G + s) + biases [16];
//              LayerNorm weight / bias [16]; post_attention_fc [4 tiles][8 tokens][64]
//              (token i's 4 k-steps) + bias [64]
//   net 0 (pi) / net 1 (vf): layer 1 [8 tiles][4 quads][64] (k-step q = 4f + s: feature
//              16f + 4G + s), layer 2 [8 tiles][8 quads][64], b1 / b2 [128], head rows
//              [4][128], head bias [4]
//   log_std / Normal constants float[16], the tanh table (kF32Tanh's)
// Both nets do not fit in LDS with the extractor (54 + 2 x 100 KB): the workgroup keeps
// the extractor, the constants and ONE net slot, and LDS-DMAs pi / vf into the slot.
constexpr int kAFMaxIn = 32;                                // fc1 inputs: 8 k-steps, 2 quads
constexpr int kAFFc1W = 0;
constexpr int kAFFc1B = kAFFc1W + 8 * 2 * 64 * 16;
constexpr int kAFKW = kAFFc1B + 128 * 4;
constexpr int kAFVW = kAFKW + 64 * 16;
constexpr int kAFQW = kAFVW + 64 * 16;
constexpr int kAFOW = kAFQW + 64 * 16;
constexpr int kAFKB = kAFOW + 64 * 16;
constexpr int kAFVB = kAFKB + 16 * 4;
constexpr int kAFQB = kAFVB + 16 * 4;
constexpr int kAFOB = kAFQB + 16 * 4;
constexpr int kAFGam = kAFOB + 16 * 4;
constexpr int kAFBet = kAFGam + 16 * 4;
constexpr int kAFPostW = kAFBet + 16 * 4;
constexpr int kAFPostB = kAFPostW + 4 * 8 * 64 * 16;
constexpr int kAFExt = kAFPostB + 64 * 4;                   // 54,400 B
constexpr int kAFN1 = 0;
constexpr int kAFN2 = kAFN1 + 8 * 4 * 64 * 16;
constexpr int kAFNB1 = kAFN2 + 8 * 8 * 64 * 16;
constexpr int kAFNB2 = kAFNB1 + 128 * 4;
constexpr int kAFNH = kAFNB2 + 128 * 4;
constexpr int kAFNHB = kAFNH + 4 * 128 * 4;
constexpr int kAFNet = 100 * 1024;                          // 101,392 B padded to whole 1-KiB DMA pieces
static_assert(kAFNHB + 16 <= kAFNet, "attention net slot");
constexpr int kAFPi = kAFExt, kAFVf = kAFExt + kAFNet;
constexpr int kAFConst = 64 + kTanhSegs * 32;               // log_std consts + tanh table
constexpr int kAFLogStd = kAFExt + 2 * kAFNet;
constexpr int kAFTanh = kAFLogStd + 64;
constexpr int kAFBlobBytes = kAFLogStd + kAFConst;          // 261,600 B (device)
constexpr int kAFLdsBytes = kAFExt + kAFConst + kAFNet;     // 159,200 B (LDS)
// The opt-in "i8x4" nets (lz_attn_policy_pack_i8x4, LZ_POLICY_I8X4): the same blob, the
// same extractor, the same offsets -- the two wide layers' float32 weights replaced by
// their four int8 digits (4 B per weight either way, v_mfma_i32_16x16x64_i8 A operands)
// and two int16 tables of per-row shifts after the head bias.  Layer 1 tile t, digit i:
// lane (G, m) 16 B, byte 4f + r = digit i of W1[16t + m][16f + 4G + r]; layer 2 tile t,
// k-block kb, digit i: byte 4f + r = digit i of W2[16t + m][64kb + 16f + 4G + r].
// Shift of unit u: 24 - q_u (layer 1, the input's q subtracted in the kernel) and
// 24 - q_u - 28 (layer 2; its inputs are tanh outputs at q = 28).
constexpr int kAXN1 = kAFN1;                                // [8][4][64][16 B]
constexpr int kAXN2 = kAFN2;                                // [8][2][4][64][16 B]
static_assert(kAXN2 == kAXN1 + 8 * 4 * 64 * 16 && kAFNB1 == kAXN2 + 8 * 2 * 4 * 64 * 16, "i8x4 layout");
constexpr int kAXSh1 = kAFNHB + 16;                         // int16 [128]
constexpr int kAXSh2 = kAXSh1 + 128 * 2;                    // int16 [128]
// post_attention_fc in i8x4 too: its float32 weights at kAFPostW become digits ([4 tiles]
// [2 k-blocks][4 digits][64][16 B], byte 4f + r of lane (G, m) = digit of post_w[16u + m]
// [64kb + 16f + 4G + r]); the 64 row shifts (24 - q, int16) ride in the pi slot's spare bytes
// at kAXPostSh and are copied into LDS once per launch (the slot itself is overwritten).
constexpr int kAXPostSh = kAXSh2 + 128 * 2;                 // int16 [64], pi slot only
static_assert(kAXPostSh + 64 * 2 <= kAFNet, "i8x4 net slot");

// Blob format tag: the float32 and i8x4 blobs of one policy family have the
// same size and offsets, so only the launch's LZ_POLICY_I8X4 flag (and the entry point:
// attention vs attention + LayerNorm) says how to read one.  Every packer of those blobs
// writes a 16-B tag into spare bytes -- {kBlobMagic, format, ~format, kBlobMagic ^ format}
// -- and every float32 / i8x4 policy kernel compares it with the format its launch
// expects; on a mismatch the kernel's LDS copy of the blob is NaN (weights, Normal
// constants, tanh table), so every action, value, log-prob, reward and observation the
// launch writes is NaN instead of a silently wrong rollout.
constexpr uint32_t kBlobMagic = 0x42505A4Cu;  // "LZPB"
constexpr int kF32Tag = kF32HB + 48;          // net 0 (pi): the head bias uses 16 of its 64 B
constexpr int kAXTag = kAXPostSh + 64 * 2;    // the pi slot's spare bytes (f32 and i8x4 alike)
static_assert(kAXTag + 16 <= kAFNet, "blob tag in the attention net slot");
constexpr int kAFTag = kAFPi + kAXTag;
__host__ __device__ inline void blob_tag(uint32_t fmt, uint32_t t[4]) {
  t[0] = kBlobMagic;
  t[1] = fmt;
  t[2] = ~fmt;
  t[3] = kBlobMagic ^ fmt;
}
__host__ __device__ inline bool blob_tag_ok(const uint32_t t[4], uint32_t fmt) {
  return t[0] == kBlobMagic && t[1] == fmt && t[2] == ~fmt && t[3] == (kBlobMagic ^ fmt);
}

struct PArgs {
  const uint8_t* blob;     // device copy of the packed policy
  const float* obs_in;     // [N, O] raw observation at rollout start
  float* obs_last;         // [N, O] raw observation after K steps
  const double* norm;      // VecNormalize obs_rms: mean[O], var[O] (nullable)
  double eps, clip;
  float gamma;             // truncation bootstrap discount
  float act_lo, act_hi;    // action-space clip before env.step
  uint32_t pflags;         // LZ_POLICY_*
  float* act;              // [K, N, A] sampled (unclipped) actions
  float* logp;             // [K, N]
  float* val;              // [K, N]
  float* last_val;         // [N]
  double* partials;        // [grid * waves][2 * O] obs moment partials (nullable)
  const float* stack_in;   // kPair 4: [N, n_stack * O] VecFrameStack obs at rollout start
  float* stack_out;        // kPair 4: [N, n_stack * O] after the K steps
};

// SB3-exact VecNormalize in the float32 policy rollout (lz_policy_step_f32): one env
// step per launch, because step k's policy input is normalised with statistics that
// include step k's whole batch (VecNormalize.step_wait updates obs_rms, then normalises).
// Launch k < K: deferred truncation bootstrap of step k-1, normalise obs_src with the
// statistics p.norm holds (S_k), forward, sample, env step, raw obs -> p.obs_last, the
// float64 tile moments of that raw obs -> tiles; then k_vn_tile_update (lz_rms.hip)
// turns snap (= S_k) + the tile moments into S_{k+1} in place.  Launch K (final): the
// bootstrap of step K-1 and the last values only.
//
// Moment order (restated by oracle/lz_oracle.c orc_vn_tile_totals): tile t = envs
// 32t .. 32t+31 (0.0 past n); per tile a 32-lane butterfly v_l += v_{l ^ m}, m = 16, 8,
// 4, 2, 1 of (double)x (sums) and (double)x * (double)x (squares); per column thread
// tau < 256 sums tiles tau, tau + 256, ... from 0.0 in order, then the LDS tree
// s[tau] += s[tau + m], m = 128 .. 1; then RunningMeanStd.update_from_moments
// (lz_rms_math.h rms_new) with batch count n.
constexpr int kVnTile = 32;
struct PStepArgs {
  int32_t k;            // step of the collect (the tick advances once per step launch)
  int32_t final_;       // the epilogue launch (k == K)
  int64_t ntiles;       // ceil(n / kVnTile): column stride of tiles
  double* tiles;        // [2 O][ntiles] float64 tile moments of the step's raw obs
  double* snap;         // [2 O + 1] the statistics this launch normalised with (block 0)
  float* term;          // [N, O] raw terminal obs of the step's done envs (carry)
  const float* obs_src; // [N, O] raw obs the policy sees this step
};
// S_{k+1} from snap + tiles (moments == nullptr), or (moments != nullptr) the batch
// moments (n, sums[O], sums of squares[O]) for a multi-GPU all-reduce + lz_rms_update
int launch_vn_tile_update(const double* tiles, int64_t ntiles, int O, double batch,
                          const double* snap, double* state, double* moments, void* stream);
// tile moments of x [n, O] float32 in the order above (block 0 snapshots state -> snap)
int launch_obs_tile_moments(const float* x, int64_t n, int O, double* tiles, const double* state,
                            double* snap, void* stream);

// lz_rms internals for the fused VecNormalize step (lz_rms.hip)
int rms_dim(const lz_rms* r);
int rms_device(const lz_rms* r);
double* rms_state(lz_rms* r);  // mean[dim], var[dim], count
// RunningMeanStd.update_from_moments on `stream` (moments: count, sums, sums of squares)
int launch_rms_update(lz_rms* r, const double* moments, void* stream);
// The RunningMeanStd updates folded into the normalise pass (training, not deferred):
// every workgroup reduces the step's moment partials and derives the new statistics
// from them and the snapshot the step's block 0 took; workgroup 0 writes them back.
struct VnUpdate {
  const double* part;  // [2 (O + 1)][n_wg] partials to reduce here (fused), or nullptr
  int n_wg;
  const double* tot;   // [2 (O + 1)] totals k_vn_colsum left (split), or nullptr
                       // (both nullptr: no update in this pass)
  const double* old;   // [2O+1 obs][3 returns] snapshot of the statistics
  double batch;        // batch count n
  int upd_obs;         // obs_rms.update (TRAINING and NORM_OBS)
};
// normalised obs [n, O] / reward [n] / 0-1 dones [n] / terminal rows [*n_done, O]
// (lz_vecnorm_apply)
int launch_vn_apply(int f64, int O, int64_t n, const void* obs, const void* rew,
                    const uint8_t* done, const void* term, const int32_t* n_done,
                    double* obs_state, double* ret_state, int norm_obs, int norm_rew,
                    double eps, double clip_obs, double clip_rew, float* obs_n, float* rew_n,
                    uint8_t* dones, float* term_n, const VnUpdate& upd, const int32_t* counter,
                    int32_t* n_done_out, void* stream);

// The integrator picks the system's instantiation: the launchers' `system` argument is
// lz_config.system + kSysRK4 for an LZ_INT_RK4 handle of LORENZ3 / LORENZ4 (SysL3RK4 /
// SysL4RK4, lz_systems.h), else lz_config.system.
constexpr int kSysRK4 = 256;

// record the thread-local message lz_last_error() returns; returns s
lz_status set_error(lz_status s, const char* msg);

// host-side launchers (lz_kernels.hip)
int launch_reset(int system, int f64, const KArgs& a, void* stream);
int launch_step(int system, int f64, const KArgs& a, void* stream);

// Resident step server (lz_resident_step): ONE launch per process and device serves
// every handle that steps through lz_resident_step -- one wave per handle (n <= 64 envs
// each, up to kRsMaxHandles handles) plus ONE poller wave, so a DummyVecEnv of several
// drop-in envs shares one launch on one stream (one hardware queue).
//
// Requests travel in the server's REQUEST LINES: one 64-B line per member in mapped,
// coherent host memory (kRsLineWords 8-byte granules; 16 lines = 1 KiB).  Every granule
// is {tag = the request number's low 31 bits (bits 63..32), one 32-bit data word (bits
// 31..0)}, written by ONE aligned 8-byte host store, so a granule is read whole or not
// at all and needs no ordering (the handoff-granule form of the MI355X guide's hand-off
// table).  A request whose inputs fit in 8 words -- a 1-env handle: its actions (A
// float32 words) and injected noise (3 float64 = 6 words: PMSM / HR / TP / SC) -- travels
// INSIDE its line: the poller reads every member's line with one wave-wide load per poll
// (lanes 4k..4k+3 = line k, two granules each), accepts line k when all its used
// granules carry the same new tag (a torn read shows mixed tags and is simply read again
// at the next poll), copies the data words into LDS and hands the tag to member wave k
// through LDS.  One PCIe read round trip per request.  Larger handles (n > 1 env) use
// granule 0 as a command word only and their member wave reads the inputs from the
// handle's mailbox (the round-2 path: a second round trip).  (Rounds 2-3: one command
// word per member, payload always from the mailbox -- 6.0 us per call; a poller wave per
// handle slowed every request as handles were added: 5.3 -> 11.4 us at 8, 24.9 at 16,
// profiles/r03/resident.)  A member wave holds its handle's state in registers, serves
// requests `next`, `next + 1`, ... each exactly as one k_step launch would (step_body),
// writes obs | reward | done and the handle's state planes (pub: the copy
// lz_resident_read_state returns without stopping the server) into the mailbox and then
// *resp = the request's number (release, system scope).  All waves leave together: on an
// all-ones granule 0 in any line (stop), or after idle_ticks wall-clock ticks without a
// new request; each member stores its state back to the planes.  The host relaunches the
// server (with every registered handle) when a request finds it gone.
constexpr int kRsMaxHandles = 15;  // + the poller: 16 waves, one 1024-thread workgroup
constexpr int kRsLineWords = 8;    // granules per request line (64 B)
constexpr uint32_t kRsTagMask = 0x7fffffffu;  // tags: 31 bits (an all-ones granule = stop)
constexpr int kRsReplyWords = 64;  // tagged reply granules of a one-env handle (one per lane)
struct ResBox {
  int64_t* resp;        // device -> host: number of the last request served (mailbox path)
  const float* act;     // [n, A] (mailbox path)
  const double* noise;  // [n, 3] (mailbox path, with use_noise)
  void* obs;            // T [n, O]
  void* rew;            // T [n]
  uint8_t* done;        // [n]
  void* pub[kMaxPlanes];  // the published state planes [n] each (nullptr past n_planes)
  int32_t pub_es[kMaxPlanes];  // their element sizes
  int64_t next;         // first request this launch serves
  int32_t use_noise;
  int32_t inline_words; // >= 0: the request's inputs travel in its line (that many data
                        // words: act_words actions, then 6 noise words); -1: mailbox path
  int32_t act_words;    // action words in the line (0 for a system without actions)
  // The reply of a one-env handle (inline_words >= 0): rep_words 8-byte granules
  // {tag = request number (31 bits) << 32 | data word}, written by one wave-wide store (lane g
  // granule g) with no ordering among them -- the host accepts the reply when every granule
  // carries the request's tag.  Data words: obs at rep_obs, reward at rep_rew, the done byte
  // at rep_done, published plane p at rep_pub[p] (8-byte values at even offsets); nullptr
  // reply: the mailbox path (obs / rew / done / pub, then resp)
  uint64_t* reply;
  int32_t rep_words, rep_obs, rep_rew, rep_done;
  int32_t rep_pub[kMaxPlanes];
};
struct ResMember {      // one wave of the server
  KArgs a;
  ResBox box;
  int32_t system, f64;
};
// table: device copy of n members; one workgroup of 64 (n + 1) threads, wave n the poller
int launch_resident_multi(const ResMember* table, int n, const uint64_t* lines, uint64_t idle_ticks,
                          void* stream);
int launch_rollout(int system, int f64, const KArgs& a, void* stream);
// lz_get_launch_shape of lz_step (which = 1) / lz_rollout (which = 2): out[5] = kernel,
// envs per wave, waves per workgroup, workgroups, flags
int env_launch_shape(int which, int system, int f64, const KArgs& a, int32_t* out);
// gather (scatter = false: buf[i] = plane[idx[i]]) / scatter (plane[idx[i]] = buf[i]) of
// es-byte elements; indices outside [0, n) skipped / read as zero
int launch_plane_index(bool scatter, int es, void* plane, int64_t n, const int64_t* idx, int64_t count,
                       void* buf, void* stream);
int launch_step_vecnorm(int system, int f64, const KArgs& a, const VArgs& v, void* stream);
// Launch shape of the policy rollout (one workgroup per CU: the weights fill LDS).
//   >= 131,072 envs: 64 envs per wave (two 32-env MFMA column tiles, every lane steps
//                    an env), 8 waves per workgroup (2 per SIMD);
//   fewer, but enough for 2 waves per SIMD of 32 envs: 32 envs per wave, 8 waves;
//   fewer still (e.g. cfg5's 32,768 envs per GPU): 32 envs per wave, 4 waves (one per
//                    SIMD) running the policy and value nets interleaved in one
//                    instruction stream for ILP, with the 512 registers one wave per
//                    SIMD allows.
// Measured (profiles/r01/policy/ab_shapes.json): 32,768 envs +56% for the interleaved
// shape over 8 serial waves; 65,536 envs 8 serial waves +21% over it; 262,144 envs
// 64-env waves +30% over it.  lz_config.reserved[0] bit 5 / bit 6 force the
// (32, 8, serial) / interleaved shape, bit 7 selects the interleaved nets without the
// pipelined weight loads (A/B experiments).  The kernel's grid-stride
// tile loop is correct for any grid.
struct PolShape {
  int envs_per_wave, waves, pair, grid;
};
inline PolShape policy_shape(int64_t n, int variant, int num_cus) {
  PolShape s;
  const int64_t waves32 = (n + 31) / 32;
  if (variant & 32) s = {32, 8, 0, 0};
  else if ((variant & 64) || waves32 < 8 * (int64_t)num_cus) s = {32, 4, (variant & 128) ? 1 : 2, 0};
  else if (n < 131072) s = {32, 8, 0, 0};
  else s = {64, 8, 0, 0};
  const int64_t groups = ((n + s.envs_per_wave - 1) / s.envs_per_wave + s.waves - 1) / s.waves;
  s.grid = (int)(groups < num_cus ? groups : num_cus);
  return s;
}
int launch_rollout_policy(int system, const KArgs& a, const PArgs& p, const PolShape& sh,
                          void* stream);
// the float32 MlpPolicy (kF32* blob): 32 envs per wave, 8 waves (two per SIMD; the
// 146 KB blob leaves room for one workgroup per CU, the obs moments live in registers);
// below 8 tiles per CU 4 tiles per workgroup on 8 waves, the pi net and the env step in
// waves 0-3, the value net in waves 4-7 (pair = 1); the per-step kernel runs 4 waves there
PolShape f32_policy_shape(int64_t n, int num_cus, int variant);
int launch_rollout_policy_f32(int system, const KArgs& a, const PArgs& p, const PolShape& sh,
                              void* stream);
// SB3-exact VecNormalize: one step of the float32 policy rollout (PStepArgs above)
int launch_policy_step_f32(int system, const KArgs& a, const PArgs& p, const PStepArgs& s,
                           const PolShape& sh, void* stream);
// the attention-extractor policy (kAtt* blob): one shape, 32 envs per wave, 4 waves
// (one per SIMD: the 137 KB blob leaves room for one workgroup per CU)
PolShape attn_policy_shape(int64_t n, int num_cus);
int launch_rollout_policy_attn(int system, const KArgs& a, const PArgs& p, const PolShape& sh,
                               void* stream);
// the residual + LayerNorm extractor on VecFrameStack(n_stack) obs (kLn* blob);
// n_stack 1 or 4, same shape as attn_policy_shape
int launch_rollout_policy_attn_ln(int system, int n_stack, const KArgs& a, const PArgs& p,
                                  const PolShape& sh, void* stream);
// the attention actor-critics in float32 (kAF* blob): ln = 0 code/train.py's extractor,
// 1 the residual + LayerNorm variant on VecFrameStack(n_stack = 1 or 4); systems LORENZ3 /
// PMSM / HR; attn_f32_policy_shape's grid (16 envs per wave, 8 or 4 waves)
PolShape attn_f32_policy_shape(int64_t n, int num_cus, int ln);
int launch_rollout_policy_attn_f32(int system, int ln, int n_stack, const KArgs& a, const PArgs& p,
                                   const PolShape& sh, void* stream);
int launch_policy_moments_final(const double* partials, int nparts, int width, double count,
                                double* out, void* stream);

}  // namespace lz
