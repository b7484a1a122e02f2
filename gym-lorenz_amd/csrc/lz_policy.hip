// Policy in the loop: the SB3 actor-critic forward fused with the env
// step in a K-step rollout, plus RolloutBuffer.compute_returns_and_advantage.
//
// What the reference's learners run per env step (stable-baselines3 2.7.1, absent
// from the image; call sites code/lorenz_pmsm/train.py:155-178, code/lorenz_filter/
// train.py:117-127, code/gym_try.py:106-116):
//   OnPolicyAlgorithm.collect_rollouts:
//     actions, values, log_probs = policy(obs)       ActorCriticPolicy.forward
//     clipped = np.clip(actions, low, high); env.step(clipped)
//     truncated & terminal_observation: rewards += gamma * V(terminal_obs)
//     rollout_buffer.add(last_obs, actions, rewards, last_episode_starts, values, log_probs)
//   ActorCriticPolicy (MlpPolicy, net_arch pi=[128,128] vf=[128,128], Tanh):
//     latent_pi = tanh(W2 tanh(W1 obs + b1) + b2)   (mlp_extractor.policy_net)
//     mean = action_net(latent_pi); DiagGaussian(mean, exp(log_std)): a = mean + std*z
//     log_prob = sum_j Normal(mean_j, std_j).log_prob(a_j); value = value_net(latent_vf)
//
// MI355X mapping.  One wave owns a tile of 32 envs for all K steps.  Each 128-wide
// layer is a chain of v_mfma_f32_32x32x16_bf16 with the WEIGHTS as the A operand
// (32 output units x 16 inputs) and the ACTIVATIONS as the B operand (16 inputs x 32
// envs): the f32 accumulator of layer l (output units in the 16 registers, env on the
// lane) is, after tanh and a pairwise bf16 conversion, exactly the B fragment of layer
// l+1 -- no LDS round trip, no lane shuffles.  The k order inside such a fragment is
// permuted (register j of lane half h of k-step s holds unit 16s + 8(j>>2) + 4h + (j&3)
// of its 32-unit tile), so the packer stores W2/W3 columns in that order.  Biases are
// the accumulator initialisers.  All weights (92.5 KB as bf16 fragments) stay in LDS
// for the whole launch; a workgroup is 8 waves on one CU.
//   Per env-step: pi 6->128->128->A and vf 6->128->128->1 = 69 kFLOP useful (padded
//   MFMA work 90 kFLOP: K=16 for the 6 inputs, M=32 for the heads); 512 tanh.
// Lane halves: lanes l and l+32 hold the two k-halves of the same env column.  The env
// step, the sample and every store run in the h = 0 half (the head's rows 0..3 land
// there); the h = 1 half only contributes its MFMA operands (zero obs inputs).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lz_body.h"
#include "lz_internal.h"
#include "lz_philox.h"
#include "lz_systems.h"

namespace lz {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// tanh(x) = 1 - 2 / (exp(2x) + 1) = 1 - 2 / (2^(s x) + 1), s = 2 / ln 2: v_exp_f32 +
// v_rcp_f32; |error| <= 2e-7 over all x (+-inf limits exact), far below the bf16
// rounding every activation takes next.  The packer folds s into the tanh layers'
// weights and biases (bf16(s W), s b), so the accumulator already holds s x and the
// multiply is gone (one VALU op of five per activation).
__device__ __forceinline__ float tanh_scaled(float sx) {
  const float e = __builtin_amdgcn_exp2f(sx);
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int S>
__device__ __forceinline__ bf16x8 act8(const f32x16& c) {  // registers 8S..8S+7
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {  // one v_cvt_pk_bf16_f32 per pair (RNE)
    const f32x2 t = {tanh_scaled(c[8 * S + j]), tanh_scaled(c[8 * S + j + 1])};
    const bf16x2 b = __builtin_convertvector(t, bf16x2);
    r[j] = b[0];
    r[j + 1] = b[1];
  }
  return r;
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// One net (3 linear layers) on this wave's 32-env tile.  x = the layer-1 B fragment
// (lane half 0: obs[0..7], half 1: zeros).  Returns the head accumulator: lane (env
// l & 31, half h) register g = head row (g & 3) + 8 (g >> 2) + 4 h.
__device__ __forceinline__ f32x16 mlp_tile(const uint8_t* net, bf16x8 x, int lane) {
  // The weight fragments are loop-invariant LDS loads: without this barrier LLVM hoists
  // all 44 of them (176 VGPRs per net) out of the step loop and spills.  Re-reading
  // them from LDS every step costs ~0.7 KB/lane of LDS bandwidth, far from the limit.
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1 = reinterpret_cast<const bf16x8*>(net + kPolW1) + lane;
  const bf16x8* w2 = reinterpret_cast<const bf16x8*>(net + kPolW2) + lane;
  const bf16x8* w3 = reinterpret_cast<const bf16x8*>(net + kPolW3) + lane;
  const f32x16* b1 = reinterpret_cast<const f32x16*>(net + kPolB1) + h;
  const f32x16* b2 = reinterpret_cast<const f32x16*>(net + kPolB2) + h;
  const f32x16* b3 = reinterpret_cast<const f32x16*>(net + kPolB3) + h;
  bf16x8 h1[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 c = mfma(w1[t * 64], x, b1[2 * t]);
    h1[2 * t] = act8<0>(c);
    h1[2 * t + 1] = act8<1>(c);
  }
  // layer 2 tile by tile, each tile's two activation fragments consumed by the head
  // at once (k-steps 2t, 2t+1): only 2 of layer 2's 8 fragments are ever live
  f32x16 head = *b3;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    // the tile's 8 W2 fragments are issued together (32 VGPRs) so the MFMA chain
    // does not pay one LDS round trip per MFMA; the barriers keep the loads of
    // different tiles from piling up
    asm volatile("" ::: "memory");
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = w2[(t * 8 + kk) * 64];
    f32x16 c = b2[2 * t];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) c = mfma(wf[kk], h1[kk], c);
    head = mfma(w3[(2 * t) * 64], act8<0>(c), head);
    head = mfma(w3[(2 * t + 1) * 64], act8<1>(c), head);
  }
  return head;
}

// Both nets on the same 32-env tile in one instruction stream (layer by layer, tile by
// tile): two independent MFMA / tanh chains the scheduler can interleave, for the
// one-wave-per-SIMD small-batch shape where no other wave hides the latencies.
__device__ __forceinline__ void mlp_pair(const uint8_t* na, const uint8_t* nb, bf16x8 x, int lane,
                                         f32x16& head_a, f32x16& head_b) {
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1a = reinterpret_cast<const bf16x8*>(na + kPolW1) + lane;
  const bf16x8* w1b = reinterpret_cast<const bf16x8*>(nb + kPolW1) + lane;
  const bf16x8* w2a = reinterpret_cast<const bf16x8*>(na + kPolW2) + lane;
  const bf16x8* w2b = reinterpret_cast<const bf16x8*>(nb + kPolW2) + lane;
  const bf16x8* w3a = reinterpret_cast<const bf16x8*>(na + kPolW3) + lane;
  const bf16x8* w3b = reinterpret_cast<const bf16x8*>(nb + kPolW3) + lane;
  const f32x16* b1a = reinterpret_cast<const f32x16*>(na + kPolB1) + h;
  const f32x16* b1b = reinterpret_cast<const f32x16*>(nb + kPolB1) + h;
  const f32x16* b2a = reinterpret_cast<const f32x16*>(na + kPolB2) + h;
  const f32x16* b2b = reinterpret_cast<const f32x16*>(nb + kPolB2) + h;
  bf16x8 h1a[8], h1b[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 ca = mfma(w1a[t * 64], x, b1a[2 * t]);
    const f32x16 cb = mfma(w1b[t * 64], x, b1b[2 * t]);
    h1a[2 * t] = act8<0>(ca);
    h1b[2 * t] = act8<0>(cb);
    h1a[2 * t + 1] = act8<1>(ca);
    h1b[2 * t + 1] = act8<1>(cb);
  }
  head_a = *(reinterpret_cast<const f32x16*>(na + kPolB3) + h);
  head_b = *(reinterpret_cast<const f32x16*>(nb + kPolB3) + h);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    asm volatile("" ::: "memory");
    bf16x8 wfa[8], wfb[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      wfa[kk] = w2a[(t * 8 + kk) * 64];
      wfb[kk] = w2b[(t * 8 + kk) * 64];
    }
    f32x16 ca = b2a[2 * t], cb = b2b[2 * t];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      ca = mfma(wfa[kk], h1a[kk], ca);
      cb = mfma(wfb[kk], h1b[kk], cb);
    }
    head_a = mfma(w3a[(2 * t) * 64], act8<0>(ca), head_a);
    head_b = mfma(w3b[(2 * t) * 64], act8<0>(cb), head_b);
    head_a = mfma(w3a[(2 * t + 1) * 64], act8<1>(ca), head_a);
    head_b = mfma(w3b[(2 * t + 1) * 64], act8<1>(cb), head_b);
  }
}

// mlp_pair with the layer-2 weight fragments software-pipelined: tile t+1's 16
// fragments are issued before tile t's MFMAs (LDS returns in order, so tile t waits
// with 16 newer loads still in flight), and the head fragments up front.  Register
// hungry (two tiles of fragments for both nets): for the one-wave-per-SIMD shape.
__device__ __forceinline__ void mlp_pair_pipe(const uint8_t* na, const uint8_t* nb, bf16x8 x,
                                              int lane, f32x16& head_a, f32x16& head_b) {
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1a = reinterpret_cast<const bf16x8*>(na + kPolW1) + lane;
  const bf16x8* w1b = reinterpret_cast<const bf16x8*>(nb + kPolW1) + lane;
  const bf16x8* w2a = reinterpret_cast<const bf16x8*>(na + kPolW2) + lane;
  const bf16x8* w2b = reinterpret_cast<const bf16x8*>(nb + kPolW2) + lane;
  const bf16x8* w3a = reinterpret_cast<const bf16x8*>(na + kPolW3) + lane;
  const bf16x8* w3b = reinterpret_cast<const bf16x8*>(nb + kPolW3) + lane;
  const f32x16* b1a = reinterpret_cast<const f32x16*>(na + kPolB1) + h;
  const f32x16* b1b = reinterpret_cast<const f32x16*>(nb + kPolB1) + h;
  const f32x16* b2a = reinterpret_cast<const f32x16*>(na + kPolB2) + h;
  const f32x16* b2b = reinterpret_cast<const f32x16*>(nb + kPolB2) + h;
  bf16x8 l1a[4], l1b[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) { l1a[t] = w1a[t * 64]; l1b[t] = w1b[t * 64]; }
  bf16x8 cur_a[8], cur_b[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) { cur_a[kk] = w2a[kk * 64]; cur_b[kk] = w2b[kk * 64]; }
  asm volatile("" ::: "memory");
  bf16x8 h1a[8], h1b[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 ca = mfma(l1a[t], x, b1a[2 * t]);
    const f32x16 cb = mfma(l1b[t], x, b1b[2 * t]);
    h1a[2 * t] = act8<0>(ca);
    h1b[2 * t] = act8<0>(cb);
    h1a[2 * t + 1] = act8<1>(ca);
    h1b[2 * t + 1] = act8<1>(cb);
  }
  head_a = *(reinterpret_cast<const f32x16*>(na + kPolB3) + h);
  head_b = *(reinterpret_cast<const f32x16*>(nb + kPolB3) + h);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bf16x8 nxt_a[8], nxt_b[8], h3a[2], h3b[2];
    if (t < 3) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        nxt_a[kk] = w2a[((t + 1) * 8 + kk) * 64];
        nxt_b[kk] = w2b[((t + 1) * 8 + kk) * 64];
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) { h3a[q] = w3a[(2 * t + q) * 64]; h3b[q] = w3b[(2 * t + q) * 64]; }
    f32x16 ca = b2a[2 * t], cb = b2b[2 * t];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      ca = mfma(cur_a[kk], h1a[kk], ca);
      cb = mfma(cur_b[kk], h1b[kk], cb);
    }
    head_a = mfma(h3a[0], act8<0>(ca), head_a);
    head_b = mfma(h3b[0], act8<0>(cb), head_b);
    head_a = mfma(h3a[1], act8<1>(ca), head_a);
    head_b = mfma(h3b[1], act8<1>(cb), head_b);
    if (t < 3) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) { cur_a[kk] = nxt_a[kk]; cur_b[kk] = nxt_b[kk]; }
    }
  }
}

// ------------------------------------------------------------------ attention extractor
// code/train.py:52-95 AttentionFeaturesExtractor, shared by pi and vf (SB3
// share_features_extractor=True):
//   x = relu(fc1(obs))                      [128] = 8 tokens x 16
//   q, k, v = in_proj(token)                nn.MultiheadAttention(16, 4 heads of 4)
//   a_i = sum_j softmax_j(q_i . k_j / 2) v_j   per head
//   features = relu(post_fc(concat_i out_proj(a_i)))   [64]
// MI355X mapping (one wave = 32 envs, lanes l and l + 32 = the same env):
// - fc1 is one 32x32x16 MFMA per 32 units.  Its accumulator registers 0..7 / 8..15 of
//   lane half h hold units 32t + 16S + 8(j>>2) + 4h + (j&3): after ReLU and bf16
//   packing they ARE token 2t + S's B fragment (token dim (j&3) + 8(j>>2) + 4h at k =
//   8h + j), so the per-token projections need no data movement.
// - K|V: one MFMA per token with the rows permuted so that lane half h receives the
//   keys and values of heads 2h and 2h+1 (registers 0-3 k of head 2h, 4-7 k of 2h+1,
//   8-11 v of 2h, 12-15 v of 2h+1).  Q: one MFMA per token, rows 0-7 of each half the
//   queries of the same two heads, pre-scaled by log2(e) / sqrt(4) so the softmax is an
//   exp2.  Each lane then runs its two heads' attention in fp32 VALU for all 8 query
//   tokens (keys and values of the 8 tokens live in registers).
// - The head outputs of token i (half h: dims 8h..8h+7, heads 2h, 2h+1) are, packed to
//   bf16, the B fragment of a K=16 MFMA in natural order; out_proj is folded into
//   post_attention_fc on the host (W_post[:, 16i:16i+16] W_out per token, the biases
//   likewise), so post_fc is 2 tiles x 8 tokens of accumulation.
// - ReLU keeps NaN (torch.relu), as the env's own non-finite states reach the policy.
template <int S>
__device__ __forceinline__ bf16x8 relu8(const f32x16& c) {  // registers 8S..8S+7
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const float u = c[8 * S + j], w = c[8 * S + j + 1];
    const f32x2 t = {u < 0.0f ? 0.0f : u, w < 0.0f ? 0.0f : w};
    const bf16x2 b = __builtin_convertvector(t, bf16x2);
    r[j] = b[0];
    r[j + 1] = b[1];
  }
  return r;
}

__device__ __forceinline__ void attn_extract(const uint8_t* ext, bf16x8 x, int lane, bf16x8* feat) {
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1 = reinterpret_cast<const bf16x8*>(ext + kAttFc1W) + lane;
  const f32x16* b1 = reinterpret_cast<const f32x16*>(ext + kAttFc1B) + h;
  bf16x8 tok[kAttTokens];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 c = mfma(w1[t * 64], x, b1[2 * t]);
    tok[2 * t] = relu8<0>(c);
    tok[2 * t + 1] = relu8<1>(c);
  }
  const bf16x8 wkv = reinterpret_cast<const bf16x8*>(ext + kAttKvW)[lane];
  const f32x16 bkv = reinterpret_cast<const f32x16*>(ext + kAttKvB)[h];
  f32x16 kv[kAttTokens];
#pragma unroll
  for (int t = 0; t < kAttTokens; ++t) kv[t] = mfma(wkv, tok[t], bkv);
  const bf16x8 wq = reinterpret_cast<const bf16x8*>(ext + kAttQW)[lane];
  const f32x16 bq = reinterpret_cast<const f32x16*>(ext + kAttQB)[h];
  const bf16x8* wp = reinterpret_cast<const bf16x8*>(ext + kAttPostW) + lane;
  f32x16 f0 = reinterpret_cast<const f32x16*>(ext + kAttPostB)[h];
  f32x16 f1 = reinterpret_cast<const f32x16*>(ext + kAttPostB)[2 + h];
#pragma unroll
  for (int i = 0; i < kAttTokens; ++i) {
    // token i's two post_fc fragments, issued ahead of the attention math they wait on
    const bf16x8 wpa = wp[(2 * i) * 64], wpb = wp[(2 * i + 1) * 64];
    const f32x16 q = mfma(wq, tok[i], bq);
    float o[8];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      // scores q . k (log2 domain): the 4-term dots as two packed-f32 lanes
      // (v_pk_mul_f32 + v_pk_fma_f32) and one add
      const f32x2 q01 = {q[4 * hh], q[4 * hh + 1]}, q23 = {q[4 * hh + 2], q[4 * hh + 3]};
      float s[kAttTokens];
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < kAttTokens; ++j) {
        const f32x2 k01 = {kv[j][4 * hh], kv[j][4 * hh + 1]};
        const f32x2 k23 = {kv[j][4 * hh + 2], kv[j][4 * hh + 3]};
        const f32x2 t = __builtin_elementwise_fma(q23, k23, q01 * k01);
        s[j] = t[0] + t[1];
        m = fmaxf(m, s[j]);
      }
      // softmax numerators, their sum, then sum_j p_j v_j (packed FMAs over the 4 dims)
      // normalised once by 1 / sum
      float sum = 0.0f;
      f32x2 o01, o23;
#pragma unroll
      for (int j = 0; j < kAttTokens; ++j) {
        const float p = __builtin_amdgcn_exp2f(s[j] - m);
        sum = j == 0 ? p : sum + p;
        const f32x2 pp = {p, p};
        const f32x2 v01 = {kv[j][8 + 4 * hh], kv[j][9 + 4 * hh]};
        const f32x2 v23 = {kv[j][10 + 4 * hh], kv[j][11 + 4 * hh]};
        o01 = j == 0 ? pp * v01 : __builtin_elementwise_fma(pp, v01, o01);
        o23 = j == 0 ? pp * v23 : __builtin_elementwise_fma(pp, v23, o23);
      }
      const float rs = __builtin_amdgcn_rcpf(sum);
      const f32x2 rr = {rs, rs};
      o01 = o01 * rr;
      o23 = o23 * rr;
      o[4 * hh] = o01[0];
      o[4 * hh + 1] = o01[1];
      o[4 * hh + 2] = o23[0];
      o[4 * hh + 3] = o23[1];
    }
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x2 t = {o[j], o[j + 1]};
      const bf16x2 b = __builtin_convertvector(t, bf16x2);
      a[j] = b[0];
      a[j + 1] = b[1];
    }
    f0 = mfma(wpa, a, f0);
    f1 = mfma(wpb, a, f1);
  }
  feat[0] = relu8<0>(f0);
  feat[1] = relu8<1>(f0);
  feat[2] = relu8<0>(f1);
  feat[3] = relu8<1>(f1);
}

// One [128,128] Tanh net + head on the 64 features (layer 1: 4 k-steps of 16 features,
// columns in the relu8 order unit_of(s, h, j)).
__device__ __forceinline__ f32x16 attn_net(const uint8_t* net, const bf16x8* feat, int lane) {
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1 = reinterpret_cast<const bf16x8*>(net + kAttW1) + lane;
  const bf16x8* w2 = reinterpret_cast<const bf16x8*>(net + kAttW2) + lane;
  const bf16x8* w3 = reinterpret_cast<const bf16x8*>(net + kAttW3) + lane;
  const f32x16* b1 = reinterpret_cast<const f32x16*>(net + kAttB1) + h;
  const f32x16* b2 = reinterpret_cast<const f32x16*>(net + kAttB2) + h;
  bf16x8 h1[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 c = b1[2 * t];
#pragma unroll
    for (int s = 0; s < 4; ++s) c = mfma(w1[(t * 4 + s) * 64], feat[s], c);
    h1[2 * t] = act8<0>(c);
    h1[2 * t + 1] = act8<1>(c);
  }
  f32x16 head = reinterpret_cast<const f32x16*>(net + kAttB3)[h];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    asm volatile("" ::: "memory");
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = w2[(t * 8 + kk) * 64];
    f32x16 c = b2[2 * t];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) c = mfma(wf[kk], h1[kk], c);
    head = mfma(w3[(2 * t) * 64], act8<0>(c), head);
    head = mfma(w3[(2 * t + 1) * 64], act8<1>(c), head);
  }
  return head;
}

// code/lorenz_filter/train.py:54-103: the same extractor with out_proj, a residual
// connection and LayerNorm(16) per token before post_attention_fc, on up to 32 stacked
// input dims (VecFrameStack): fc1 is KS k-steps of 16.  Per query token i: attention
// as attn_extract, out_proj (one MFMA: rows 0-15 = W_out, so registers 0..7 of lane
// half h hold the token dims (g&3) + 8(g>>2) + 4h -- exactly the order of the token's
// own fragment, so the residual adds register to register), LayerNorm over the 16
// dims (8 per half, the two halves' partial sums exchanged with a lane-32 swap), the
// affine, bf16, and post_fc's two MFMAs.  The residual uses the bf16 token values the
// projections consumed (the torch restatement does the same).
template <int KS>
__device__ __forceinline__ void attn_ln_extract(const uint8_t* ext, const bf16x8* x, int lane,
                                                bf16x8* feat) {
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1 = reinterpret_cast<const bf16x8*>(ext + kLnFc1W) + lane;
  const f32x16* b1 = reinterpret_cast<const f32x16*>(ext + kLnFc1B) + h;
  bf16x8 tok[kAttTokens];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 c = b1[2 * t];
#pragma unroll
    for (int s = 0; s < KS; ++s) c = mfma(w1[(t * 2 + s) * 64], x[s], c);
    tok[2 * t] = relu8<0>(c);
    tok[2 * t + 1] = relu8<1>(c);
  }
  const bf16x8 wkv = reinterpret_cast<const bf16x8*>(ext + kLnKvW)[lane];
  const f32x16 bkv = reinterpret_cast<const f32x16*>(ext + kLnKvB)[h];
  f32x16 kv[kAttTokens];
#pragma unroll
  for (int t = 0; t < kAttTokens; ++t) kv[t] = mfma(wkv, tok[t], bkv);
  const bf16x8 wq = reinterpret_cast<const bf16x8*>(ext + kLnQW)[lane];
  const f32x16 bq = reinterpret_cast<const f32x16*>(ext + kLnQB)[h];
  const bf16x8 wo = reinterpret_cast<const bf16x8*>(ext + kLnOutW)[lane];
  const f32x16 bo = reinterpret_cast<const f32x16*>(ext + kLnOutB)[h];
  const float* gam = reinterpret_cast<const float*>(ext + kLnGamma) + 8 * h;
  const float* bet = reinterpret_cast<const float*>(ext + kLnBeta) + 8 * h;
  const bf16x8* wp = reinterpret_cast<const bf16x8*>(ext + kLnPostW) + lane;
  f32x16 f0 = reinterpret_cast<const f32x16*>(ext + kLnPostB)[h];
  f32x16 f1 = reinterpret_cast<const f32x16*>(ext + kLnPostB)[2 + h];
#pragma unroll
  for (int i = 0; i < kAttTokens; ++i) {
    const bf16x8 wpa = wp[(2 * i) * 64], wpb = wp[(2 * i + 1) * 64];
    const f32x16 q = mfma(wq, tok[i], bq);
    float o[8];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const f32x2 q01 = {q[4 * hh], q[4 * hh + 1]}, q23 = {q[4 * hh + 2], q[4 * hh + 3]};
      float sc[kAttTokens];
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < kAttTokens; ++j) {
        const f32x2 k01 = {kv[j][4 * hh], kv[j][4 * hh + 1]};
        const f32x2 k23 = {kv[j][4 * hh + 2], kv[j][4 * hh + 3]};
        const f32x2 t = __builtin_elementwise_fma(q23, k23, q01 * k01);
        sc[j] = t[0] + t[1];
        m = fmaxf(m, sc[j]);
      }
      float sum = 0.0f;
      f32x2 o01, o23;
#pragma unroll
      for (int j = 0; j < kAttTokens; ++j) {
        const float pj = __builtin_amdgcn_exp2f(sc[j] - m);
        sum = j == 0 ? pj : sum + pj;
        const f32x2 pp = {pj, pj};
        const f32x2 v01 = {kv[j][8 + 4 * hh], kv[j][9 + 4 * hh]};
        const f32x2 v23 = {kv[j][10 + 4 * hh], kv[j][11 + 4 * hh]};
        o01 = j == 0 ? pp * v01 : __builtin_elementwise_fma(pp, v01, o01);
        o23 = j == 0 ? pp * v23 : __builtin_elementwise_fma(pp, v23, o23);
      }
      const float rs = __builtin_amdgcn_rcpf(sum);
      const f32x2 rr = {rs, rs};
      o01 = o01 * rr;
      o23 = o23 * rr;
      o[4 * hh] = o01[0];
      o[4 * hh + 1] = o01[1];
      o[4 * hh + 2] = o23[0];
      o[4 * hh + 3] = o23[1];
    }
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x2 t = {o[j], o[j + 1]};
      const bf16x2 b = __builtin_convertvector(t, bf16x2);
      a[j] = b[0];
      a[j + 1] = b[1];
    }
    const f32x16 y = mfma(wo, a, bo);  // out_proj
    float z[8];
    float s1 = 0.0f;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      z[g] = y[g] + (float)tok[i][g];  // residual
      s1 = g == 0 ? z[g] : s1 + z[g];
    }
    s1 = s1 + __shfl_xor(s1, 32, 64);
    const float mean = s1 * 0.0625f;
    float s2 = 0.0f;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      z[g] = z[g] - mean;
      s2 = g == 0 ? z[g] * z[g] : s2 + z[g] * z[g];
    }
    s2 = s2 + __shfl_xor(s2, 32, 64);
    const float r = __builtin_amdgcn_rsqf(s2 * 0.0625f + 1e-5f);  // LayerNorm eps 1e-5
    bf16x8 u;
#pragma unroll
    for (int g = 0; g < 8; g += 2) {
      const f32x2 t = {(z[g] * r) * gam[g] + bet[g], (z[g + 1] * r) * gam[g + 1] + bet[g + 1]};
      const bf16x2 b = __builtin_convertvector(t, bf16x2);
      u[g] = b[0];
      u[g + 1] = b[1];
    }
    f0 = mfma(wpa, u, f0);
    f1 = mfma(wpb, u, f1);
  }
  feat[0] = relu8<0>(f0);
  feat[1] = relu8<1>(f0);
  feat[2] = relu8<0>(f1);
  feat[3] = relu8<1>(f1);
}

// the KS fc1 B fragments of a VecFrameStack obs of SO dims held by both lane halves:
// k-step s, half h, element j = stacked dim 16s + 8h + j (zero past SO or if !use)
template <int SO, int KS>
__device__ __forceinline__ void stack_frags(const float* st, int h, bool use, bf16x8* xs) {
#pragma unroll
  for (int s = 0; s < KS; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d0 = 16 * s + j, d1 = 16 * s + 8 + j;
      const float v0 = d0 < SO ? st[d0 < SO ? d0 : 0] : 0.0f;
      const float v1 = d1 < SO ? st[d1 < SO ? d1 : 0] : 0.0f;
      xs[s][j] = (__bf16)(use ? (h ? v1 : v0) : 0.0f);
    }
  }
}

// pi and vf nets on the same features, interleaved layer by layer (two independent
// MFMA / tanh chains for the one-wave-per-SIMD shape)
__device__ __forceinline__ void attn_nets_pair(const uint8_t* na, const uint8_t* nb,
                                               const bf16x8* feat, int lane, f32x16& head_a,
                                               f32x16& head_b) {
  // weight fragments software-pipelined one tile ahead (as mlp_pair_pipe): with one
  // wave per SIMD nothing else hides the LDS latency of a tile's loads
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const bf16x8* w1a = reinterpret_cast<const bf16x8*>(na + kAttW1) + lane;
  const bf16x8* w1b = reinterpret_cast<const bf16x8*>(nb + kAttW1) + lane;
  const bf16x8* w2a = reinterpret_cast<const bf16x8*>(na + kAttW2) + lane;
  const bf16x8* w2b = reinterpret_cast<const bf16x8*>(nb + kAttW2) + lane;
  const bf16x8* w3a = reinterpret_cast<const bf16x8*>(na + kAttW3) + lane;
  const bf16x8* w3b = reinterpret_cast<const bf16x8*>(nb + kAttW3) + lane;
  const f32x16* b1a = reinterpret_cast<const f32x16*>(na + kAttB1) + h;
  const f32x16* b1b = reinterpret_cast<const f32x16*>(nb + kAttB1) + h;
  const f32x16* b2a = reinterpret_cast<const f32x16*>(na + kAttB2) + h;
  const f32x16* b2b = reinterpret_cast<const f32x16*>(nb + kAttB2) + h;
  bf16x8 c1a[4], c1b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) { c1a[s] = w1a[s * 64]; c1b[s] = w1b[s * 64]; }
  asm volatile("" ::: "memory");
  bf16x8 h1a[8], h1b[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bf16x8 n1a[4], n1b[4];
    if (t < 3) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        n1a[s] = w1a[((t + 1) * 4 + s) * 64];
        n1b[s] = w1b[((t + 1) * 4 + s) * 64];
      }
    }
    f32x16 ca = b1a[2 * t], cb = b1b[2 * t];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ca = mfma(c1a[s], feat[s], ca);
      cb = mfma(c1b[s], feat[s], cb);
    }
    h1a[2 * t] = act8<0>(ca);
    h1b[2 * t] = act8<0>(cb);
    h1a[2 * t + 1] = act8<1>(ca);
    h1b[2 * t + 1] = act8<1>(cb);
    if (t < 3) {
#pragma unroll
      for (int s = 0; s < 4; ++s) { c1a[s] = n1a[s]; c1b[s] = n1b[s]; }
    }
  }
  bf16x8 cur_a[8], cur_b[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) { cur_a[kk] = w2a[kk * 64]; cur_b[kk] = w2b[kk * 64]; }
  asm volatile("" ::: "memory");
  head_a = reinterpret_cast<const f32x16*>(na + kAttB3)[h];
  head_b = reinterpret_cast<const f32x16*>(nb + kAttB3)[h];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bf16x8 nxt_a[8], nxt_b[8], h3a[2], h3b[2];
    if (t < 3) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        nxt_a[kk] = w2a[((t + 1) * 8 + kk) * 64];
        nxt_b[kk] = w2b[((t + 1) * 8 + kk) * 64];
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) { h3a[q] = w3a[(2 * t + q) * 64]; h3b[q] = w3b[(2 * t + q) * 64]; }
    f32x16 ca = b2a[2 * t], cb = b2b[2 * t];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      ca = mfma(cur_a[kk], h1a[kk], ca);
      cb = mfma(cur_b[kk], h1b[kk], cb);
    }
    head_a = mfma(h3a[0], act8<0>(ca), head_a);
    head_b = mfma(h3b[0], act8<0>(cb), head_b);
    head_a = mfma(h3a[1], act8<1>(ca), head_a);
    head_b = mfma(h3b[1], act8<1>(cb), head_b);
    if (t < 3) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) { cur_a[kk] = nxt_a[kk]; cur_b[kk] = nxt_b[kk]; }
    }
  }
}

// VecNormalize.normalize_obs (float64, then float32 for the policy: obs_as_tensor)
template <int O>
__device__ __forceinline__ void normalize(const float* o, float* x, bool on, const double* mu,
                                          const double* sd, double clip) {  // mu, sd: LDS
#pragma unroll
  for (int j = 0; j < O; ++j) {
    if (!on) {
      x[j] = o[j];
      continue;
    }
    double v = ((double)o[j] - mu[j]) / sd[j];
    v = v < -clip ? -clip : (v > clip ? clip : v);  // np.clip (NaN-propagating)
    x[j] = (float)v;
  }
}

template <int O>
__device__ __forceinline__ bf16x8 obs_frag(const float* x, bool use) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (__bf16)((use && j < O) ? x[j < O ? j : 0] : 0.0f);
  return b;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// One net's forward for the wave's E envs (E = 32: lane r and r + 32 both stand for env
// r; E = 64: lane l owns env l and the wave runs two 32-env MFMA column tiles, the
// upper half's observations moved to the lower lanes for tile B and its results moved
// back).  Each lane gets its own env's head rows 0..N-1 in out[] (E = 32: h = 0 lanes).
template <int E, int O, int N>
__device__ __forceinline__ void net_fwd(const uint8_t* net, const float* x, bool use, int lane,
                                        float* out) {
  const int h = lane >> 5;
  const bf16x8 own = obs_frag<O>(x, use);
  const bf16x8 zero = obs_frag<O>(x, false);
  if constexpr (E == 32) {
    const f32x16 c = mlp_tile(net, h == 0 ? own : zero, lane);
#pragma unroll
    for (int j = 0; j < N; ++j) out[j] = c[j];
  } else {
    const u32x4 ou = __builtin_bit_cast(u32x4, own);
    u32x4 sw;
#pragma unroll
    for (int q = 0; q < 4; ++q) sw[q] = (uint32_t)__shfl_xor((int)ou[q], 32, 64);
    const f32x16 ca = mlp_tile(net, h == 0 ? own : zero, lane);
    const f32x16 cb = mlp_tile(net, h == 0 ? __builtin_bit_cast(bf16x8, sw) : zero, lane);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float b = __shfl_xor(cb[j], 32, 64);
      out[j] = h == 0 ? ca[j] : b;
    }
  }
}

// ---------------------------------------------------------------------------------------
// The MlpPolicy at SB3's precision (kMlpF32, kF32* blob).  Float32 operands end to end;
// every output is a fixed sequence of correctly rounded IEEE operations, so the C
// oracle (oracle/lz_oracle.c orc_mlp_f32) reproduces it bit for bit:
//   * hidden layers on v_mfma_f32_32x32x2_f32 (gfx950: bit-for-bit the k-ordered fmaf
//     chain D = fma(a_k1, b_k1, fma(a_k0, b_k0, C)), k0 = lane half 0's operand).  Same
//     dataflow as the bf16 kernel: weights = A (32 units x 2 inputs), activations = B
//     (2 inputs x 32 envs); layer 1's accumulator register g of lane half h (unit
//     row(g, h) of its tile, env on the lane) is exactly layer 2's B operand for
//     k-step 16 ti + g, so layer 2 sums its 128 inputs in the order
//     ti = 0..3, g = 0..15, h = 0, 1 -- the packer permutes W2's columns to match;
//   * the heads (2-4 rows: a 32-row MFMA tile would waste 90% of it) as one fmaf chain
//     per lane half over that half's 64 units (t, g ascending), the halves' partial
//     sums added once (__shfl_xor 32), then the bias;
//   * tanh as a piecewise polynomial (tanh_tab: 72 segments of width 1/8, degree 5,
//     Horner in fmaf; coefficients from tools/tanh_table.py in the blob) -- no
//     v_exp_f32 / v_rcp_f32, whose bits no CPU reproduces, and no division.  Max error
//     vs tanh in float64: 1.01 ulp (tests/test_policy_f32_host.py).
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// tanh(x) = sign(x) p_k(|x| - k/8), k = floor(8|x|) < 72, p_k a degree-5 polynomial
// (tools/tanh_table.py; segment 0 is t q(t): full relative accuracy near 0); 1 for
// |x| >= 9 (1 - tanh(9) < 2^-25).  The blob holds c_j 8^-j (exact scaling) so Horner
// runs in u = fract(8|x|) = 8 t: every Horner step is the oracle's (t-form) value times
// 8^-j exactly -- scaling by a power of two commutes with rounding -- so the result has
// the oracle's bits with v_fract replacing a convert + fma.  11 VALU instructions and two
// LDS reads of the segment's coefficients (the table sits in the blob, tab = LDS).
__device__ __forceinline__ float tanh_tab(float x, const float* tab) {
  const float ax = fabsf(x);
  // 8|x| exactly, clamped to 72 with NaN kept: |x| >= 9 (inf too) lands on segment 72,
  // the constant 1 -- the oracle's "1 for |x| >= 9" without a compare and select
  const float m = __builtin_elementwise_minimum(ax * 8.0f, 72.0f);
  const int k = (int)m;                     // NaN -> 0
  const f32x4 lo = reinterpret_cast<const f32x4*>(tab)[2 * k];
  const f32x4 hi = reinterpret_cast<const f32x4*>(tab)[2 * k + 1];
  const float u = __builtin_amdgcn_fractf(m);  // m - floor(m), exact
  float y = fmaf(hi[1], u, hi[0]);
  y = fmaf(y, u, lo[3]);
  y = fmaf(y, u, lo[2]);
  y = fmaf(y, u, lo[1]);
  y = fmaf(y, u, lo[0]);      // NaN: u (so y) is NaN
  return __builtin_copysignf(y, x);
}

// tanh_tab of four values with all eight coefficient reads issued before the first
// Horner step (one LDS round trip for the four instead of four in a row); the same bits
template <class V4>
__device__ __forceinline__ V4 tanh_tab4(V4 x, const float* tab) {
  f32x4 lo[4], hi[4];
  float u[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float m = __builtin_elementwise_minimum(fabsf(x[r]) * 8.0f, 72.0f);
    const int k = (int)m;
    lo[r] = reinterpret_cast<const f32x4*>(tab)[2 * k];
    hi[r] = reinterpret_cast<const f32x4*>(tab)[2 * k + 1];
    u[r] = __builtin_amdgcn_fractf(m);
  }
  V4 out;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float y = fmaf(hi[r][1], u[r], hi[r][0]);
    y = fmaf(y, u[r], lo[r][3]);
    y = fmaf(y, u[r], lo[r][2]);
    y = fmaf(y, u[r], lo[r][1]);
    y = fmaf(y, u[r], lo[r][0]);
    out[r] = __builtin_copysignf(y, x[r]);
  }
  return out;
}

// Layer 2 (128 -> 128, tanh_tab) and the NH head rows of a float32 net, from layer 1's
// activations a1[4] (accumulator layout: tile t register g of half h = unit 32t +
// row(g, h)).  w2 [4 out tiles][16 quads][64 lanes][4] (k-step q: input unit 32 (q >> 4)
// + row(q & 15, h)), b2 [4][2][16], head rows [NH][2 halves][64], head bias [NH].
// Returns the head rows in head[] on every lane (both halves hold the same values).
template <int NH>
__device__ __forceinline__ void mlp_f32_tail(const uint8_t* w2p, const uint8_t* b2p, const uint8_t* whp,
                                             const uint8_t* bhp, const f32x16* a1, int lane,
                                             float* head, const float* ttab) {
  const int h = lane >> 5;
  const f32x4* w2 = reinterpret_cast<const f32x4*>(w2p) + lane;
  const f32x16* b2 = reinterpret_cast<const f32x16*>(b2p) + h;
  const float* wh = reinterpret_cast<const float*>(whp) + h * 64;
  const float* bh = reinterpret_cast<const float*>(bhp);
  float acc[NH];
#pragma unroll
  for (int j = 0; j < NH; ++j) acc[j] = 0.0f;  // first step fmaf(w, v, +0)
  // one output tile at a time (not unrolled: four tiles' tanh chains in flight at once
  // would spill)
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    f32x16 c = b2[2 * t];
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
      // the tile's 16 k-steps of weights in four 16-B loads, issued together
      asm volatile("" ::: "memory");
      f32x4 wq[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) wq[e] = w2[((t * 16) + ti * 4 + e) * 64];
#pragma unroll
      for (int g = 0; g < 16; ++g) c = mfma_f32(wq[g >> 2][g & 3], a1[ti][g], c);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float v = tanh_tab(c[g], ttab);
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const float w = wh[j * 128 + t * 16 + g];
        acc[j] = fmaf(w, v, acc[j]);
      }
      if ((g & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int j = 0; j < NH; ++j) {
    const float o = __shfl_xor(acc[j], 32, 64);
    head[j] = (acc[j] + o) + bh[j];  // IEEE add commutes: both halves get the same bits
  }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// the digits of the 4 values of v at scale 2^q: d[i] byte r = digit i of v[r] (the i8x4
// fixed point of lz_attn_policy_pack_i8x4: V = rint(v 2^q), U = V + 0x808080, digits
// 0-2 = bytes 0-2 of U minus 128, digit 3 = U >> 24), four bytes per v_perm
__device__ __forceinline__ void i8x_digits4(const f32x4& v, int q, uint32_t* d) {
  uint32_t U[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    U[r] = (uint32_t)(int32_t)__builtin_rintf(__builtin_ldexpf(v[r], q)) + 0x808080u;
  const uint32_t t0 = __builtin_amdgcn_perm(U[1], U[0], 0x05010400u);  // U0.b0 U1.b0 U0.b1 U1.b1
  const uint32_t t1 = __builtin_amdgcn_perm(U[1], U[0], 0x07030602u);  // U0.b2 U1.b2 U0.b3 U1.b3
  const uint32_t t2 = __builtin_amdgcn_perm(U[3], U[2], 0x05010400u);
  const uint32_t t3 = __builtin_amdgcn_perm(U[3], U[2], 0x07030602u);
  d[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u) ^ 0x80808080u;
  d[1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u) ^ 0x80808080u;
  d[2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u) ^ 0x80808080u;
  d[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
}

__device__ __forceinline__ float i8x_recombine(int l6, int l5, int l4, int l3, int sh) {
  const int hi = l6 * 256 + l5, lo = l4 * 256 + l3;
  return __builtin_ldexpf(fmaf((float)hi, 65536.0f, (float)lo), sh);
}

__device__ __forceinline__ i32x16 mfma_i8_32(i32x4 a, i32x4 b, i32x16 c) {
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}

// mlp_f32_tail with layer 2 as exact i8x4 fixed-point products (LZ_POLICY_I8X4,
// lz_policy_pack_i8x4; oracle orc_mlp_i8x4).  Layer 1's tanh outputs at scale 2^28 are
// the B operand of v_mfma_i32_32x32x32_i8 as they sit: k-block kb = layer-1 tile kb, byte
// j of lane (env, h) = its register j (unit 32 kb + row(j, h)); the packer lays W2 out to
// match ([T][kb][digit][64 lanes][16 B]).  xd[kb][i] = digit i of tile kb (made by
// mlp_f32 right after each tile's tanh, so the float activations never all live at once).
// The 10 digit products of levels 6..3 accumulate in int32 (exact, order-free) in two
// passes per output tile -- levels 6 + 5 (-> hi = L6 256 + L5), then 4 + 3 (-> lo) -- so
// two 16-register accumulators are live instead of four (the 512-lane kernels' 256-VGPR
// budget; the weight digits of w3 / w2 are read twice);
// y = ldexp(fma(float(hi), 2^16, float(lo)), 24 - q_row - 28) + b2, then tanh_tab and the
// heads exactly as the float32 tail.  The int8 MFMA issues beside the VALU (the float32
// one shares it).  An env with a NaN among its layer-1 outputs (bad) gets NaN heads.
template <int NH>
__device__ __forceinline__ void mlp_i8_tail(const uint8_t* net, const i32x4 (*xd)[4], bool bad, int lane,
                                            float* head, const float* ttab) {
  const int h = lane >> 5;
  const i32x4* w2 = reinterpret_cast<const i32x4*>(net + kF32W2) + lane;
  const f32x16* b2 = reinterpret_cast<const f32x16*>(net + kF32B2) + h;
  const int16_t* sh2 = reinterpret_cast<const int16_t*>(net + kF32Sh2) + h * 16;
  const float* wh = reinterpret_cast<const float*>(net + kF32H) + h * 64;
  const float* bh = reinterpret_cast<const float*>(net + kF32HB);
  float acc[NH];
#pragma unroll
  for (int j = 0; j < NH; ++j) acc[j] = 0.0f;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    __builtin_amdgcn_sched_barrier(0);
    // (software-pipelining tile t + 1's passes around tile t's VALU work measured 3-10 %
    // slower, profiles/r05/mlp_i8/pipe_rejected/)
    const i32x16 z = {};
    const i32x4* wt = w2 + t * 4 * 4 * 64;
    // hi = L6 256 + L5 and lo = L4 256 + L3 accumulated directly: the first pass sums the
    // levels 6 and 4 over the k-blocks, both accumulators are shifted left 8 bits, the
    // second adds levels 5 and 3 (exact: |hi| < 2^24, |lo| < 2^31)
    i32x16 Hi = z, Lo = z;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      asm volatile("" ::: "memory");
      const i32x4* wp = wt + kb * 4 * 64;
      const i32x4 w1 = wp[64], w2d = wp[128], w3 = wp[192];
      Hi = mfma_i8_32(w3, xd[kb][3], Hi);
      Lo = mfma_i8_32(w3, xd[kb][1], Lo);
      Lo = mfma_i8_32(w2d, xd[kb][2], Lo);
      Lo = mfma_i8_32(w1, xd[kb][3], Lo);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      Hi[g] <<= 8;
      Lo[g] <<= 8;
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      asm volatile("" ::: "memory");
      const i32x4* wp = wt + kb * 4 * 64;
      const i32x4 w0 = wp[0], w1 = wp[64], w2d = wp[128], w3 = wp[192];
      Hi = mfma_i8_32(w3, xd[kb][2], Hi);
      Hi = mfma_i8_32(w2d, xd[kb][3], Hi);
      Lo = mfma_i8_32(w3, xd[kb][0], Lo);
      Lo = mfma_i8_32(w2d, xd[kb][1], Lo);
      Lo = mfma_i8_32(w1, xd[kb][2], Lo);
      Lo = mfma_i8_32(w0, xd[kb][3], Lo);
    }
    const float* bias = reinterpret_cast<const float*>(b2 + 2 * t);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float y = __builtin_ldexpf(fmaf((float)Hi[g], 65536.0f, (float)Lo[g]), sh2[t * 32 + g]) + bias[g];
      const float v = tanh_tab(y, ttab);
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const float w = wh[j * 128 + t * 16 + g];
        acc[j] = fmaf(w, v, acc[j]);
      }
      if ((g & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int j = 0; j < NH; ++j) {
    const float o = __shfl_xor(acc[j], 32, 64);
    const float r = (acc[j] + o) + bh[j];
    head[j] = bad ? __builtin_nanf("") : r;
  }
}

// One net on the wave's 32-env tile.  xs[s] = this lane's layer-1 input for k-step s
// (obs[2s + h] of env lane & 31).  Returns the NH head rows in head[] on every lane
// (both halves hold the same values).  kI8: layer 2 as mlp_i8_tail, layer 1's outputs
// turned into digits tile by tile.
template <int KS1, int NH, bool kI8 = false>
__device__ __forceinline__ void mlp_f32(const uint8_t* net, const float* xs, int lane, float* head,
                                        const float* ttab) {
  asm volatile("" ::: "memory");
  const int h = lane >> 5;
  const f32x4* w1 = reinterpret_cast<const f32x4*>(net + kF32W1) + lane;
  const f32x16* b1 = reinterpret_cast<const f32x16*>(net + kF32B1) + h;
  f32x16 a1[kI8 ? 1 : 4];
  i32x4 xd[kI8 ? 4 : 1][4];
  float chk = 0.0f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x4 w = w1[t * 64];
    f32x16 c = b1[2 * t];
#pragma unroll
    for (int s = 0; s < KS1; ++s) c = mfma_f32(w[s], xs[s], c);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      c[g] = tanh_tab(c[g], ttab);
    }
    if constexpr (kI8) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x4 v = {c[4 * e], c[4 * e + 1], c[4 * e + 2], c[4 * e + 3]};
        chk += (v[0] + v[1]) + (v[2] + v[3]);  // |v| <= 1: NaN iff a NaN among them
        uint32_t d[4];
        i8x_digits4(v, 28, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) xd[t][i][e] = (int)d[i];
      }
    } else {
      a1[t] = c;
    }
  }
  if constexpr (kI8) {
    const bool bad = __builtin_isnan(chk + __shfl_xor(chk, 32, 64));
    mlp_i8_tail<NH>(net, xd, bad, lane, head, ttab);
  } else {
    mlp_f32_tail<NH>(net + kF32W2, net + kF32B2, net + kF32H, net + kF32HB, a1, lane, head, ttab);
  }
}

// this lane's layer-1 inputs from the env-owning lane (half 0) of its env
template <int O, int KS1>
__device__ __forceinline__ void f32_inputs(const float* x, int lane, float* xs) {
  const int src = lane & 31;
#pragma unroll
  for (int s = 0; s < KS1; ++s) {
    const float lo = __shfl(x[2 * s], src, 64);
    const float hi = __shfl(2 * s + 1 < O ? x[2 * s + 1 < O ? 2 * s + 1 : 0] : 0.0f, src, 64);
    xs[s] = lane < 32 ? lo : hi;
  }
}

// The kernel variants (template parameter kPair of k_rollout_policy): the MlpPolicy
// nets one after the other / interleaved / interleaved with pipelined weight loads,
// code/train.py's attention actor-critic, code/lorenz_filter/train.py's residual +
// LayerNorm attention actor-critic on VecFrameStack observations.
constexpr int kMlpSerial = 0, kMlpPair = 1, kMlpPairPipe = 2, kAttn = 3, kAttnLn = 4,
              kMlpF32 = 5, kMlpI8 = 6;  // kMlpI8: kMlpF32 with layer 2 as mlp_i8_tail
constexpr bool mlp_f32_kind(int k) { return k == kMlpF32 || k == kMlpI8; }

// The blob's format tag (lz_internal.h kBlobMagic) against the format this launch expects.
__device__ inline bool blob_is(const uint8_t* blob, int off, uint32_t fmt) {
  const uint32_t* t = reinterpret_cast<const uint32_t*>(blob + off);
  const uint32_t w[4] = {t[0], t[1], t[2], t[3]};
  return blob_tag_ok(w, fmt);
}

// Copy n16 16-B pieces of the blob into LDS -- or, when its tag does not match the
// launch (`bad`, workgroup-uniform), fill them with NaN: every weight, Normal constant
// and tanh-table entry is NaN, so every output of the launch is NaN.
__device__ inline void blob_to_lds(f4v* dst, const f4v* src, int n16, int tid, int stride, bool bad) {
  if (bad) {
    const float q = __builtin_nanf("");
    const f4v nan4 = {q, q, q, q};
    for (int v = tid; v < n16; v += stride) dst[v] = nan4;
  } else {
    for (int v = tid; v < n16; v += stride) dst[v] = src[v];
  }
}

// V(x) alone (truncation bootstrap, last values): the value net, after the shared
// attention extractor for kPair == kAttn
template <int E, int O, int kPair>
__device__ __forceinline__ void value_fwd(const uint8_t* blob, const uint8_t* vf_net, const float* x,
                                          bool use, int lane, float* out) {
  if constexpr (kPair == kAttn) {
    bf16x8 f[4];
    attn_extract(blob, obs_frag<O>(x, use), lane, f);
    out[0] = attn_net(blob + kAttVf, f, lane)[0];
  } else if constexpr (mlp_f32_kind(kPair)) {
    float xs[(O + 1) / 2];
    f32_inputs<O, (O + 1) / 2>(x, lane, xs);
    mlp_f32<(O + 1) / 2, 1, kPair == kMlpI8>(vf_net, xs, lane, out,
                            reinterpret_cast<const float*>(blob + kF32Tanh));
  } else {
    net_fwd<E, O, 1>(vf_net, x, use, lane, out);
  }
}

// kPair (see kMlpSerial ...): kMlpPair = mlp_pair, kMlpPairPipe = mlp_pair_pipe,
// kAttn = attn_extract + attn_nets_pair (kAtt* blob), kAttnLn = attn_ln_extract +
// attn_nets_pair (kLn* blob) with the S-frame stack in the registers of both lane
// halves of the env, kMlpF32 = mlp_f32 twice (kF32* blob; the obs moments accumulate
// in registers: the blob leaves too little LDS for them)
template <class Sys, int W, int E, int kPair, int S = 1>
__global__ __launch_bounds__(W * 64) void k_rollout_policy(KArgs a, PArgs p) {
  static_assert(kPair == kMlpSerial || E == 32, "the paired / attention kernels run 32-env tiles");
  constexpr int kBlob = kPair == kAttnLn ? kLnBlobBytes
                        : kPair == kAttn ? kAttBlobBytes
                        : mlp_f32_kind(kPair) ? kF32BlobBytes : kPolBlobBytes;
  constexpr bool kRegMom = mlp_f32_kind(kPair);  // obs moments in registers, not LDS
  constexpr int O = Sys::O, A = Sys::A;
  constexpr int SO = S * O, KS = (SO + 15) / 16;  // kAttnLn: stacked dims, fc1 k-steps
  static_assert(kPair == kAttnLn || S == 1, "frame stacking is the kAttnLn path");
  static_assert(SO <= kLnMaxIn, "stacked obs dims");
  static_assert(O <= kPolMaxObs && A <= kPolMaxAct, "policy tile shape");
  static_assert(E == 32 || E == 64, "envs per wave");
  __shared__ __attribute__((aligned(64))) uint8_t s_blob[kBlob];
  __shared__ double s_norm[2 * kPolMaxObs];
  __shared__ double s_mom[(kPair == kAttnLn || kRegMom) ? 1 : W * E * 2 * O];  // kAttnLn: none
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int slot = E == 64 ? lane : (lane & 31);  // this lane's env within the tile
  const bool owner = E == 64 || h == 0;           // lanes that step an env
  {
    bool bad = false;
    if constexpr (mlp_f32_kind(kPair))
      bad = !blob_is(p.blob, kF32Tag, kPair == kMlpI8 ? LZ_BLOB_MLP_I8X4 : LZ_BLOB_MLP_F32);
    blob_to_lds(reinterpret_cast<f4v*>(s_blob), reinterpret_cast<const f4v*>(p.blob), kBlob / 16,
                tid, W * 64, bad);
  }
  if (tid < O) {  // VecNormalize: mean and sqrt(var + eps) per obs dim
    s_norm[tid] = p.norm ? p.norm[tid] : 0.0;
    s_norm[kPolMaxObs + tid] = p.norm ? sqrt(p.norm[O + tid] + p.eps) : 1.0;
  }
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  __syncthreads();
  const uint8_t* pi_net = s_blob + (kPair == kAttnLn ? kLnPi : kPair == kAttn ? kAttPi : 0);
  const uint8_t* vf_net =
      s_blob + (kPair == kAttnLn ? kLnVf : kPair == kAttn ? kAttVf : mlp_f32_kind(kPair) ? kF32Net : kPolNet);
  // torch.distributions.Normal constants, computed by the packer: scale = exp(log_std),
  // 2 * scale**2, log(scale) (LDS, wave-uniform broadcast reads)
  const float* g_scale =
      reinterpret_cast<const float*>(
          s_blob + (kPair == kAttnLn   ? kLnLogStd
                    : kPair == kAttn   ? kAttLogStd
                    : mlp_f32_kind(kPair) ? kF32LogStd : kPolLogStd)) + 4;
  const float* g_var2 = g_scale + 4;
  const float* g_lscale = g_scale + 8;
  const bool norm = p.norm != nullptr;
  const double* mu = s_norm;
  const double* sd = s_norm + kPolMaxObs;
  const bool det = (p.pflags & LZ_POLICY_DETERMINISTIC) != 0;
  const bool boot = (p.pflags & LZ_POLICY_BOOTSTRAP) != 0;
  const float gamma = p.gamma;
  // per-lane float64 obs-moment accumulators of the env-owning lanes, in LDS; kRegMom:
  // in registers, split over the env's two lanes (half 0 the sums, half 1 the squares)
  double mom_r[kRegMom ? O : 1];
  double* mom = kRegMom ? mom_r : s_mom + (kPair == kAttnLn ? 0 : (wave * E + slot) * (2 * O));
  if constexpr (kRegMom) {
#pragma unroll
    for (int j = 0; j < O; ++j) mom_r[j] = 0.0;
  } else if constexpr (kPair != kAttnLn) {
    if (owner) {
#pragma unroll
      for (int j = 0; j < 2 * O; ++j) mom[j] = 0.0;
    }
  }

  Sys sys;
  sys.setup(a);
  float* obs_buf = static_cast<float*>(a.obs);
  float* rew_buf = static_cast<float*>(a.rew);
  const int64_t ntiles = (a.n + E - 1) / E;
  for (int64_t tile = (int64_t)blockIdx.x * W + wave; tile < ntiles; tile += (int64_t)gridDim.x * W) {
    const int64_t i = tile * E + slot;
    const bool live = owner && i < a.n;
    int32_t steps = 0;
    bool any_reset = false;
    float o[O];
#pragma unroll
    for (int j = 0; j < O; ++j) o[j] = 0.0f;
    if (live) {
      sys.load(a, i);
      if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
#pragma unroll
      for (int j = 0; j < O; ++j) o[j] = p.obs_in[i * O + j];
    }
    const bool valid = i < a.n;  // kAttnLn: both halves of the env's lanes
    float st[kPair == kAttnLn ? SO : 1];
    if constexpr (kPair == kAttnLn) {
#pragma unroll
      for (int j = 0; j < SO; ++j) st[j] = valid ? p.stack_in[i * SO + j] : 0.0f;
    }
    // settle the tile's loads (state planes, obs_in) here: otherwise
    // hipcc places their first-use waits inside the step loop, where a vmcnt(0) also
    // drains every store of the previous step -- a store round trip per step
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched
    for (int k = 0; k < a.K; ++k) {
      const int64_t off = (int64_t)k * a.n + i;
      float x[O];
      if constexpr (kPair == kAttnLn) {
        if (live) {  // the stacked observation the policy sees
#pragma unroll
          for (int j = 0; j < SO; ++j) obs_buf[off * SO + j] = st[j];
        }
      } else {
        normalize<O>(o, x, norm, mu, sd, p.clip);
        if (live) {  // the observation the policy sees (SB3 rollout_buffer.add(_last_obs))
#pragma unroll
          for (int j = 0; j < O; ++j) obs_buf[off * O + j] = x[j];
        }
      }
      float mean[A], val[1];
      if constexpr (kPair == kAttnLn) {
        f32x16 hp, hv;
        bf16x8 xs[KS], f[4];
        stack_frags<SO, KS>(st, h, valid, xs);
        attn_ln_extract<KS>(s_blob, xs, lane, f);
        attn_nets_pair(pi_net, vf_net, f, lane, hp, hv);
#pragma unroll
        for (int j = 0; j < A; ++j) mean[j] = hp[j];
        val[0] = hv[0];
      } else if constexpr (kPair == kAttn) {
        f32x16 hp, hv;
        bf16x8 f[4];
        attn_extract(s_blob, obs_frag<O>(x, live), lane, f);
        attn_nets_pair(pi_net, vf_net, f, lane, hp, hv);
#pragma unroll
        for (int j = 0; j < A; ++j) mean[j] = hp[j];
        val[0] = hv[0];
      } else if constexpr (mlp_f32_kind(kPair)) {
        constexpr bool kI8 = kPair == kMlpI8;
        float xs[(O + 1) / 2];
        f32_inputs<O, (O + 1) / 2>(x, lane, xs);
        const float* ttab = reinterpret_cast<const float*>(s_blob + kF32Tanh);
        mlp_f32<(O + 1) / 2, A, kI8>(pi_net, xs, lane, mean, ttab);
        __builtin_amdgcn_sched_barrier(0);  // the two nets one after the other
        mlp_f32<(O + 1) / 2, 1, kI8>(vf_net, xs, lane, val, ttab);
      } else if constexpr (kPair == kMlpPair || kPair == kMlpPairPipe) {
        f32x16 hp, hv;
        if constexpr (kPair == kMlpPairPipe)
          mlp_pair_pipe(pi_net, vf_net, obs_frag<O>(x, live), lane, hp, hv);
        else mlp_pair(pi_net, vf_net, obs_frag<O>(x, live), lane, hp, hv);
#pragma unroll
        for (int j = 0; j < A; ++j) mean[j] = hp[j];
        val[0] = hv[0];
      } else {
        net_fwd<E, O, A>(pi_net, x, live, lane, mean);
        net_fwd<E, O, 1>(vf_net, x, live, lane, val);
      }
      float act_c[A];
      if (live) {
        float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (!det) {
          if constexpr (A <= 2) normal2(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k, z);
          else normal4(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k, z);
        }
        float lp = 0.0f;
#pragma unroll
        for (int j = 0; j < A; ++j) {
          const float aj = det ? mean[j] : mean[j] + z[j] * g_scale[j];  // Normal.rsample
          const float d = aj - mean[j];
          const float lpj = (-(d * d)) / g_var2[j] - g_lscale[j] - 0.91893853320467274f;
          lp = j == 0 ? lpj : lp + lpj;
          act_c[j] = clip(aj, p.act_lo, p.act_hi);
          p.act[off * A + j] = aj;
        }
        p.logp[off] = lp;
        p.val[off] = val[0];
      }
      float on[O], ot[O];
      float rew = 0.0f;
      bool did_reset;
      const uint8_t df = step_body<Sys, float, true, true>(sys, steps, a, i, live, act_c,
                                                           tick + (uint64_t)k, k, on, rew,
                                                           did_reset, ot);
      any_reset = any_reset || did_reset;
      if constexpr (kPair == kAttnLn) {
        // VecFrameStack (SB3 StackedObservations.update): the partner half receives the
        // env's new / terminal frames and done byte; both halves roll the stack; a done
        // env's terminal observation is [rolled stack, terminal frame], its stack
        // restarts from zeros; the new frame goes last
        const int src = lane & 31;
        const uint8_t db = (uint8_t)__shfl((int)df, src, 64);
        float nb[O], tb[O];
#pragma unroll
        for (int j = 0; j < O; ++j) {
          nb[j] = __shfl(on[j], src, 64);
          tb[j] = __shfl(ot[j], src, 64);
        }
        float stt[SO];
#pragma unroll
        for (int j = 0; j < SO - O; ++j) stt[j] = st[j + O];
#pragma unroll
        for (int j = 0; j < O; ++j) stt[SO - O + j] = tb[j];
        if (boot) {
          const bool bt = valid && (db & LZ_DONE_TRUNCATED) && !(db & LZ_DONE_TERMINATED);
          if (__ballot(bt) != 0ull) {
            bf16x8 xs[KS], f[4];
            stack_frags<SO, KS>(stt, h, bt, xs);
            attn_ln_extract<KS>(s_blob, xs, lane, f);
            const float vt = attn_net(vf_net, f, lane)[0];
            if (bt) rew = rew + gamma * vt;
          }
        }
#pragma unroll
        for (int j = 0; j < SO - O; ++j) st[j] = db ? 0.0f : stt[j];
#pragma unroll
        for (int j = 0; j < O; ++j) st[SO - O + j] = nb[j];
      } else if (boot) {  // SB3: truncated (not terminated) -> rewards += gamma * V(terminal obs)
        const bool bt = live && (df & LZ_DONE_TRUNCATED) && !(df & LZ_DONE_TERMINATED);
        if (__ballot(bt) != 0ull) {  // wave-uniform branch
          float xt[O], vt[1];
          normalize<O>(ot, xt, norm, mu, sd, p.clip);
          value_fwd<E, O, kPair>(s_blob, vf_net, xt, bt, lane, vt);
          if (bt) rew = rew + gamma * vt[0];
        }
      }
      if (live) {
        rew_buf[off] = rew;
        a.done[off] = df;
        if (kPair != kAttnLn && !kRegMom && p.partials) {
#pragma unroll
          for (int j = 0; j < O; ++j) {
            const double v = (double)on[j];
            mom[j] += v;
            mom[O + j] += v * v;
          }
        }
      }
      if constexpr (kRegMom) {
        if (p.partials) {
#pragma unroll
          for (int j = 0; j < O; ++j) {
            const double v = (double)__shfl(on[j], lane & 31, 64);
            if (i < a.n) mom_r[j] += h ? v * v : v;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < O; ++j) o[j] = on[j];
    }
    float vl[1];
    if constexpr (kPair == kAttnLn) {
      bf16x8 xs[KS], f[4];
      stack_frags<SO, KS>(st, h, valid, xs);
      attn_ln_extract<KS>(s_blob, xs, lane, f);
      vl[0] = attn_net(vf_net, f, lane)[0];
      if (live) {
#pragma unroll
        for (int j = 0; j < SO; ++j) p.stack_out[i * SO + j] = st[j];
      }
    } else {
      float x[O];
      normalize<O>(o, x, norm, mu, sd, p.clip);
      value_fwd<E, O, kPair>(s_blob, vf_net, x, live, lane, vl);
    }
    if (live) {
      p.last_val[i] = vl[0];
#pragma unroll
      for (int j = 0; j < O; ++j) p.obs_last[i * O + j] = o[j];
      sys.store(a, i);
      if (any_reset) sys.store_autoreset_extra(a, i);
      if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
    }
  }
  if (kPair != kAttnLn && p.partials) {  // fixed-order butterfly over the wave: deterministic
    double* dst = p.partials + ((int64_t)blockIdx.x * W + wave) * (2 * O);
#pragma unroll
    for (int j = 0; j < 2 * O; ++j) {
      double v;
      if constexpr (kRegMom) v = (j < O ? h == 0 : h == 1) ? mom_r[j < O ? j : j - O] : 0.0;
      else v = owner ? mom[j] : 0.0;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
      if (lane == 0) dst[j] = v;
    }
  }
}

// Workgroup barrier for LDS hand-overs: this wave's LDS ops complete, then s_barrier.
// __syncthreads() would also drain vmcnt (every outstanding global store of the wave).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------------------
// The float32 MlpPolicy rollout with the two nets in different waves (f32_policy_shape
// pair = 1: fewer than 8 32-env tiles per CU, e.g. cfg5's 32,768 envs = 1,024 tiles).
// With both nets in one wave such a grid has one wave per SIMD, and every MFMA chain's
// and tanh's latency is exposed.  Here waves 0-3 (actors) each step a 32-env tile: the
// pi net, the sample, the env step; waves 4-7 (critics; wave w + 4 shares wave w's SIMD)
// run the value net on the same tiles: V(x_k) for the values, the truncation bootstraps
// and V(x_K) -- two waves per SIMD, each computing what k_rollout_policy<kMlpF32>
// computes (the same bits; the same moment partials, one per actor wave, the same tile
// order).  Hand-over through LDS, one slot per env and no double buffer: the actor
// writes step k's next obs, terminal obs, reward and done code between barriers M_k and
// B_k; the critic reads them between B_k and M_{k+1}, then evaluates V(x_{k+1}) (and
// step k's bootstraps) while the actor runs step k + 1.
template <class Sys, bool kI8 = false>
__global__ __launch_bounds__(512) void k_rollout_policy_f32_split(KArgs a, PArgs p) {
  constexpr int kKind = kI8 ? kMlpI8 : kMlpF32;
  constexpr int O = Sys::O, A = Sys::A, KS1 = (O + 1) / 2, T = 4;  // T tiles per workgroup
  static_assert(O <= kPolMaxObs && A <= kPolMaxAct, "policy tile shape");
  __shared__ __attribute__((aligned(64))) uint8_t s_blob[kF32BlobBytes];
  __shared__ double s_norm[2 * kPolMaxObs];
  __shared__ float s_on[T][O][32], s_ot[T][O][32], s_rew[T][32];
  __shared__ uint32_t s_df[T][32];
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63, h = lane >> 5, slot = lane & 31;
  // wave-uniform in an SGPR: the actor / critic branches below hold barriers, so they
  // must be scalar branches, never exec-masked
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tw = wave & (T - 1);
  const bool owner = h == 0;
  blob_to_lds(reinterpret_cast<f4v*>(s_blob), reinterpret_cast<const f4v*>(p.blob), kF32BlobBytes / 16,
              tid, 2 * T * 64, !blob_is(p.blob, kF32Tag, kI8 ? LZ_BLOB_MLP_I8X4 : LZ_BLOB_MLP_F32));
  if (tid < O) {
    s_norm[tid] = p.norm ? p.norm[tid] : 0.0;
    s_norm[kPolMaxObs + tid] = p.norm ? sqrt(p.norm[O + tid] + p.eps) : 1.0;
  }
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  __syncthreads();
  const uint8_t* pi_net = s_blob;
  const uint8_t* vf_net = s_blob + kF32Net;
  const float* ttab = reinterpret_cast<const float*>(s_blob + kF32Tanh);
  const float* g_scale = reinterpret_cast<const float*>(s_blob + kF32LogStd) + 4;
  const float* g_var2 = g_scale + 4;
  const float* g_lscale = g_scale + 8;
  const bool norm = p.norm != nullptr;
  const double* mu = s_norm;
  const double* sd = s_norm + kPolMaxObs;
  const bool det = (p.pflags & LZ_POLICY_DETERMINISTIC) != 0;
  const bool boot = (p.pflags & LZ_POLICY_BOOTSTRAP) != 0;
  const float gamma = p.gamma;
  double mom_r[O];  // actors: the env's two lanes, half 0 the sums, half 1 the squares
#pragma unroll
  for (int j = 0; j < O; ++j) mom_r[j] = 0.0;
  float* obs_buf = static_cast<float*>(a.obs);
  float* rew_buf = static_cast<float*>(a.rew);
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t base = (int64_t)blockIdx.x * T; base < ntiles; base += (int64_t)gridDim.x * T) {
    const int64_t i = (base + tw) * 32 + slot;
    const bool live = owner && i < a.n;
    if (wave < T) {  // ---- actor
      Sys sys;
      sys.setup(a);
      int32_t steps = 0;
      bool any_reset = false;
      float o[O];
#pragma unroll
      for (int j = 0; j < O; ++j) o[j] = 0.0f;
      if (live) {
        sys.load(a, i);
        if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
#pragma unroll
        for (int j = 0; j < O; ++j) o[j] = p.obs_in[i * O + j];
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): see k_rollout_policy
      for (int k = 0; k < a.K; ++k) {
        lds_barrier();  // M_k: the critic has read step k - 1's hand-over
        const int64_t off = (int64_t)k * a.n + i;
        float x[O];
        normalize<O>(o, x, norm, mu, sd, p.clip);
        if (live) {
#pragma unroll
          for (int j = 0; j < O; ++j) obs_buf[off * O + j] = x[j];
        }
        float xs[KS1], mean[A];
        f32_inputs<O, KS1>(x, lane, xs);
        mlp_f32<KS1, A, kI8>(pi_net, xs, lane, mean, ttab);
        float act_c[A];
        if (live) {
          float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
          if (!det) {
            if constexpr (A <= 2) normal2(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k, z);
            else normal4(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k, z);
          }
          float lp = 0.0f;
#pragma unroll
          for (int j = 0; j < A; ++j) {
            const float aj = det ? mean[j] : mean[j] + z[j] * g_scale[j];
            const float d = aj - mean[j];
            const float lpj = (-(d * d)) / g_var2[j] - g_lscale[j] - 0.91893853320467274f;
            lp = j == 0 ? lpj : lp + lpj;
            act_c[j] = clip(aj, p.act_lo, p.act_hi);
            p.act[off * A + j] = aj;
          }
          p.logp[off] = lp;
        }
        float on[O], ot[O];
        float rew = 0.0f;
        bool did_reset;
        const uint8_t df = step_body<Sys, float, true, true>(sys, steps, a, i, live, act_c,
                                                             tick + (uint64_t)k, k, on, rew,
                                                             did_reset, ot);
        any_reset = any_reset || did_reset;
        if (live) {
          a.done[off] = df;
#pragma unroll
          for (int j = 0; j < O; ++j) {
            s_on[tw][j][slot] = on[j];
            s_ot[tw][j][slot] = ot[j];
          }
          s_rew[tw][slot] = rew;
          s_df[tw][slot] = df;
        }
        if (p.partials) {
#pragma unroll
          for (int j = 0; j < O; ++j) {
            const double v = (double)__shfl(on[j], slot, 64);
            if (i < a.n) mom_r[j] += h ? v * v : v;
          }
        }
#pragma unroll
        for (int j = 0; j < O; ++j) o[j] = on[j];
        lds_barrier();  // B_k: step k's hand-over is written
      }
      if (live) {
#pragma unroll
        for (int j = 0; j < O; ++j) p.obs_last[i * O + j] = o[j];
        sys.store(a, i);
        if (any_reset) sys.store_autoreset_extra(a, i);
        if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
      }
    } else {  // ---- critic
      float o[O], ot[O];
      float rew = 0.0f;
      uint32_t df = 0;
#pragma unroll
      for (int j = 0; j < O; ++j) o[j] = live ? p.obs_in[i * O + j] : 0.0f;
      // step kk's hand-over -> registers (between B_kk and M_{kk+1})
      auto take = [&]() {
        if (live) {
#pragma unroll
          for (int j = 0; j < O; ++j) {
            o[j] = s_on[tw][j][slot];
            ot[j] = s_ot[tw][j][slot];
          }
          rew = s_rew[tw][slot];
          df = s_df[tw][slot];
        }
      };
      // step kk's truncation bootstrap (SB3: rewards += gamma * V(terminal obs)), reward out
      auto settle = [&](int kk) {
        if (boot) {
          const bool bt = live && (df & LZ_DONE_TRUNCATED) && !(df & LZ_DONE_TERMINATED);
          if (__ballot(bt) != 0ull) {
            float xt[O], vt[1];
            normalize<O>(ot, xt, norm, mu, sd, p.clip);
            value_fwd<32, O, kKind>(s_blob, vf_net, xt, bt, lane, vt);
            if (bt) rew = rew + gamma * vt[0];
          }
        }
        if (live) rew_buf[(int64_t)kk * a.n + i] = rew;
      };
      for (int k = 0; k < a.K; ++k) {
        if (k > 0) take();
        lds_barrier();  // M_k
        if (k > 0) settle(k - 1);
        float x[O], xs[KS1], val[1];
        normalize<O>(o, x, norm, mu, sd, p.clip);
        f32_inputs<O, KS1>(x, lane, xs);
        mlp_f32<KS1, 1, kI8>(vf_net, xs, lane, val, ttab);
        if (live) p.val[(int64_t)k * a.n + i] = val[0];
        lds_barrier();  // B_k
      }
      take();
      settle(a.K - 1);
      float x[O], vl[1];
      normalize<O>(o, x, norm, mu, sd, p.clip);
      value_fwd<32, O, kKind>(s_blob, vf_net, x, live, lane, vl);
      if (live) p.last_val[i] = vl[0];
    }
  }
  if (wave < T && p.partials) {  // fixed-order butterfly over the wave, as k_rollout_policy
    double* dst = p.partials + ((int64_t)blockIdx.x * T + wave) * (2 * O);
#pragma unroll
    for (int j = 0; j < 2 * O; ++j) {
      double v = (j < O ? h == 0 : h == 1) ? mom_r[j < O ? j : j - O] : 0.0;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
      if (lane == 0) dst[j] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// SB3-exact VecNormalize in the float32 rollout (lz_policy_step_f32).  SB3 2.7.1's
// collect_rollouts under VecNormalize(training=True) (code/lorenz_pmsm/train.py:170-181):
//   step k:   actions, values = policy(_last_obs)            (_last_obs normalised by S_k)
//             obs, rew, done, infos = venv.step(clip(actions))  -> raw obs_{k+1}
//             VecNormalize.step_wait: S_{k+1} = obs_rms.update(S_k, raw obs_{k+1} batch);
//               obs_{k+1} = normalise(raw, S_{k+1}); infos' terminal obs normalised by
//               S_{k+1} too
//             truncated: rew += gamma * V(terminal obs)       (needs S_{k+1})
// Step k's input depends on a reduction over the whole batch of step k's outputs, so
// the collect runs one launch per step with the statistics update between launches
// (k_vn_tile_update), and each launch first settles the previous step's truncation
// bootstraps with the statistics that step produced.  Per launch: the blob to LDS, the
// env state from / to its planes (no VGPR residency across steps), the raw obs carry.
// The forward is mlp_f32 (the same bits as k_rollout_policy<kMlpF32>); the obs moments
// are float64 sums per 32-env tile (lz_internal.h PStepArgs: the order the oracle
// restates).  32 envs per wave: lane r (h = 0) owns env r, lane r + 32 its second half.
template <class Sys, int W>
__global__ __launch_bounds__(W * 64) void k_policy_step_f32(KArgs a, PArgs p, PStepArgs s) {
  constexpr int O = Sys::O, A = Sys::A, KS1 = (O + 1) / 2;
  static_assert(O <= kPolMaxObs && A <= kPolMaxAct, "policy tile shape");
  __shared__ __attribute__((aligned(64))) uint8_t s_blob[kF32BlobBytes];
  __shared__ double s_norm[2 * kPolMaxObs];
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int slot = lane & 31;
  blob_to_lds(reinterpret_cast<f4v*>(s_blob), reinterpret_cast<const f4v*>(p.blob), kF32BlobBytes / 16,
              tid, W * 64, !blob_is(p.blob, kF32Tag, LZ_BLOB_MLP_F32));
  if (tid < O) {
    s_norm[tid] = p.norm[tid];
    s_norm[kPolMaxObs + tid] = sqrt(p.norm[O + tid] + p.eps);
  }
  // S_k for the update after this launch (read-only there: no race with the write-back)
  if (blockIdx.x == 0 && s.snap && tid < 2 * O + 1) s.snap[tid] = p.norm[tid];
  const uint64_t tick = *a.tick_in;
  // a step launch flips the handle's call parity: advance the tick and zero the done
  // cursor the handle's next launch (outside the collect) starts from
  if (blockIdx.x == 0 && tid == 0 && !s.final_) {
    *a.tick_out = tick + 1;
    *a.counter_next = 0;
  }
  __syncthreads();
  const uint8_t* pi_net = s_blob;
  const uint8_t* vf_net = s_blob + kF32Net;
  const float* ttab = reinterpret_cast<const float*>(s_blob + kF32Tanh);
  const float* g_scale = reinterpret_cast<const float*>(s_blob + kF32LogStd) + 4;
  const float* g_var2 = g_scale + 4;
  const float* g_lscale = g_scale + 8;
  const double* mu = s_norm;
  const double* sd = s_norm + kPolMaxObs;
  const bool det = (p.pflags & LZ_POLICY_DETERMINISTIC) != 0;
  const bool boot = (p.pflags & LZ_POLICY_BOOTSTRAP) != 0;
  const int k = s.k;
  Sys sys;
  sys.setup(a);
  float* obs_buf = static_cast<float*>(a.obs);
  float* rew_buf = static_cast<float*>(a.rew);
  const int64_t ntiles = (a.n + kVnTile - 1) / kVnTile;
  for (int64_t tile = (int64_t)blockIdx.x * W + wave; tile < ntiles; tile += (int64_t)gridDim.x * W) {
    const int64_t i = tile * kVnTile + slot;
    const bool valid = i < a.n;
    const bool live = h == 0 && valid;
    // 1. the truncation bootstraps of step k - 1: V(terminal obs normalised by S_k)
    if (boot && k > 0) {
      const int64_t po = (int64_t)(k - 1) * a.n + i;
      const uint8_t d = live ? a.done[po] : (uint8_t)0;
      const bool bt = live && (d & LZ_DONE_TRUNCATED) && !(d & LZ_DONE_TERMINATED);
      if (__ballot(bt) != 0ull) {  // wave-uniform
        float ot[O], xt[O], vt[1];
#pragma unroll
        for (int j = 0; j < O; ++j) ot[j] = bt ? s.term[i * O + j] : 0.0f;
        normalize<O>(ot, xt, true, mu, sd, p.clip);
        value_fwd<32, O, kMlpF32>(s_blob, vf_net, xt, bt, lane, vt);
        if (bt) rew_buf[po] = rew_buf[po] + p.gamma * vt[0];
      }
    }
    // 2. the observation the policy sees: the raw obs normalised by S_k
    float o[O], x[O];
#pragma unroll
    for (int j = 0; j < O; ++j) o[j] = live ? s.obs_src[i * O + j] : 0.0f;
    normalize<O>(o, x, true, mu, sd, p.clip);
    if (s.final_) {  // the epilogue: last values (SB3 compute_returns_and_advantage input)
      float vl[1];
      value_fwd<32, O, kMlpF32>(s_blob, vf_net, x, live, lane, vl);
      if (live) p.last_val[i] = vl[0];
      continue;
    }
    int32_t steps = 0;
    if (live) {
      sys.load(a, i);
      if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
    }
    const int64_t off = (int64_t)k * a.n + i;
    if (live) {
#pragma unroll
      for (int j = 0; j < O; ++j) obs_buf[off * O + j] = x[j];
    }
    float mean[A], val[1];
    {
      float xs[KS1];
      f32_inputs<O, KS1>(x, lane, xs);
      mlp_f32<KS1, A>(pi_net, xs, lane, mean, ttab);
      __builtin_amdgcn_sched_barrier(0);
      mlp_f32<KS1, 1>(vf_net, xs, lane, val, ttab);
    }
    float act_c[A];
    if (live) {
      float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (!det) {
        if constexpr (A <= 2) normal2(a.seed, (uint64_t)(a.gid0 + i), tick, z);
        else normal4(a.seed, (uint64_t)(a.gid0 + i), tick, z);
      }
      float lp = 0.0f;
#pragma unroll
      for (int j = 0; j < A; ++j) {
        const float aj = det ? mean[j] : mean[j] + z[j] * g_scale[j];
        const float dd = aj - mean[j];
        const float lpj = (-(dd * dd)) / g_var2[j] - g_lscale[j] - 0.91893853320467274f;
        lp = j == 0 ? lpj : lp + lpj;
        act_c[j] = clip(aj, p.act_lo, p.act_hi);
        p.act[off * A + j] = aj;
      }
      p.logp[off] = lp;
      p.val[off] = val[0];
    }
    float on[O], ot[O];
    float rew = 0.0f;
    bool did_reset;
    const uint8_t df = step_body<Sys, float, true, true>(sys, steps, a, i, live, act_c, tick, k, on,
                                                         rew, did_reset, ot);
    if (live) {
      rew_buf[off] = rew;
      a.done[off] = df;
#pragma unroll
      for (int j = 0; j < O; ++j) p.obs_last[i * O + j] = on[j];
      if (df) {
#pragma unroll
        for (int j = 0; j < O; ++j) s.term[i * O + j] = ot[j];
      }
      sys.store(a, i);
      if (did_reset) sys.store_autoreset_extra(a, i);
      if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
    }
    // 3. the tile's float64 moments of the raw obs VecNormalize updates obs_rms with:
    // half 0 sums, half 1 squares, a 32-lane butterfly within each half
    if (s.tiles) {
#pragma unroll
      for (int j = 0; j < O; ++j) {
        const double v = (double)__shfl(on[j], slot, 64);
        double m = valid ? (h ? v * v : v) : 0.0;
#pragma unroll
        for (int q = 16; q >= 1; q >>= 1) m += __shfl_xor(m, q, 64);
        if (slot == 0) s.tiles[(int64_t)(h * O + j) * s.ntiles + tile] = m;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// The attention actor-critics at SB3's precision: code/train.py:52-112 (PPO, the
// AttentionFeaturesExtractor shared by pi and vf) and code/lorenz_filter/train.py:54-132
// (the residual + LayerNorm variant on VecFrameStack(4)), float32 end to end -- the
// oracle (lz_oracle.c orc_attn_f32) restates every operation in this order, bit for bit.
// Layout (lz_internal.h kAF*): v_mfma_f32_16x16x4_f32, 16 envs per wave, lane group
// G = lane >> 4 holds units 4G .. 4G+3 of every 16-unit tile, which is also the k order
// of the next projection -- so token t is fc1 tile t, lane group G holds head G's query,
// keys and values and runs head G's softmax, and nothing moves between lanes:
//   fc1 + ReLU            (relu keeps NaN)
//   K, V, Q per token     Q with the exact 1/sqrt(4) = 0.5 folded (torch scales q)
//   attention, head G     scores as fmaf chains, NaN-propagating max, exp_att, the sum in
//                         key order, one division 1 / sum, weights e_j * (1 / sum), outputs
//                         as fmaf chains over the keys (torch: softmax, then weights @ v)
//   out_proj
//   [LayerNorm]           (x + attn): per lane group the sum of its 4 dims in order, the
//                         groups' partials combined by a lane-16 then a lane-32 swap
//                         ((p0 + p1) + (p2 + p3) on every lane), * 1/16; the biased
//                         variance the same way; rstd = 1 / sqrtf(var + 1e-5);
//                         fmaf(z * rstd, w, b)
//   post_fc + ReLU, the pi / vf nets (layer 1 over the 64 features, tanh_tab, layer 2,
//   tanh_tab) and the heads (per lane group an fmaf chain over its units, the groups
//   combined like the LayerNorm sums, then the bias).
// All four lanes of an env (c, c + 16, c + 32, c + 48) also run the env step, the sample
// and the frame stack redundantly (step_body's lead flag: only lane group 0 takes a slot
// in the compact done list; only lane group 0 stores), so every lane has the inputs its
// k-steps need without a shuffle.
// Both nets do not fit in LDS beside the extractor: the workgroup keeps the extractor,
// the constants and ONE net slot, and LDS-DMAs (global_load_lds_dwordx4, 1 KiB per wave
// instruction, no VGPR staging) pi into it while the step's features are extracted and
// vf while the env steps.  The value of the step and the truncation bootstrap of the
// PREVIOUS step (its terminal input extracted while vf lands) run from the vf slot after
// the env step; the last step's bootstrap and the last values close the tile.  8 waves
// (two per SIMD), every wave of the workgroup in lockstep through the swaps.

// exp(x) for the softmax (x <= 0, or NaN): orc_exp_f32's operations exactly
__device__ __forceinline__ float exp_att(float x) {
  const float k = __builtin_rintf(x * 1.44269504088896341f);
  float r = fmaf(k, -0.693145751953125f, x);
  r = fmaf(k, -1.42860682030941723e-6f, r);
  float p = fmaf(1.38888892e-3f, r, 8.33333377e-3f);
  p = fmaf(p, r, 4.16666679e-2f);
  p = fmaf(p, r, 1.66666672e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  const float y = __builtin_ldexpf(p, (int)k);
  // a NaN x is NaN here already (k, r and p are NaN; (int)NaN = 0): the oracle's explicit
  // NaN return needs no select (any NaN is the oracle's NaN)
  return x < -86.0f ? 0.0f : y;
}

__device__ __forceinline__ float relu_f(float v) { return v < 0.0f ? 0.0f : v; }  // NaN kept

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// (p0 + p1) + (p2 + p3) of the four lane groups' values, on every lane (IEEE addition
// commutes, so each lane's order gives the same bits)
__device__ __forceinline__ float group_sum4(float v) {
  v = v + __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}


__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// one 16-unit tile over KB k-blocks: w(kb, i) the weight digits, x[kb][i] the inputs'
// -> the four level accumulators
template <int KB, class WF>
__device__ __forceinline__ void i8x_tile(WF w, const i32x4 (*x)[4], i32x4* L) {
  const i32x4 z = {0, 0, 0, 0};
  L[0] = L[1] = L[2] = L[3] = z;  // levels 6, 5, 4, 3
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const i32x4 w3 = w(kb, 3), w2 = w(kb, 2), w1 = w(kb, 1), w0 = w(kb, 0);
    L[0] = mfma_i8(w3, x[kb][3], L[0]);
    L[1] = mfma_i8(w3, x[kb][2], L[1]);
    L[1] = mfma_i8(w2, x[kb][3], L[1]);
    L[2] = mfma_i8(w3, x[kb][1], L[2]);
    L[2] = mfma_i8(w2, x[kb][2], L[2]);
    L[2] = mfma_i8(w1, x[kb][3], L[2]);
    L[3] = mfma_i8(w3, x[kb][0], L[3]);
    L[3] = mfma_i8(w2, x[kb][1], L[3]);
    L[3] = mfma_i8(w1, x[kb][2], L[3]);
    L[3] = mfma_i8(w0, x[kb][3], L[3]);
  }
}

// the 64 features (4 tiles) of one input; xs[s] = this lane group's fc1 input of k-step
// s (input 4s + G)
template <int KS, bool kLn, bool kI8 = false>
__device__ __forceinline__ void attn16_extract(const uint8_t* ext, const float* xs, int lane,
                                               f32x4* feat, const int16_t* psh = nullptr) {
  asm volatile("" ::: "memory");
  const int G = lane >> 4;
  constexpr int KQ = (KS + 3) / 4;
  const f32x4* wf = reinterpret_cast<const f32x4*>(ext + kAFFc1W) + lane;
  const f32x4* bf = reinterpret_cast<const f32x4*>(ext + kAFFc1B) + G;
  // token t = fc1 tile t, computed twice (for the keys / values first, then again for
  // the query and the residual): 8 KS MFMAs instead of 32 registers held through the
  // attention
  auto token = [&](int t) __attribute__((always_inline)) {
    asm volatile("" ::: "memory");  // keep the LDS weight loads of different tiles apart
    f32x4 c = bf[4 * t];
#pragma unroll
    for (int qd = 0; qd < KQ; ++qd) {
      const f32x4 w = wf[(t * 2 + qd) * 64];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * qd + e < KS) c = mfma16(w[e], xs[4 * qd + e], c);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = relu_f(c[r]);
    return c;
  };
  const f32x4 wk = reinterpret_cast<const f32x4*>(ext + kAFKW)[lane];
  const f32x4 wv = reinterpret_cast<const f32x4*>(ext + kAFVW)[lane];
  const f32x4 bk = reinterpret_cast<const f32x4*>(ext + kAFKB)[G];
  const f32x4 bv = reinterpret_cast<const f32x4*>(ext + kAFVB)[G];
  f32x4 K[kAttTokens], V[kAttTokens];  // head G's 4 key / value dims of each token
#pragma unroll
  for (int T = 0; T < kAttTokens; ++T) {
    const f32x4 tk = token(T);
    f32x4 ck = bk, cv = bv;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ck = mfma16(wk[s], tk[s], ck);
      cv = mfma16(wv[s], tk[s], cv);
    }
    K[T] = ck;
    V[T] = cv;
  }
  const f32x4 wq = reinterpret_cast<const f32x4*>(ext + kAFQW)[lane];
  const f32x4 wo = reinterpret_cast<const f32x4*>(ext + kAFOW)[lane];
  const f32x4 bq = reinterpret_cast<const f32x4*>(ext + kAFQB)[G];
  const f32x4 bo = reinterpret_cast<const f32x4*>(ext + kAFOB)[G];
  const f32x4 gam = reinterpret_cast<const f32x4*>(ext + kAFGam)[G];
  const f32x4 bet = reinterpret_cast<const f32x4*>(ext + kAFBet)[G];
  const f32x4* wp = reinterpret_cast<const f32x4*>(ext + kAFPostW) + lane;
  f32x4 post[4];
  f32x4 uall[kI8 ? kAttTokens : 1];  // kI8: every token's attention outputs (dims 4G..4G+3)
  if constexpr (!kI8) {  // (kI8: the bias is read after the token loop: fewer live registers)
#pragma unroll
    for (int u = 0; u < 4; ++u) post[u] = reinterpret_cast<const f32x4*>(ext + kAFPostB)[4 * u + G];
  }
#pragma unroll
  for (int i = 0; i < kAttTokens; ++i) {
    asm volatile("" ::: "memory");  // one query token's weights in flight at a time
    f32x4 pw[4];  // token i's post_fc weights, issued ahead of the attention math
    if constexpr (!kI8) {
#pragma unroll
      for (int u = 0; u < 4; ++u) pw[u] = wp[(u * 8 + i) * 64];
    }
    const f32x4 tk = token(i);
    f32x4 q = bq;
#pragma unroll
    for (int s = 0; s < 4; ++s) q = mfma16(wq[s], tk[s], q);
    float sc[kAttTokens];
#pragma unroll
    for (int j = 0; j < kAttTokens; ++j) {
      float t = q[0] * K[j][0];
      t = fmaf(q[1], K[j][1], t);
      t = fmaf(q[2], K[j][2], t);
      t = fmaf(q[3], K[j][3], t);
      sc[j] = t;
    }
    float m = sc[0];
#pragma unroll
    // NaN-propagating max (v_maximum_f32): the oracle's NaN-keeping select, except that
    // +0 beats -0 -- which cannot change sc[j] - m or its exp
    for (int j = 1; j < kAttTokens; ++j) m = __builtin_elementwise_maximum(m, sc[j]);
    float e[kAttTokens], sum = 0.0f;
#pragma unroll
    for (int j = 0; j < kAttTokens; ++j) {
      e[j] = exp_att(sc[j] - m);
      sum = j == 0 ? e[0] : sum + e[j];
    }
    const float r = 1.0f / sum;
    float o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float acc = (e[0] * r) * V[0][d];
#pragma unroll
      for (int j = 1; j < kAttTokens; ++j) acc = fmaf(e[j] * r, V[j][d], acc);
      o[d] = acc;
    }
    f32x4 y = bo;
#pragma unroll
    for (int s = 0; s < 4; ++s) y = mfma16(wo[s], o[s], y);
    float u[4];
    if constexpr (kLn) {
      float z[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) z[d] = y[d] + tk[d];
      const float mean = group_sum4(((z[0] + z[1]) + z[2]) + z[3]) * 0.0625f;
#pragma unroll
      for (int d = 0; d < 4; ++d) z[d] = z[d] - mean;
      float s2 = z[0] * z[0];
#pragma unroll
      for (int d = 1; d < 4; ++d) s2 = fmaf(z[d], z[d], s2);
      const float rstd = 1.0f / sqrtf(group_sum4(s2) * 0.0625f + 1e-5f);
#pragma unroll
      for (int d = 0; d < 4; ++d) u[d] = fmaf(z[d] * rstd, gam[d], bet[d]);
    } else {
#pragma unroll
      for (int d = 0; d < 4; ++d) u[d] = y[d];
    }
    if constexpr (kI8) {
#pragma unroll
      for (int d = 0; d < 4; ++d) uall[i][d] = u[d];
    } else {
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
#pragma unroll
        for (int s = 0; s < 4; ++s) post[uu] = mfma16(pw[uu][s], u[s], post[uu]);
      }
    }
  }
  if constexpr (kI8) {
    // post_attention_fc as i8x4 products (lz_oracle.c i8x_post): the env's 128 attention
    // outputs at the scale of their largest magnitude, k-block kb = tokens 4kb .. 4kb + 3
    // (byte 4f + r of lane group G = dim 4G + r of token 4kb + f)
    float m = 0.0f;
#pragma unroll
    for (int i = 0; i < kAttTokens; ++i)
#pragma unroll
      for (int d = 0; d < 4; ++d) m = __builtin_elementwise_maximum(m, fabsf(uall[i][d]));
    m = __builtin_elementwise_maximum(m, __shfl_xor(m, 16, 64));
    m = __builtin_elementwise_maximum(m, __shfl_xor(m, 32, 64));
    const bool bad = !(m <= 3.40282347e38f);
    const int qu = 28 - __builtin_amdgcn_frexp_expf(m);
    i32x4 xu[2][4];
#pragma unroll
    for (int i = 0; i < kAttTokens; ++i) {
      uint32_t d[4];
      i8x_digits4(uall[i], qu, d);
#pragma unroll
      for (int q = 0; q < 4; ++q) xu[i >> 2][q][i & 3] = (int)d[q];
    }
    const i32x4* w8 = reinterpret_cast<const i32x4*>(ext + kAFPostW) + lane;
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
      i32x4 L[4];
      i8x_tile<2>([&](int kb, int q) { return w8[((uu * 2 + kb) * 4 + q) * 64]; }, xu, L);
      post[uu] = reinterpret_cast<const f32x4*>(ext + kAFPostB)[4 * uu + G];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float y = i8x_recombine(L[0][r], L[1][r], L[2][r], L[3][r], psh[16 * uu + 4 * G + r] - qu) +
                        post[uu][r];
        feat[uu][r] = relu_f(bad ? __builtin_nanf("") : y);
      }
    }
    return;
  }
#pragma unroll
  for (int uu = 0; uu < 4; ++uu) {
#pragma unroll
    for (int r = 0; r < 4; ++r) post[uu][r] = relu_f(post[uu][r]);
    feat[uu] = post[uu];
  }
}

// one [128, 128] Tanh net + NH head rows on the 64 features (a kAFN* net slot)
template <int NH>
__device__ __forceinline__ void attn16_net(const uint8_t* net, const f32x4* feat, int lane,
                                           float* head, const float* ttab) {
  asm volatile("" ::: "memory");
  const int G = lane >> 4;
  const f32x4* w1 = reinterpret_cast<const f32x4*>(net + kAFN1) + lane;
  const f32x4* b1 = reinterpret_cast<const f32x4*>(net + kAFNB1) + G;
  f32x4 a1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    asm volatile("" ::: "memory");
    f32x4 w[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) w[f] = w1[(t * 4 + f) * 64];
    f32x4 c = b1[4 * t];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
#pragma unroll
      for (int s = 0; s < 4; ++s) c = mfma16(w[f][s], feat[f][s], c);
    }
    a1[t] = tanh_tab4(c, ttab);
  }
  const f32x4* w2 = reinterpret_cast<const f32x4*>(net + kAFN2) + lane;
  const f32x4* b2 = reinterpret_cast<const f32x4*>(net + kAFNB2) + G;
  const f32x4* wh = reinterpret_cast<const f32x4*>(net + kAFNH) + G;
  const float* bh = reinterpret_cast<const float*>(net + kAFNHB);
  float acc[NH];
#pragma unroll
  for (int j = 0; j < NH; ++j) acc[j] = 0.0f;  // first step fmaf(w, v, +0)
#pragma unroll 1
  for (int t = 0; t < 8; ++t) {
    asm volatile("" ::: "memory");
    f32x4 w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = w2[(t * 8 + q) * 64];
    f32x4 c = b2[4 * t];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int s = 0; s < 4; ++s) c = mfma16(w[q][s], a1[q][s], c);
    }
    const f32x4 v = tanh_tab4(c, ttab);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int j = 0; j < NH; ++j) acc[j] = fmaf(wh[j * 32 + 4 * t][r], v[r], acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NH; ++j) head[j] = group_sum4(acc[j]) + bh[j];
}

// ---------------------------------------------------------------------------------------
// attn16_net with the opt-in i8x4 wide layers (kAX* net slot, LZ_POLICY_I8X4; oracle:
// lz_oracle.c orc_attn_i8x4).  Each float32 input / weight is V = rint(v 2^q), |V| <=
// 2^28, as four balanced int8 digits (U = V + 0x808080: bytes 0..2 of U ^ 0x80, byte 3);
// a 16-unit tile's dot products are the 10 digit pairs (i, j), i + j >= 3, on
// v_mfma_i32_16x16x64_i8 into four int32 accumulators (levels 6..3) -- exact, so their
// order is free -- then hi = L6 * 256 + L5 (< 2^24), lo = L4 * 256 + L3 and
// y = ldexp(fmaf(float(hi), 2^16, float(lo)), shift) + bias.  The B operand of k-block
// digit i is lane (G, env) 16 B with byte 4f + r = digit i of input 16f + 4G + r of the
// block (the A operand's byte of the same k: the k order inside the instruction does not
// matter for an exact sum); the 16x16 accumulator's register r of lane (G, env) is unit
// 16t + 4G + r -- the f32 path's layout, so the inputs of layer 2 are layer 1's registers.
// the 64 features of a tile's envs as i8x4 digits at the env's scale (its largest
// feature; ReLU outputs >= 0, a NaN propagates): computed once per extraction and shared
// by the pi and vf nets.  x[i] byte 4f + r = digit i of feature 16f + 4G + r.
struct I8Feat {
  i32x4 x[4];
  int qa;
  bool bad;  // a NaN / inf feature: every output of the env is NaN
};

__device__ __forceinline__ I8Feat i8x_feat(const f32x4* feat) {
  float m = feat[0][0];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = __builtin_elementwise_maximum(m, feat[f][r]);
  m = __builtin_elementwise_maximum(m, __shfl_xor(m, 16, 64));
  m = __builtin_elementwise_maximum(m, __shfl_xor(m, 32, 64));
  I8Feat fi;
  fi.bad = !(m <= 3.40282347e38f);
  fi.qa = 28 - __builtin_amdgcn_frexp_expf(m);
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    uint32_t d[4];
    i8x_digits4(feat[f], fi.qa, d);
#pragma unroll
    for (int i = 0; i < 4; ++i) fi.x[i][f] = (int)d[i];
  }
  return fi;
}

template <int NH>
__device__ __forceinline__ void attn16_net_i8(const uint8_t* net, const I8Feat& fi, int lane,
                                              float* head, const float* ttab) {
  asm volatile("" ::: "memory");
  const int G = lane >> 4;
  const bool bad = fi.bad;
  const int qa = fi.qa;
  const i32x4(*xf)[4] = reinterpret_cast<const i32x4(*)[4]>(fi.x);
  const i32x4* w1 = reinterpret_cast<const i32x4*>(net + kAXN1) + lane;
  const f32x4* b1 = reinterpret_cast<const f32x4*>(net + kAFNB1) + G;
  const int16_t* s1 = reinterpret_cast<const int16_t*>(net + kAXSh1) + 4 * G;
  i32x4 xa[2][4];  // layer 2's inputs: k-block kb = tiles 4kb .. 4kb + 3
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    asm volatile("" ::: "memory");
    i32x4 L[4];
    i8x_tile<1>([&](int, int i) { return w1[(t * 4 + i) * 64]; }, xf, L);
    const f32x4 bb = b1[4 * t];
    f32x4 y;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      y[r] = i8x_recombine(L[0][r], L[1][r], L[2][r], L[3][r], s1[16 * t + r] - qa) + bb[r];
    const f32x4 a = tanh_tab4(y, ttab);  // (a bad env's garbage is replaced by NaN at the heads)
    uint32_t d[4];
    i8x_digits4(a, 28, d);
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[t >> 2][i][t & 3] = (int)d[i];
  }
  const i32x4* w2 = reinterpret_cast<const i32x4*>(net + kAXN2) + lane;
  const f32x4* b2 = reinterpret_cast<const f32x4*>(net + kAFNB2) + G;
  const int16_t* s2 = reinterpret_cast<const int16_t*>(net + kAXSh2) + 4 * G;
  const f32x4* wh = reinterpret_cast<const f32x4*>(net + kAFNH) + G;
  const float* bh = reinterpret_cast<const float*>(net + kAFNHB);
  float acc[NH];
#pragma unroll
  for (int j = 0; j < NH; ++j) acc[j] = 0.0f;  // first step fmaf(w, v, +0)
  // software-pipelined: tile t + 1's MFMAs are issued before tile t's recombination /
  // tanh / head work, so the matrix pipe runs under that VALU work
  auto tile2 = [&](int t, i32x4* L) __attribute__((always_inline)) {
    i8x_tile<2>([&](int kb, int i) { return w2[((t * 2 + kb) * 4 + i) * 64]; }, xa, L);
  };
#ifndef LZ_I8_PIPE
#define LZ_I8_PIPE 1
#endif
  i32x4 Lc[4];
  if (LZ_I8_PIPE) tile2(0, Lc);
#pragma unroll 1
  for (int t = 0; t < 8; ++t) {
    asm volatile("" ::: "memory");
    i32x4 Ln[4];
    if (!LZ_I8_PIPE) tile2(t, Lc);
    if (LZ_I8_PIPE && t + 1 < 8) tile2(t + 1, Ln);
    const f32x4 bb = b2[4 * t];
    f32x4 y;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      y[r] = i8x_recombine(Lc[0][r], Lc[1][r], Lc[2][r], Lc[3][r], s2[16 * t + r]) + bb[r];
    const f32x4 v = tanh_tab4(y, ttab);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int j = 0; j < NH; ++j) acc[j] = fmaf(wh[j * 32 + 4 * t][r], v[r], acc[j]);
    }
    if (LZ_I8_PIPE) {
#pragma unroll
      for (int q = 0; q < 4; ++q) Lc[q] = Ln[q];
    }
  }
#pragma unroll
  for (int j = 0; j < NH; ++j) {
    const float r = group_sum4(acc[j]) + bh[j];
    head[j] = bad ? __builtin_nanf("") : r;
  }
}

template <int NH, bool kI8>
__device__ __forceinline__ void attn16_net_sel(const uint8_t* net, const f32x4* feat, const I8Feat& fi,
                                               int lane, float* head, const float* ttab) {
  if constexpr (kI8) attn16_net_i8<NH>(net, fi, lane, head, ttab);
  else attn16_net<NH>(net, feat, lane, head, ttab);
}

typedef __attribute__((address_space(3))) void* las_p;
// 1 KiB per wave instruction from global (L2-resident weights: default cache policy)
// into LDS at M0 + 16 lane; issued from inline asm, so hipcc neither sees nor waits for
// it -- the caller waits with vmcnt(0) and a barrier before reading the slot.
__device__ __forceinline__ void dma16_keep(const void* g, uint32_t m0) {
  uint32_t saved;  // M0 is a reserved register hipcc may hold a value in: save/restore
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(m0)
               : "memory");
}

template <class Sys, bool kLn, int S, int W, bool kI8 = false>
__global__ __launch_bounds__(W * 64) void k_rollout_policy_attn_f32(KArgs a, PArgs p) {
  constexpr int E = 16;
  constexpr int O = Sys::O, A = Sys::A;
  constexpr int SO = S * O, KS = (SO + 3) / 4;
  static_assert(kLn || S == 1, "frame stacking is the LayerNorm variant's");
  static_assert(SO <= kAFMaxIn && O <= kPolMaxObs && A <= kPolMaxAct, "policy tile shape");
  constexpr int SZ = SO - O;  // the stack's older frames
  __shared__ __attribute__((aligned(16))) uint8_t s_lds[kAFLdsBytes];
  __shared__ double s_norm[2 * kPolMaxObs];
  __shared__ __attribute__((aligned(16))) int16_t s_psh[kI8 ? kAttFeat : 8];  // kI8: post_fc row shifts
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, G = lane >> 4, col = lane & 15;
  {
    const bool bad = !blob_is(p.blob, kAFTag,
                              kLn ? (kI8 ? LZ_BLOB_ATTN_LN_I8X4 : LZ_BLOB_ATTN_LN_F32)
                                  : (kI8 ? LZ_BLOB_ATTN_I8X4 : LZ_BLOB_ATTN_F32));
    // (a mismatch poisons the resident extractor and constants: the features, and with
    // them both nets' outputs, are NaN whatever the DMA'd net slots hold)
    blob_to_lds(reinterpret_cast<f4v*>(s_lds), reinterpret_cast<const f4v*>(p.blob), kAFExt / 16, tid,
                W * 64, bad);
    blob_to_lds(reinterpret_cast<f4v*>(s_lds + kAFExt), reinterpret_cast<const f4v*>(p.blob + kAFLogStd),
                kAFConst / 16, tid, W * 64, bad);
    if constexpr (kI8) {
      if (tid < kAttFeat * 2 / 16)
        reinterpret_cast<f4v*>(s_psh)[tid] = reinterpret_cast<const f4v*>(p.blob + kAFPi + kAXPostSh)[tid];
    }
  }
  if (tid < O) {
    s_norm[tid] = p.norm ? p.norm[tid] : 0.0;
    s_norm[kPolMaxObs + tid] = p.norm ? sqrt(p.norm[O + tid] + p.eps) : 1.0;
  }
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  __syncthreads();
  const uint8_t* s_ext = s_lds;
  const float* cst = reinterpret_cast<const float*>(s_lds + kAFExt);
  const float* g_scale = cst + 4;
  const float* g_var2 = cst + 8;
  const float* g_lscale = cst + 12;
  const float* ttab = cst + 16;
  const uint8_t* s_net = s_lds + kAFExt + kAFConst;
  const uint32_t m0_net = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(las_p)(const_cast<uint8_t*>(s_net)));
  const uint8_t* g_pi = p.blob + kAFPi;
  const uint8_t* g_vf = p.blob + kAFVf;
  auto net_dma = [&](const uint8_t* g) {  // this wave's share of the 100 1-KiB pieces
    const int wv = __builtin_amdgcn_readfirstlane(wave);  // M0 takes a wave-uniform SGPR
    for (int c = wv; c < kAFNet / 1024; c += W)
      dma16_keep(g + c * 1024 + lane * 16, (uint32_t)__builtin_amdgcn_readfirstlane(m0_net + 1024u * c));
  };
  const bool norm = p.norm != nullptr;
  const double* mu = s_norm;
  const double* sd = s_norm + kPolMaxObs;
  const bool det = (p.pflags & LZ_POLICY_DETERMINISTIC) != 0;
  const bool boot = (p.pflags & LZ_POLICY_BOOTSTRAP) != 0;
  const float gamma = p.gamma;
  double mom_r[O];  // pooled obs moments (code/train.py's variant): group 0 sums, 1 squares
#pragma unroll
  for (int j = 0; j < O; ++j) mom_r[j] = 0.0;
  Sys sys;
  sys.setup(a);
  float* obs_buf = static_cast<float*>(a.obs);
  float* rew_buf = static_cast<float*>(a.rew);
  const int64_t ntiles = (a.n + E - 1) / E;
  const int64_t per_round = (int64_t)gridDim.x * W;
  const int64_t rounds = (ntiles + per_round - 1) / per_round;
  // this lane group's fc1 inputs: input 4s + G of the stacked / normalised input
  auto inputs = [&](const float* src, float* xs) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float v = 0.0f;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (4 * s + g < SO) v = G == g ? src[4 * s + g < SO ? 4 * s + g : 0] : v;
      xs[s] = v;
    }
  };
  // kLn: the frame stack lives distributed like the fc1 inputs it feeds -- lane group G
  // holds entries 4s + G (s < KS) of its env's stack, 1/4 of it.  The policy's input
  // (the deferred zeroing applied) / the stacked terminal observation of a pending
  // bootstrap ([older frames, terminal frame]) are then per-lane selects.
  auto cur_stack = [&](const float* stv, bool z, float* xs) {
#pragma unroll
    for (int s = 0; s < KS; ++s) xs[s] = (z && 4 * s + G < SZ) ? 0.0f : stv[s];
  };
  auto frame_at = [&](const float* f, int q) {  // f[q] for a lane-varying q in [0, O)
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < O; ++j) v = q == j ? f[j] : v;
    return v;
  };
  auto term_stack = [&](const float* stv, const float* tf, float* xs) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int q = 4 * s + G;
      xs[s] = q < SZ ? stv[s] : (q < SO ? frame_at(tf, q - SZ) : 0.0f);
    }
  };
  // VecFrameStack roll (SB3 StackedObservations.update): entry q takes q + O, the new
  // frame lands in the last O.  Entry q + O lives in lane group (G + O) & 3, slot
  // s + O / 4 (+1 when G + O % 4 wraps): one lane permute per slot pair.
  auto roll_stack = [&](float* stv, const float* nf) {
    const int src = (((G + O) & 3) << 4) | col;
    const bool carry = G + (O & 3) >= 4;
    float nst[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      constexpr int D = O / 4;
      const float va = __shfl(s + D < KS ? stv[s + D < KS ? s + D : 0] : 0.0f, src, 64);
      const float vb = __shfl(s + D + 1 < KS ? stv[s + D + 1 < KS ? s + D + 1 : 0] : 0.0f, src, 64);
      const int q = 4 * s + G;
      const float v = carry ? vb : va;
      nst[s] = q < SZ ? v : (q < SO ? frame_at(nf, q - SZ) : 0.0f);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) stv[s] = nst[s];
  };
  for (int64_t rd = 0; rd < rounds; ++rd) {
    const int64_t tile = (rd * gridDim.x + blockIdx.x) * W + wave;
    const bool active = tile < ntiles;  // wave-uniform; inactive waves still swap the slot
    const int64_t i = tile * E + col;
    const bool valid = active && i < a.n;  // all four lanes of the env compute it
    const bool own = valid && G == 0;      // ... lane group 0 stores it
    int32_t steps = 0;
    bool any_reset = false;
    // pt: the raw terminal obs of a pending bootstrap.  kLn: st is the rolled stack with
    // the zeroing of a done env's older frames deferred (zf) until the bootstrap of the
    // step has read [st[0 .. SZ), pt] (SB3's stacked terminal observation)
    float o[O], st[kLn ? KS : 1], pt[O];
    bool zf = false;
#pragma unroll
    for (int j = 0; j < O; ++j) o[j] = pt[j] = 0.0f;
    if (valid) {
      sys.load(a, i);
      if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
#pragma unroll
      for (int j = 0; j < O; ++j) o[j] = p.obs_in[i * O + j];
    }
    if constexpr (kLn) {
#pragma unroll
      for (int s = 0; s < KS; ++s)
        st[s] = (valid && 4 * s + G < SO) ? p.stack_in[i * SO + (4 * s + G < SO ? 4 * s + G : 0)] : 0.0f;
    }
    bool pend = false;  // this env's step truncated: its bootstrap value comes next step
    float prew = 0.0f;  // ... and its reward before the bootstrap
    __builtin_amdgcn_s_waitcnt(0x0F70);
    for (int k = 0; k < a.K; ++k) {
      const int64_t off = (int64_t)k * a.n + i;
      // [1] pi into the slot, meanwhile the features of this step's input
      __syncthreads();
      net_dma(g_pi);
      const bool pb = pend;
      const bool any_pb = __ballot(pb) != 0ull;
      f32x4 F[4], Ft[4];
      I8Feat FI, FIt;  // kI8: F / Ft as digits (unused otherwise)
      if (active) {
        float xs[KS];
        if constexpr (kLn) {
          cur_stack(st, zf, xs);
          if (valid) {  // every lane group stores its entries of the stacked row
#pragma unroll
            for (int s = 0; s < KS; ++s)
              if (4 * s + G < SO) obs_buf[off * SO + 4 * s + G] = xs[s];
          }
        } else {
          float x[O];
          normalize<O>(o, x, norm, mu, sd, p.clip);
          if (own) {
#pragma unroll
            for (int j = 0; j < O; ++j) obs_buf[off * O + j] = x[j];
          }
          inputs(x, xs);
        }
        attn16_extract<KS, kLn, kI8>(s_ext, xs, lane, F, s_psh);
        if constexpr (kI8) FI = i8x_feat(F);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's DMA pieces have landed
      __syncthreads();
      // [2] the policy head: sample (every lane of the env, same Philox draw), log-prob, clip
      float act_c[A];
#pragma unroll
      for (int j = 0; j < A; ++j) act_c[j] = 0.0f;
      if (active) {
        float mean[A];
        attn16_net_sel<A, kI8>(s_net, F, FI, lane, mean, ttab);
        if (valid) {
          float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
          if (!det) {
            if constexpr (A <= 2) normal2(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k, z);
            else normal4(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k, z);
          }
          float lp = 0.0f;
#pragma unroll
          for (int j = 0; j < A; ++j) {
            const float aj = det ? mean[j] : mean[j] + z[j] * g_scale[j];
            const float dd = aj - mean[j];
            const float lpj = (-(dd * dd)) / g_var2[j] - g_lscale[j] - 0.91893853320467274f;
            lp = j == 0 ? lpj : lp + lpj;
            act_c[j] = clip(aj, p.act_lo, p.act_hi);
            if (own) p.act[off * A + j] = aj;
          }
          if (own) p.logp[off] = lp;
        }
      }
      // [3] vf into the slot while the previous step's pending terminal input is
      //     extracted and the env steps (which overwrites pt)
      __syncthreads();
      net_dma(g_vf);
      float rew = 0.0f;
      bool pn = false;
      if (active) {
        if (any_pb) {
          float xt[KS];
          if constexpr (kLn) {
            term_stack(st, pt, xt);
          } else {
            float x[O];
            normalize<O>(pt, x, norm, mu, sd, p.clip);
            inputs(x, xt);
          }
          attn16_extract<KS, kLn, kI8>(s_ext, xt, lane, Ft, s_psh);
          if constexpr (kI8) FIt = i8x_feat(Ft);
        }
        if constexpr (kLn) {  // the deferred zeroing, now that the bootstrap has its input
#pragma unroll
          for (int s = 0; s < KS; ++s) st[s] = (zf && 4 * s + G < SZ) ? 0.0f : st[s];
        }
        float on[O], ot[O];
        bool did_reset;
        const uint8_t df = step_body<Sys, float, true, true>(sys, steps, a, i, valid, act_c,
                                                             tick + (uint64_t)k, k, on, rew,
                                                             did_reset, ot, G == 0);
        any_reset = any_reset || did_reset;
        pn = boot && valid && (df & LZ_DONE_TRUNCATED) && !(df & LZ_DONE_TERMINATED);
        if (pn) {
#pragma unroll
          for (int j = 0; j < O; ++j) pt[j] = ot[j];
        }
        if constexpr (kLn) {
          // VecFrameStack (SB3 StackedObservations.update): roll by O, the new frame last;
          // a done env's older frames become zeros (deferred: zf) -- its stacked terminal
          // observation is [rolled older frames, terminal frame]
          roll_stack(st, on);
          zf = df != 0;
        } else {
          if (p.partials && valid && G < 2) {
#pragma unroll
            for (int j = 0; j < O; ++j) {
              const double v = (double)on[j];
              mom_r[j] += G ? v * v : v;
            }
          }
        }
        if (own) {
          rew_buf[off] = rew;
          a.done[off] = df;
        }
#pragma unroll
        for (int j = 0; j < O; ++j) o[j] = on[j];
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
      // [4] V(this step's input); the previous step's truncation bootstrap
      if (active) {
        float v[1];
        attn16_net_sel<1, kI8>(s_net, F, FI, lane, v, ttab);
        if (own) p.val[off] = v[0];
        if (any_pb) {
          float vt[1];
          attn16_net_sel<1, kI8>(s_net, Ft, FIt, lane, vt, ttab);
          if (own && pb) rew_buf[off - a.n] = prew + gamma * vt[0];
        }
      }
      pend = pn;
      prew = rew;
    }
    // the slot holds vf: the last step's bootstrap and the last values
    if (active) {
      const bool pb = pend;
      const bool any_pb = __ballot(pb) != 0ull;
      f32x4 F[4];
      I8Feat FI;
      float xs[KS];
      if constexpr (kLn) {
        cur_stack(st, zf, xs);
      } else {
        float x[O];
        normalize<O>(o, x, norm, mu, sd, p.clip);
        inputs(x, xs);
      }
      attn16_extract<KS, kLn, kI8>(s_ext, xs, lane, F, s_psh);
        if constexpr (kI8) FI = i8x_feat(F);
      float vl[1];
      attn16_net_sel<1, kI8>(s_net, F, FI, lane, vl, ttab);
      if (any_pb) {
        float xt[KS];
        if constexpr (kLn) {
          term_stack(st, pt, xt);
        } else {
          float x[O];
          normalize<O>(pt, x, norm, mu, sd, p.clip);
          inputs(x, xt);
        }
        attn16_extract<KS, kLn, kI8>(s_ext, xt, lane, F, s_psh);
        if constexpr (kI8) FI = i8x_feat(F);
        float vt[1];
        attn16_net_sel<1, kI8>(s_net, F, FI, lane, vt, ttab);
        if (own && pb) rew_buf[(int64_t)(a.K - 1) * a.n + i] = prew + gamma * vt[0];
      }
      if (own) {
        p.last_val[i] = vl[0];
#pragma unroll
        for (int j = 0; j < O; ++j) p.obs_last[i * O + j] = o[j];
        sys.store(a, i);
        if (any_reset) sys.store_autoreset_extra(a, i);
        if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
      }
      if constexpr (kLn) {
        if (valid) {
#pragma unroll
          for (int s = 0; s < KS; ++s)
            if (4 * s + G < SO) p.stack_out[i * SO + 4 * s + G] = xs[s];
        }
      }
    }
  }
  if (!kLn && p.partials) {  // fixed-order butterfly over the wave: deterministic
    double* dst = p.partials + ((int64_t)blockIdx.x * W + wave) * (2 * O);
#pragma unroll
    for (int j = 0; j < 2 * O; ++j) {
      double v = (j < O ? G == 0 : G == 1) ? mom_r[j < O ? j : j - O] : 0.0;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
      if (lane == 0) dst[j] = v;
    }
  }
}

// obs moments: out = (count, column sums, column sums of squares) from the per-wave
// partials, summed in a fixed order.  One workgroup per column (the column loop ran in
// a single workgroup before: 22.9 us per collect at 262,144 envs, 2.8% of K=16); the
// per-column order -- lane t takes partials t, t+256, ..., then a fixed LDS tree -- is
// unchanged, so the totals are the same bits.
__global__ __launch_bounds__(256) void k_pol_moments_final(const double* part, int nparts, int width,
                                                          double count, double* out) {
  __shared__ double s[256];
  const int c = (int)blockIdx.x;
  double v = 0.0;
  for (int q = (int)threadIdx.x; q < nparts; q += 256) v += part[(int64_t)q * width + c];
  s[threadIdx.x] = v;
  __syncthreads();
  for (int m = 128; m >= 1; m >>= 1) {
    if ((int)threadIdx.x < m) s[threadIdx.x] += s[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[1 + c] = s[0];
    if (c == 0) out[0] = count;
  }
}

// RolloutBuffer.compute_returns_and_advantage (SB3 2.7.1 common/buffers.py), float32:
//   delta = rewards[t] + gamma * next_values * next_non_terminal - values[t]
//   last_gae_lam = delta + gamma * gae_lambda * next_non_terminal * last_gae_lam
//   returns = advantages + values
// with next_non_terminal = 1 - episode_starts[t+1] = 1 - done[t].
// One lane per env walks k = K-1 .. 0 (the recursion runs backwards in time); the next
// value is carried in a register instead of re-read, and one-wave workgroups spread a
// small batch (cfg5: 32,768 envs) over all CUs.  Loads are issued in batches of U steps
// ahead of their arithmetic (restrict pointers: the outputs never alias the inputs).
// Two schedules, picked by batch size (profiles/r01/policy/gae_ab.json):
//   DB = true : double-buffered, batch j+1 issued before batch j's arithmetic (U = 4):
//               a latency-bound small batch (32,768 envs = 512 waves) keeps loads in
//               flight across batches -- 830 -> 450 us at 32,768 envs x 2048 steps,
//               312 -> 214 us at 131,072 x 512 (gae_threshold.json);
//   DB = false: one batch of U = 8 at a time: with >= 4,096 waves the other waves hide
//               the gaps, and this schedule runs 5.4 TB/s at 262,144 envs (DB: 4.9).
// Same expressions, same order: bit-identical to the straightforward loop either way.
constexpr int kGaeBlock = 64;
template <int U, bool DB>
__global__ __launch_bounds__(kGaeBlock) void k_gae(int64_t n, int K, const float* __restrict__ rew,
                                                  const float* __restrict__ val,
                                                  const uint8_t* __restrict__ done,
                                                  const float* __restrict__ last_val, float gamma,
                                                  float gl, float* __restrict__ adv,
                                                  float* __restrict__ ret) {
  const int64_t i = (int64_t)blockIdx.x * kGaeBlock + threadIdx.x;
  if (i >= n) return;
  float last = 0.0f;
  float nv = last_val[i];  // next step's value: V(last obs) for k = K-1
  auto one = [&](int64_t off, float r, float v, uint8_t d) __attribute__((always_inline)) {
    const float nnt = 1.0f - (d ? 1.0f : 0.0f);
    const float delta = (r + (gamma * nv) * nnt) - v;
    last = delta + (gl * nnt) * last;
    __builtin_nontemporal_store(last, adv + off);
    __builtin_nontemporal_store(last + v, ret + off);
    nv = v;
  };
  float ra[U], va[U], rb[U], vb[U];
  uint8_t da[U], db[U];
  auto load = [&](int k0, float* r, float* v, uint8_t* d) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (int64_t)(k0 - u) * n + i;
      r[u] = __builtin_nontemporal_load(rew + off);
      v[u] = __builtin_nontemporal_load(val + off);
      d[u] = __builtin_nontemporal_load(done + off);
    }
  };
  auto run = [&](int k0, const float* r, const float* v, const uint8_t* d)
      __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) one((int64_t)(k0 - u) * n + i, r[u], v[u], d[u]);
  };
  int k = K - 1;
  if (!DB) {
    for (; k >= U - 1; k -= U) {
      float r[U], v[U];  // batch-local arrays: the scheduler interleaves the next
      uint8_t d[U];      // batch's loads with this one's stores
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = (int64_t)(k - u) * n + i;
        r[u] = __builtin_nontemporal_load(rew + off);
        v[u] = __builtin_nontemporal_load(val + off);
        d[u] = __builtin_nontemporal_load(done + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) one((int64_t)(k - u) * n + i, r[u], v[u], d[u]);
    }
  } else if (k >= U - 1) {
    load(k, ra, va, da);
    // two batches per iteration (a, b) so the buffers swap by name, not by moves
    for (; k >= 3 * U - 1; k -= 2 * U) {
      load(k - U, rb, vb, db);
      run(k, ra, va, da);
      load(k - 2 * U, ra, va, da);
      run(k - U, rb, vb, db);
    }
    if (k >= 2 * U - 1) {
      load(k - U, rb, vb, db);
      run(k, ra, va, da);
      run(k - U, rb, vb, db);
      k -= 2 * U;
    } else {
      run(k, ra, va, da);
      k -= U;
    }
  }
  for (; k >= 0; --k) {
    const int64_t off = (int64_t)k * n + i;
    one(off, rew[off], val[off], done[off]);
  }
}

// RolloutBuffer.episode_starts of one collect, from the done codes the rollout wrote
// (SB3 collect_rollouts: episode_starts[0] = the previous collect's last dones,
// episode_starts[k] = dones[k-1]): one pass instead of the compare + convert + copy
// torch launches it replaces.  Thread e of the grid-stride loop writes element e of
// the [K, N] float32 buffer; the first N lanes also write the next collect's carry.
__global__ __launch_bounds__(256) void k_episode_starts(int64_t n, int K, const uint8_t* __restrict__ done,
                                                        const float* __restrict__ last_in,
                                                        float* __restrict__ starts,
                                                        float* __restrict__ last_out) {
  const int64_t total = (int64_t)K * n;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const float v = e < n ? last_in[e] : (done[e - n] != 0 ? 1.0f : 0.0f);
    __builtin_nontemporal_store(v, starts + e);
    if (e < n) last_out[e] = done[(int64_t)(K - 1) * n + e] != 0 ? 1.0f : 0.0f;
  }
}

template <class Sys>
static int launch_pol(const KArgs& a, const PArgs& p, const PolShape& sh, hipStream_t s) {
  const dim3 grid((unsigned)sh.grid);
  if (sh.envs_per_wave == 64)
    hipLaunchKernelGGL((k_rollout_policy<Sys, 8, 64, kMlpSerial>), grid, dim3(8 * 64), 0, s, a, p);
  else if (sh.pair == 2)
    hipLaunchKernelGGL((k_rollout_policy<Sys, 4, 32, kMlpPairPipe>), grid, dim3(4 * 64), 0, s, a, p);
  else if (sh.pair)
    hipLaunchKernelGGL((k_rollout_policy<Sys, 4, 32, kMlpPair>), grid, dim3(4 * 64), 0, s, a, p);
  else
    hipLaunchKernelGGL((k_rollout_policy<Sys, 8, 32, kMlpSerial>), grid, dim3(8 * 64), 0, s, a, p);
  return (int)hipGetLastError();
}

template <class Sys, bool kI8>
static void launch_pol_f32_k(const KArgs& a, const PArgs& p, const PolShape& sh, hipStream_t s) {
  constexpr int kKind = kI8 ? kMlpI8 : kMlpF32;
  if (sh.pair == 1)
    hipLaunchKernelGGL((k_rollout_policy_f32_split<Sys, kI8>), dim3((unsigned)sh.grid), dim3(8 * 64), 0, s,
                       a, p);
  else if (sh.waves == 4)
    hipLaunchKernelGGL((k_rollout_policy<Sys, 4, 32, kKind>), dim3((unsigned)sh.grid), dim3(4 * 64), 0, s,
                       a, p);
  else
    hipLaunchKernelGGL((k_rollout_policy<Sys, 8, 32, kKind>), dim3((unsigned)sh.grid), dim3(8 * 64), 0, s,
                       a, p);
}

// kI8: LZ_POLICY_I8X4 is built for the four systems of the reference's training scripts
// (LORENZ3 / LORENZ4 / PMSM / HR); the others refuse it
template <class Sys, bool kHasI8 = false>
static int launch_pol_f32(const KArgs& a, const PArgs& p, const PolShape& sh, hipStream_t s) {
  if (p.pflags & LZ_POLICY_I8X4) {
    if constexpr (kHasI8) launch_pol_f32_k<Sys, true>(a, p, sh, s);
    else return (int)hipErrorInvalidValue;
  } else {
    launch_pol_f32_k<Sys, false>(a, p, sh, s);
  }
  return (int)hipGetLastError();
}

// 8 waves (two per SIMD) when there are enough 32-env tiles for every CU, else 4 tiles
// per workgroup with the nets split over 8 waves (pair = 1, k_rollout_policy_f32_split:
// cfg5's 32,768 envs are 1,024 tiles = 128 eight-tile groups, half the CUs).
// LZ_POL_F32_WAVES=4|8 forces the one-wave-per-tile kernel at that width, lz_config
// reserved[0] bit 8192 keeps it at 4 waves (A/B knobs).  waves = tiles per workgroup:
// the moment partials are one per tile-wave either way.
PolShape f32_policy_shape(int64_t n, int num_cus, int variant) {
  const int64_t tiles = (n + 31) / 32;
  static const int forced = [] {
    const char* e = std::getenv("LZ_POL_F32_WAVES");
    const int w = e ? std::atoi(e) : 0;
    return w == 4 || w == 8 ? w : 0;
  }();
  PolShape s = {32, forced ? forced : tiles >= 8 * (int64_t)num_cus ? 8 : 4, 0, 0};
  if (!forced && s.waves == 4 && !(variant & 8192)) s.pair = 1;
  const int64_t groups = (tiles + s.waves - 1) / s.waves;
  s.grid = (int)(groups < num_cus ? groups : num_cus);
  return s;
}

int launch_rollout_policy_f32(int system, const KArgs& a, const PArgs& p, const PolShape& grid,
                              void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3: return launch_pol_f32<SysL3<float>, true>(a, p, grid, s);
    case LZ_SYS_LORENZ4: return launch_pol_f32<SysL4<float>, true>(a, p, grid, s);
    case LZ_SYS_PMSM: return launch_pol_f32<SysPMSM, true>(a, p, grid, s);
    case LZ_SYS_HR: return launch_pol_f32<SysHR<float>, true>(a, p, grid, s);
    case LZ_SYS_T1: return launch_pol_f32<SysT1<float>>(a, p, grid, s);
    case LZ_SYS_T2: return launch_pol_f32<SysT2<float>>(a, p, grid, s);
    case LZ_SYS_TP: return launch_pol_f32<SysTP<float>>(a, p, grid, s);
    case LZ_SYS_SC: return launch_pol_f32<SysSC<float>>(a, p, grid, s);
  }
  return (int)hipErrorInvalidValue;
}

template <class Sys>
static int launch_step_f32(const KArgs& a, const PArgs& p, const PStepArgs& st, const PolShape& sh,
                           hipStream_t s) {
  if (sh.waves == 4)
    hipLaunchKernelGGL((k_policy_step_f32<Sys, 4>), dim3((unsigned)sh.grid), dim3(4 * 64), 0, s, a, p, st);
  else
    hipLaunchKernelGGL((k_policy_step_f32<Sys, 8>), dim3((unsigned)sh.grid), dim3(8 * 64), 0, s, a, p, st);
  return (int)hipGetLastError();
}

int launch_policy_step_f32(int system, const KArgs& a, const PArgs& p, const PStepArgs& st,
                           const PolShape& grid, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3: return launch_step_f32<SysL3<float>>(a, p, st, grid, s);
    case LZ_SYS_LORENZ4: return launch_step_f32<SysL4<float>>(a, p, st, grid, s);
    case LZ_SYS_PMSM: return launch_step_f32<SysPMSM>(a, p, st, grid, s);
    case LZ_SYS_HR: return launch_step_f32<SysHR<float>>(a, p, st, grid, s);
    case LZ_SYS_T1: return launch_step_f32<SysT1<float>>(a, p, st, grid, s);
    case LZ_SYS_T2: return launch_step_f32<SysT2<float>>(a, p, st, grid, s);
    case LZ_SYS_TP: return launch_step_f32<SysTP<float>>(a, p, st, grid, s);
    case LZ_SYS_SC: return launch_step_f32<SysSC<float>>(a, p, st, grid, s);
  }
  return (int)hipErrorInvalidValue;
}

int launch_rollout_policy(int system, const KArgs& a, const PArgs& p, const PolShape& grid,
                          void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3: return launch_pol<SysL3<float>>(a, p, grid, s);
    case LZ_SYS_LORENZ4: return launch_pol<SysL4<float>>(a, p, grid, s);
    case LZ_SYS_PMSM: return launch_pol<SysPMSM>(a, p, grid, s);
    case LZ_SYS_HR: return launch_pol<SysHR<float>>(a, p, grid, s);
    case LZ_SYS_T1: return launch_pol<SysT1<float>>(a, p, grid, s);
    case LZ_SYS_T2: return launch_pol<SysT2<float>>(a, p, grid, s);
    case LZ_SYS_TP: return launch_pol<SysTP<float>>(a, p, grid, s);
    case LZ_SYS_SC: return launch_pol<SysSC<float>>(a, p, grid, s);
  }
  return (int)hipErrorInvalidValue;
}

// waves of 16 envs, one workgroup per CU (the LDS holds one): 8 (two per SIMD, 256
// registers) for both extractors -- the LayerNorm variant ran 4 (one per SIMD, 512
// registers) until its frame stack was distributed over the lane groups; then 8 waves
// measured 5.96e8 vs 4.50e8 env-steps/s at HR 32,768 x 2048 (profiles/r03/attn_f32) with
// 20 spilled VGPRs; LZ_ATTN_F32_WAVES=4|8 forces
PolShape attn_f32_policy_shape(int64_t n, int num_cus, int ln) {
  static const int forced = [] {
    const char* e = std::getenv("LZ_ATTN_F32_WAVES");
    const int w = e ? std::atoi(e) : 0;
    return w == 4 || w == 8 ? w : 0;
  }();
  (void)ln;
  PolShape s = {16, forced ? forced : 8, 0, 0};
  const int64_t groups = ((n + 15) / 16 + s.waves - 1) / s.waves;
  s.grid = (int)(groups < num_cus ? groups : num_cus);
  return s;
}

PolShape attn_policy_shape(int64_t n, int num_cus) {
  PolShape s = {32, 4, 3, 0};
  const int64_t groups = ((n + 31) / 32 + 3) / 4;
  s.grid = (int)(groups < num_cus ? groups : num_cus);
  return s;
}

template <class Sys>
static int launch_pol_attn(const KArgs& a, const PArgs& p, const PolShape& sh, hipStream_t s) {
  hipLaunchKernelGGL((k_rollout_policy<Sys, 4, 32, kAttn>), dim3((unsigned)sh.grid), dim3(4 * 64), 0, s,
                     a, p);
  return (int)hipGetLastError();
}

int launch_rollout_policy_attn(int system, const KArgs& a, const PArgs& p, const PolShape& grid,
                               void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3: return launch_pol_attn<SysL3<float>>(a, p, grid, s);
    case LZ_SYS_LORENZ4: return launch_pol_attn<SysL4<float>>(a, p, grid, s);
    case LZ_SYS_PMSM: return launch_pol_attn<SysPMSM>(a, p, grid, s);
    case LZ_SYS_HR: return launch_pol_attn<SysHR<float>>(a, p, grid, s);
    case LZ_SYS_T1: return launch_pol_attn<SysT1<float>>(a, p, grid, s);
    case LZ_SYS_T2: return launch_pol_attn<SysT2<float>>(a, p, grid, s);
    case LZ_SYS_TP: return launch_pol_attn<SysTP<float>>(a, p, grid, s);
    case LZ_SYS_SC: return launch_pol_attn<SysSC<float>>(a, p, grid, s);
  }
  return (int)hipErrorInvalidValue;
}

template <class Sys>
static int launch_pol_attn_ln(int n_stack, const KArgs& a, const PArgs& p, const PolShape& sh,
                              hipStream_t s) {
  const dim3 grid((unsigned)sh.grid), block(4 * 64);
  if (n_stack == 4) hipLaunchKernelGGL((k_rollout_policy<Sys, 4, 32, kAttnLn, 4>), grid, block, 0, s, a, p);
  else if (n_stack == 1) hipLaunchKernelGGL((k_rollout_policy<Sys, 4, 32, kAttnLn, 1>), grid, block, 0, s, a, p);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

template <class Sys>
static int launch_pol_attn_f32(int ln, int n_stack, const KArgs& a, const PArgs& p, const PolShape& sh,
                               hipStream_t s) {
  const dim3 grid((unsigned)sh.grid), block(sh.waves * 64);
  const bool i8 = (p.pflags & LZ_POLICY_I8X4) != 0;
#define LZ_ATTN_F32(LN, S_)                                                                        \
  if (i8) {                                                                                        \
    if (sh.waves == 8) hipLaunchKernelGGL((k_rollout_policy_attn_f32<Sys, LN, S_, 8, true>), grid, block, 0, s, a, p); \
    else hipLaunchKernelGGL((k_rollout_policy_attn_f32<Sys, LN, S_, 4, true>), grid, block, 0, s, a, p); \
  } else if (sh.waves == 8) hipLaunchKernelGGL((k_rollout_policy_attn_f32<Sys, LN, S_, 8>), grid, block, 0, s, a, p); \
  else hipLaunchKernelGGL((k_rollout_policy_attn_f32<Sys, LN, S_, 4>), grid, block, 0, s, a, p);
  if (!ln) { LZ_ATTN_F32(false, 1) }
  else if (n_stack == 4) { LZ_ATTN_F32(true, 4) }
  else if (n_stack == 1) { LZ_ATTN_F32(true, 1) }
  else return (int)hipErrorInvalidValue;
#undef LZ_ATTN_F32
  return (int)hipGetLastError();
}

int launch_rollout_policy_attn_f32(int system, int ln, int n_stack, const KArgs& a, const PArgs& p,
                                   const PolShape& grid, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {  // code/train.py's learner is HR; lorenz_filter's is HR on VecFrameStack(4)
    case LZ_SYS_LORENZ3: return launch_pol_attn_f32<SysL3<float>>(ln, n_stack, a, p, grid, s);
    case LZ_SYS_PMSM: return launch_pol_attn_f32<SysPMSM>(ln, n_stack, a, p, grid, s);
    case LZ_SYS_HR: return launch_pol_attn_f32<SysHR<float>>(ln, n_stack, a, p, grid, s);
  }
  return (int)hipErrorInvalidValue;
}

int launch_rollout_policy_attn_ln(int system, int n_stack, const KArgs& a, const PArgs& p,
                                  const PolShape& grid, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {  // the reference's frame-stacked learner is HR (lorenz_filter/train.py)
    case LZ_SYS_LORENZ3: return launch_pol_attn_ln<SysL3<float>>(n_stack, a, p, grid, s);
    case LZ_SYS_PMSM: return launch_pol_attn_ln<SysPMSM>(n_stack, a, p, grid, s);
    case LZ_SYS_HR: return launch_pol_attn_ln<SysHR<float>>(n_stack, a, p, grid, s);
  }
  return (int)hipErrorInvalidValue;
}

int launch_policy_moments_final(const double* partials, int nparts, int width, double count,
                                double* out, void* stream) {
  hipLaunchKernelGGL(k_pol_moments_final, dim3((unsigned)width), dim3(256), 0, static_cast<hipStream_t>(stream),
                     partials, nparts, width, count, out);
  return (int)hipGetLastError();
}

}  // namespace lz

// ------------------------------------------------------------------ GAE / episode starts
extern "C" {

lz_status lz_gae(int64_t n, int32_t K, const float* rew, const float* values, const uint8_t* done,
                 const float* last_values, double gamma, double gae_lambda, float* advantages,
                 float* returns, int32_t device, void* stream) {
  if (!rew || !values || !done || !last_values || !advantages || !returns)
    return lz::set_error(LZ_ERR_INVALID, "NULL buffer");
  if (n < 0 || K < 1) return lz::set_error(LZ_ERR_INVALID, "n >= 0 and K >= 1 required");
  if (n == 0) return LZ_OK;
  if (hipSetDevice(device) != hipSuccess) return lz::set_error(LZ_ERR_HIP, "hipSetDevice failed");
  // NumPy: python-float gamma * float32 array -> float32(gamma); gamma * gae_lambda is a
  // python-float product rounded once to float32
  // below 4,096 one-wave groups the batch is latency-bound: double-buffered loads
  auto kern = n < 262144 ? lz::k_gae<4, true> : lz::k_gae<8, false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)((n + lz::kGaeBlock - 1) / lz::kGaeBlock)),
                     dim3(lz::kGaeBlock), 0,
                     static_cast<hipStream_t>(stream), n, K, rew, values, done, last_values,
                     (float)gamma, (float)(gamma * gae_lambda), advantages, returns);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lz::set_error(LZ_ERR_HIP, hipGetErrorString(e));
  return LZ_OK;
}

lz_status lz_episode_starts(int64_t n, int32_t K, const uint8_t* done, const float* last_in,
                            float* starts, float* last_out, int32_t device, void* stream) {
  if (!done || !last_in || !starts || !last_out) return lz::set_error(LZ_ERR_INVALID, "NULL buffer");
  if (n < 0 || K < 1) return lz::set_error(LZ_ERR_INVALID, "n >= 0 and K >= 1 required");
  if (last_in == last_out) return lz::set_error(LZ_ERR_INVALID, "last_in and last_out must not alias");
  if (n == 0) return LZ_OK;
  if (hipSetDevice(device) != hipSuccess) return lz::set_error(LZ_ERR_HIP, "hipSetDevice failed");
  const int64_t total = (int64_t)K * n;
  const int64_t want = (total + 255) / 256;
  const unsigned grid = (unsigned)(want < 8192 ? want : 8192);  // grid-stride beyond 2M
  hipLaunchKernelGGL(lz::k_episode_starts, dim3(grid), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, K, done, last_in, starts, last_out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lz::set_error(LZ_ERR_HIP, hipGetErrorString(e));
  return LZ_OK;
}

}  // extern "C"
