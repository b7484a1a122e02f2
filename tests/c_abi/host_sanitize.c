/* The library's host-side C-ABI code (argument validation, config defaults, the policy
 * packer's index maps, error paths) under AddressSanitizer + UndefinedBehaviorSanitizer,
 * without a GPU: every buffer is heap-allocated to its exact documented size, so an
 * out-of-bounds read/write in lz_policy_pack or a validation path aborts with a report.
 * Built by tests/test_sanitizers.py with hipcc -Xarch_host -fsanitize=... over the
 * library sources (device code compiled as usual, never launched here). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lorenz_env.h"

static float* w(size_t count, float scale) {
  float* p = malloc(count * sizeof(float));
  for (size_t i = 0; i < count; ++i) p[i] = scale * (float)((int)(i % 13) - 6);
  return p;
}

int main(void) {
  if (lz_abi_version() != LZ_ABI_VERSION) return 1;
  lz_config cfg;
  for (int s = LZ_SYS_LORENZ3; s <= LZ_SYS_SC; ++s)
    if (lz_config_init(&cfg, s) != LZ_OK) return 2;
  if (lz_config_init(&cfg, 99) != LZ_ERR_INVALID || lz_config_init(NULL, 0) != LZ_ERR_INVALID) return 3;
  /* no GPU here: creation fails cleanly with a message */
  lz_config_init(&cfg, LZ_SYS_LORENZ3);
  lz_handle* h = NULL;
  if (lz_create(&cfg, &h) == LZ_OK || h != NULL || strlen(lz_last_error()) == 0) return 4;
  cfg.num_envs = 0;
  if (lz_create(&cfg, &h) != LZ_ERR_INVALID) return 5;
  if (lz_step(NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL) != LZ_ERR_INVALID) return 6;
  if (lz_rollout_policy(NULL, NULL) != LZ_ERR_INVALID) return 7;
  if (lz_step_host(NULL, NULL, NULL, NULL, NULL, NULL) != LZ_ERR_INVALID) return 20;
  if (lz_gae(10, 2, NULL, NULL, NULL, NULL, 0.99, 0.95, NULL, NULL, 0, NULL) != LZ_ERR_INVALID) return 8;
  if (lz_frame_stack(NULL, NULL, NULL, 1, 4, 6, 0, 0, NULL) != LZ_ERR_INVALID) return 9;
  lz_rms* r = NULL;
  if (lz_rms_create(6, 0, 1e-4, &r) == LZ_OK) return 10;
  /* the packer, every supported shape, exact-size inputs and output */
  const int64_t bytes = lz_policy_blob_bytes();
  for (int O = 1; O <= 8; ++O)
    for (int A = 1; A <= 4; ++A) {
      const int H = LZ_POLICY_HIDDEN;
      lz_mlp_policy p;
      p.obs_dim = O;
      p.act_dim = A;
      p.pi_w1 = w((size_t)H * O, 0.1f); p.pi_b1 = w(H, 0.01f);
      p.pi_w2 = w((size_t)H * H, 0.05f); p.pi_b2 = w(H, 0.01f);
      p.vf_w1 = w((size_t)H * O, 0.1f); p.vf_b1 = w(H, 0.01f);
      p.vf_w2 = w((size_t)H * H, 0.05f); p.vf_b2 = w(H, 0.01f);
      p.act_w = w((size_t)A * H, 0.02f); p.act_b = w(A, 0.01f);
      p.val_w = w(H, 0.02f); p.val_b = w(1, 0.01f);
      p.log_std = w(A, 0.1f);
      void* blob = malloc((size_t)bytes);
      if (lz_policy_pack(&p, blob, bytes) != LZ_OK) return 11;
      if (lz_policy_pack(&p, blob, bytes - 1) != LZ_ERR_INVALID) return 12;
      free(blob);
      free((void*)p.pi_w1); free((void*)p.pi_b1); free((void*)p.pi_w2); free((void*)p.pi_b2);
      free((void*)p.vf_w1); free((void*)p.vf_b1); free((void*)p.vf_w2); free((void*)p.vf_b2);
      free((void*)p.act_w); free((void*)p.act_b); free((void*)p.val_w); free((void*)p.val_b);
      free((void*)p.log_std);
    }
  /* the attention-extractor packer (code/train.py's policy), every supported shape */
  const int64_t abytes = lz_attn_policy_blob_bytes();
  for (int O = 1; O <= 8; ++O)
    for (int A = 1; A <= 4; ++A) {
      const int H = LZ_POLICY_HIDDEN, F = 64;
      lz_attn_policy p;
      p.obs_dim = O;
      p.act_dim = A;
      p.fc1_w = w((size_t)H * O, 0.1f); p.fc1_b = w(H, 0.01f);
      p.in_proj_w = w(48 * 16, 0.1f); p.in_proj_b = w(48, 0.01f);
      p.out_proj_w = w(16 * 16, 0.1f); p.out_proj_b = w(16, 0.01f);
      p.post_w = w((size_t)F * H, 0.05f); p.post_b = w(F, 0.01f);
      p.pi_w1 = w((size_t)H * F, 0.1f); p.pi_b1 = w(H, 0.01f);
      p.pi_w2 = w((size_t)H * H, 0.05f); p.pi_b2 = w(H, 0.01f);
      p.vf_w1 = w((size_t)H * F, 0.1f); p.vf_b1 = w(H, 0.01f);
      p.vf_w2 = w((size_t)H * H, 0.05f); p.vf_b2 = w(H, 0.01f);
      p.act_w = w((size_t)A * H, 0.02f); p.act_b = w(A, 0.01f);
      p.val_w = w(H, 0.02f); p.val_b = w(1, 0.01f);
      p.log_std = w(A, 0.1f);
      void* blob = malloc((size_t)abytes);
      if (lz_attn_policy_pack(&p, blob, abytes) != LZ_OK) return 14;
      if (lz_attn_policy_pack(&p, blob, abytes - 1) != LZ_ERR_INVALID) return 15;
      free(blob);
      const float* all[] = {p.fc1_w, p.fc1_b, p.in_proj_w, p.in_proj_b, p.out_proj_w,
                            p.out_proj_b, p.post_w, p.post_b, p.pi_w1, p.pi_b1, p.pi_w2,
                            p.pi_b2, p.vf_w1, p.vf_b1, p.vf_w2, p.vf_b2, p.act_w, p.act_b,
                            p.val_w, p.val_b, p.log_std};
      for (size_t i = 0; i < sizeof all / sizeof all[0]; ++i) free((void*)all[i]);
    }
  if (lz_rollout_policy_attn(NULL, NULL) != LZ_ERR_INVALID) return 16;
  /* the residual + LayerNorm packer (code/lorenz_filter/train.py), input dims 1..32 */
  const int64_t lbytes = lz_attn_ln_policy_blob_bytes();
  for (int I = 1; I <= 32; I += 3)
    for (int A = 1; A <= 4; A += 3) {
      const int H = LZ_POLICY_HIDDEN, F = 64;
      lz_attn_ln_policy q;
      lz_attn_policy* p = &q.attn;
      p->obs_dim = I;
      p->act_dim = A;
      p->fc1_w = w((size_t)H * I, 0.1f); p->fc1_b = w(H, 0.01f);
      p->in_proj_w = w(48 * 16, 0.1f); p->in_proj_b = w(48, 0.01f);
      p->out_proj_w = w(16 * 16, 0.1f); p->out_proj_b = w(16, 0.01f);
      p->post_w = w((size_t)F * H, 0.05f); p->post_b = w(F, 0.01f);
      p->pi_w1 = w((size_t)H * F, 0.1f); p->pi_b1 = w(H, 0.01f);
      p->pi_w2 = w((size_t)H * H, 0.05f); p->pi_b2 = w(H, 0.01f);
      p->vf_w1 = w((size_t)H * F, 0.1f); p->vf_b1 = w(H, 0.01f);
      p->vf_w2 = w((size_t)H * H, 0.05f); p->vf_b2 = w(H, 0.01f);
      p->act_w = w((size_t)A * H, 0.02f); p->act_b = w(A, 0.01f);
      p->val_w = w(H, 0.02f); p->val_b = w(1, 0.01f);
      p->log_std = w(A, 0.1f);
      q.ln_w = w(16, 0.1f); q.ln_b = w(16, 0.01f);
      void* blob = malloc((size_t)lbytes);
      if (lz_attn_ln_policy_pack(&q, blob, lbytes) != LZ_OK) return 17;
      if (lz_attn_ln_policy_pack(&q, blob, lbytes - 1) != LZ_ERR_INVALID) return 18;
      free(blob);
      const float* all[] = {p->fc1_w, p->fc1_b, p->in_proj_w, p->in_proj_b, p->out_proj_w,
                            p->out_proj_b, p->post_w, p->post_b, p->pi_w1, p->pi_b1, p->pi_w2,
                            p->pi_b2, p->vf_w1, p->vf_b1, p->vf_w2, p->vf_b2, p->act_w, p->act_b,
                            p->val_w, p->val_b, p->log_std, q.ln_w, q.ln_b};
      for (size_t i = 0; i < sizeof all / sizeof all[0]; ++i) free((void*)all[i]);
    }
  if (lz_rollout_policy_attn_stack(NULL, NULL, 4, NULL, NULL) != LZ_ERR_INVALID) return 19;
  lz_mlp_policy bad;
  memset(&bad, 0, sizeof bad);
  bad.obs_dim = 9;
  bad.act_dim = 2;
  char tiny[8];
  if (lz_policy_pack(&bad, tiny, sizeof tiny) == LZ_OK) return 13;
  printf("host ABI: clean under ASan + UBSan\n");
  return 0;
}
