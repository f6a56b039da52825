/*
 * sac_fused.h — C ABI of the fused SAC update kernels (gfx950), libsacfused.so.
 *
 * Replaces the per-op PyTorch graph of one SACTrainer.train_from_torch call
 * (ast_sac/torch/sac/sac.py:102-154 compute_loss + train_from_torch, :156-166 soft update,
 * torch.optim.Adam for log_alpha / policy / qf1 / qf2) for the runner's networks:
 *   policy  TanhGaussianPolicy(obs_dim -> H -> H -> (mean, log_std)), act_dim = 1
 *   qf1/qf2 ConcatMlp(obs_dim + 1 -> H -> H -> 1), targets likewise
 * as batched fp32 GEMMs on the matrix cores (v_mfma_f32_32x32x2_f32):
 *   sacf_grads : three dependent launches per grad step — the forward pass (batch gather/sampling,
 *                actor on obs / next_obs, critics on the (obs, a) rows); the critics on (obs, ã) with
 *                the forward-mode tangent of Q along the action, the target critics, and the backward
 *                factors of layer 2; the weight-gradient kernel (flat fp32 gradient of
 *                [log_alpha | policy | qf1 | qf2], losses, d log α). With world_size == 1 that kernel
 *                also applies Adam (torch.optim.Adam semantics, betas/eps as configured), the soft
 *                target update and the refresh of the library's transposed weight copies.
 *   sacf_apply : world_size > 1 or split_update only (a no-op otherwise): the same update as a fourth
 *                launch, after the caller all-reduced the flat gradient; the gradient is divided by
 *                world_size.
 *
 * Memory: the caller owns the flat buffers (torch tensors) bound with sacf_bind; the library owns
 * its scratch (per-row activations, ≈10·B·H floats) and transposed copies of the H×H weights.
 * Flat layout (fp32, torch parameter order and (out, in) row-major weights):
 *   params : [log_alpha] policy{fc0.w (H×O), fc0.b (H), fc1.w (H×H), fc1.b (H), last_fc.w (H),
 *            last_fc.b (1), last_fc_log_std.w (H), last_fc_log_std.b (1)}
 *            qf1{fc0.w (H×(O+1)), fc0.b, fc1.w (H×H), fc1.b, last_fc.w (H), last_fc.b (1)} qf2{…}
 *   targets: target_qf1{…} target_qf2{…}  (same layout as the qf part)
 * Conventions: 0 = success, negative SACF_E* otherwise; asynchronous on the handle's stream;
 * a handle is not thread-safe.
 */
#ifndef SAC_FUSED_H
#define SAC_FUSED_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SACF_ABI_VERSION 4 /* 4: SACF_CHAIN_NO_GRADS; 3: sacf_grads_chain (steps in a chain stage the next batch); 2: three-pass step */
#define SACF_OK 0
#define SACF_EINVAL -1
#define SACF_EHIP -2
#define SACF_ESTATE -3
#define SACF_MAX_OBS 16
#define SACF_MAX_HIDDEN 512 /* hidden: any multiple of 32 up to 256, or 320 / 384 / 448 / 512 */
#define SACF_MAX_BATCH 8192 /* per-rank batch bound (any size 1..8192; rows padded to a multiple of 32) */

typedef struct sacf_config {
  int32_t abi_version;   /* = SACF_ABI_VERSION */
  int32_t obs_dim;       /* <= SACF_MAX_OBS (8 for the AST env) */
  int32_t hidden;        /* H: see SACF_MAX_HIDDEN and sacf_hidden_supported (runner: 256) */
  int32_t batch;         /* B per call (per rank), 1 ..= SACF_MAX_BATCH */
  float discount;        /* sac.py:31  γ */
  float reward_scale;    /* sac.py:32 */
  float soft_target_tau; /* sac.py:37  τ */
  float action_reg_coeff;/* runner: 0.01 (0 disables) */
  float clip_val;        /* q-target clamp (runner: 100; +inf disables) */
  float target_entropy;  /* sac.py:62-64: −|A| */
  float policy_lr;       /* lr of log_alpha and the policy */
  float qf_lr;
  float beta1, beta2, adam_eps; /* torch.optim.Adam defaults 0.9, 0.999, 1e-8 */
  int32_t auto_entropy;  /* use_automatic_entropy_tuning */
  int32_t world_size;    /* gradient is divided by this in sacf_apply */
  int32_t split_update;  /* 1: keep the update out of sacf_grads even with world_size 1 (the data-parallel
                            call pattern grads | all-reduce | apply on one rank); 0: fused when world_size 1 */
  int32_t reserved[5];   /* must be 0 */
} sacf_config;

typedef struct sacf_handle sacf_handle;

int32_t sacf_abi_version(void);
/* "sacfused gfx950 HIP src <hash>": the content hash of the sources this library was built from */
const char* sacf_build_info(void);
/* 1 if kernels for this hidden width are compiled in, else 0 */
int sacf_hidden_supported(int32_t hidden);
int sacf_create(const sacf_config* cfg, int device, void* stream, sacf_handle** out);
int sacf_destroy(sacf_handle* h);
const char* sacf_last_error(const sacf_handle* h);
/* launches go to this stream from now on (e.g. torch's current / capturing stream) */
int sacf_set_stream(sacf_handle* h, void* stream);
/* element counts of the flat params / targets buffers */
int64_t sacf_param_count(const sacf_handle* h);
int64_t sacf_target_count(const sacf_handle* h);
/* stats buffer: [policy_loss, qf1_loss, qf2_loss, alpha_loss, alpha, Adam step sizes (pi, q) and
 * sqrt(1 - beta2^t) of this step] then per row
 * q1_pred[B], q2_pred[B], q_target[B], log_pi[B], tanh(mean)[B], std[B] */
int64_t sacf_stats_count(const sacf_handle* h);
/* Bind caller-owned device buffers (params/targets/grads/adam_m/adam_v: param or target count
 * floats; step: one int64 = number of completed updates, read by Adam bias correction and the RNG). */
int sacf_bind(sacf_handle* h, float* params, float* targets, float* grads, float* adam_m, float* adam_v,
              int64_t* step, float* stats);
/* Re-derive the library's transposed weight copies after params/targets changed outside the library. */
int sacf_sync_params(sacf_handle* h);
/* Replay ring (DeviceReplayBuffer storage, float32 rows) sampled uniformly with replacement. */
int sacf_set_replay(sacf_handle* h, const float* obs, const float* act, const float* rew, const float* term,
                    const float* next_obs, const int64_t* size_dev, int64_t capacity, uint64_t seed);
/* Gradient of one update into `grads` (and step += 1); with world_size == 1 and no split_update also the
 * update itself
 * (grads keeps the gradient for inspection). With obs == NULL the batch is sampled from
 * the replay ring; with eps == NULL the 2·B reparameterisation normals come from the in-kernel
 * Philox stream, else eps = [B normals for obs rows | B normals for next_obs rows]. */
int sacf_grads(sacf_handle* h, const float* obs, const float* act, const float* rew, const float* term,
               const float* next_obs, const float* eps);
/* A step of a chain of replay-sampled steps (the trainer's multi-step graph; no replay change between the steps):
 * sacf_grads(h, NULL x 5, eps) with `flags`:
 *   SACF_CHAIN_STAGE_NEXT   the weight-gradient pass also gathers the NEXT step's batch (its Philox row draw, the
 *                           replay rows, the reparameterisation normals) into library buffers;
 *   SACF_CHAIN_FROM_STAGED  the forward pass starts from the batch the previous call staged instead of gathering
 *                           it (the same rows and normals: results are bitwise those of sacf_grads). Only right
 *                           after a call with SACF_CHAIN_STAGE_NEXT on this handle (SACF_ESTATE otherwise), and
 *                           the caller guarantees the replay ring and its size did not change in between.
 * A replay ring must be bound (sacf_set_replay). With either staging flag eps must be NULL (the normals then come from the
 * in-kernel Philox stream, and a staged batch carries the ones of the call that staged it): SACF_EINVAL otherwise.
 *   SACF_CHAIN_NO_GRADS     with the update applied in the same call (world_size == 1, no split_update): the step
 *                           does not write `grads` (it keeps its previous contents; the update, the parameters,
 *                           targets and Adam state are bitwise those of the step without the flag). The trainer's
 *                           multi-step graph sets it on every step but its last, whose gradient stays inspectable.
 *                           Ignored when the update is a separate sacf_apply (which reads `grads`).
 * flags == 0 is sacf_grads(h, NULL x 5, eps). */
#define SACF_CHAIN_STAGE_NEXT 1
#define SACF_CHAIN_FROM_STAGED 2
#define SACF_CHAIN_NO_GRADS 4
int sacf_grads_chain(sacf_handle* h, const float* eps, int32_t flags);
/* Adam + soft target update from `grads` (divided by world_size); a no-op when sacf_grads applied it. */
int sacf_apply(sacf_handle* h);

/* Collector actions from the CURRENT policy parameters (the bound params and the library's W2ᵀ copy):
 * TanhGaussianPolicy.forward + TanhNormal.sample (gaussian_policy.py:105-118, distributions.py:394-425)
 * for n rows obs[i * obs_stride + 0..obs_dim), act[i] = tanh(mean + std·ε) with ε ~ N(0, 1) from
 * Philox(seed, *counter, i) (the caller advances *counter between calls), or tanh(mean) with
 * deterministic != 0 (MakeDeterministic). Rows with mask[i] == 0 keep act[i] (mask may be NULL).
 * eps_out (NULL or n floats) receives ε. Two launches on the handle's stream; graph-capturable once
 * sacf_policy_reserve(h, >= n) has sized the scratch (outside the capture). */
int sacf_policy_reserve(sacf_handle* h, int64_t n);
int sacf_policy_act(sacf_handle* h, const float* obs, int64_t n, int32_t obs_stride, const uint8_t* mask,
                    int32_t deterministic, uint64_t seed, const int64_t* counter, float* act, float* eps_out);
/* The policy's device parameters (torch order, at the bound params) and the library's current W2ᵀ copy,
 * with obs_dim and hidden: what shipsim_run_policy reads (each output may be NULL). */
int sacf_policy_weights(const sacf_handle* h, const float** params, const float** w2t, int32_t* obs_dim,
                        int32_t* hidden);

#ifdef __cplusplus
}
#endif
#endif
