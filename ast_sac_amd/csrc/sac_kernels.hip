// sac_kernels.hip — fused SAC update for gfx950 (C ABI: include/sac_fused.h) -> libsacfused.so
//
// One grad step of ast_sac/torch/sac/sac.py (compute_loss :156-270, train_from_torch :102-154,
// update_target_networks :160-166) for TanhGaussianPolicy + twin ConcatMlp critics with two hidden
// layers of width H and act_dim 1, in three kernels:
//
//   sac_rows_g4_kernel: one batch row per block (default; sac_rows_kernel<RR, KS> is the general
//                      shape). Gathers the batch (or samples it from the replay ring with Philox),
//                      runs actor(obs), actor(next_obs), Q1/Q2 on (obs, ã) and (obs, a), target
//                      Q1/Q2 on (next_obs, ã'), the per-row losses, and the whole per-row backward.
//                      Everything in one SAC update is row-local except the batch means, whose 1/B
//                      factors are constants, so no grid-wide step is needed until the weight
//                      gradients. Bound: every block streams 8 H x H fp32 matrices (2 MB at H = 256)
//                      from L2; scripts/mb_weight_read.hip measures that alone at ≈19 µs on MI355X.
//   sac_wgrad_kernel : every weight/bias gradient = Σ_rows dY[r]ᵀ X[r] (64×64 tiles, 4×4 per thread,
//                      LDS-staged row chunks, rows split kParts ways into partial gradients) + the loss
//                      scalars, d(log α) and this step's Adam bias corrections.
//   sac_gsum_kernel  : (data parallel only) Σ of the partials into the flat gradient before the all-reduce.
//   sac_apply_kernel : Σ partials (single process), torch.optim.Adam on every element (two lr groups),
//                      soft target update θ' ← θ'(1−τ) + θτ, and the transposed H×H copies the rows
//                      kernel reads (32×32 tiles through LDS).
//
// Only the four gradients the reference keeps are formed: the π-loss gradient w.r.t. the critics
// (which sac.py:123-133 discards with qf*_optimizer.zero_grad()) is never computed; α is treated as a
// constant inside the π- and Q-losses exactly as after alpha_optimizer.step() in the reference
// (its grad there is also discarded).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "sac_fused.h"

namespace {

constexpr int kThreads = 256;

#ifdef SACF_PHASE_TIMING
// timing build only: shader-clock stamps of block 0 at the phase boundaries of sac_rows_g4_kernel
__device__ unsigned long long g_sac_stamp[16];
#define SAC_MARK(k)                                                              \
  do {                                                                           \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_sac_stamp[k] = clock64();         \
  } while (0)
#else
#define SAC_MARK(k) \
  do {              \
  } while (0)
#endif
constexpr int R = 4;           // batch granularity: B must be a multiple of R (rows-kernel tiles)
constexpr int kXLd = 16;       // leading dim of the per-row input scratch (obs | act)
constexpr float kLog2 = 0.69314718055994530942f;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;

struct Layout {
  int O, H, B;
  int64_t p_w1, p_b1, p_w2, p_b2, p_wm, p_bm, p_ws, p_bs;  // policy (params)
  int64_t q_base[2];                                      // start of qf1 / qf2 in params
  int64_t q_size;                                         // floats of one critic
  // offsets inside one critic block
  int64_t c_w1, c_b1, c_w2, c_b2, c_w3, c_b3;
  int64_t n_params, n_targets;
};

struct Scratch {
  float *a_x, *a_h1, *a_h2, *a_dh1, *a_dh2, *a_dhead;  // actor, obs rows [B][..]
  float *q_x[2], *q_g1[2], *q_g2[2], *q_dg1[2], *q_dg2[2], *q_dq[2];  // critics, (obs, a) rows
  float *p_pl, *p_q1l, *p_q2l, *p_la, *p_ga;  // per-row loss partials
};

struct Hyper {
  float gamma, rscale, tau, areg, clip, tent, lr_pi, lr_q, beta1, beta2, eps;
  int auto_ent;
  float inv_world;
};

struct RowsArgs {
  const float* params;
  const float* targets;
  const float* T;  // transposed copies: [actor W2ᵀ | q1 W2ᵀ | q2 W2ᵀ | t1 W2ᵀ | t2 W2ᵀ], each H×H
  const float *obs, *act, *rew, *term, *nobs;
  const int64_t* size_dev;
  int64_t capacity;
  uint64_t seed;
  int sampled;
  const float* eps;
  const int64_t* step;
  float* stats;
  Scratch sc;
  Layout L;
  Hyper hp;
};

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based; one 4-word draw per batch row and step)
// ---------------------------------------------------------------------------------------------
__device__ inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// block-wide sum of n (<= 32) per-thread partials; result in out[0..n) (LDS), visible after return
template <int N>
__device__ inline void block_sum(float (&v)[N], float (*red)[32], float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float x = v[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (lane == 0) red[wave][i] = x;
  }
  __syncthreads();
  if ((int)threadIdx.x < N) out[threadIdx.x] = (red[0][threadIdx.x] + red[1][threadIdx.x]) +
                                                (red[2][threadIdx.x] + red[3][threadIdx.x]);
  __syncthreads();
}

__device__ __forceinline__ float relu(float x) { return fmaxf(x, 0.0f); }
__device__ __forceinline__ float softplus(float x) { return x > 20.0f ? x : log1pf(expf(x)); }

// ---------------------------------------------------------------------------------------------
// rows kernel: RR batch rows per block, KS k-groups of kCols threads (split-K matvecs)
// ---------------------------------------------------------------------------------------------
constexpr int kCols = 256;  // column threads per k-group (>= H)

// acc[i] += Σ_{k in this k-group's slice} WT[k*H + j] · in[i][k]. With W row-major (out, in) the
// same indexing computes the backward product Σ_jj W[jj][m] · d[i][jj] for column m.
template <int NR, int KS>
__device__ __forceinline__ void mv_part(const float* __restrict__ WT, int H, const float* in, int ld, int j, int kg,
                                        float (&acc)[NR]) {
  const int len = H / KS, k0 = kg * len, k1 = k0 + len;
#pragma unroll 2
  for (int k = k0; k < k1; k += 8) {
    float w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = WT[(size_t)(k + u) * H + j];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const float4 x0 = *reinterpret_cast<const float4*>(in + i * ld + k);
      const float4 x1 = *reinterpret_cast<const float4*>(in + i * ld + k + 4);
      acc[i] = fmaf(w[0], x0.x, acc[i]);
      acc[i] = fmaf(w[1], x0.y, acc[i]);
      acc[i] = fmaf(w[2], x0.z, acc[i]);
      acc[i] = fmaf(w[3], x0.w, acc[i]);
      acc[i] = fmaf(w[4], x1.x, acc[i]);
      acc[i] = fmaf(w[5], x1.y, acc[i]);
      acc[i] = fmaf(w[6], x1.z, acc[i]);
      acc[i] = fmaf(w[7], x1.w, acc[i]);
    }
  }
}

// sum the k-groups' partials into the kg == 0 threads (every thread of the block must call this)
template <int NR, int KS>
__device__ __forceinline__ void kreduce(float (&acc)[NR], float* part, int j, int kg) {
  if (KS == 1) return;
  if (kg > 0)
#pragma unroll
    for (int i = 0; i < NR; ++i) part[((kg - 1) * NR + i) * kCols + j] = acc[i];
  __syncthreads();
  if (kg == 0)
    for (int g = 1; g < KS; ++g)
#pragma unroll
      for (int i = 0; i < NR; ++i) acc[i] += part[((g - 1) * NR + i) * kCols + j];
  __syncthreads();
}

// block-wide sum over NW waves of N (<= 32) per-thread partials -> out[0..N)
template <int N, int NW>
__device__ inline void block_sum_w(float (&v)[N], float (*red)[32], float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float x = v[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (lane == 0) red[wave][i] = x;
  }
  __syncthreads();
  if ((int)threadIdx.x < N) {
    float t = 0.0f;
    for (int w = 0; w < NW; ++w) t += red[w][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// per-row scalar slots in LDS
enum { S_MEAN, S_LSRAW, S_STD, S_Z, S_A, S_LOGP, S_Q1, S_Q2, S_T1, S_T2, S_DQ1, S_DQ2, S_DMEAN, S_DLS, S_NSLOT };

template <int RR, int KS>
__global__ __launch_bounds__(kCols* KS) void sac_rows_kernel(RowsArgs a) {
  constexpr int NW = kCols * KS / 64;
  const Layout& L = a.L;
  const int H = L.H, O = L.O, B = L.B;
  const int tid = threadIdx.x;
  const int j = tid % kCols, kg = tid / kCols;
  const bool col = j < H;
  const bool lead = kg == 0 && col;  // finalises column j
  const int r0 = blockIdx.x * RR;
  const float* P = a.params;
  const float* TG = a.targets;

  __shared__ float s_x[2 * RR][kXLd];  // actor inputs: obs rows | next_obs rows
  __shared__ float s_act[RR], s_rew[RR], s_term[RR], s_eps[2 * RR];
  __shared__ __attribute__((aligned(16))) float s_h1[2 * RR][SACF_MAX_HIDDEN];
  __shared__ __attribute__((aligned(16))) float s_h2[2 * RR][SACF_MAX_HIDDEN];
  __shared__ __attribute__((aligned(16))) float s_g1[2][2 * RR][SACF_MAX_HIDDEN];  // critic rows: (obs, ã) | (obs, a)
  __shared__ __attribute__((aligned(16))) float s_g2[2][2 * RR][SACF_MAX_HIDDEN];
  __shared__ float s_part[(KS > 1 ? KS - 1 : 1) * 2 * RR * kCols];
  __shared__ float s_red[NW][32];
  __shared__ float s_sum[32];
  __shared__ float s_row[S_NSLOT][2 * RR];

  // ---- batch rows + reparameterisation noise ----
  if (tid < RR) {
    const int r = r0 + tid;
    int64_t idx = r;
    uint32_t c[4] = {(uint32_t)r, (uint32_t)*a.step, (uint32_t)((uint64_t)*a.step >> 32), 0x5AC0u};
    if (a.sampled || !a.eps) philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    if (a.sampled) {
      const int64_t size = *a.size_dev > 0 ? *a.size_dev : 1;
      const double u = ((double)c[0] + 0.5) * (1.0 / 4294967296.0);
      idx = (int64_t)(u * (double)size);
      if (idx >= a.capacity) idx = a.capacity - 1;
    }
    float e0, e1;
    if (a.eps) {
      e0 = a.eps[r];
      e1 = a.eps[B + r];
    } else {  // Box-Muller on two 32-bit uniforms
      const float u1 = ((float)c[1] + 1.0f) * 2.3283064365386963e-10f;
      const float u2 = (float)c[2] * 2.3283064365386963e-10f;
      const float rad = sqrtf(-2.0f * logf(u1));
      e0 = rad * cosf(6.283185307179586f * u2);
      e1 = rad * sinf(6.283185307179586f * u2);
    }
    for (int m = 0; m < O; ++m) {
      s_x[tid][m] = a.obs[idx * O + m];
      s_x[RR + tid][m] = a.nobs[idx * O + m];
    }
    s_act[tid] = a.act[idx];
    s_rew[tid] = a.rew[idx];
    s_term[tid] = a.term[idx];
    s_eps[tid] = e0;
    s_eps[RR + tid] = e1;
  }
  __syncthreads();

  // ---- actor forward on 2RR rows (gaussian_policy.py:105-118) ----
  if (lead) {
    float acc[2 * RR];
    const float b = P[L.p_b1 + j];
#pragma unroll
    for (int i = 0; i < 2 * RR; ++i) acc[i] = b;
    for (int m = 0; m < O; ++m) {
      const float w = P[L.p_w1 + (int64_t)j * O + m];
#pragma unroll
      for (int i = 0; i < 2 * RR; ++i) acc[i] = fmaf(w, s_x[i][m], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 2 * RR; ++i) s_h1[i][j] = relu(acc[i]);
  }
  __syncthreads();
  {
    float acc[2 * RR];
    const float b = lead ? P[L.p_b2 + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2 * RR; ++i) acc[i] = b;
    if (col) mv_part<2 * RR, KS>(a.T, H, &s_h1[0][0], SACF_MAX_HIDDEN, j, kg, acc);
    kreduce<2 * RR, KS>(acc, s_part, j, kg);
    if (lead)
#pragma unroll
      for (int i = 0; i < 2 * RR; ++i) s_h2[i][j] = relu(acc[i]);
  }
  __syncthreads();
  {
    float v[4 * RR];
    const float wm = lead ? P[L.p_wm + j] : 0.0f, ws = lead ? P[L.p_ws + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2 * RR; ++i) {
      const float h = lead ? s_h2[i][j] : 0.0f;
      v[i] = wm * h;
      v[2 * RR + i] = ws * h;
    }
    block_sum_w<4 * RR, NW>(v, s_red, s_sum);
  }
  if (tid < 2 * RR) {  // TanhNormal.rsample_and_logprob (distributions.py:346-392)
    const int i = tid;
    const float mean = s_sum[i] + P[L.p_bm];
    const float ls_raw = s_sum[2 * RR + i] + P[L.p_bs];
    const float log_std = fminf(fmaxf(ls_raw, -20.0f), 2.0f);
    const float std = expf(log_std);
    const float z = mean + std * s_eps[i];
    const float act = tanhf(z);
    const float var = std * std;
    const float d = z - mean;
    const float lp = -(d * d) / (2.0f * var) - logf(std) - kLogSqrt2Pi;
    const float corr = -2.0f * (kLog2 - z - softplus(-2.0f * z));
    s_row[S_MEAN][i] = mean;
    s_row[S_LSRAW][i] = ls_raw;
    s_row[S_STD][i] = std;
    s_row[S_Z][i] = z;
    s_row[S_A][i] = act;
    s_row[S_LOGP][i] = lp + corr;
  }
  __syncthreads();

  // ---- critics on (obs, ã) rows 0..RR-1 and (obs, a) rows RR..2RR-1 ----
  if (lead) {
    for (int k = 0; k < 2; ++k) {
      const float* C = P + L.q_base[k];
      float base[RR];
      const float b = C[L.c_b1 + j];
#pragma unroll
      for (int i = 0; i < RR; ++i) base[i] = b;
      for (int m = 0; m < O; ++m) {
        const float w = C[L.c_w1 + (int64_t)j * (O + 1) + m];
#pragma unroll
        for (int i = 0; i < RR; ++i) base[i] = fmaf(w, s_x[i][m], base[i]);
      }
      const float wa = C[L.c_w1 + (int64_t)j * (O + 1) + O];
#pragma unroll
      for (int i = 0; i < RR; ++i) {
        s_g1[k][i][j] = relu(fmaf(wa, s_row[S_A][i], base[i]));
        s_g1[k][RR + i][j] = relu(fmaf(wa, s_act[i], base[i]));
      }
    }
  }
  __syncthreads();
  for (int k = 0; k < 2; ++k) {
    const float* C = P + L.q_base[k];
    float acc[2 * RR];
    const float b = lead ? C[L.c_b2 + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2 * RR; ++i) acc[i] = b;
    if (col) mv_part<2 * RR, KS>(a.T + (size_t)(1 + k) * H * H, H, &s_g1[k][0][0], SACF_MAX_HIDDEN, j, kg, acc);
    kreduce<2 * RR, KS>(acc, s_part, j, kg);
    if (lead)
#pragma unroll
      for (int i = 0; i < 2 * RR; ++i) s_g2[k][i][j] = relu(acc[i]);
  }
  __syncthreads();
  {
    float v[4 * RR];
    const float w0 = lead ? P[L.q_base[0] + L.c_w3 + j] : 0.0f, w1 = lead ? P[L.q_base[1] + L.c_w3 + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2 * RR; ++i) {
      v[i] = lead ? w0 * s_g2[0][i][j] : 0.0f;
      v[2 * RR + i] = lead ? w1 * s_g2[1][i][j] : 0.0f;
    }
    block_sum_w<4 * RR, NW>(v, s_red, s_sum);
  }
  if (tid < 2 * RR) {
    s_row[S_Q1][tid] = s_sum[tid] + P[L.q_base[0] + L.c_b3];
    s_row[S_Q2][tid] = s_sum[2 * RR + tid] + P[L.q_base[1] + L.c_b3];
  }
  __syncthreads();

  // ---- target critics on (next_obs, ã') (rows RR..2RR-1 of s_h1/s_h2 are free now) ----
  for (int k = 0; k < 2; ++k) {
    const float* C = TG + (int64_t)k * L.q_size;
    if (lead) {
      float acc[RR];
      const float b = C[L.c_b1 + j];
#pragma unroll
      for (int i = 0; i < RR; ++i) acc[i] = b;
      for (int m = 0; m < O; ++m) {
        const float w = C[L.c_w1 + (int64_t)j * (O + 1) + m];
#pragma unroll
        for (int i = 0; i < RR; ++i) acc[i] = fmaf(w, s_x[RR + i][m], acc[i]);
      }
      const float wa = C[L.c_w1 + (int64_t)j * (O + 1) + O];
#pragma unroll
      for (int i = 0; i < RR; ++i) s_h1[RR + i][j] = relu(fmaf(wa, s_row[S_A][RR + i], acc[i]));
    }
    __syncthreads();
    {
      float acc[RR];
      const float b = lead ? C[L.c_b2 + j] : 0.0f;
#pragma unroll
      for (int i = 0; i < RR; ++i) acc[i] = b;
      if (col) mv_part<RR, KS>(a.T + (size_t)(3 + k) * H * H, H, &s_h1[RR][0], SACF_MAX_HIDDEN, j, kg, acc);
      kreduce<RR, KS>(acc, s_part, j, kg);
      if (lead)
#pragma unroll
        for (int i = 0; i < RR; ++i) s_h2[RR + i][j] = relu(acc[i]);
    }
    __syncthreads();
    float v[RR];
    const float w3 = lead ? C[L.c_w3 + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < RR; ++i) v[i] = lead ? w3 * s_h2[RR + i][j] : 0.0f;
    block_sum_w<RR, NW>(v, s_red, s_sum);
    if (tid < RR) s_row[k == 0 ? S_T1 : S_T2][tid] = s_sum[tid] + C[L.c_b3];
    __syncthreads();
  }

  // ---- losses and output gradients per row (sac.py:170-247) ----
  const float log_alpha = P[0];
  const float alpha = a.hp.auto_ent ? expf(log_alpha) : 1.0f;
  const float invB = 1.0f / (float)B;
  if (tid < RR) {
    const int i = tid, r = r0 + i;
    const float q1a = s_row[S_Q1][i], q2a = s_row[S_Q2][i];
    const float q1b = s_row[S_Q1][RR + i], q2b = s_row[S_Q2][RR + i];
    const float tq = fminf(s_row[S_T1][i], s_row[S_T2][i]) - alpha * s_row[S_LOGP][RR + i];
    float qt = a.hp.rscale * s_rew[i] + ((1.0f - s_term[i]) * a.hp.gamma) * tq;
    qt = fminf(fmaxf(qt, -a.hp.clip), a.hp.clip);
    const float qmin = fminf(q1a, q2a);
    // torch.minimum backward: the smaller input takes the gradient, ties split it in half
    const float w1 = (q1a < q2a) ? 1.0f : ((q1a == q2a) ? 0.5f : 0.0f);
    const float w2 = 1.0f - w1;
    s_row[S_DQ1][i] = -w1 * invB;
    s_row[S_DQ2][i] = -w2 * invB;
    const float dq1b = (2.0f * invB) * (q1b - qt), dq2b = (2.0f * invB) * (q2b - qt);
    s_row[S_DQ1][RR + i] = dq1b;
    s_row[S_DQ2][RR + i] = dq2b;
    a.sc.q_dq[0][r] = dq1b;
    a.sc.q_dq[1][r] = dq2b;
    const float logp = s_row[S_LOGP][i], act = s_row[S_A][i];
    a.sc.p_pl[r] = alpha * logp - qmin + (a.hp.areg != 0.0f ? a.hp.areg * (act * act) : 0.0f);
    a.sc.p_q1l[r] = (q1b - qt) * (q1b - qt);
    a.sc.p_q2l[r] = (q2b - qt) * (q2b - qt);
    a.sc.p_la[r] = -(log_alpha * (logp + a.hp.tent));
    a.sc.p_ga[r] = -(logp + a.hp.tent);
    float* st = a.stats + 8;
    st[r] = q1b;
    st[B + r] = q2b;
    st[2 * B + r] = qt;
    st[3 * B + r] = logp;
    st[4 * B + r] = tanhf(s_row[S_MEAN][i]);
    st[5 * B + r] = s_row[S_STD][i];
    for (int m = 0; m < kXLd; ++m) {
      const float x = m < O ? s_x[i][m] : (m == O ? s_act[i] : 0.0f);
      a.sc.q_x[0][(int64_t)r * kXLd + m] = x;
      a.sc.q_x[1][(int64_t)r * kXLd + m] = x;
      a.sc.a_x[(int64_t)r * kXLd + m] = m < O ? s_x[i][m] : 0.0f;
    }
  }
  __syncthreads();

  // ---- critic backward: dg2 = dq·w3 ⊙ [g2 > 0], dg1 = (W2ᵀ dg2) ⊙ [g1 > 0] ----
  if (lead) {
    for (int k = 0; k < 2; ++k) {
      const float* C = P + L.q_base[k];
      const float* dq = s_row[k == 0 ? S_DQ1 : S_DQ2];
      const float w3 = C[L.c_w3 + j];
#pragma unroll
      for (int i = 0; i < 2 * RR; ++i) {
        const float g2 = s_g2[k][i][j];
        const float dg2 = g2 > 0.0f ? dq[i] * w3 : 0.0f;
        if (i >= RR) {
          const int64_t o = (int64_t)(r0 + i - RR) * H + j;
          a.sc.q_g2[k][o] = g2;
          a.sc.q_dg2[k][o] = dg2;
        }
        s_g2[k][i][j] = dg2;
      }
    }
  }
  __syncthreads();
  {
    float v[2 * RR];  // d(ã) partials for the policy rows, both critics
    for (int k = 0; k < 2; ++k) {
      const float* C = P + L.q_base[k];
      float acc[2 * RR];
#pragma unroll
      for (int i = 0; i < 2 * RR; ++i) acc[i] = 0.0f;
      // Σ_jj W2[jj][m]·dg2[i][jj] with m = this column: W2 row-major reads are coalesced over m
      if (col) mv_part<2 * RR, KS>(C + L.c_w2, H, &s_g2[k][0][0], SACF_MAX_HIDDEN, j, kg, acc);
      kreduce<2 * RR, KS>(acc, s_part, j, kg);
      const float wa = lead ? C[L.c_w1 + (int64_t)j * (O + 1) + O] : 0.0f;
#pragma unroll
      for (int i = 0; i < 2 * RR; ++i) {
        const float g1 = lead ? s_g1[k][i][j] : 0.0f;
        const float dg1 = g1 > 0.0f ? acc[i] : 0.0f;
        if (i < RR) {
          v[k * RR + i] = wa * dg1;
        } else if (lead) {
          const int64_t o = (int64_t)(r0 + i - RR) * H + j;
          a.sc.q_g1[k][o] = g1;  // (obs, a) rows feed the weight gradients
          a.sc.q_dg1[k][o] = dg1;
        }
      }
    }
    block_sum_w<2 * RR, NW>(v, s_red, s_sum);
  }

  // ---- actor backward on the obs rows ----
  if (tid < RR) {
    const int i = tid, r = r0 + i;
    const float act = s_row[S_A][i], z = s_row[S_Z][i], mean = s_row[S_MEAN][i], std = s_row[S_STD][i];
    const float ls_raw = s_row[S_LSRAW][i];
    float dA = s_sum[i] + s_sum[RR + i];
    if (a.hp.areg != 0.0f) dA += (a.hp.areg * invB) * (2.0f * act);
    const float ainv = alpha * invB;
    const float d = z - mean, var = std * std;
    const float sig = 1.0f / (1.0f + expf(2.0f * z));  // sigmoid(-2z)
    const float gz = dA * (1.0f - act * act) + ainv * (-(d / var) + (2.0f - 4.0f * sig));
    const float dmean = gz + ainv * (d / var);
    const float dstd = gz * s_eps[i] + ainv * ((d * d) / (var * std) - 1.0f / std);
    const float dls = (ls_raw >= -20.0f && ls_raw <= 2.0f) ? dstd * std : 0.0f;
    s_row[S_DMEAN][i] = dmean;
    s_row[S_DLS][i] = dls;
    a.sc.a_dhead[(int64_t)r * 2] = dmean;
    a.sc.a_dhead[(int64_t)r * 2 + 1] = dls;
  }
  __syncthreads();
  if (lead) {
    const float wm = P[L.p_wm + j], ws = P[L.p_ws + j];
#pragma unroll
    for (int i = 0; i < RR; ++i) {
      const float h2 = s_h2[i][j];
      const float dh2 = h2 > 0.0f ? (wm * s_row[S_DMEAN][i] + ws * s_row[S_DLS][i]) : 0.0f;
      const int64_t o = (int64_t)(r0 + i) * H + j;
      a.sc.a_h2[o] = h2;
      a.sc.a_dh2[o] = dh2;
      s_h2[i][j] = dh2;
    }
  }
  __syncthreads();
  {
    float acc[RR];
#pragma unroll
    for (int i = 0; i < RR; ++i) acc[i] = 0.0f;
    if (col) mv_part<RR, KS>(P + L.p_w2, H, &s_h2[0][0], SACF_MAX_HIDDEN, j, kg, acc);
    kreduce<RR, KS>(acc, s_part, j, kg);
    if (lead) {
#pragma unroll
      for (int i = 0; i < RR; ++i) {
        const float h1 = s_h1[i][j];
        const int64_t o = (int64_t)(r0 + i) * H + j;
        a.sc.a_h1[o] = h1;
        a.sc.a_dh1[o] = h1 > 0.0f ? acc[i] : 0.0f;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// rows kernel, one batch row per block, four 256-thread groups working on independent matrices:
// the six critic / target-critic rows of the forward pass are one phase (group g = Q1, Q2, T1, T2,
// each over the full K), the twin-critic backward is one phase (two groups per critic, split-K 2).
// Same math as sac_rows_kernel<1, 4>; 4 H x H matvec phases per block instead of 8.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kCols * 4) void sac_rows_g4_kernel(RowsArgs a) {
  constexpr int NW = kCols * 4 / 64;
  const Layout& L = a.L;
  const int H = L.H, O = L.O, B = L.B;
  const int tid = threadIdx.x;
  const int j = tid % kCols, kg = tid / kCols;
  const bool col = j < H;
  const bool lead = kg == 0 && col;
  const int r = blockIdx.x;
  const float* P = a.params;
  const float* TG = a.targets;
  SAC_MARK(0);

  __shared__ float s_x[2][kXLd];  // obs row | next_obs row
  __shared__ float s_act, s_rew, s_term, s_eps[2];
  __shared__ __attribute__((aligned(16))) float s_h1[2][SACF_MAX_HIDDEN];     // actor: obs | next_obs
  __shared__ __attribute__((aligned(16))) float s_h2[2][SACF_MAX_HIDDEN];
  __shared__ __attribute__((aligned(16))) float s_g1[4][2][SACF_MAX_HIDDEN];  // Q1, Q2: (obs, ã) | (obs, a); T1, T2: row 0
  __shared__ __attribute__((aligned(16))) float s_g2[4][2][SACF_MAX_HIDDEN];
  __shared__ float s_part[3 * 2 * kCols];
  __shared__ float s_red[NW][32];
  __shared__ float s_sum[32];
  __shared__ float s_row[S_NSLOT][2];

  // ---- batch row + reparameterisation noise ----
  if (tid == 0) {
    int64_t idx = r;
    uint32_t c[4] = {(uint32_t)r, (uint32_t)*a.step, (uint32_t)((uint64_t)*a.step >> 32), 0x5AC0u};
    if (a.sampled || !a.eps) philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    if (a.sampled) {
      const int64_t size = *a.size_dev > 0 ? *a.size_dev : 1;
      const double u = ((double)c[0] + 0.5) * (1.0 / 4294967296.0);
      idx = (int64_t)(u * (double)size);
      if (idx >= a.capacity) idx = a.capacity - 1;
    }
    float e0, e1;
    if (a.eps) {
      e0 = a.eps[r];
      e1 = a.eps[B + r];
    } else {
      const float u1 = ((float)c[1] + 1.0f) * 2.3283064365386963e-10f;
      const float u2 = (float)c[2] * 2.3283064365386963e-10f;
      const float rad = sqrtf(-2.0f * logf(u1));
      e0 = rad * cosf(6.283185307179586f * u2);
      e1 = rad * sinf(6.283185307179586f * u2);
    }
    for (int m = 0; m < O; ++m) {
      s_x[0][m] = a.obs[idx * O + m];
      s_x[1][m] = a.nobs[idx * O + m];
    }
    s_act = a.act[idx];
    s_rew = a.rew[idx];
    s_term = a.term[idx];
    s_eps[0] = e0;
    s_eps[1] = e1;
  }
  __syncthreads();
  SAC_MARK(1);

  // ---- actor forward on obs and next_obs ----
  if (lead) {
    float acc[2];
    const float b = P[L.p_b1 + j];
    acc[0] = b;
    acc[1] = b;
    for (int m = 0; m < O; ++m) {
      const float w = P[L.p_w1 + (int64_t)j * O + m];
      acc[0] = fmaf(w, s_x[0][m], acc[0]);
      acc[1] = fmaf(w, s_x[1][m], acc[1]);
    }
    s_h1[0][j] = relu(acc[0]);
    s_h1[1][j] = relu(acc[1]);
  }
  __syncthreads();
  SAC_MARK(2);
  {
    float acc[2];
    const float b = lead ? P[L.p_b2 + j] : 0.0f;
    acc[0] = b;
    acc[1] = b;
    if (col) mv_part<2, 4>(a.T, H, &s_h1[0][0], SACF_MAX_HIDDEN, j, kg, acc);
    kreduce<2, 4>(acc, s_part, j, kg);
    if (lead) {
      s_h2[0][j] = relu(acc[0]);
      s_h2[1][j] = relu(acc[1]);
    }
  }
  __syncthreads();
  SAC_MARK(3);
  {
    float v[4];
    const float wm = lead ? P[L.p_wm + j] : 0.0f, ws = lead ? P[L.p_ws + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float h = lead ? s_h2[i][j] : 0.0f;
      v[i] = wm * h;
      v[2 + i] = ws * h;
    }
    block_sum_w<4, NW>(v, s_red, s_sum);
  }
  if (tid < 2) {  // TanhNormal.rsample_and_logprob (distributions.py:346-392)
    const int i = tid;
    const float mean = s_sum[i] + P[L.p_bm];
    const float ls_raw = s_sum[2 + i] + P[L.p_bs];
    const float log_std = fminf(fmaxf(ls_raw, -20.0f), 2.0f);
    const float std = expf(log_std);
    const float z = mean + std * s_eps[i];
    const float act = tanhf(z);
    const float var = std * std;
    const float d = z - mean;
    const float lp = -(d * d) / (2.0f * var) - logf(std) - kLogSqrt2Pi;
    const float corr = -2.0f * (kLog2 - z - softplus(-2.0f * z));
    s_row[S_MEAN][i] = mean;
    s_row[S_LSRAW][i] = ls_raw;
    s_row[S_STD][i] = std;
    s_row[S_Z][i] = z;
    s_row[S_A][i] = act;
    s_row[S_LOGP][i] = lp + corr;
  }
  __syncthreads();
  SAC_MARK(4);

  // ---- first layers: group g = Q1, Q2 on (obs, ã) | (obs, a); T1, T2 on (next_obs, ã') ----
  const bool is_t = kg >= 2;
  const float* C = is_t ? TG + (int64_t)(kg - 2) * L.q_size : P + L.q_base[kg];
  if (col) {
    const float* xin = s_x[is_t ? 1 : 0];
    float base = C[L.c_b1 + j];
    for (int m = 0; m < O; ++m) base = fmaf(C[L.c_w1 + (int64_t)j * (O + 1) + m], xin[m], base);
    const float wa = C[L.c_w1 + (int64_t)j * (O + 1) + O];
    if (is_t) {
      s_g1[kg][0][j] = relu(fmaf(wa, s_row[S_A][1], base));
    } else {
      s_g1[kg][0][j] = relu(fmaf(wa, s_row[S_A][0], base));
      s_g1[kg][1][j] = relu(fmaf(wa, s_act, base));
    }
  }
  __syncthreads();
  SAC_MARK(5);
  // ---- second layers, all four at once (full K per group) ----
  if (col) {
    const float b = C[L.c_b2 + j];
    float acc[2] = {b, b};
    const float* WT = a.T + (size_t)(1 + kg) * H * H;  // [q1 | q2 | t1 | t2] W2ᵀ
    if (is_t) {
      float a1[1] = {b};
      mv_part<1, 1>(WT, H, &s_g1[kg][0][0], SACF_MAX_HIDDEN, j, 0, a1);
      acc[0] = a1[0];
    } else {
      mv_part<2, 1>(WT, H, &s_g1[kg][0][0], SACF_MAX_HIDDEN, j, 0, acc);
    }
    s_g2[kg][0][j] = relu(acc[0]);
    if (!is_t) s_g2[kg][1][j] = relu(acc[1]);
  }
  __syncthreads();
  SAC_MARK(6);
  {
    // heads: Q1 (2 rows), Q2 (2 rows), T1, T2 -> v[0..5]
    float v[6] = {0, 0, 0, 0, 0, 0};
    if (col) {
      const float w3 = C[L.c_w3 + j];
      if (is_t) {
        v[4 + (kg - 2)] = w3 * s_g2[kg][0][j];
      } else {
        v[2 * kg] = w3 * s_g2[kg][0][j];
        v[2 * kg + 1] = w3 * s_g2[kg][1][j];
      }
    }
    block_sum_w<6, NW>(v, s_red, s_sum);
  }
  const float log_alpha = P[0];
  const float alpha = a.hp.auto_ent ? expf(log_alpha) : 1.0f;
  const float invB = 1.0f / (float)B;
  if (tid == 0) {  // losses and output gradients (sac.py:170-247)
    const float q1a = s_sum[0] + P[L.q_base[0] + L.c_b3], q1b = s_sum[1] + P[L.q_base[0] + L.c_b3];
    const float q2a = s_sum[2] + P[L.q_base[1] + L.c_b3], q2b = s_sum[3] + P[L.q_base[1] + L.c_b3];
    const float t1 = s_sum[4] + TG[L.c_b3], t2 = s_sum[5] + TG[L.q_size + L.c_b3];
    const float tq = fminf(t1, t2) - alpha * s_row[S_LOGP][1];
    float qt = a.hp.rscale * s_rew + ((1.0f - s_term) * a.hp.gamma) * tq;
    qt = fminf(fmaxf(qt, -a.hp.clip), a.hp.clip);
    const float qmin = fminf(q1a, q2a);
    const float w1 = (q1a < q2a) ? 1.0f : ((q1a == q2a) ? 0.5f : 0.0f);
    const float w2 = 1.0f - w1;
    s_row[S_DQ1][0] = -w1 * invB;
    s_row[S_DQ2][0] = -w2 * invB;
    const float dq1b = (2.0f * invB) * (q1b - qt), dq2b = (2.0f * invB) * (q2b - qt);
    s_row[S_DQ1][1] = dq1b;
    s_row[S_DQ2][1] = dq2b;
    a.sc.q_dq[0][r] = dq1b;
    a.sc.q_dq[1][r] = dq2b;
    const float logp = s_row[S_LOGP][0], act = s_row[S_A][0];
    a.sc.p_pl[r] = alpha * logp - qmin + (a.hp.areg != 0.0f ? a.hp.areg * (act * act) : 0.0f);
    a.sc.p_q1l[r] = (q1b - qt) * (q1b - qt);
    a.sc.p_q2l[r] = (q2b - qt) * (q2b - qt);
    a.sc.p_la[r] = -(log_alpha * (logp + a.hp.tent));
    a.sc.p_ga[r] = -(logp + a.hp.tent);
    float* st = a.stats + 8;
    st[r] = q1b;
    st[B + r] = q2b;
    st[2 * B + r] = qt;
    st[3 * B + r] = logp;
    st[4 * B + r] = tanhf(s_row[S_MEAN][0]);
    st[5 * B + r] = s_row[S_STD][0];
  } else if (tid >= 64 && tid < 64 + kXLd) {
    const int m = tid - 64;
    const float x = m < O ? s_x[0][m] : (m == O ? s_act : 0.0f);
    a.sc.q_x[0][(int64_t)r * kXLd + m] = x;
    a.sc.q_x[1][(int64_t)r * kXLd + m] = x;
    a.sc.a_x[(int64_t)r * kXLd + m] = m < O ? s_x[0][m] : 0.0f;
  }
  __syncthreads();
  SAC_MARK(7);

  // ---- critic backward: dg2 = dq·w3 ⊙ [g2 > 0] (groups 0, 1), then dg1 = (W2ᵀ dg2) ⊙ [g1 > 0] ----
  if (col && kg < 2) {
    const float* dq = s_row[kg == 0 ? S_DQ1 : S_DQ2];
    const float w3 = C[L.c_w3 + j];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float g2 = s_g2[kg][i][j];
      const float dg2 = g2 > 0.0f ? dq[i] * w3 : 0.0f;
      if (i == 1) {
        const int64_t o = (int64_t)r * H + j;
        a.sc.q_g2[kg][o] = g2;
        a.sc.q_dg2[kg][o] = dg2;
      }
      s_g2[kg][i][j] = dg2;
    }
  }
  __syncthreads();
  SAC_MARK(8);
  {
    // groups 0, 1 -> critic 0 (k halves), groups 2, 3 -> critic 1
    const int k = kg >> 1, half = kg & 1;
    const float* Ck = P + L.q_base[k];
    float acc[2] = {0.0f, 0.0f};
    if (col) mv_part<2, 2>(Ck + L.c_w2, H, &s_g2[k][0][0], SACF_MAX_HIDDEN, j, half, acc);
    if (half) {
      s_part[(k * 2 + 0) * kCols + j] = acc[0];
      s_part[(k * 2 + 1) * kCols + j] = acc[1];
    }
    __syncthreads();
    float v[2] = {0.0f, 0.0f};
    if (!half && col) {
      acc[0] += s_part[(k * 2 + 0) * kCols + j];
      acc[1] += s_part[(k * 2 + 1) * kCols + j];
      const float wa = Ck[L.c_w1 + (int64_t)j * (O + 1) + O];
      const float g1a = s_g1[k][0][j], g1b = s_g1[k][1][j];
      v[k] = wa * (g1a > 0.0f ? acc[0] : 0.0f);
      const int64_t o = (int64_t)r * H + j;
      a.sc.q_g1[k][o] = g1b;
      a.sc.q_dg1[k][o] = g1b > 0.0f ? acc[1] : 0.0f;
    }
    block_sum_w<2, NW>(v, s_red, s_sum);
  }

  // ---- actor backward on the obs row ----
  if (tid == 0) {
    const float act = s_row[S_A][0], z = s_row[S_Z][0], mean = s_row[S_MEAN][0], std = s_row[S_STD][0];
    const float ls_raw = s_row[S_LSRAW][0];
    float dA = s_sum[0] + s_sum[1];
    if (a.hp.areg != 0.0f) dA += (a.hp.areg * invB) * (2.0f * act);
    const float ainv = alpha * invB;
    const float d = z - mean, var = std * std;
    const float sig = 1.0f / (1.0f + expf(2.0f * z));  // sigmoid(-2z)
    const float gz = dA * (1.0f - act * act) + ainv * (-(d / var) + (2.0f - 4.0f * sig));
    const float dmean = gz + ainv * (d / var);
    const float dstd = gz * s_eps[0] + ainv * ((d * d) / (var * std) - 1.0f / std);
    const float dls = (ls_raw >= -20.0f && ls_raw <= 2.0f) ? dstd * std : 0.0f;
    s_row[S_DMEAN][0] = dmean;
    s_row[S_DLS][0] = dls;
    a.sc.a_dhead[(int64_t)r * 2] = dmean;
    a.sc.a_dhead[(int64_t)r * 2 + 1] = dls;
  }
  __syncthreads();
  SAC_MARK(9);
  if (lead) {
    const float wm = P[L.p_wm + j], ws = P[L.p_ws + j];
    const float h2 = s_h2[0][j];
    const float dh2 = h2 > 0.0f ? (wm * s_row[S_DMEAN][0] + ws * s_row[S_DLS][0]) : 0.0f;
    const int64_t o = (int64_t)r * H + j;
    a.sc.a_h2[o] = h2;
    a.sc.a_dh2[o] = dh2;
    s_h2[0][j] = dh2;
  }
  __syncthreads();
  SAC_MARK(10);
  {
    float acc[1] = {0.0f};
    if (col) mv_part<1, 4>(P + L.p_w2, H, &s_h2[0][0], SACF_MAX_HIDDEN, j, kg, acc);
    kreduce<1, 4>(acc, s_part, j, kg);
    if (lead) {
      const float h1 = s_h1[0][j];
      const int64_t o = (int64_t)r * H + j;
      a.sc.a_h1[o] = h1;
      a.sc.a_dh1[o] = h1 > 0.0f ? acc[0] : 0.0f;
    }
  }
  SAC_MARK(11);
}

// ---------------------------------------------------------------------------------------------
// weight gradients: out[j][k] = Σ_r dY[r·ldY + j] · X[r·ldX + k]  (X == nullptr: ones -> bias)
// ---------------------------------------------------------------------------------------------
struct GMat {
  const float* dY;
  const float* X;
  int ldY, ldX, M, N;
  int64_t out_off;
};
struct GTask {
  int mat, j0, k0;
};
constexpr int kMaxMats = 24;
// Row split of the weight gradients: grid.y = kParts blocks per tile each reduce B / kParts rows
// into partial gradient p (same layout as the flat gradient); sac_gsum_kernel adds the kParts
// partials in a fixed order (deterministic) into the gradient.
#ifndef SAC_KPARTS
#define SAC_KPARTS 8
#endif
constexpr int kParts = SAC_KPARTS;
struct WgradArgs {
  GMat mats[kMaxMats];
  const GTask* tasks;
  int n_tasks;
  float* partials;          // [kParts][n_params]
  int64_t n_params;
  float* grads;
  int B;
  Scratch sc;
  const float* params;
  int64_t* step;
  float* stats;
  Hyper hp;
};

__global__ __launch_bounds__(kThreads) void sac_wgrad_kernel(WgradArgs a) {
  const int tid = threadIdx.x;
  if ((int)blockIdx.x == a.n_tasks) {  // scalars: losses, α and d(log α); step += 1
    if (blockIdx.y != 0) return;
    float v[5] = {0, 0, 0, 0, 0};
    for (int r = tid; r < a.B; r += kThreads) {
      v[0] += a.sc.p_pl[r];
      v[1] += a.sc.p_q1l[r];
      v[2] += a.sc.p_q2l[r];
      v[3] += a.sc.p_la[r];
      v[4] += a.sc.p_ga[r];
    }
    __shared__ float red[4][32];
    __shared__ float sum[32];
    block_sum<5>(v, red, sum);
    if (tid == 0) {
      const float invB = 1.0f / (float)a.B;
      a.stats[0] = sum[0] * invB;
      a.stats[1] = sum[1] * invB;
      a.stats[2] = sum[2] * invB;
      a.stats[3] = a.hp.auto_ent ? sum[3] * invB : 0.0f;
      a.stats[4] = a.hp.auto_ent ? expf(a.params[0]) : 1.0f;
      a.grads[0] = a.hp.auto_ent ? sum[4] * invB : 0.0f;
      const int64_t step = *a.step + 1;
      *a.step = step;
      // Adam bias corrections of this step for sac_apply_kernel (stats[5..7])
      const double t = (double)step;
      const double bc1 = 1.0 - pow((double)a.hp.beta1, t);
      const double bc2 = 1.0 - pow((double)a.hp.beta2, t);
      a.stats[5] = (float)(a.hp.lr_pi / bc1);
      a.stats[6] = (float)(a.hp.lr_q / bc1);
      a.stats[7] = (float)sqrt(bc2);
    }
    return;
  }
  const GTask t = a.tasks[blockIdx.x];
  const GMat m = a.mats[t.mat];
  __shared__ float sY[32][64 + 1];
  __shared__ float sX[32][64 + 1];
  const int tj = tid >> 4, tk = tid & 15;
  float acc[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.0f;
  const int part = blockIdx.y;
  const int rows = (a.B + kParts - 1) / kParts;
  const int r_lo = part * rows, r_hi = min(a.B, r_lo + rows);
  for (int rb = r_lo; rb < r_hi; rb += 32) {
    for (int e = tid; e < 32 * 64; e += kThreads) {
      const int rr = e >> 6, cc = e & 63, r = rb + rr;
      const int jj = t.j0 + cc, kk = t.k0 + cc;
      sY[rr][cc] = (r < r_hi && jj < m.M) ? m.dY[(int64_t)r * m.ldY + jj] : 0.0f;
      sX[rr][cc] = (r < r_hi && kk < m.N) ? (m.X ? m.X[(int64_t)r * m.ldX + kk] : 1.0f) : 0.0f;
    }
    __syncthreads();
#pragma unroll 4
    for (int rr = 0; rr < 32; ++rr) {
      float y[4], x[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) y[p] = sY[rr][tj * 4 + p];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = sX[rr][tk * 4 + q];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = fmaf(y[p], x[q], acc[p][q]);
    }
    __syncthreads();
  }
  float* P = a.partials + (size_t)part * a.n_params;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int jj = t.j0 + tj * 4 + p;
    if (jj >= m.M) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = t.k0 + tk * 4 + q;
      if (kk < m.N) P[m.out_off + (int64_t)jj * m.N + kk] = acc[p][q];
    }
  }
}

// gradient = Σ_p partial_p (p = 0..kParts-1 in order); element 0 (d log α) is the scalar block's
__global__ __launch_bounds__(kThreads) void sac_gsum_kernel(const float* __restrict__ partials, float* grads,
                                                            int64_t n_params) {
  const int64_t e = 1 + (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= n_params) return;
  float g = partials[e];
#pragma unroll
  for (int p = 1; p < kParts; ++p) g += partials[(size_t)p * n_params + e];
  grads[e] = g;
}

// ---------------------------------------------------------------------------------------------
// Adam (torch.optim.Adam, amsgrad=False, no weight decay) + soft target update + transposes
// ---------------------------------------------------------------------------------------------
struct ApplyArgs {
  float* params;
  float* targets;
  float* grads;
  const float* partials;  // non-null: the gradient is Σ of the kParts partials (single process, no all-reduce)
  float* m;
  float* v;
  const int64_t* step;
  float* T;
  const float* stats;
  Layout L;
  Hyper hp;
  int n_tile_blocks;      // blocks [0, n_tile_blocks) take 32x32 tiles of the three H x H W2 matrices
};

constexpr int kTile = 32;

// Adam bias corrections of this step, computed once by the weight-gradient kernel (stats[5..7])
struct AdamStep {
  float step_pi, step_q, bc2_sqrt;
};

// one element: gradient (Σ partials or the all-reduced flat gradient), torch.optim.Adam, soft update
__device__ __forceinline__ float adam_elem(const ApplyArgs& a, const AdamStep& st, int64_t e, float* tp_out) {
  const Layout& L = a.L;
  float g;
  if (a.partials && e != 0) {
    g = a.partials[e];
#pragma unroll
    for (int p = 1; p < kParts; ++p) g += a.partials[(size_t)p * L.n_params + e];
    a.grads[e] = g;
  } else {
    g = a.grads[e];
  }
  g *= a.hp.inv_world;
  const bool is_q = e >= L.q_base[0];
  float m = a.m[e], v = a.v[e];
  m = m + (1.0f - a.hp.beta1) * (g - m);             // exp_avg.lerp_(grad, 1 - beta1)
  v = v * a.hp.beta2 + (1.0f - a.hp.beta2) * (g * g);  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / st.bc2_sqrt + a.hp.eps;
  const float p = a.params[e] + (-(is_q ? st.step_q : st.step_pi)) * (m / denom);
  a.m[e] = m;
  a.v[e] = v;
  a.params[e] = p;
  if (is_q) {
    const int64_t qe = e - L.q_base[0];
    const float tp = a.targets[qe] * (1.0f - a.hp.tau) + p * a.hp.tau;
    a.targets[qe] = tp;
    *tp_out = tp;
  }
  return p;
}

__global__ __launch_bounds__(kThreads) void sac_apply_kernel(ApplyArgs a) {
  __shared__ float tile[2][kTile][kTile + 1];
  const AdamStep st{a.stats[5], a.stats[6], a.stats[7]};
  const Layout& L = a.L;
  const int H = L.H;
  const int64_t HH = (int64_t)H * H;
  const int64_t w2[3] = {L.p_w2, L.q_base[0] + L.c_w2, L.q_base[1] + L.c_w2};
  if ((int)blockIdx.x < a.n_tile_blocks) {
    // 32 x 32 tile of one W2: Adam on row-major elements, transposed copies written through LDS
    const int tpm = (H / kTile) * (H / kTile);
    const int mat = blockIdx.x / tpm, t = blockIdx.x % tpm;
    const int r0 = (t / (H / kTile)) * kTile, c0 = (t % (H / kTile)) * kTile;
    const int tc = threadIdx.x % kTile, tr = threadIdx.x / kTile;  // 8 rows per pass
    for (int rr = tr; rr < kTile; rr += kThreads / kTile) {
      float tp = 0.0f;
      const int64_t l = (int64_t)(r0 + rr) * H + c0 + tc;
      const float p = adam_elem(a, st, w2[mat] + l, &tp);
      tile[0][tc][rr] = p;
      tile[1][tc][rr] = tp;
    }
    __syncthreads();
    for (int cc = tr; cc < kTile; cc += kThreads / kTile) {
      const int64_t o = (int64_t)(c0 + cc) * H + r0 + tc;  // T[col][row]
      if (mat == 0) {
        a.T[o] = tile[0][cc][tc];
      } else {
        a.T[(size_t)mat * HH + o] = tile[0][cc][tc];
        a.T[(size_t)(2 + mat) * HH + o] = tile[1][cc][tc];
      }
    }
    return;
  }
  // every other element: flat index over the parameters outside the three W2 blocks
  int64_t f = (int64_t)(blockIdx.x - a.n_tile_blocks) * kThreads + threadIdx.x;
  int64_t e = f;
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (e >= w2[k]) e += HH;
  if (e >= L.n_params) return;
  if (e == 0 && !a.hp.auto_ent) return;
  float tp;
  adam_elem(a, st, e, &tp);
}

__global__ void sac_transpose_kernel(const float* params, const float* targets, float* T, Layout L) {
  const int64_t HH = (int64_t)L.H * L.H;
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= 5 * HH) return;
  const int which = (int)(e / HH);
  const int64_t l = e % HH;
  const float* src = which == 0 ? params + L.p_w2
                     : which <= 2 ? params + L.q_base[which - 1] + L.c_w2
                                  : targets + (int64_t)(which - 3) * L.q_size + L.c_w2;
  T[which * HH + (l % L.H) * L.H + l / L.H] = src[l];
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
struct sacf_handle {
  sacf_config cfg;
  Layout L;
  Hyper hp;
  int device;
  hipStream_t stream;
  float *params, *targets, *grads, *adam_m, *adam_v, *stats;
  int64_t* step;
  const float *r_obs, *r_act, *r_rew, *r_term, *r_nobs;
  const int64_t* r_size;
  int64_t r_cap;
  uint64_t seed;
  float* T;
  float* scratch;
  Scratch sc;
  GTask* tasks;
  int n_tasks;
  float* partials;
  GMat mats[kMaxMats];
  int n_mats;
  char err[512];
};

static int sfail(sacf_handle* h, int code, const char* fmt, ...) {
  if (h) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(h->err, sizeof(h->err), fmt, ap);
    va_end(ap);
  }
  return code;
}

struct SDev {
  int prev;
  explicit SDev(int d) {
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(d);
  }
  ~SDev() { (void)hipSetDevice(prev); }
};

extern "C" {

int32_t sacf_abi_version(void) { return SACF_ABI_VERSION; }

#ifndef SACF_SRC_HASH
#define SACF_SRC_HASH "unknown"
#endif
const char* sacf_build_info(void) { return "sacfused gfx950 HIP src " SACF_SRC_HASH; }

int sacf_create(const sacf_config* cfg, int device, void* stream, sacf_handle** out) {
  if (!out) return SACF_EINVAL;
  *out = nullptr;
  if (!cfg || cfg->abi_version != SACF_ABI_VERSION) return SACF_EINVAL;
  const int O = cfg->obs_dim, H = cfg->hidden, B = cfg->batch;
  if (O < 1 || O + 1 > kXLd || H < 32 || H > SACF_MAX_HIDDEN || H % 32 || B < R || B % R || cfg->world_size < 1)
    return SACF_EINVAL;
  sacf_handle* h = new (std::nothrow) sacf_handle();
  if (!h) return SACF_EINVAL;
  h->cfg = *cfg;
  h->device = device;
  h->stream = (hipStream_t)stream;
  Layout& L = h->L;
  L.O = O;
  L.H = H;
  L.B = B;
  int64_t o = 1;  // log_alpha at 0
  L.p_w1 = o; o += (int64_t)H * O;
  L.p_b1 = o; o += H;
  L.p_w2 = o; o += (int64_t)H * H;
  L.p_b2 = o; o += H;
  L.p_wm = o; o += H;
  L.p_bm = o; o += 1;
  L.p_ws = o; o += H;
  L.p_bs = o; o += 1;
  int64_t c = 0;
  L.c_w1 = c; c += (int64_t)H * (O + 1);
  L.c_b1 = c; c += H;
  L.c_w2 = c; c += (int64_t)H * H;
  L.c_b2 = c; c += H;
  L.c_w3 = c; c += H;
  L.c_b3 = c; c += 1;
  L.q_size = c;
  L.q_base[0] = o;
  L.q_base[1] = o + c;
  L.n_params = o + 2 * c;
  L.n_targets = 2 * c;
  Hyper& hp = h->hp;
  hp.gamma = cfg->discount;
  hp.rscale = cfg->reward_scale;
  hp.tau = cfg->soft_target_tau;
  hp.areg = cfg->action_reg_coeff;
  hp.clip = cfg->clip_val;
  hp.tent = cfg->target_entropy;
  hp.lr_pi = cfg->policy_lr;
  hp.lr_q = cfg->qf_lr;
  hp.beta1 = cfg->beta1;
  hp.beta2 = cfg->beta2;
  hp.eps = cfg->adam_eps;
  hp.auto_ent = cfg->auto_entropy;
  hp.inv_world = 1.0f / (float)cfg->world_size;

  SDev g(device);
  // scratch: actor 4·B·H + B·16 + 2B; critics 2·(4·B·H + B·16 + B); partials 5B
  const int64_t BH = (int64_t)B * H;
  const int64_t n_scr = 4 * BH + B * kXLd + 2 * B + 2 * (4 * BH + B * kXLd + B) + 5 * B;
  hipError_t e = hipMalloc(&h->scratch, sizeof(float) * n_scr);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "hipMalloc(scratch): %s", hipGetErrorString(e));
  }
  float* s = h->scratch;
  Scratch& sc = h->sc;
  sc.a_x = s; s += B * kXLd;
  sc.a_h1 = s; s += BH;
  sc.a_h2 = s; s += BH;
  sc.a_dh1 = s; s += BH;
  sc.a_dh2 = s; s += BH;
  sc.a_dhead = s; s += 2 * B;
  for (int k = 0; k < 2; ++k) {
    sc.q_x[k] = s; s += B * kXLd;
    sc.q_g1[k] = s; s += BH;
    sc.q_g2[k] = s; s += BH;
    sc.q_dg1[k] = s; s += BH;
    sc.q_dg2[k] = s; s += BH;
    sc.q_dq[k] = s; s += B;
  }
  sc.p_pl = s; s += B;
  sc.p_q1l = s; s += B;
  sc.p_q2l = s; s += B;
  sc.p_la = s; s += B;
  sc.p_ga = s; s += B;
  e = hipMalloc(&h->T, sizeof(float) * 5 * (size_t)H * H);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "hipMalloc(T): %s", hipGetErrorString(e));
  }
  // weight-gradient matrices and their 64×64 tiles
  int nm = 0;
  auto add = [&](const float* dY, int ldY, const float* X, int ldX, int M, int N, int64_t off) {
    h->mats[nm++] = GMat{dY, X, ldY, ldX, M, N, off};
  };
  add(sc.a_dh1, H, sc.a_x, kXLd, H, O, L.p_w1);
  add(sc.a_dh1, H, nullptr, 0, H, 1, L.p_b1);
  add(sc.a_dh2, H, sc.a_h1, H, H, H, L.p_w2);
  add(sc.a_dh2, H, nullptr, 0, H, 1, L.p_b2);
  add(sc.a_dhead, 2, sc.a_h2, H, 1, H, L.p_wm);
  add(sc.a_dhead, 2, nullptr, 0, 1, 1, L.p_bm);
  add(sc.a_dhead + 1, 2, sc.a_h2, H, 1, H, L.p_ws);
  add(sc.a_dhead + 1, 2, nullptr, 0, 1, 1, L.p_bs);
  for (int k = 0; k < 2; ++k) {
    const int64_t b = L.q_base[k];
    add(sc.q_dg1[k], H, sc.q_x[k], kXLd, H, O + 1, b + L.c_w1);
    add(sc.q_dg1[k], H, nullptr, 0, H, 1, b + L.c_b1);
    add(sc.q_dg2[k], H, sc.q_g1[k], H, H, H, b + L.c_w2);
    add(sc.q_dg2[k], H, nullptr, 0, H, 1, b + L.c_b2);
    add(sc.q_dq[k], 1, sc.q_g2[k], H, 1, H, b + L.c_w3);
    add(sc.q_dq[k], 1, nullptr, 0, 1, 1, b + L.c_b3);
  }
  h->n_mats = nm;
  std::vector<GTask> tasks;
  // the big H×H tiles first so they start early
  for (int pass = 0; pass < 2; ++pass)
    for (int mi = 0; mi < nm; ++mi) {
      const GMat& m = h->mats[mi];
      const bool big = m.M == H && m.N == H;
      if ((pass == 0) != big) continue;
      for (int j0 = 0; j0 < m.M; j0 += 64)
        for (int k0 = 0; k0 < m.N; k0 += 64) tasks.push_back(GTask{mi, j0, k0});
    }
  h->n_tasks = (int)tasks.size();
  e = hipMalloc(&h->partials, sizeof(float) * kParts * L.n_params);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "partials: %s", hipGetErrorString(e));
  }
  e = hipMalloc(&h->tasks, sizeof(GTask) * tasks.size());
  if (e == hipSuccess) e = hipMemcpy(h->tasks, tasks.data(), sizeof(GTask) * tasks.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "tasks: %s", hipGetErrorString(e));
  }
  *out = h;
  return SACF_OK;
}

int sacf_destroy(sacf_handle* h) {
  if (!h) return SACF_OK;
  SDev g(h->device);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->T) (void)hipFree(h->T);
  if (h->tasks) (void)hipFree(h->tasks);
  if (h->partials) (void)hipFree(h->partials);
  delete h;
  return SACF_OK;
}

#ifdef SACF_PHASE_TIMING
int sacf_debug_stamps(unsigned long long* out16) {
  return hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_sac_stamp), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -1;
}
#endif

const char* sacf_last_error(const sacf_handle* h) { return h ? h->err : "null handle"; }
int64_t sacf_param_count(const sacf_handle* h) { return h ? h->L.n_params : -1; }
int64_t sacf_target_count(const sacf_handle* h) { return h ? h->L.n_targets : -1; }
int64_t sacf_stats_count(const sacf_handle* h) { return h ? 8 + 6 * (int64_t)h->L.B : -1; }

int sacf_set_stream(sacf_handle* h, void* stream) {
  if (!h) return SACF_EINVAL;
  h->stream = (hipStream_t)stream;
  return SACF_OK;
}

int sacf_bind(sacf_handle* h, float* params, float* targets, float* grads, float* adam_m, float* adam_v,
              int64_t* step, float* stats) {
  if (!h || !params || !targets || !grads || !adam_m || !adam_v || !step || !stats)
    return sfail(h, SACF_EINVAL, "sacf_bind: null buffer");
  h->params = params;
  h->targets = targets;
  h->grads = grads;
  h->adam_m = adam_m;
  h->adam_v = adam_v;
  h->step = step;
  h->stats = stats;
  return sacf_sync_params(h);
}

int sacf_sync_params(sacf_handle* h) {
  if (!h || !h->params) return sfail(h, SACF_ESTATE, "sacf_sync_params: not bound");
  SDev g(h->device);
  const int64_t n = 5 * (int64_t)h->L.H * h->L.H;
  hipLaunchKernelGGL(sac_transpose_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     h->stream, h->params, h->targets, h->T, h->L);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "transpose: %s", hipGetErrorString(e));
}

int sacf_set_replay(sacf_handle* h, const float* obs, const float* act, const float* rew, const float* term,
                    const float* next_obs, const int64_t* size_dev, int64_t capacity, uint64_t seed) {
  if (!h || !obs || !act || !rew || !term || !next_obs || !size_dev || capacity < 1)
    return sfail(h, SACF_EINVAL, "sacf_set_replay: bad argument");
  h->r_obs = obs;
  h->r_act = act;
  h->r_rew = rew;
  h->r_term = term;
  h->r_nobs = next_obs;
  h->r_size = size_dev;
  h->r_cap = capacity;
  h->seed = seed;
  return SACF_OK;
}

int sacf_grads(sacf_handle* h, const float* obs, const float* act, const float* rew, const float* term,
               const float* next_obs, const float* eps) {
  if (!h || !h->params) return sfail(h, SACF_ESTATE, "sacf_grads: buffers not bound");
  RowsArgs a;
  memset(&a, 0, sizeof(a));
  a.params = h->params;
  a.targets = h->targets;
  a.T = h->T;
  if (obs) {
    if (!act || !rew || !term || !next_obs) return sfail(h, SACF_EINVAL, "sacf_grads: partial batch");
    a.obs = obs; a.act = act; a.rew = rew; a.term = term; a.nobs = next_obs;
    a.sampled = 0;
  } else {
    if (!h->r_obs) return sfail(h, SACF_ESTATE, "sacf_grads: no batch and no replay bound");
    a.obs = h->r_obs; a.act = h->r_act; a.rew = h->r_rew; a.term = h->r_term; a.nobs = h->r_nobs;
    a.size_dev = h->r_size;
    a.capacity = h->r_cap;
    a.sampled = 1;
  }
  a.seed = h->seed;
  a.eps = eps;
  a.step = h->step;
  a.stats = h->stats;
  a.sc = h->sc;
  a.L = h->L;
  a.hp = h->hp;
  SDev g(h->device);
  // rows-kernel shape: RR batch rows per block x KS k-groups (SACF_ROWS=RRxKS overrides, e.g. 4x1).
  // Measured on MI355X, H = 256, B = 256 (grad steps/s): 4x1 5131, 2x2 7430, 2x4 8364, 1x4 9682.
  int rr = 1, ks = 4;
  if (const char* e = getenv("SACF_ROWS")) {
    if (sscanf(e, "%dx%d", &rr, &ks) != 2) rr = 1, ks = 4;
  }
  if (h->L.H / ks < 8 || (h->L.H / ks) % 8) ks = 1;
#define ROWS(RR_, KS_) \
  hipLaunchKernelGGL((sac_rows_kernel<RR_, KS_>), dim3(h->L.B / RR_), dim3(kCols * KS_), 0, h->stream, a)
  if (!getenv("SACF_ROWS") && h->L.H <= kCols) {  // default: the four-group one-row kernel
    hipLaunchKernelGGL(sac_rows_g4_kernel, dim3(h->L.B), dim3(kCols * 4), 0, h->stream, a);
  } else if (rr == 4 && ks == 1) ROWS(4, 1);
  else if (rr == 4 && ks == 2) ROWS(4, 2);
  else if (rr == 2 && ks == 2) ROWS(2, 2);
  else if (rr == 1 && ks == 4) ROWS(1, 4);
  else if (rr == 2 && ks == 4) ROWS(2, 4);
  else if (ks == 1) ROWS(2, 1);
  else ROWS(1, 4);
#undef ROWS
  WgradArgs w;
  memset(&w, 0, sizeof(w));
  for (int i = 0; i < h->n_mats; ++i) w.mats[i] = h->mats[i];
  w.tasks = h->tasks;
  w.n_tasks = h->n_tasks;
  w.partials = h->partials;
  w.n_params = h->L.n_params;
  w.grads = h->grads;
  w.B = h->L.B;
  w.sc = h->sc;
  w.params = h->params;
  w.step = h->step;
  w.stats = h->stats;
  w.hp = h->hp;
  hipLaunchKernelGGL(sac_wgrad_kernel, dim3(h->n_tasks + 1, kParts), dim3(kThreads), 0, h->stream, w);
  if (h->cfg.world_size > 1)  // the flat gradient is all-reduced before sacf_apply; single process: summed there
    hipLaunchKernelGGL(sac_gsum_kernel, dim3((unsigned)((h->L.n_params - 1 + kThreads - 1) / kThreads)), dim3(kThreads),
                       0, h->stream, h->partials, h->grads, h->L.n_params);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_grads: %s", hipGetErrorString(e));
}

int sacf_apply(sacf_handle* h) {
  if (!h || !h->params) return sfail(h, SACF_ESTATE, "sacf_apply: buffers not bound");
  ApplyArgs a;
  a.params = h->params;
  a.targets = h->targets;
  a.grads = h->grads;
  a.m = h->adam_m;
  a.v = h->adam_v;
  a.step = h->step;
  a.T = h->T;
  a.L = h->L;
  a.hp = h->hp;
  a.partials = h->cfg.world_size > 1 ? nullptr : h->partials;
  a.stats = h->stats;
  const int64_t HH = (int64_t)h->L.H * h->L.H;
  a.n_tile_blocks = 3 * (h->L.H / kTile) * (h->L.H / kTile);
  const int64_t rest = h->L.n_params - 3 * HH;
  SDev g(h->device);
  hipLaunchKernelGGL(sac_apply_kernel, dim3((unsigned)(a.n_tile_blocks + (rest + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, h->stream, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_apply: %s", hipGetErrorString(e));
}

}  // extern "C"
