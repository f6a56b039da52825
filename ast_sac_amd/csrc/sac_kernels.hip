// sac_kernels.hip — fused SAC update for gfx950 (C ABI: include/sac_fused.h) -> libsacfused.so
//
// One grad step of ast_sac/torch/sac/sac.py (compute_loss :156-270, train_from_torch :102-154,
// update_target_networks :160-166) for TanhGaussianPolicy + twin ConcatMlp critics with two hidden
// layers of width H and act_dim 1, as batched GEMMs on the matrix cores (v_mfma_f32_32x32x2_f32,
// exact fp32) in six launches:
//
//   sac_actor_fwd_kernel / sac_critic_fwd_kernel / sac_critic_bwd_kernel / sac_actor_bwd_kernel:
//       the forward and backward passes over the batch (2B actor rows [obs; next_obs], 2B critic
//       rows [(obs, ã); (obs, a)] per critic, B target rows), each a 32 x 32-tiled GEMM with the
//       elementwise work (input layer, bias, ReLU, heads, TanhNormal, losses, masks) fused into
//       the operand fetch or the epilogue; see the MFMA-path section below.
//   sac_wgrad_mfma_kernel: every weight/bias gradient = Σ_rows dY[r]ᵀ X[r] (the H x H ones on MFMA,
//       the rest on the VALU) straight into the flat gradient, plus the loss scalars, d(log α) and
//       this step's Adam bias corrections.
//   sac_apply_kernel : torch.optim.Adam on every element (two lr groups; the gradient divided by the
//       world size after the caller's all-reduce), soft target update θ' ← θ'(1−τ) + θτ, and the
//       transposed H×H copies the forward kernels read (32×32 tiles through LDS).
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
// weight-gradient matrices: out[j][k] = Σ_r dY[r·ldY + j] · X[r·ldX + k]  (X == nullptr: ones -> bias)
// ---------------------------------------------------------------------------------------------
struct GMat {
  const float* dY;
  const float* X;
  int ldY, ldX, M, N;
  int64_t out_off;
};
constexpr int kMaxMats = 24;

// ---------------------------------------------------------------------------------------------
// MFMA path: the grad step as batched GEMMs on v_mfma_f32_32x32x2_f32 (exact fp32: an fmaf chain
// in k order, MI355X_MICROARCH.md "Matrix cores"). Every GEMM runs in 32-row x 32-column output
// tiles, one 256-thread block (4 waves) per tile, the K dimension split over the 4 waves and the 4
// partial tiles summed in LDS in a fixed order. MFMA operand maps (cdna_hip_programming.md §3):
// lane l holds A[l & 31][k] and B[k][l & 31] with k = kb + (l >> 5)·K/8 + i for MFMA i of the wave's
// K/4-slice (a permuted k order: the sum is the same, the loads stay contiguous per lane / per half
// wave); C/D: col = l & 31, row = (reg & 3) + 8·(reg >> 2) + 4·(l >> 5).
//   sac_actor_fwd_kernel  : batch gather (replay sampling), h1 (VALU), h2 = relu(h1 W2ᵀ + b2) on 2B rows
//   sac_critic_fwd_kernel : actor heads + TanhNormal sample per row, g1 (VALU), g2 = relu(g1 W2ᵀ + b2) for
//                           Q1, Q2 on [(obs, ã); (obs, a)] and T1, T2 on (next_obs, ã')
//   sac_critic_bwd_kernel : q heads, losses, dq, dg2 = dq·w3 ⊙ [g2 > 0], dg1 = (dg2 W2) ⊙ [g1 > 0]
//   sac_actor_bwd_kernel  : dA, TanhNormal backward, dh2 = (wm dmean + ws dls) ⊙ [h2 > 0], dh1 = (dh2 W2) ⊙ [h1 > 0]
//   sac_wgrad_mfma_kernel : dW = dYᵀ X for the H x H matrices (rows = K), the small ones on the VALU,
//                           the loss scalars and d(log α)
// ---------------------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kTile2 = 32;  // output tile edge of the MFMA kernels
constexpr int kMaxN2 = 32;  // MFMAs per wave per tile (K / 8 <= 32, i.e. K <= 256)

struct MScratch {
  float *x, *xn, *act, *rew, *term, *eps;  // gathered batch: obs / next_obs [B][kXLd], per row [B] (eps [2][B])
  float *h2n;                              // actor h2 of the next_obs rows [B][H]
  float *hd;                               // actor head of the obs rows [6][B]: mean, ls_raw, std, z, a, logp
  float *hdn;                              // actor head of the next_obs rows [6][B]
  float *g1pi[2], *g2pi[2];                // critics on (obs, ã) rows [B][H]
  float *tg2[2];                           // target critics on (next_obs, ã') [B][H]
  float *dg1pi[2];                         // critic input gradient on (obs, ã) rows [B][H]
};
enum { HD_MEAN, HD_LSRAW, HD_STD, HD_Z, HD_A, HD_LOGP };

struct MArgs {
  const float* params;
  const float* targets;
  const float* T;  // [actor W2ᵀ | q1 W2ᵀ | q2 W2ᵀ | t1 W2ᵀ | t2 W2ᵀ]
  const float *obs, *act, *rew, *term, *nobs;
  const int64_t* size_dev;
  int64_t capacity;
  uint64_t seed;
  int sampled;
  const float* eps;
  const int64_t* step;
  float* stats;
  Scratch sc;
  MScratch ms;
  Layout L;
  Hyper hp;
};

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int g = 0; g < 16; ++g) z[g] = 0.0f;
  return z;
}

// acc += Σ_i A_i ⊗ B_i over the wave's n2 MFMAs (a[i], b[i]: this lane's operands, see above)
__device__ __forceinline__ void mfma_chain(f32x16& acc, const float (&a)[kMaxN2], const float (&b)[kMaxN2], int n2) {
#pragma unroll
  for (int i = 0; i < kMaxN2; ++i)
    if (i < n2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[i], acc, 0, 0, 0);
}

// Sum of the 4 waves' partial tiles (wave 0 + 1 + 2 + 3, in that order), then epi(row, col, v) on the
// 1024 outputs: wave w finishes accumulator registers 4w .. 4w + 3.
template <class EPI>
__device__ __forceinline__ void splitk_finish(const f32x16& acc, float* lds, EPI&& epi) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 16; ++g) lds[(w * 16 + g) * 64 + lane] = acc[g];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int g = 4 * w + q;
    float v = lds[(0 * 16 + g) * 64 + lane];
    v += lds[(1 * 16 + g) * 64 + lane];
    v += lds[(2 * 16 + g) * 64 + lane];
    v += lds[(3 * 16 + g) * 64 + lane];
    epi((g & 3) + 8 * (g >> 2) + 4 * (lane >> 5), lane & 31, v);
  }
}

// Σ_j x[j] w[j] over the row, split between the lane and its partner lane ^ 32 (halves of j);
// both lanes return the same value (the two halves added in one order: lower half + upper half)
__device__ __forceinline__ float row_dot(const float* __restrict__ x, const float* __restrict__ w, int H) {
  const int h = (threadIdx.x >> 5) & 1, half = H / 2;
  float s = 0.0f;
  for (int j = h * half; j < (h + 1) * half; ++j) s = fmaf(x[j], w[j], s);  // w: flat params, not 16-B aligned
  const float o = __shfl_xor(s, 32, 64);
  return h ? o + s : s + o;
}

// one batch item (replay sample or given batch) and its two reparameterisation normals
__device__ __forceinline__ int64_t batch_item(const MArgs& a, int r, float& e0, float& e1) {
  int64_t idx = r;
  uint32_t c[4] = {(uint32_t)r, (uint32_t)*a.step, (uint32_t)((uint64_t)*a.step >> 32), 0x5AC0u};
  if (a.sampled || !a.eps) philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
  if (a.sampled) {
    const int64_t size = *a.size_dev > 0 ? *a.size_dev : 1;
    const double u = ((double)c[0] + 0.5) * (1.0 / 4294967296.0);
    idx = (int64_t)(u * (double)size);
    if (idx >= a.capacity) idx = a.capacity - 1;
  }
  if (a.eps) {
    e0 = a.eps[r];
    e1 = a.eps[a.L.B + r];
  } else {
    const float u1 = ((float)c[1] + 1.0f) * 2.3283064365386963e-10f;
    const float u2 = (float)c[2] * 2.3283064365386963e-10f;
    const float rad = sqrtf(-2.0f * logf(u1));
    e0 = rad * cosf(6.283185307179586f * u2);
    e1 = rad * sinf(6.283185307179586f * u2);
  }
  return idx;
}

// grid (2B / 32, H / 32): rows [0, B) are the obs rows, [B, 2B) the next_obs rows of the batch
__global__ __launch_bounds__(256) void sac_actor_fwd_kernel(MArgs a) {
  __shared__ float lds[4 * 16 * 64];
  const Layout& L = a.L;
  const int H = L.H, O = L.O, B = L.B;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int r0 = blockIdx.x * kTile2, c0 = blockIdx.y * kTile2;
  const int row = r0 + (lane & 31);
  const bool nrow = row >= B;
  const int item = nrow ? row - B : row;
  float e0, e1;
  const int64_t idx = batch_item(a, item, e0, e1);
  const float* src = nrow ? a.nobs : a.obs;
  float x[kXLd];
#pragma unroll
  for (int m = 0; m < kXLd; ++m) x[m] = m < O ? src[idx * O + m] : 0.0f;
  if (blockIdx.y == 0 && w == 0 && h == 0) {  // the gathered batch for the later kernels
    float* xd = (nrow ? a.ms.xn : a.ms.x) + (int64_t)item * kXLd;
    for (int m = 0; m < kXLd; ++m) xd[m] = x[m];
    if (!nrow) {
      a.ms.act[item] = a.act[idx];
      a.ms.rew[item] = a.rew[idx];
      a.ms.term[item] = a.term[idx];
      a.ms.eps[item] = e0;
      a.ms.eps[B + item] = e1;
      for (int m = 0; m < kXLd; ++m) a.sc.a_x[(int64_t)item * kXLd + m] = m < O ? x[m] : 0.0f;
    }
  }
  // h1 for this lane's k (fmaf chain from the bias, as fc0 computes it) and the W2ᵀ operand
  const int n2 = H / 8, kb = w * (H / 4) + h * n2;
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < kMaxN2; ++i) {
    if (i >= n2) break;
    const int k = kb + i;
    float acc = P[L.p_b1 + k];
    for (int m = 0; m < O; ++m) acc = fmaf(P[L.p_w1 + (int64_t)k * O + m], x[m], acc);
    av[i] = relu(acc);
    bv[i] = a.T[(int64_t)k * H + c0 + (lane & 31)];
  }
  if (blockIdx.y == 0 && !nrow)
    for (int i = 0; i < n2; ++i) a.sc.a_h1[(int64_t)item * H + kb + i] = av[i];
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const int r = r0 + rr, col = c0 + cc;
    const float y = relu(v + P[L.p_b2 + col]);
    if (r < B) a.sc.a_h2[(int64_t)r * H + col] = y;
    else a.ms.h2n[(int64_t)(r - B) * H + col] = y;
  });
}

// TanhNormal.rsample_and_logprob (distributions.py:346-392) of one row's head
__device__ __forceinline__ void tanh_normal(float mean, float ls_raw, float eps, float out[6]) {
  const float log_std = fminf(fmaxf(ls_raw, -20.0f), 2.0f);
  const float std = expf(log_std);
  const float z = mean + std * eps;
  const float act = tanhf(z);
  const float var = std * std;
  const float d = z - mean;
  const float lp = -(d * d) / (2.0f * var) - logf(std) - kLogSqrt2Pi;
  const float corr = -2.0f * (kLog2 - z - softplus(-2.0f * z));
  out[HD_MEAN] = mean; out[HD_LSRAW] = ls_raw; out[HD_STD] = std; out[HD_Z] = z; out[HD_A] = act;
  out[HD_LOGP] = lp + corr;
}

// grid (row tiles of [Q1: 2B | Q2: 2B | T1: B | T2: B], H / 32). Q rows [0, B): (obs, ã), [B, 2B): (obs, a)
__global__ __launch_bounds__(256) void sac_critic_fwd_kernel(MArgs a) {
  __shared__ float lds[4 * 16 * 64];
  const Layout& L = a.L;
  const int H = L.H, O = L.O, B = L.B;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int qt = 2 * B / kTile2, tt = B / kTile2;  // row tiles per critic / per target critic
  int net, rt = blockIdx.x;
  if (rt < 2 * qt) { net = rt / qt; rt %= qt; }
  else { rt -= 2 * qt; net = 2 + rt / tt; rt %= tt; }
  const bool is_t = net >= 2;
  const float* C = is_t ? a.targets + (int64_t)(net - 2) * L.q_size : P + L.q_base[net];
  const int r0 = rt * kTile2, c0 = blockIdx.y * kTile2;
  const int row = r0 + (lane & 31);
  const bool data = !is_t && row >= B;  // (obs, a) row
  const int item = data ? row - B : row;
  const bool store_rows = blockIdx.y == 0 && w == 0 && h == 0;
  // input row: (obs, ã) / (obs, a) / (next_obs, ã')
  const float* xr = (is_t ? a.ms.xn : a.ms.x) + (int64_t)item * kXLd;
  float act;
  if (data) {
    act = a.ms.act[item];
  } else {  // actor head of the row and its sample
    const float* h2 = (is_t ? a.ms.h2n : a.sc.a_h2) + (int64_t)item * H;
    const float mean = row_dot(h2, P + L.p_wm, H) + P[L.p_bm];
    const float ls = row_dot(h2, P + L.p_ws, H) + P[L.p_bs];
    float hd[6];
    tanh_normal(mean, ls, a.ms.eps[(is_t ? B : 0) + item], hd);
    act = hd[HD_A];
    if (store_rows && (net == 0 || net == 2))
      for (int q = 0; q < 6; ++q) (is_t ? a.ms.hdn : a.ms.hd)[q * B + item] = hd[q];
  }
  const int n2 = H / 8, kb = w * (H / 4) + h * n2;
  float av[kMaxN2], bv[kMaxN2];
  const float* WT = a.T + (int64_t)(1 + net) * H * H;  // [q1 | q2 | t1 | t2] W2ᵀ
#pragma unroll
  for (int i = 0; i < kMaxN2; ++i) {
    if (i >= n2) break;
    const int k = kb + i;
    float base = C[L.c_b1 + k];
    for (int m = 0; m < O; ++m) base = fmaf(C[L.c_w1 + (int64_t)k * (O + 1) + m], xr[m], base);
    av[i] = relu(fmaf(C[L.c_w1 + (int64_t)k * (O + 1) + O], act, base));
    bv[i] = WT[(int64_t)k * H + c0 + (lane & 31)];
  }
  if (blockIdx.y == 0 && !is_t) {
    float* g1 = (data ? a.sc.q_g1[net] : a.ms.g1pi[net]) + (int64_t)item * H;
    for (int i = 0; i < n2; ++i) g1[kb + i] = av[i];
    if (data && w == 0 && h == 0)
      for (int m = 0; m < kXLd; ++m) a.sc.q_x[net][(int64_t)item * kXLd + m] = m < O ? xr[m] : (m == O ? act : 0.0f);
  }
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const int r = r0 + rr, col = c0 + cc;
    const float y = relu(v + C[L.c_b2 + col]);
    if (is_t) a.ms.tg2[net - 2][(int64_t)r * H + col] = y;
    else if (r >= B) a.sc.q_g2[net][(int64_t)(r - B) * H + col] = y;
    else a.ms.g2pi[net][(int64_t)r * H + col] = y;
  });
}

// grid (2 critics x 2B / 32 row tiles, H / 32): losses and dq (sac.py:170-247), dg2, dg1 = (dg2 W2) ⊙ [g1 > 0]
__global__ __launch_bounds__(256) void sac_critic_bwd_kernel(MArgs a) {
  __shared__ float lds[4 * 16 * 64];
  const Layout& L = a.L;
  const int H = L.H, B = L.B;
  const float* P = a.params;
  const float* TG = a.targets;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int qt = 2 * B / kTile2;
  const int net = blockIdx.x / qt, rt = blockIdx.x % qt;
  const float* C = P + L.q_base[net];
  const int r0 = rt * kTile2, c0 = blockIdx.y * kTile2;
  const int row = r0 + (lane & 31);
  const bool data = row >= B;
  const int item = data ? row - B : row;
  const bool store_rows = net == 0 && blockIdx.y == 0 && w == 0 && h == 0;
  const float log_alpha = P[0];
  const float alpha = a.hp.auto_ent ? expf(log_alpha) : 1.0f;
  const float invB = 1.0f / (float)B;
  const float* g2row;
  float dq;
  if (data) {  // Q losses on (obs, a)
    const float q1b = row_dot(a.sc.q_g2[0] + (int64_t)item * H, P + L.q_base[0] + L.c_w3, H) + P[L.q_base[0] + L.c_b3];
    const float q2b = row_dot(a.sc.q_g2[1] + (int64_t)item * H, P + L.q_base[1] + L.c_w3, H) + P[L.q_base[1] + L.c_b3];
    const float t1 = row_dot(a.ms.tg2[0] + (int64_t)item * H, TG + L.c_w3, H) + TG[L.c_b3];
    const float t2 = row_dot(a.ms.tg2[1] + (int64_t)item * H, TG + L.q_size + L.c_w3, H) + TG[L.q_size + L.c_b3];
    const float tq = fminf(t1, t2) - alpha * a.ms.hdn[HD_LOGP * B + item];
    float qtv = a.hp.rscale * a.ms.rew[item] + ((1.0f - a.ms.term[item]) * a.hp.gamma) * tq;
    qtv = fminf(fmaxf(qtv, -a.hp.clip), a.hp.clip);
    const float dq1b = (2.0f * invB) * (q1b - qtv), dq2b = (2.0f * invB) * (q2b - qtv);
    dq = net == 0 ? dq1b : dq2b;
    g2row = a.sc.q_g2[net] + (int64_t)item * H;
    if (store_rows) {
      a.sc.q_dq[0][item] = dq1b;
      a.sc.q_dq[1][item] = dq2b;
      a.sc.p_q1l[item] = (q1b - qtv) * (q1b - qtv);
      a.sc.p_q2l[item] = (q2b - qtv) * (q2b - qtv);
      float* st = a.stats + 8;
      st[item] = q1b;
      st[B + item] = q2b;
      st[2 * B + item] = qtv;
    }
  } else {  // policy loss through min(Q1, Q2)(obs, ã)
    const float q1a = row_dot(a.ms.g2pi[0] + (int64_t)item * H, P + L.q_base[0] + L.c_w3, H) + P[L.q_base[0] + L.c_b3];
    const float q2a = row_dot(a.ms.g2pi[1] + (int64_t)item * H, P + L.q_base[1] + L.c_w3, H) + P[L.q_base[1] + L.c_b3];
    const float w1 = (q1a < q2a) ? 1.0f : ((q1a == q2a) ? 0.5f : 0.0f);
    dq = net == 0 ? -w1 * invB : -(1.0f - w1) * invB;
    g2row = a.ms.g2pi[net] + (int64_t)item * H;
    if (store_rows) {
      const float logp = a.ms.hd[HD_LOGP * B + item], act = a.ms.hd[HD_A * B + item];
      const float qmin = fminf(q1a, q2a);
      a.sc.p_pl[item] = alpha * logp - qmin + (a.hp.areg != 0.0f ? a.hp.areg * (act * act) : 0.0f);
      a.sc.p_la[item] = -(log_alpha * (logp + a.hp.tent));
      a.sc.p_ga[item] = -(logp + a.hp.tent);
      float* st = a.stats + 8;
      st[3 * B + item] = logp;
      st[4 * B + item] = tanhf(a.ms.hd[HD_MEAN * B + item]);
      st[5 * B + item] = a.ms.hd[HD_STD * B + item];
    }
  }
  const int n2 = H / 8, kb = w * (H / 4) + h * n2;
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < kMaxN2; ++i) {
    if (i >= n2) break;
    const int j = kb + i;
    const float g2 = g2row[j];
    av[i] = g2 > 0.0f ? dq * C[L.c_w3 + j] : 0.0f;
    bv[i] = C[L.c_w2 + (int64_t)j * H + c0 + (lane & 31)];
  }
  if (data && blockIdx.y == 0)
    for (int i = 0; i < n2; ++i) a.sc.q_dg2[net][(int64_t)item * H + kb + i] = av[i];
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const int r = r0 + rr, col = c0 + cc;
    if (r >= B) {
      const int64_t o = (int64_t)(r - B) * H + col;
      a.sc.q_dg1[net][o] = a.sc.q_g1[net][o] > 0.0f ? v : 0.0f;
    } else {
      const int64_t o = (int64_t)r * H + col;
      a.ms.dg1pi[net][o] = a.ms.g1pi[net][o] > 0.0f ? v : 0.0f;
    }
  });
}

// grid (B / 32, H / 32): policy backward through the action (obs rows)
__global__ __launch_bounds__(256) void sac_actor_bwd_kernel(MArgs a) {
  __shared__ float lds[4 * 16 * 64];
  const Layout& L = a.L;
  const int H = L.H, O = L.O, B = L.B;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int r0 = blockIdx.x * kTile2, c0 = blockIdx.y * kTile2;
  const int item = r0 + (lane & 31);
  const float log_alpha = P[0];
  const float alpha = a.hp.auto_ent ? expf(log_alpha) : 1.0f;
  const float invB = 1.0f / (float)B;
  // dA = Σ_m wa1[m] dg1_Q1[m] + Σ_m wa2[m] dg1_Q2[m] (wa: the action column of each critic's fc0)
  float dA;
  {
    const int half = H / 2;
    float s[2] = {0.0f, 0.0f};
    for (int k = 0; k < 2; ++k) {
      const float* dg = a.ms.dg1pi[k] + (int64_t)item * H;
      const float* C = P + L.q_base[k];
      for (int m = h * half; m < (h + 1) * half; ++m) s[k] = fmaf(C[L.c_w1 + (int64_t)m * (O + 1) + O], dg[m], s[k]);
      const float o = __shfl_xor(s[k], 32, 64);
      s[k] = h ? o + s[k] : s[k] + o;
    }
    dA = s[0] + s[1];
  }
  const float act = a.ms.hd[HD_A * B + item], z = a.ms.hd[HD_Z * B + item], mean = a.ms.hd[HD_MEAN * B + item];
  const float std = a.ms.hd[HD_STD * B + item], ls_raw = a.ms.hd[HD_LSRAW * B + item];
  if (a.hp.areg != 0.0f) dA += (a.hp.areg * invB) * (2.0f * act);
  const float ainv = alpha * invB;
  const float d = z - mean, var = std * std;
  const float sig = 1.0f / (1.0f + expf(2.0f * z));  // sigmoid(-2z)
  const float gz = dA * (1.0f - act * act) + ainv * (-(d / var) + (2.0f - 4.0f * sig));
  const float dmean = gz + ainv * (d / var);
  const float dstd = gz * a.ms.eps[item] + ainv * ((d * d) / (var * std) - 1.0f / std);
  const float dls = (ls_raw >= -20.0f && ls_raw <= 2.0f) ? dstd * std : 0.0f;
  if (blockIdx.y == 0 && w == 0 && h == 0) {
    a.sc.a_dhead[(int64_t)item * 2] = dmean;
    a.sc.a_dhead[(int64_t)item * 2 + 1] = dls;
  }
  const int n2 = H / 8, kb = w * (H / 4) + h * n2;
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < kMaxN2; ++i) {
    if (i >= n2) break;
    const int j = kb + i;
    const float h2 = a.sc.a_h2[(int64_t)item * H + j];
    av[i] = h2 > 0.0f ? (P[L.p_wm + j] * dmean + P[L.p_ws + j] * dls) : 0.0f;
    bv[i] = P[L.p_w2 + (int64_t)j * H + c0 + (lane & 31)];
  }
  if (blockIdx.y == 0)
    for (int i = 0; i < n2; ++i) a.sc.a_dh2[(int64_t)item * H + kb + i] = av[i];
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const int64_t o = (int64_t)(r0 + rr) * H + c0 + cc;
    a.sc.a_dh1[o] = a.sc.a_h1[o] > 0.0f ? v : 0.0f;
  });
}

// weight gradients into the flat gradient: out[j][k] = Σ_r dY[r][j] X[r][k] (X null: ones -> bias).
// Blocks [0, n_mfma): 32 x 32 tiles of the H x H matrices on MFMA (rows split over the 4 waves);
// then VALU blocks, one output element per thread (rows summed in order); the last block: the loss
// scalars, d(log α), α, the Adam bias corrections of this step and step += 1.
struct WgArgs {
  GMat mats[kMaxMats];
  int n_mats;
  int big[3];        // indices of the H x H matrices in mats
  int n_mfma;        // MFMA tile blocks
  int n_small;       // elements of the other matrices
  int small_mat[kMaxMats];
  int64_t small_start[kMaxMats + 1];  // prefix sums of M·N over the non-big matrices
  int n_small_mats;
  float* grads;
  int B;
  Scratch sc;
  const float* params;
  int64_t* step;
  float* stats;
  Hyper hp;
};

__global__ __launch_bounds__(256) void sac_wgrad_mfma_kernel(WgArgs a) {
  __shared__ float lds[4 * 16 * 64];
  const int tid = threadIdx.x;
  const int n_small_blocks = (a.n_small + 255) / 256;
  if ((int)blockIdx.x == a.n_mfma + n_small_blocks) {  // scalars
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
      const double t = (double)step;
      const double bc1 = 1.0 - pow((double)a.hp.beta1, t);
      const double bc2 = 1.0 - pow((double)a.hp.beta2, t);
      a.stats[5] = (float)(a.hp.lr_pi / bc1);
      a.stats[6] = (float)(a.hp.lr_q / bc1);
      a.stats[7] = (float)sqrt(bc2);
    }
    return;
  }
  if ((int)blockIdx.x >= a.n_mfma) {  // VALU elements
    const int64_t e = (int64_t)(blockIdx.x - a.n_mfma) * 256 + tid;
    if (e >= a.n_small) return;
    int s = 0;
    while (s + 1 < a.n_small_mats && e >= a.small_start[s + 1]) ++s;
    const GMat m = a.mats[a.small_mat[s]];
    const int64_t l = e - a.small_start[s];
    const int j = (int)(l / m.N), k = (int)(l % m.N);
    float acc = 0.0f;
    for (int r = 0; r < a.B; ++r) {
      const float x = m.X ? m.X[(int64_t)r * m.ldX + k] : 1.0f;
      acc = fmaf(m.dY[(int64_t)r * m.ldY + j], x, acc);
    }
    a.grads[m.out_off + l] = acc;
    return;
  }
  // MFMA tile of an H x H matrix: A[j][r] = dY[r][j], B[r][k] = X[r][k]
  const int H = a.mats[a.big[0]].M;
  const int tiles = (H / kTile2) * (H / kTile2);
  const GMat m = a.mats[a.big[blockIdx.x / tiles]];
  const int t = blockIdx.x % tiles;
  const int j0 = (t / (H / kTile2)) * kTile2, k0 = (t % (H / kTile2)) * kTile2;
  const int w = tid >> 6, lane = tid & 63, h = lane >> 5;
  const int rows_w = a.B / 4;  // this wave's rows, in chunks of up to 64 (32 MFMAs)
  f32x16 acc = zero16();
  for (int rc = 0; rc < rows_w; rc += 2 * kMaxN2) {
    const int n2 = min(kMaxN2, (rows_w - rc) / 2), rb = w * rows_w + rc + h * n2;
    float av[kMaxN2], bv[kMaxN2];
#pragma unroll
    for (int i = 0; i < kMaxN2; ++i) {
      if (i >= n2) break;
      const int64_t r = rb + i;
      av[i] = m.dY[r * m.ldY + j0 + (lane & 31)];
      bv[i] = m.X[r * m.ldX + k0 + (lane & 31)];
    }
    mfma_chain(acc, av, bv, n2);
  }
  splitk_finish(acc, lds, [&](int rr, int cc, float v) { a.grads[m.out_off + (int64_t)(j0 + rr) * m.N + k0 + cc] = v; });
}


// ---------------------------------------------------------------------------------------------
// Adam (torch.optim.Adam, amsgrad=False, no weight decay) + soft target update + transposes
// ---------------------------------------------------------------------------------------------
struct ApplyArgs {
  float* params;
  float* targets;
  float* grads;
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

// one element: gradient (the flat gradient, all-reduced when data parallel), torch.optim.Adam, soft update
__device__ __forceinline__ float adam_elem(const ApplyArgs& a, const AdamStep& st, int64_t e, float* tp_out) {
  const Layout& L = a.L;
  float g = a.grads[e];
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
  MScratch ms;
  WgArgs wg;
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
  if (O < 1 || O + 1 > kXLd || H < 32 || H > SACF_MAX_HIDDEN || H % 32 || B < kTile2 || B % kTile2 || B > 1024 ||
      cfg->world_size < 1)
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
  // scratch: actor 4·B·H + B·16 + 2B; critics 2·(4·B·H + B·16 + B); per-row losses 5B;
  // MFMA path: batch 2·B·16 + 5B, h2n B·H, heads 12B, (g1, g2, dg1) on (obs, ã) 6·B·H, targets 2·B·H
  const int64_t BH = (int64_t)B * H;
  const int64_t n_scr = 4 * BH + B * kXLd + 2 * B + 2 * (4 * BH + B * kXLd + B) + 5 * B +
                        2 * B * kXLd + 5 * B + BH + 12 * B + 6 * BH + 2 * BH;
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
  MScratch& ms = h->ms;
  ms.x = s; s += B * kXLd;
  ms.xn = s; s += B * kXLd;
  ms.act = s; s += B;
  ms.rew = s; s += B;
  ms.term = s; s += B;
  ms.eps = s; s += 2 * B;
  ms.h2n = s; s += BH;
  ms.hd = s; s += 6 * B;
  ms.hdn = s; s += 6 * B;
  for (int k = 0; k < 2; ++k) {
    ms.g1pi[k] = s; s += BH;
    ms.g2pi[k] = s; s += BH;
    ms.dg1pi[k] = s; s += BH;
    ms.tg2[k] = s; s += BH;
  }
  e = hipMalloc(&h->T, sizeof(float) * 5 * (size_t)H * H);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "hipMalloc(T): %s", hipGetErrorString(e));
  }
  // weight-gradient matrices: the three H x H ones on MFMA tiles, the rest one element per thread
  WgArgs& wg = h->wg;
  memset(&wg, 0, sizeof(wg));
  int nm = 0;
  auto add = [&](const float* dY, int ldY, const float* X, int ldX, int M, int N, int64_t off) {
    wg.mats[nm++] = GMat{dY, X, ldY, ldX, M, N, off};
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
  wg.n_mats = nm;
  int nb = 0;
  wg.n_small_mats = 0;
  wg.small_start[0] = 0;
  for (int mi = 0; mi < nm; ++mi) {
    const GMat& m = wg.mats[mi];
    if (m.M == H && m.N == H && m.X) {
      wg.big[nb++] = mi;
    } else {
      wg.small_mat[wg.n_small_mats] = mi;
      wg.small_start[wg.n_small_mats + 1] = wg.small_start[wg.n_small_mats] + (int64_t)m.M * m.N;
      wg.n_small_mats++;
    }
  }
  wg.n_small = (int)wg.small_start[wg.n_small_mats];
  wg.n_mfma = nb * (H / kTile2) * (H / kTile2);
  wg.B = B;
  wg.sc = sc;
  wg.hp = h->hp;
  *out = h;
  return SACF_OK;
}

int sacf_destroy(sacf_handle* h) {
  if (!h) return SACF_OK;
  SDev g(h->device);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->T) (void)hipFree(h->T);
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
  MArgs a;
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
  a.ms = h->ms;
  a.L = h->L;
  a.hp = h->hp;
  const int B = h->L.B, H = h->L.H, ct = H / kTile2;
  SDev g(h->device);
  hipLaunchKernelGGL(sac_actor_fwd_kernel, dim3(2 * B / kTile2, ct), dim3(256), 0, h->stream, a);
  hipLaunchKernelGGL(sac_critic_fwd_kernel, dim3(6 * B / kTile2, ct), dim3(256), 0, h->stream, a);
  hipLaunchKernelGGL(sac_critic_bwd_kernel, dim3(4 * B / kTile2, ct), dim3(256), 0, h->stream, a);
  hipLaunchKernelGGL(sac_actor_bwd_kernel, dim3(B / kTile2, ct), dim3(256), 0, h->stream, a);
  WgArgs& w = h->wg;
  w.grads = h->grads;
  w.params = h->params;
  w.step = h->step;
  w.stats = h->stats;
  hipLaunchKernelGGL(sac_wgrad_mfma_kernel, dim3(w.n_mfma + (w.n_small + 255) / 256 + 1), dim3(256), 0, h->stream, w);
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
