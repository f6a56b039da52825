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
#include <type_traits>
#include <string.h>

#include <new>
#include <vector>

#include "sac_fused.h"

namespace {

constexpr int kThreads = 256;

#ifdef SACF_PHASE_TIMING
// timing build only (scripts/build_timing.sh): wall-clock stamps of block (0, 0) thread 0 at phase
// boundaries, each after waiting for that wave's outstanding memory operations
__device__ unsigned long long g_sac_stamp[64];
__device__ unsigned long long g_wg_blk[3 * 1024];  // weight-gradient pass: per block start, end, XCC id
__device__ unsigned long long g_wg_wave[1024 * 4 * 4];  // ... per block, wave, stage (MFMA tiles)
#define SAC_WAVE(bx, k)                                                                              \
  do {                                                                                              \
    if ((threadIdx.x & 63) == 0 && (bx) < 1024) {                                                   \
      __builtin_amdgcn_s_waitcnt(0);                                                                \
      g_wg_wave[((bx) * 4 + (threadIdx.x >> 6)) * 4 + (k)] = wall_clock64();                         \
    }                                                                                               \
  } while (0)
#define SAC_TB(kern, k, cond)                                    \
  do {                                                           \
    if ((cond) && threadIdx.x == 0) {                            \
      __builtin_amdgcn_s_waitcnt(0);                             \
      g_sac_stamp[(kern) * 12 + (k)] = wall_clock64();           \
    }                                                            \
  } while (0)
#else
#define SAC_TB(kern, k, cond) \
  do {                        \
  } while (0)
#endif
#ifndef SACF_PHASE_TIMING
#define SAC_WAVE(bx, k) \
  do {                  \
  } while (0)
#endif
#define SAC_T(kern, k) SAC_TB(kern, k, blockIdx.x == 0 && blockIdx.y == 0)
#ifdef SACF_PHASE_TIMING
// every block: earliest start (slot 9) and latest end (slot 10) of the kernel, via vector atomics
#define SAC_SPAN_BEGIN(kern)                                                                  \
  if (threadIdx.x == 0) atomicMin(&g_sac_stamp[(kern) * 12 + 9], (unsigned long long)wall_clock64())
#define SAC_SPAN_END(kern)                                                                    \
  if (threadIdx.x == 0) {                                                                     \
    const unsigned long long t_ = (unsigned long long)wall_clock64();                        \
    atomicMax(&g_sac_stamp[(kern) * 12 + 10], t_);                                            \
    atomicMax(&g_sac_stamp[(kern) * 12 + 11], (t_ << 12) | (blockIdx.x & 4095));             \
  }
#else
#define SAC_SPAN_BEGIN(kern)
#define SAC_SPAN_END(kern)
#endif

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

// Adam bias corrections of step t (torch.optim.Adam: step_size = lr / (1 - beta1^t), denominator
// sqrt(v) / sqrt(1 - beta2^t) + eps), in double as torch computes them on the host, then rounded once
struct AdamStep {
  float step_pi, step_q, bc2_sqrt;
};
__device__ __forceinline__ AdamStep adam_step(const Hyper& hp, int64_t step) {
  const double t = (double)step;
  const double bc1 = 1.0 - pow((double)hp.beta1, t);
  const double bc2 = 1.0 - pow((double)hp.beta2, t);
  return AdamStep{(float)(hp.lr_pi / bc1), (float)(hp.lr_q / bc1), (float)sqrt(bc2)};
}

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
// a pointer read from LDS has no address space for the compiler (flat loads, which also count on the
// LDS counter and get conservative waits): these matrices are all device memory
typedef const float __attribute__((address_space(1)))* gptr;
__device__ __forceinline__ gptr as_global(const float* p) { return (gptr)p; }

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
//   sac_actor_fwd_kernel  : batch gather (replay sampling), h1 (VALU), h2 = relu(h1 W2ᵀ + b2) on 2B rows;
//                           beside them the critics' (obs, a) row tiles of critic_fwd (SACF_EARLY_DATA)
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
  // per-row dot products of a layer output with a head weight vector, one partial per 32-column
  // block (the epilogue of the tile that produced those columns), summed in block order by the consumer
  // (row-major per row: a consumer's CB parts of one row are contiguous, float4 loads when CB % 4 == 0)
  float *hpart;  // actor heads: [2B][mean | log_std][H/32] over the obs and next_obs rows
  float *qpart;  // critic heads g2 · w3: [Q1 | Q2 | T1 | T2][2B][H/32] (targets: rows [0, B))
  float *apart;  // dg1 · (fc0 action column) on the (obs, ã) rows: [Q1 | Q2][B][H/32]
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
__device__ __forceinline__ void splitk_finish_q(const f32x16& acc, float* lds, EPI&& epi) {
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
    epi(q, (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5), lane & 31, v);
  }
}

template <class EPI>
__device__ __forceinline__ void splitk_finish(const f32x16& acc, float* lds, EPI&& epi) {
  splitk_finish_q(acc, lds, [&](int, int rr, int cc, float v) { epi(rr, cc, v); });
}
// the row of output register q (0..3) of this wave in splitk_finish's order
__device__ __forceinline__ int finish_row(int q) {
  const int g = 4 * (threadIdx.x >> 6) + q;
  return (g & 3) + 8 * (g >> 2) + 4 * ((threadIdx.x & 63) >> 5);
}

// Σ of x over the 32 lanes of this half-wave (the 32 columns of one output row in the C/D layout),
// butterfly order: every lane gets the same bits
__device__ __forceinline__ float halfwave_sum(float x) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Σ over the CB column blocks of one row's head partials (block order), from part[cb * stride + row]
// (unrolled: the CB loads are in flight together)
template <int CB>
__device__ __forceinline__ float sum_parts(const float* part, int64_t stride, int64_t row) {
  float v[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) v[cb] = part[cb * stride + row];
  float s = v[0];
#pragma unroll
  for (int cb = 1; cb < CB; ++cb) s += v[cb];
  return s;
}

// n (compile-time) contiguous floats from p, 16-byte aligned when n % 4 == 0: float4 loads then (fewer
// vector-memory instructions in flight: a wave stalls issuing its 64th outstanding load)
template <int N>
__device__ __forceinline__ void load_run(const float* p, float (&v)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const float4 x = reinterpret_cast<const float4*>(p)[q];
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = p[i];
  }
}

// a contiguous run of n floats of the parameters into LDS (the block's first-layer weights)
__device__ __forceinline__ void stage(float* dst, const float* src, int n) {
  for (int e = threadIdx.x; e < n; e += kThreads) dst[e] = src[e];
}

// W1 [H][nin] (row-major in the parameters) into LDS as W1ᵀ [nin][H], and b1 [H] after it. Every
// thread issues all its loads before its first LDS store (a load-store loop would wait on each load
// in turn); element e = tid + 256 i sits at row e / nin, column e % nin, kept incrementally.
template <int H>
__device__ __forceinline__ void stage_w1t(float* dst, const float* w1, const float* b1, int nin) {
  constexpr int kIt = (H * kXLd + kThreads - 1) / kThreads;
  const int n = H * nin, tid = threadIdx.x;
  float v[kIt];
#pragma unroll
  for (int i = 0; i < kIt; ++i) v[i] = tid + i * kThreads < n ? w1[tid + i * kThreads] : 0.0f;
  const float bb = tid < H ? b1[tid] : 0.0f;
  int q = tid / nin, r = tid - q * nin;
  const int dq = kThreads / nin, dr = kThreads - dq * nin;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    if (tid + i * kThreads < n) dst[r * H + q] = v[i];
    q += dq;
    r += dr;
    if (r >= nin) {
      r -= nin;
      ++q;
    }
  }
  if (tid < H) dst[nin * H + tid] = bb;
}

// av[i] = relu(b1[k] + Σ_{m < nin} W1[k][m] · in[m]) for k = kb + i: an fmaf chain from the bias in
// input order, as fc0 computes one output. W1ᵀ | b1 and the row's inputs come from LDS; the input loop
// stays rolled (nin is a run-time size) around the unrolled k loop.
template <int H>
__device__ __forceinline__ void first_layer(const float* lw1t, const float* xin, int nin, int kb, float (&av)[kMaxN2]) {
  constexpr int n2 = H / 8;
#pragma unroll
  for (int i = 0; i < n2; ++i) av[i] = lw1t[nin * H + kb + i];
  for (int m = 0; m < nin; ++m) {
    const float xm = xin[m];
#pragma unroll
    for (int i = 0; i < n2; ++i) av[i] = fmaf(lw1t[m * H + kb + i], xm, av[i]);
  }
#pragma unroll
  for (int i = 0; i < n2; ++i) av[i] = relu(av[i]);
}

// LDS of the forward/backward kernels. Region A: split-K partial tiles / a 32-row
// tile of this lane-per-row operand layout. Region B: first-layer weights (W1ᵀ | b1) and the tile's
// input rows (forward kernels), or a 32-row activation tile and head weights (backward kernels).
constexpr int kLdsSplit = 4 * 16 * 64;
constexpr int kTileLd = SACF_MAX_HIDDEN + 4;  // row pitch bound of a 32-row tile (H + 4 floats)
constexpr int kLdsTile = 32 * kTileLd;
constexpr int kLdsA = kLdsSplit > kLdsTile ? kLdsSplit : kLdsTile;
constexpr int kLdsW1 = SACF_MAX_HIDDEN * kXLd + SACF_MAX_HIDDEN;
constexpr int kLdsX = 32 * (kXLd + 1);
constexpr int kLdsB = (kLdsW1 + kLdsX > kLdsTile + 2 * SACF_MAX_HIDDEN) ? kLdsW1 + kLdsX : kLdsTile + 2 * SACF_MAX_HIDDEN;
constexpr int kLdsFloats = kLdsA + kLdsB;
constexpr int kLdsW1Off = kLdsA;
constexpr int kLdsXOff = kLdsA + kLdsW1;
constexpr int kLdsTileOff = kLdsA;
constexpr int kLdsHeadWOff = kLdsA + kLdsTile;

// 32 consecutive rows of a row-major [*][H] activation matrix -> an LDS tile of pitch H + 4, in
// float4 pieces (coalesced: a wave moves whole 1 KiB rows). The MFMA A operand wants one row per lane
// (lane & 31), which read straight from the matrix would touch 32 rows per instruction.
template <int H>
__device__ __forceinline__ void tile_load(float* t, const float* src) {
  constexpr int C4 = H / 4, kIt = (32 * C4 + kThreads - 1) / kThreads;
  constexpr bool kFull = (32 * C4) % kThreads == 0;
  float vx[kIt], vy[kIt], vz[kIt], vw[kIt];  // every load in flight before the first LDS store
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int e = threadIdx.x + i * kThreads, r = e / C4, c = e % C4;
    float4 x = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (kFull || e < 32 * C4) x = *reinterpret_cast<const float4*>(src + (int64_t)r * H + 4 * c);
    vx[i] = x.x; vy[i] = x.y; vz[i] = x.z; vw[i] = x.w;
  }
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int e = threadIdx.x + i * kThreads, r = e / C4, c = e % C4;
    if (kFull || e < 32 * C4) *reinterpret_cast<float4*>(t + r * (H + 4) + 4 * c) = make_float4(vx[i], vy[i], vz[i], vw[i]);
  }
}

// this lane's operands (row lane & 31, columns kb .. kb + H/8) straight to its row of the matrix, by the
// column block whose columns they are (kb / 32 == by): float4 stores, no LDS staging or block barrier,
// and the rows' stores spread over the column blocks instead of delaying block column 0
template <int H>
__device__ __forceinline__ void store_slice(float* base, int r0, int by, const float (&av)[kMaxN2], int kb) {
  constexpr int n2 = H / 8;
  if (kb / kTile2 != by) return;
  float4* d = reinterpret_cast<float4*>(base + (int64_t)(r0 + (threadIdx.x & 31)) * H + kb);
#pragma unroll
  for (int q = 0; q < n2 / 4; ++q) d[q] = make_float4(av[4 * q], av[4 * q + 1], av[4 * q + 2], av[4 * q + 3]);
}
// XCD-aware block -> tile map of the forward/backward grids (gx row tiles x H/32 column tiles). The hardware
// deals consecutive blocks round-robin over the 8 XCDs, each with its own L2; every block of one column tile
// reads that column's 32 KB weight slice. With 8 column tiles (H = 256), column tile = linear block id mod 8
// puts them all on one XCD, which then brings only its slice into its L2 instead of all eight (fabric
// traffic / 8). Any placement gives the same results (the map is a bijection of the same grid).
template <int H>
__device__ __forceinline__ void xcd_tile(int& bx, int& by) {
  if constexpr (H / kTile2 == 8) {
    const int L = (int)(blockIdx.x + blockIdx.y * gridDim.x);
    by = L & 7;
    bx = L >> 3;
  } else {
    bx = (int)blockIdx.x;
    by = (int)blockIdx.y;
  }
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
template <int H>
__device__ __forceinline__ void actor_fwd_tile(const MArgs& a, int bx, int by, float* lds) {
  SAC_T(0, 0);
  SAC_SPAN_BEGIN(0);
  const Layout& L = a.L;
  const int O = L.O, B = L.B;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int r0 = bx * kTile2, c0 = by * kTile2;
  constexpr int n2 = H / 8;
  const int kb = w * (H / 4) + h * n2;
  // the batch gather first: its chain (step / size -> Philox -> replay row) is the longest of the
  // prologue, and vector loads complete in issue order, so the staging loads queue behind it
  const int row = r0 + (lane & 31);
  const bool nrow = row >= B;
  const int item = nrow ? row - B : row;
  float e0, e1;
  const int64_t idx = batch_item(a, item, e0, e1);
  const float* src = nrow ? a.nobs : a.obs;
  float x[kXLd];
#pragma unroll
  for (int m = 0; m < kXLd; ++m) x[m] = m < O ? src[idx * O + m] : 0.0f;
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < n2; ++i) bv[i] = a.T[(int64_t)(kb + i) * H + c0 + (lane & 31)];  // W2ᵀ operand
  // the epilogue's per-column operands, in flight with the rest (one column per lane)
  const float b2c = P[L.p_b2 + c0 + (lane & 31)];
  const float wm = P[L.p_wm + c0 + (lane & 31)], ws = P[L.p_ws + c0 + (lane & 31)];
  float* lw1 = lds + kLdsW1Off;  // W1ᵀ [O][H] | b1 [H]
  float* lx = lds + kLdsXOff;    // the tile's input rows [32][kXLd + 1]
  stage_w1t<H>(lw1, P + L.p_w1, P + L.p_b1, O);
  if (w == 0 && h == 0)
    for (int m = 0; m < O; ++m) lx[(lane & 31) * (kXLd + 1) + m] = x[m];
  if (by == 0 && w == 0 && h == 0) {  // the gathered batch for the later kernels
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
  SAC_T(0, 1);
  __syncthreads();  // lw1 staged
  SAC_T(0, 2);
  // h1 for this lane's k (fmaf chain from the bias, as fc0 computes it)
  first_layer<H>(lw1, lx + (lane & 31) * (kXLd + 1), O, kb, av);
  if (r0 < B) store_slice<H>(a.sc.a_h1, r0, by, av, kb);
  SAC_T(0, 3);
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  SAC_T(0, 4);
  constexpr int CB = H / kTile2;
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const int r = r0 + rr, col = c0 + cc;
    const float y = relu(v + b2c);
    if (r < B) a.sc.a_h2[(int64_t)r * H + col] = y;
    else a.ms.h2n[(int64_t)(r - B) * H + col] = y;
    // this column block's part of the mean / log_std heads of row r (rows [0, 2B))
    const float pm = halfwave_sum(y * wm), ps = halfwave_sum(y * ws);
    if (cc == 0) {
      a.ms.hpart[(int64_t)r * 2 * CB + by] = pm;
      a.ms.hpart[(int64_t)r * 2 * CB + CB + by] = ps;
    }
  });
  SAC_T(0, 5);
  SAC_SPAN_END(0);
}


template <int H, bool kGather = false>
__device__ __forceinline__ void critic_fwd_tile(const MArgs& a, int bx, int by, float* lds);

// SACF_EARLY_DATA (default): the critics' (obs, a) row tiles need nothing from the actor forward pass, so they
// run in this launch beside the actor tiles (row tiles [2B/32, 4B/32) of the grid: Q1 then Q2 data rows), and
// the critic_fwd launch keeps only the rows that need the actor head — 2 x 128 blocks at B = 256 instead of
// 128 + 384 (one block per CU in both passes)
#ifndef SACF_EARLY_DATA
#define SACF_EARLY_DATA 1
#endif
template <int H>
__global__ __launch_bounds__(256) void sac_actor_fwd_kernel(MArgs a) {
  __shared__ float lds[kLdsFloats];
  int bx, by;
  xcd_tile<H>(bx, by);
  const int at = 2 * a.L.B / kTile2;
  if (!SACF_EARLY_DATA || bx < at) {
    actor_fwd_tile<H>(a, bx, by, lds);
  } else {
    const int d = bx - at, dt = a.L.B / kTile2;  // data row tile d % dt of critic d / dt
    critic_fwd_tile<H, true>(a, (d / dt) * 2 * dt + dt + d % dt, by, lds);
  }
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
// kGather (a data-row tile run in the actor_fwd launch, SACF_EARLY_DATA): the row's observation and replayed
// action come straight from the replay buffer (the same Philox draw as actor_fwd's gather, so the same values
// as the gathered copies), since the gathered batch is being written by that same launch
template <int H, bool kGather>
__device__ __forceinline__ void critic_fwd_tile(const MArgs& a, int bx, int by, float* lds) {
  SAC_T(1, 0);
  SAC_SPAN_BEGIN(1);
  const Layout& L = a.L;
  const int O = L.O, B = L.B;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int qt = 2 * B / kTile2, tt = B / kTile2;  // row tiles per critic / per target critic
  int net, rt = bx;
  if (rt < 2 * qt) { net = rt / qt; rt %= qt; }
  else { rt -= 2 * qt; net = 2 + rt / tt; rt %= tt; }
  const bool is_t = net >= 2;
  const float* C = is_t ? a.targets + (int64_t)(net - 2) * L.q_size : P + L.q_base[net];
  const int r0 = rt * kTile2, c0 = by * kTile2;
  constexpr int n2 = H / 8;
  constexpr int CB = H / kTile2;
  const int kb = w * (H / 4) + h * n2;
  const int row = r0 + (lane & 31);
  const bool data = !is_t && row >= B;  // (obs, a) row (block-uniform: B is a multiple of 32)
  const int item = data ? row - B : row;
  const bool store_rows = by == 0 && w == 0 && h == 0;
  // the row's inputs first — observation, actor-head partials (or the replayed action), noise — as
  // they end the prologue's longest chain; vector loads complete in issue order, so the staging loads
  // below queue behind them instead of delaying them. Every load is issued unconditionally (the
  // addresses are valid for either row kind) so no branch splits the batch of loads.
  float xin[kXLd];
  float pm[CB], pls[CB];
  float bm = 0.0f, bs = 0.0f, ev = 0.0f, act_data;
  if constexpr (kGather) {  // (data rows only: no actor head)
    float e0, e1;
    const int64_t idx = batch_item(a, item, e0, e1);
#pragma unroll
    for (int m = 0; m < kXLd; ++m) xin[m] = m < O ? a.obs[idx * O + m] : 0.0f;
    act_data = a.act[idx];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) pm[cb] = pls[cb] = 0.0f;
  } else {
    const float* xr = (is_t ? a.ms.xn : a.ms.x) + (int64_t)item * kXLd;
    load_run<kXLd>(xr, xin);
    const int64_t hr = (is_t ? B : 0) + item;
    load_run<CB>(a.ms.hpart + hr * 2 * CB, pm);
    load_run<CB>(a.ms.hpart + hr * 2 * CB + CB, pls);
    bm = P[L.p_bm];
    bs = P[L.p_bs];
    ev = a.ms.eps[(is_t ? B : 0) + item];
    act_data = a.ms.act[item];
  }
  float av[kMaxN2], bv[kMaxN2];
  const float* WT = a.T + (int64_t)(1 + net) * H * H;  // [q1 | q2 | t1 | t2] W2ᵀ
#pragma unroll
  for (int i = 0; i < n2; ++i) bv[i] = WT[(int64_t)(kb + i) * H + c0 + (lane & 31)];
  const float b2c = C[L.c_b2 + c0 + (lane & 31)], w3 = C[L.c_w3 + c0 + (lane & 31)];  // epilogue operands
  SAC_T(1, 6);
  float* lw1 = lds + kLdsW1Off;  // W1ᵀ [O + 1][H] | b1 [H]
  float* lx = lds + kLdsXOff;    // the tile's input rows [32][kXLd + 1]: obs | action
  stage_w1t<H>(lw1, C + L.c_w1, C + L.c_b1, O + 1);
  SAC_T(1, 7);
  float act;
  if (kGather || data) {
    act = act_data;
  } else {  // actor head of the row (the column-block parts of actor_fwd's epilogue, summed in block
            // order as sum_parts does) and its sample
    float sm = pm[0], sl = pls[0];
#pragma unroll
    for (int cb = 1; cb < CB; ++cb) {
      sm += pm[cb];
      sl += pls[cb];
    }
    const float mean = sm + bm;
    const float ls = sl + bs;
    float hd[6];
    SAC_T(1, 8);
    tanh_normal(mean, ls, ev, hd);
    act = hd[HD_A];
    if (store_rows && (net == 0 || net == 2))
      for (int q = 0; q < 6; ++q) (is_t ? a.ms.hdn : a.ms.hd)[q * B + item] = hd[q];
  }
  SAC_T(1, 1);
  // the tile's input rows next to W1ᵀ | b1, both behind one barrier
  if (w == 0 && h == 0) {
#pragma unroll
    for (int m = 0; m < kXLd; ++m)
      if (m < O) lx[(lane & 31) * (kXLd + 1) + m] = xin[m];
    lx[(lane & 31) * (kXLd + 1) + O] = act;
  }
  __syncthreads();  // lw1 and the input rows staged (also when the tile computed no heads)
  SAC_T(1, 2);
  first_layer<H>(lw1, lx + (lane & 31) * (kXLd + 1), O + 1, kb, av);
  if (!is_t) {  // block-uniform
    if (by == 0 && data && w == 0 && h == 0)
#pragma unroll
      for (int m = 0; m < kXLd; ++m) a.sc.q_x[net][(int64_t)item * kXLd + m] = m < O ? xin[m] : (m == O ? act : 0.0f);
    store_slice<H>(data ? a.sc.q_g1[net] : a.ms.g1pi[net], data ? r0 - B : r0, by, av, kb);
  }
  SAC_T(1, 3);
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  SAC_T(1, 4);
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const int r = r0 + rr, col = c0 + cc;
    const float y = relu(v + b2c);
    if (is_t) a.ms.tg2[net - 2][(int64_t)r * H + col] = y;
    else if (r >= B) a.sc.q_g2[net][(int64_t)(r - B) * H + col] = y;
    else a.ms.g2pi[net][(int64_t)r * H + col] = y;
    const float pq = halfwave_sum(y * w3);  // this column block's part of g2 · w3 for row r
    if (cc == 0) a.ms.qpart[((int64_t)net * 2 * B + r) * CB + by] = pq;
  });
  SAC_T(1, 5);
  SAC_SPAN_END(1);
}


template <int H>
__global__ __launch_bounds__(256) void sac_critic_fwd_kernel(MArgs a) {
  __shared__ float lds[kLdsFloats];
  int bx, by;
  xcd_tile<H>(bx, by);
  if (SACF_EARLY_DATA) {  // row tiles: Q1 (obs, ã) | Q2 (obs, ã) | T1 | T2 (the data rows ran with the actor)
    const int dt = a.L.B / kTile2;
    bx = bx < 2 * dt ? (bx / dt) * 2 * dt + bx % dt : bx + 2 * dt;
  }
  critic_fwd_tile<H>(a, bx, by, lds);
}

// SACF_DIRECT_BWD (default): the backward passes read each lane's activation-row segment and head weights straight
// from memory (float4 runs) instead of staging a 32-row tile and the head vectors in LDS behind a block barrier
#ifndef SACF_DIRECT_BWD
#define SACF_DIRECT_BWD 1
#endif
// grid (2 critics x 2B / 32 row tiles, H / 32): losses and dq (sac.py:170-247), dg2, dg1 = (dg2 W2) ⊙ [g1 > 0]
template <int H>
__device__ __forceinline__ void critic_bwd_tile(const MArgs& a, int bx, int by, float* lds) {
  SAC_T(2, 0);
  SAC_SPAN_BEGIN(2);
  const Layout& L = a.L;
  const int B = L.B;
  const float* P = a.params;
  const float* TG = a.targets;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int qt = 2 * B / kTile2;
  if ((int)bx >= 2 * qt) {  // extra blocks (8, keeping the row-tile -> XCD map of the other kernels):
    if (bx == 2 * qt && by == 0 && threadIdx.x == 0) {  // step t and Adam's bias corrections
      const int64_t t = *a.step + 1;            // (only actor_fwd read the old value)
      *const_cast<int64_t*>(a.step) = t;
      const AdamStep st = adam_step(a.hp, t);
      a.stats[5] = st.step_pi;
      a.stats[6] = st.step_q;
      a.stats[7] = st.bc2_sqrt;
    }
    return;
  }
  const int net = bx / qt, rt = bx % qt;
  const float* C = P + L.q_base[net];
  const int r0 = rt * kTile2, c0 = by * kTile2;
  constexpr int n2 = H / 8;
  constexpr int CB = H / kTile2;
  const int kb = w * (H / 4) + h * n2;
  const int row = r0 + (lane & 31);
  const bool data = row >= B;  // (block-uniform: B is a multiple of 32)
  const int item = data ? row - B : row;
  // the row's Q / target-Q head partials and batch terms first: they end the prologue's longest chain
  // and vector loads complete in issue order, so the staging loads below queue behind them. All are
  // issued for both row kinds (valid addresses either way), keeping the batch of loads in one block.
  const float* qp = a.ms.qpart;
  const int64_t qs = (int64_t)CB * 2 * B;  // one net's parts
  const int64_t qrow = data ? B + item : item;
  float q1p[CB], q2p[CB], t1p[CB], t2p[CB];
  load_run<CB>(qp + qrow * CB, q1p);
  load_run<CB>(qp + qs + qrow * CB, q2p);
  load_run<CB>(qp + 2 * qs + (int64_t)item * CB, t1p);
  load_run<CB>(qp + 3 * qs + (int64_t)item * CB, t2p);
  const float bq1 = P[L.q_base[0] + L.c_b3], bq2 = P[L.q_base[1] + L.c_b3];
  const float bt1 = TG[L.c_b3], bt2 = TG[L.q_size + L.c_b3];
  const float logp_n = a.ms.hdn[HD_LOGP * B + item], rew_i = a.ms.rew[item], term_i = a.ms.term[item];
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < n2; ++i) bv[i] = C[L.c_w2 + (int64_t)(kb + i) * H + c0 + (lane & 31)];
  // the epilogue's operands: fc0's action column at this lane's column, and the g1 > 0 masks of the
  // four outputs this lane finishes
  const float wa = C[L.c_w1 + (int64_t)(c0 + (lane & 31)) * (L.O + 1) + L.O];
  float g1m[4];
  {
    const float* g1 = data ? a.sc.q_g1[net] + (int64_t)(r0 - B) * H : a.ms.g1pi[net] + (int64_t)r0 * H;
#pragma unroll
    for (int q = 0; q < 4; ++q) g1m[q] = g1[(int64_t)finish_row(q) * H + c0 + (lane & 31)];
  }
  const bool store_rows = net == 0 && by == 0 && w == 0 && h == 0;
  const float log_alpha = P[0];
  const float alpha = a.hp.auto_ent ? expf(log_alpha) : 1.0f;
  const float invB = 1.0f / (float)B;
  float dq;
  const int ib = data ? r0 - B : r0;  // first batch item of the tile (tiles never straddle B)
  // this lane's g2 row segment and w3 entries (columns kb .. kb + H/8), straight from memory: no LDS staging
  // and no block barrier before the dg2 operand (SACF_DIRECT_BWD)
  float g2v[n2], w3v[n2];
#if SACF_DIRECT_BWD
  load_run<n2>((data ? a.sc.q_g2[net] : a.ms.g2pi[net]) + (int64_t)(ib + (lane & 31)) * H + kb, g2v);
#pragma unroll
  for (int i = 0; i < n2; ++i) w3v[i] = C[L.c_w3 + kb + i];
#else
  float* tg = lds + kLdsTileOff;      // this critic's g2 rows of the tile
  float* lw3 = lds + kLdsHeadWOff;    // this critic's w3
  tile_load<H>(tg, (data ? a.sc.q_g2[net] : a.ms.g2pi[net]) + (int64_t)ib * H);
  stage(lw3, C + L.c_w3, H);
#endif
  // Σ of the column-block parts in block order (sum_parts), then the head bias
  float s_q1 = q1p[0], s_q2 = q2p[0], s_t1 = t1p[0], s_t2 = t2p[0];
#pragma unroll
  for (int cb = 1; cb < CB; ++cb) {
    s_q1 += q1p[cb];
    s_q2 += q2p[cb];
    s_t1 += t1p[cb];
    s_t2 += t2p[cb];
  }
  if (data) {  // Q losses on (obs, a)
    const float q1b = s_q1 + bq1;
    const float q2b = s_q2 + bq2;
    const float t1 = s_t1 + bt1;
    const float t2 = s_t2 + bt2;
    const float tq = fminf(t1, t2) - alpha * logp_n;
    float qtv = a.hp.rscale * rew_i + ((1.0f - term_i) * a.hp.gamma) * tq;
    qtv = fminf(fmaxf(qtv, -a.hp.clip), a.hp.clip);
    const float dq1b = (2.0f * invB) * (q1b - qtv), dq2b = (2.0f * invB) * (q2b - qtv);
    dq = net == 0 ? dq1b : dq2b;
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
    const float q1a = s_q1 + bq1;
    const float q2a = s_q2 + bq2;
    const float w1 = (q1a < q2a) ? 1.0f : ((q1a == q2a) ? 0.5f : 0.0f);
    dq = net == 0 ? -w1 * invB : -(1.0f - w1) * invB;
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
  SAC_T(2, 1);
#if !SACF_DIRECT_BWD
  __syncthreads();  // g2 tile and w3 staged
#pragma unroll
  for (int i = 0; i < n2; ++i) {
    g2v[i] = tg[(lane & 31) * (H + 4) + kb + i];
    w3v[i] = lw3[kb + i];
  }
#endif
#pragma unroll
  for (int i = 0; i < n2; ++i) {
    av[i] = g2v[i] > 0.0f ? dq * w3v[i] : 0.0f;
  }
  if (data) store_slice<H>(a.sc.q_dg2[net], ib, by, av, kb);
  SAC_T(2, 3);
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  SAC_T(2, 4);
  splitk_finish_q(acc, lds, [&](int q, int rr, int cc, float v) {
    const int r = r0 + rr, col = c0 + cc;
    if (r >= B) {
      const int64_t o = (int64_t)(r - B) * H + col;
      a.sc.q_dg1[net][o] = g1m[q] > 0.0f ? v : 0.0f;
    } else {  // (tile-uniform branch: the half-wave sum below runs in every lane)
      const int64_t o = (int64_t)r * H + col;
      const float d = g1m[q] > 0.0f ? v : 0.0f;
      a.ms.dg1pi[net][o] = d;
      const float pa = halfwave_sum(d * wa);  // this column block's part of dQ/dã for row r
      if (cc == 0) a.ms.apart[((int64_t)net * B + r) * CB + by] = pa;
    }
  });
  SAC_T(2, 5);
  SAC_SPAN_END(2);
}


template <int H>
__global__ __launch_bounds__(256) void sac_critic_bwd_kernel(MArgs a) {
  __shared__ float lds[kLdsFloats];
  int bx, by;
  xcd_tile<H>(bx, by);
  critic_bwd_tile<H>(a, bx, by, lds);
}

// grid (B / 32, H / 32): policy backward through the action (obs rows)
template <int H>
__device__ __forceinline__ void actor_bwd_tile(const MArgs& a, int bx, int by, float* lds) {
  SAC_T(3, 0);
  SAC_SPAN_BEGIN(3);
  const Layout& L = a.L;
  const int O = L.O, B = L.B;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int r0 = bx * kTile2, c0 = by * kTile2;
  constexpr int n2 = H / 8;
  constexpr int CB = H / kTile2;
  const int kb = w * (H / 4) + h * n2;
  const int item = r0 + (lane & 31);
  // the row's dQ/dã partials, head and noise first (the prologue's longest chain; vector loads complete
  // in issue order, so the staging loads below queue behind them)
  float ap1[CB], ap2[CB];
  load_run<CB>(a.ms.apart + (int64_t)item * CB, ap1);
  load_run<CB>(a.ms.apart + ((int64_t)B + item) * CB, ap2);
  const float act = a.ms.hd[HD_A * B + item], z = a.ms.hd[HD_Z * B + item], mean = a.ms.hd[HD_MEAN * B + item];
  const float std = a.ms.hd[HD_STD * B + item], ls_raw = a.ms.hd[HD_LSRAW * B + item];
  const float eps_i = a.ms.eps[item];
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < n2; ++i) bv[i] = P[L.p_w2 + (int64_t)(kb + i) * H + c0 + (lane & 31)];
  float h1m[4];  // the h1 > 0 masks of the four outputs this lane finishes
#pragma unroll
  for (int q = 0; q < 4; ++q) h1m[q] = a.sc.a_h1[(int64_t)(r0 + finish_row(q)) * H + c0 + (lane & 31)];
  const float log_alpha = P[0];
  const float alpha = a.hp.auto_ent ? expf(log_alpha) : 1.0f;
  const float invB = 1.0f / (float)B;
  // this lane's h2 row segment and head weights (columns kb .. kb + H/8), straight from memory (SACF_DIRECT_BWD)
  float h2v[n2], wmv[n2], wsv[n2];
#if SACF_DIRECT_BWD
  load_run<n2>(a.sc.a_h2 + (int64_t)(r0 + (lane & 31)) * H + kb, h2v);
#pragma unroll
  for (int i = 0; i < n2; ++i) {
    wmv[i] = P[L.p_wm + kb + i];
    wsv[i] = P[L.p_ws + kb + i];
  }
#else
  float* th = lds + kLdsTileOff;     // actor h2 rows of the tile
  float* lwh = lds + kLdsHeadWOff;   // wm | ws
  tile_load<H>(th, a.sc.a_h2 + (int64_t)r0 * H);
  stage(lwh, P + L.p_wm, H);
  stage(lwh + H, P + L.p_ws, H);
#endif
  // dA = Σ_m wa1[m] dg1_Q1[m] + Σ_m wa2[m] dg1_Q2[m] (wa: the action column of each critic's fc0), each
  // sum over the column-block parts in block order (sum_parts)
  float s1 = ap1[0], s2 = ap2[0];
#pragma unroll
  for (int cb = 1; cb < CB; ++cb) {
    s1 += ap1[cb];
    s2 += ap2[cb];
  }
  float dA = s1 + s2;
  SAC_T(3, 1);
  if (a.hp.areg != 0.0f) dA += (a.hp.areg * invB) * (2.0f * act);
  const float ainv = alpha * invB;
  const float d = z - mean, var = std * std;
  const float sig = 1.0f / (1.0f + expf(2.0f * z));  // sigmoid(-2z)
  const float gz = dA * (1.0f - act * act) + ainv * (-(d / var) + (2.0f - 4.0f * sig));
  const float dmean = gz + ainv * (d / var);
  const float dstd = gz * eps_i + ainv * ((d * d) / (var * std) - 1.0f / std);
  const float dls = (ls_raw >= -20.0f && ls_raw <= 2.0f) ? dstd * std : 0.0f;
  if (by == 0 && w == 0 && h == 0) {
    a.sc.a_dhead[(int64_t)item * 2] = dmean;
    a.sc.a_dhead[(int64_t)item * 2 + 1] = dls;
  }
  SAC_T(3, 2);
#if !SACF_DIRECT_BWD
  __syncthreads();  // h2 tile and head weights staged
#pragma unroll
  for (int i = 0; i < n2; ++i) {
    h2v[i] = th[(lane & 31) * (H + 4) + kb + i];
    wmv[i] = lwh[kb + i];
    wsv[i] = lwh[H + kb + i];
  }
#endif
#pragma unroll
  for (int i = 0; i < n2; ++i) av[i] = h2v[i] > 0.0f ? (wmv[i] * dmean + wsv[i] * dls) : 0.0f;
  store_slice<H>(a.sc.a_dh2, r0, by, av, kb);
  SAC_T(3, 3);
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  SAC_T(3, 4);
  splitk_finish_q(acc, lds, [&](int q, int rr, int cc, float v) {
    const int64_t o = (int64_t)(r0 + rr) * H + c0 + cc;
    a.sc.a_dh1[o] = h1m[q] > 0.0f ? v : 0.0f;
  });
  SAC_T(3, 5);
  SAC_SPAN_END(3);
}


template <int H>
__global__ __launch_bounds__(256) void sac_actor_bwd_kernel(MArgs a) {
  __shared__ float lds[kLdsFloats];
  int bx, by;
  xcd_tile<H>(bx, by);
  actor_bwd_tile<H>(a, bx, by, lds);
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


// one element: gradient (the flat gradient, all-reduced when data parallel), torch.optim.Adam, soft
// update. Loads (ld) and update/stores (st) are split so a thread can put several elements' loads in
// flight before the first update.
struct AdamElem {
  float g, m, v, p, t;
  bool q;
};

// (with_g false: the caller has the gradient in hand — the fused weight-gradient pass)
__device__ __forceinline__ AdamElem adam_ld(const ApplyArgs& a, int64_t e, bool with_g = true) {
  const Layout& L = a.L;
  AdamElem x;
  x.q = e >= L.q_base[0];
  x.g = with_g ? a.grads[e] : 0.0f;
  x.m = a.m[e];
  x.v = a.v[e];
  x.p = a.params[e];
  x.t = x.q ? a.targets[e - L.q_base[0]] : 0.0f;
  return x;
}

__device__ __forceinline__ void adam_st(const ApplyArgs& a, const AdamStep& st, int64_t e, AdamElem& x) {
  const float g = x.g * a.hp.inv_world;
  const float m = x.m + (1.0f - a.hp.beta1) * (g - x.m);         // exp_avg.lerp_(grad, 1 - beta1)
  const float v = x.v * a.hp.beta2 + (1.0f - a.hp.beta2) * (g * g);  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / st.bc2_sqrt + a.hp.eps;
  const float p = x.p + (-(x.q ? st.step_q : st.step_pi)) * (m / denom);
  a.m[e] = m;
  a.v[e] = v;
  a.params[e] = p;
  x.p = p;
  if (x.q) {
    x.t = x.t * (1.0f - a.hp.tau) + p * a.hp.tau;
    a.targets[e - a.L.q_base[0]] = x.t;
  }
}

// weight gradients into the flat gradient: out[j][k] = Σ_r dY[r][j] X[r][k] (X null: ones -> bias).
// Blocks [0, n_mfma): 32 x 32 tiles of the H x H matrices on MFMA (rows split over the 4 waves);
// then VALU blocks, one output element per thread (rows summed in order); the last block: the loss
// scalars, d(log α), α, the Adam bias corrections of this step and step += 1.
// the matrix table lives in device memory (a kernel-argument array indexed by a run-time value would
// be copied to scratch in every thread)
struct WgTable {
  GMat mats[kMaxMats];
  int n_mats;
  int big[3];                         // indices of the H x H matrices in mats
  int big_slot[3];                    // their W2ᵀ slot in T (0 actor, 1 / 2 Q1 / Q2; targets at + 2)
  int has_scalar;                     // the last block reduces the losses and updates log α
  int small_mat[kMaxMats];
  int64_t small_start[kMaxMats + 1];  // prefix sums of M·N over the non-big matrices
  int n_small_mats;
};

struct WgArgs {
  const WgTable* tab;
  int n_mfma;   // MFMA tile blocks
  int n_small;  // elements of the other matrices
  float* grads;
  int B;
  Scratch sc;
  const float* params;
  const int64_t* step;  // this step's number t (critic_fwd advanced it)
  float* stats;
  Hyper hp;
  int n_blocks;  // grid
  int blk0;      // (timing experiments, $SACF_WG_MODE) this launch's first block / block rotation
  int fuse;      // single process: each block also applies Adam / soft update / W2ᵀ to the elements it finished
  ApplyArgs ap;  // (fuse) parameters, optimizer state, targets, transposed copies
};

// the weight-gradient kernel's LDS (also one region of the persistent step kernel's)
struct WgLds {
  float lds[4 * 16 * 64];
  WgTable tab;   // one coalesced copy instead of a chain of dependent global loads
  AdamStep sst;  // this step's Adam bias corrections (critic_bwd wrote them)
  float red[4][32];
  float sum[32];
  float tt[2][kTile][kTile + 1];
};

// the matrix table and this step's Adam bias corrections into LDS (every thread of the block)
__device__ __forceinline__ void wgrad_stage(const WgArgs& a, WgLds& S) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(a.tab);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&S.tab);
  constexpr int kW = (int)(sizeof(WgTable) / 4), kIt = (kW + 255) / 256;
  uint32_t v[kIt];
#pragma unroll
  for (int i = 0; i < kIt; ++i) v[i] = threadIdx.x + i * 256 < kW ? src[threadIdx.x + i * 256] : 0u;
#pragma unroll
  for (int i = 0; i < kIt; ++i)
    if (threadIdx.x + i * 256 < kW) dst[threadIdx.x + i * 256] = v[i];
  if (threadIdx.x == 0) S.sst = AdamStep{a.stats[5], a.stats[6], a.stats[7]};
  __syncthreads();
}

// block bx of the weight-gradient pass (see above); S staged by wgrad_stage
__device__ __forceinline__ void wgrad_tile(const WgArgs& a, int bx, WgLds& S) {
  float* lds = S.lds;
  const WgTable& tab = S.tab;
  const AdamStep& sst = S.sst;
  const int tid = threadIdx.x;
  SAC_T(4, 0);
  SAC_SPAN_BEGIN(4);
  SAC_TB(4, 6, (int)bx == a.n_mfma);
  const int n_small_blocks = (a.n_small + 63) / 64;
  if (tab.has_scalar && (int)bx == a.n_mfma + n_small_blocks) {  // scalars
    float v[5] = {0, 0, 0, 0, 0};
    for (int r = tid; r < a.B; r += kThreads) {
      v[0] += a.sc.p_pl[r];
      v[1] += a.sc.p_q1l[r];
      v[2] += a.sc.p_q2l[r];
      v[3] += a.sc.p_la[r];
      v[4] += a.sc.p_ga[r];
    }
    float (*red)[32] = S.red;
    float* sum = S.sum;
    block_sum<5>(v, red, sum);
    if (tid == 0) {
      const float invB = 1.0f / (float)a.B;
      a.stats[0] = sum[0] * invB;
      a.stats[1] = sum[1] * invB;
      a.stats[2] = sum[2] * invB;
      a.stats[3] = a.hp.auto_ent ? sum[3] * invB : 0.0f;
      a.stats[4] = a.hp.auto_ent ? expf(a.params[0]) : 1.0f;
      const float g0 = a.hp.auto_ent ? sum[4] * invB : 0.0f;
      a.grads[0] = g0;
      if (a.fuse && a.hp.auto_ent) {  // log α
        AdamElem x = adam_ld(a.ap, 0);
        x.g = g0;
        adam_st(a.ap, sst, 0, x);
      }
    }
    SAC_SPAN_END(4);
    return;
  }
  if ((int)bx >= a.n_mfma) {  // VALU elements: 64 per block, wave w sums rows [wB/4, (w+1)B/4)
    const int w = tid >> 6;
    const int64_t e = (int64_t)(bx - a.n_mfma) * 64 + (tid & 63);
    float acc = 0.0f;
    int s = 0;
    int64_t l = 0;
    const GMat* m = nullptr;
    AdamElem xv;
    if (e < a.n_small) {
      const WgTable& tb = tab;
      while (s + 1 < tb.n_small_mats && e >= tb.small_start[s + 1]) ++s;
      m = &tb.mats[tb.small_mat[s]];
      l = e - tb.small_start[s];
      const int j = (int)(l / m->N), k = (int)(l % m->N);
      // the optimizer state of this output (the lane of wave 0 that finishes it), in flight with the row sums
      if (a.fuse && w == 0) xv = adam_ld(a.ap, m->out_off + l, false);
      const int rq = a.B / 4, rb = w * rq;
      const gptr dy = as_global(m->dY) + (int64_t)rb * m->ldY + j;
      const gptr x = m->X ? as_global(m->X) + (int64_t)rb * m->ldX + k : nullptr;
      for (int r0 = 0; r0 < rq; r0 += 32) {  // 32 rows' loads in flight, then the fmaf chain in row order
        float yv[32], xv[32];
        if (r0 + 32 <= rq) {  // a full batch: straight-line loads, no per-load guard (see the MFMA tiles)
          if (x) {
#pragma unroll
            for (int u = 0; u < 32; ++u) {
              yv[u] = dy[(int64_t)(r0 + u) * m->ldY];
              xv[u] = x[(int64_t)(r0 + u) * m->ldX];
            }
          } else {
#pragma unroll
            for (int u = 0; u < 32; ++u) {
              yv[u] = dy[(int64_t)(r0 + u) * m->ldY];
              xv[u] = 1.0f;
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < 32; ++u) {
            const bool ok = r0 + u < rq;
            yv[u] = ok ? dy[(int64_t)(r0 + u) * m->ldY] : 0.0f;
            xv[u] = ok ? (x ? x[(int64_t)(r0 + u) * m->ldX] : 1.0f) : 0.0f;
          }
        }
#pragma unroll
        for (int u = 0; u < 32; ++u) acc = fmaf(yv[u], xv[u], acc);
      }
    }
    SAC_TB(4, 7, (int)bx == a.n_mfma);
    float* part = lds;  // [4][64]
    part[w * 64 + (tid & 63)] = acc;
    __syncthreads();
    if (w == 0 && m) {
      const int c = tid & 63;
      const int64_t e = m->out_off + l;
      AdamElem x = xv;
      x.g = ((part[c] + part[64 + c]) + part[128 + c]) + part[192 + c];
      a.grads[e] = x.g;
      if (a.fuse) adam_st(a.ap, sst, e, x);
    }
    SAC_TB(4, 8, (int)bx == a.n_mfma);
    SAC_SPAN_END(4);
    return;
  }
  // MFMA tile of an H x H matrix: A[j][r] = dY[r][j], B[r][k] = X[r][k]
  const WgTable& tb = tab;
  const int H = tb.mats[tb.big[0]].M;
  const int tiles = (H / kTile2) * (H / kTile2);
  // XCD-aware tile map (H = 256: 64 tiles per matrix, 24 per XCD): XCD x = bx mod 8 takes, of each matrix, the
  // 2 x 4 tiles of row blocks 2(x / 2) + {0, 1} and column blocks 4(x mod 2) + {0..3}, so its L2 fetches a quarter
  // of dYᵀ's columns and half of X's instead of all of both (the fabric traffic of the pass / 2.7; any placement
  // gives the same results)
  int bm = bx / tiles, t = bx % tiles;
  if (H == 256 && a.n_mfma == 3 * tiles) {
    const int x = bx & 7, sl = bx >> 3, tt = sl & 7;
    bm = sl >> 3;
    t = ((x >> 1) * 2 + (tt >> 2)) * 8 + (x & 1) * 4 + (tt & 3);
  }
  const GMat m = tb.mats[tb.big[bm]];
  const int j0 = (t / (H / kTile2)) * kTile2, k0 = (t % (H / kTile2)) * kTile2;
  const int w = tid >> 6, lane = tid & 63, h = lane >> 5;
  const int mat = tb.big_slot[bm];  // 0: actor W2, 1 / 2: Q1 / Q2 W2
  AdamElem x[4];
  const int rows_w = a.B / 4;  // this wave's rows, in chunks of up to 64 (32 MFMAs)
  f32x16 acc = zero16();
  for (int rc = 0; rc < rows_w; rc += 2 * kMaxN2) {
    const int n2 = min(kMaxN2, (rows_w - rc) / 2), rb = w * rows_w + rc + h * n2;
    float av[kMaxN2], bv[kMaxN2];
    // the chunk's operands as one straight-line batch of loads, all in flight together (a run-time guard per
    // load would make a chain of branches with a wait after every load): n2 = 32 for B >= 256, 16 / 8 / 4 for
    // B = 128 / 64 / 32
    auto load_chunk = [&](auto n_tag) __attribute__((always_inline)) {
      constexpr int N = decltype(n_tag)::value;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int64_t r = rb + i;
        av[i] = as_global(m.dY)[r * m.ldY + j0 + (lane & 31)];
        bv[i] = as_global(m.X)[r * m.ldX + k0 + (lane & 31)];
      }
    };
    if (n2 == 32) load_chunk(std::integral_constant<int, 32>{});
    else if (n2 == 16) load_chunk(std::integral_constant<int, 16>{});
    else if (n2 == 8) load_chunk(std::integral_constant<int, 8>{});
    else if (n2 == 4) load_chunk(std::integral_constant<int, 4>{});
    else {
#pragma unroll
      for (int i = 0; i < kMaxN2; ++i) {
        if (i >= n2) continue;  // (continue, not break: the constant trip count keeps the loop unrolled)
        const int64_t r = rb + i;
        av[i] = as_global(m.dY)[r * m.ldY + j0 + (lane & 31)];
        bv[i] = as_global(m.X)[r * m.ldX + k0 + (lane & 31)];
      }
    }
    // the optimizer state of the four outputs this lane finishes, in flight during the GEMM: issued after the
    // first chunk's operands (vector loads complete in issue order, so operands first lets the MFMA chain
    // start without waiting for these)
    if (rc == 0) SAC_WAVE(bx, 0);  // (timing build: operands only)
    if (rc == 0 && a.fuse)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        x[q] = adam_ld(a.ap, m.out_off + (int64_t)(j0 + finish_row(q)) * m.N + k0 + (lane & 31), false);
    SAC_T(4, 1);
    mfma_chain(acc, av, bv, n2);
  }
  SAC_T(4, 2);
  SAC_WAVE(bx, 1);
  auto& tt = S.tt;  // (fuse) updated parameters / targets, transposed
  splitk_finish_q(acc, lds, [&](int q, int rr, int cc, float v) {
    if (q == 0) SAC_WAVE(bx, 2);
    const int64_t e = m.out_off + (int64_t)(j0 + rr) * m.N + k0 + cc;
    a.grads[e] = v;
    if (a.fuse) {
      x[q].g = v;
      adam_st(a.ap, sst, e, x[q]);
      tt[0][cc][rr] = x[q].p;
      tt[1][cc][rr] = x[q].t;
    }
  });
  if (a.fuse) {  // W2ᵀ (and the target's) for the next step's forward passes: T[col][row]
    __syncthreads();
    const int64_t HH = (int64_t)H * H;
    const int tc = tid % kTile, tr = tid / kTile;
    for (int cc = tr; cc < kTile; cc += kThreads / kTile) {
      const int64_t o = (int64_t)(k0 + cc) * H + j0 + tc;
      a.ap.T[(size_t)mat * HH + o] = tt[0][cc][tc];
      if (mat > 0) a.ap.T[(size_t)(2 + mat) * HH + o] = tt[1][cc][tc];
    }
  }
  SAC_WAVE(bx, 3);
  SAC_T(4, 3);
  SAC_SPAN_END(4);
}


__global__ __launch_bounds__(256) void sac_wgrad_mfma_kernel(WgArgs a) {
  __shared__ WgLds S;
  const int bx = ((int)blockIdx.x + a.blk0) % a.n_blocks;
#ifdef SACF_PHASE_TIMING
  if (threadIdx.x == 0 && bx < 1024) {
    g_wg_blk[3 * bx] = wall_clock64();
    g_wg_blk[3 * bx + 2] = __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 7;  // HW_REG_XCC_ID
  }
#endif
  wgrad_stage(a, S);
  wgrad_tile(a, bx, S);
#ifdef SACF_PHASE_TIMING
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0 && bx < 1024) g_wg_blk[3 * bx + 1] = wall_clock64();
#endif
}


// ---------------------------------------------------------------------------------------------
// One grad step in ONE launch (sacf_config.step_kernel = 1): the five passes above as phases of a
// persistent kernel, G co-resident blocks (2 per CU) looping over each phase's tiles and meeting at a
// grid barrier between phases. The tile code, tile order and arithmetic are the five-launch kernels'
// own (tile t of a phase = (t mod gx, t / gx), the same work), so the results are bit-identical; what
// goes is four kernel boundaries and their cold prologues (instruction fetch, kernel arguments).
// ---------------------------------------------------------------------------------------------
struct PArgs {
  MArgs m;
  WgArgs w;
  unsigned* bar;  // barrier words (kBarWords, zeroed before every launch), see grid_barrier
  int* err;       // set when a barrier wait exceeds its bound (blocks not co-resident, or not dealt evenly over
                  // the XCDs): results invalid
};

// Barrier words, each counter on a 128-byte line of its own: [0] arrivals of the XCD leaders, [32] the top
// generation, [64 + 64x] arrivals on XCD x, [96 + 64x] XCD x's generation. Zeroed by a memset node ahead of
// every launch, so counts and generations run from 0 within the launch (barrier b waits for b + 1).
constexpr int kBarWords = 64 + 64 * 8;

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 7; }  // HW_REG_XCC_ID

// bounded relaxed agent-scope poll (global_load sc1: L1 bypassed) until *w >= want; false (and *err set)
// when the bound is hit
__device__ __forceinline__ bool poll_ge(unsigned* w, unsigned want, int* err) {
  for (unsigned spins = 0; __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want;) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1u << 20)) {  // (a legitimate wait is microseconds)
      atomicOr(err, 1);
      return false;
    }
  }
  return true;
}

// Grid barrier b of a launch, XCD-hierarchical (MI355X_MICROARCH.md "barrier-xcd", cdna_hip_programming.md
// §6 Guideline 16): every wave's stores drained (vmcnt 0); one lane per block arrives on its XCD's counter;
// the XCD's last arrival writes that XCD's L2 back (agent release), arrives on the top counter and waits for
// all eight XCDs, then bumps its XCD's generation; every block then takes an agent-scope acquire (drops its
// CU's L1) before the next pass reads. Placement-independent for correctness: the XCD only groups the
// counting (nblocks / 8 per XCD, as the round-robin deal gives for a grid that is a multiple of 8; an
// uneven deal times out into *err instead of hanging).
__device__ __forceinline__ void grid_barrier(unsigned* bar, int* err, unsigned nblocks, unsigned b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned x = xcc_id(), per_xcd = nblocks / 8, epoch = b + 1;
    unsigned* xcnt = bar + 64 + 64 * x;
    unsigned* xgen = xcnt + 32;
    const unsigned old = __hip_atomic_fetch_add(xcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == epoch * per_xcd - 1) {  // this XCD's last arrival
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (kept: the fence's own wait can be dropped)
      const unsigned t = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == epoch * 8 - 1) __hip_atomic_store(bar + 32, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else poll_ge(bar + 32, epoch, err);
      __hip_atomic_store(xgen, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      poll_ge(xgen, epoch, err);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate done before the block goes on
  }
  __syncthreads();
}

// the kernel's PArgs read through the kernarg segment pointer, laundered: every field is re-read (scalar
// loads) where a tile uses it instead of ~200 argument dwords held in SGPRs across all five phases
typedef const __attribute__((address_space(4))) PArgs* PArgsPtr;
__device__ __forceinline__ const PArgs& persist_args() {
  PArgsPtr q = (PArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return *(const PArgs*)q;
}

template <int H>
__global__ __launch_bounds__(256, 2) void sac_step_persistent_kernel(PArgs p_arg) {
  (void)p_arg;  // read through persist_args()
  constexpr int kRaw = (kLdsFloats * 4 > (int)sizeof(WgLds) ? kLdsFloats * 4 : (int)sizeof(WgLds)) / 16;
  __shared__ float4 raw[kRaw];  // the passes' LDS, then (last phase) the weight-gradient pass's WgLds
  float* lds = reinterpret_cast<float*>(raw);
  const int G = gridDim.x, ct = H / kTile2;
  const int B = persist_args().m.L.B;
  if (threadIdx.x == 0) {  // diagnostics: blocks congruent mod 8 share an XCD (the deal the counting assumes)
    const unsigned xcc = xcc_id() + 1;
    unsigned* seen_at = persist_args().bar + kBarWords + 8 + blockIdx.x % 8;  // (not zeroed per launch)
    const unsigned seen = atomicCAS(seen_at, 0u, xcc);
    if (seen != 0u && seen != xcc) atomicOr(persist_args().err, 2 | (int)(xcc << 8) | (int)(seen << 16));
  }
  unsigned nb = 0;  // barriers passed in this launch
  auto barrier = [&](bool) __attribute__((always_inline)) {
    const PArgs& pa = persist_args();
    grid_barrier(pa.bar, pa.err, G, nb++);
  };
  {  // actor_fwd
    const int gx = 2 * B / kTile2, nt = gx * ct;
    for (int t = blockIdx.x; t < nt; t += G) {
      actor_fwd_tile<H>(persist_args().m, t % gx, t / gx, lds);
      __syncthreads();
    }
  }
  barrier(false);
  {  // critic_fwd
    const int gx = 6 * B / kTile2, nt = gx * ct;
    for (int t = blockIdx.x; t < nt; t += G) {
      critic_fwd_tile<H>(persist_args().m, t % gx, t / gx, lds);
      __syncthreads();
    }
  }
  barrier(false);
  {  // critic_bwd
    const int gx = 4 * B / kTile2 + 8, nt = gx * ct;
    for (int t = blockIdx.x; t < nt; t += G) {
      critic_bwd_tile<H>(persist_args().m, t % gx, t / gx, lds);
      __syncthreads();
    }
  }
  barrier(false);
  {  // actor_bwd
    const int gx = B / kTile2, nt = gx * ct;
    for (int t = blockIdx.x; t < nt; t += G) {
      actor_bwd_tile<H>(persist_args().m, t % gx, t / gx, lds);
      __syncthreads();
    }
  }
  barrier(true);
  {  // weight gradients (+ Adam / soft update / W2T when fused)
    WgLds& S = *reinterpret_cast<WgLds*>(raw);
    const int nb = persist_args().w.n_blocks;
    if ((int)blockIdx.x < nb) wgrad_stage(persist_args().w, S);
    for (int t = blockIdx.x; t < nb; t += G) {
      wgrad_tile(persist_args().w, t, S);
      __syncthreads();
    }
  }
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
    constexpr int kPer = kTile / (kThreads / kTile);  // 4 rows per thread
    const int tpm = (H / kTile) * (H / kTile);
    const int mat = blockIdx.x / tpm, t = blockIdx.x % tpm;
    const int r0 = (t / (H / kTile)) * kTile, c0 = (t % (H / kTile)) * kTile;
    const int tc = threadIdx.x % kTile, tr = threadIdx.x / kTile;  // 8 rows per pass
    AdamElem x[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) x[u] = adam_ld(a, w2[mat] + (int64_t)(r0 + tr + u * 8) * H + c0 + tc);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int rr = tr + u * 8;
      adam_st(a, st, w2[mat] + (int64_t)(r0 + rr) * H + c0 + tc, x[u]);
      tile[0][tc][rr] = x[u].p;
      tile[1][tc][rr] = x[u].t;
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
  AdamElem x = adam_ld(a, e);
  adam_st(a, st, e, x);
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


// ---------------------------------------------------------------------------------------------
// Policy actions for the collector (sacf_policy_act): TanhGaussianPolicy.forward + TanhNormal.sample
// (gaussian_policy.py:105-118, distributions.py:394-425; MakeDeterministic: tanh(mean), policies/base.py:
// 54-64) for n observation rows, from the trainer's own parameters and transposed W2 copy.
//   sac_act_fwd_kernel  : grid (n / 32, H / 32): h1 (VALU), h2 = relu(h1 W2ᵀ + b2) on MFMA, and this column
//                         block's part of the mean / log_std heads of each row (as actor_fwd's epilogue)
//   sac_act_head_kernel : per row: the parts summed in block order + biases, log_std clamped, std = exp,
//                         a = tanh(mean + std·ε) (ε from Philox(seed, counter, row)) or tanh(mean); rows
//                         whose mask byte is 0 keep their previous action
// ---------------------------------------------------------------------------------------------
struct ActArgs {
  const float* params;
  const float* T;
  const float* obs;    // [n][obs_stride]
  int64_t n;
  int obs_stride;
  Layout L;
  float* hpart;        // [2][H/32][n_pad]
  int64_t n_pad;
  const uint8_t* mask;
  int deterministic;
  uint64_t seed;
  const int64_t* counter;
  float* act;          // [n]
  float* eps_out;      // [n] or null
};

template <int H>
__global__ __launch_bounds__(256) void sac_act_fwd_kernel(ActArgs a) {
  __shared__ float lds[kLdsFloats];
  const Layout& L = a.L;
  const int O = L.O;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int r0 = blockIdx.x * kTile2, c0 = blockIdx.y * kTile2;
  constexpr int n2 = H / 8;
  const int kb = w * (H / 4) + h * n2;
  const int64_t row = r0 + (lane & 31);
  const int64_t rowc = row < a.n ? row : a.n - 1;  // rows past n (last tile) repeat the last row
  float x[kXLd];
#pragma unroll
  for (int m = 0; m < kXLd; ++m) x[m] = m < O ? a.obs[rowc * a.obs_stride + m] : 0.0f;
  float av[kMaxN2], bv[kMaxN2];
#pragma unroll
  for (int i = 0; i < n2; ++i) bv[i] = a.T[(int64_t)(kb + i) * H + c0 + (lane & 31)];  // policy W2ᵀ
  const float b2c = P[L.p_b2 + c0 + (lane & 31)];
  const float wm = P[L.p_wm + c0 + (lane & 31)], ws = P[L.p_ws + c0 + (lane & 31)];
  float* lw1 = lds + kLdsW1Off;
  float* lx = lds + kLdsXOff;
  stage_w1t<H>(lw1, P + L.p_w1, P + L.p_b1, O);
  if (w == 0 && h == 0)
    for (int m = 0; m < O; ++m) lx[(lane & 31) * (kXLd + 1) + m] = x[m];
  __syncthreads();
  first_layer<H>(lw1, lx + (lane & 31) * (kXLd + 1), O, kb, av);
  f32x16 acc = zero16();
  mfma_chain(acc, av, bv, n2);
  constexpr int CB = H / kTile2;
  splitk_finish(acc, lds, [&](int rr, int cc, float v) {
    const float y = relu(v + b2c);
    const float pm = halfwave_sum(y * wm), ps = halfwave_sum(y * ws);
    if (cc == 0) {
      a.hpart[(int64_t)blockIdx.y * a.n_pad + r0 + rr] = pm;
      a.hpart[(int64_t)(CB + blockIdx.y) * a.n_pad + r0 + rr] = ps;
    }
  });
}

template <int H>
__global__ __launch_bounds__(256) void sac_act_head_kernel(ActArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  constexpr int CB = H / kTile2;
  const float* P = a.params;
  const float mean = sum_parts<CB>(a.hpart, a.n_pad, r) + P[a.L.p_bm];
  const float ls = sum_parts<CB>(a.hpart + CB * a.n_pad, a.n_pad, r) + P[a.L.p_bs];
  float eps = 0.0f;
  if (!a.deterministic) {
    const uint64_t ctr = a.counter ? (uint64_t)*a.counter : 0;
    uint32_t c[4] = {(uint32_t)r, (uint32_t)ctr, (uint32_t)(ctr >> 32), 0xAC70u};
    philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    const float u1 = ((float)c[0] + 1.0f) * 2.3283064365386963e-10f;
    const float u2 = (float)c[1] * 2.3283064365386963e-10f;
    eps = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
  }
  const float log_std = fminf(fmaxf(ls, -20.0f), 2.0f);
  const float z = a.deterministic ? mean : mean + expf(log_std) * eps;
  if (a.eps_out) a.eps_out[r] = eps;
  if (a.mask && !a.mask[r]) return;
  a.act[r] = tanhf(z);
}

template <int H>
void launch_act(const ActArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sac_act_fwd_kernel<H>, dim3((unsigned)(a.n_pad / kTile2), H / kTile2), dim3(256), 0, st, a);
  hipLaunchKernelGGL(sac_act_head_kernel<H>, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
}

// the four forward/backward passes of one grad step for hidden width H (a compile-time tile count)
template <int H>
void launch_passes(const MArgs& a, hipStream_t st, int part) {
  const int B = a.L.B, ct = H / kTile2;
  if (part == 0) {
    hipLaunchKernelGGL(sac_actor_fwd_kernel<H>, dim3((SACF_EARLY_DATA ? 4 : 2) * B / kTile2, ct), dim3(256), 0, st, a);
    hipLaunchKernelGGL(sac_critic_fwd_kernel<H>, dim3((SACF_EARLY_DATA ? 4 : 6) * B / kTile2, ct), dim3(256), 0, st, a);
    // (grid x a multiple of 8 everywhere: block i runs on XCD i % 8, so row tile r of every kernel
    //  lands on XCD r % 8, the L2 that holds what the previous kernel wrote for those rows)
    hipLaunchKernelGGL(sac_critic_bwd_kernel<H>, dim3(4 * B / kTile2 + 8, ct), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(sac_actor_bwd_kernel<H>, dim3(B / kTile2, ct), dim3(256), 0, st, a);
  }
}

template <int H>
hipError_t occupancy_of(int* per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, sac_step_persistent_kernel<H>, 256, 0);
}
hipError_t persistent_occupancy(int H, int* per_cu) {
  switch (H) {
    case 32: return occupancy_of<32>(per_cu);
    case 64: return occupancy_of<64>(per_cu);
    case 96: return occupancy_of<96>(per_cu);
    case 128: return occupancy_of<128>(per_cu);
    case 160: return occupancy_of<160>(per_cu);
    case 192: return occupancy_of<192>(per_cu);
    case 224: return occupancy_of<224>(per_cu);
    case 256: return occupancy_of<256>(per_cu);
    default: return hipErrorInvalidValue;
  }
}

template <int H>
void launch_persistent(const PArgs& p, int grid, hipStream_t st) {
  hipLaunchKernelGGL(sac_step_persistent_kernel<H>, dim3(grid), dim3(256), 0, st, p);
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
  WgArgs wg[1];       // weight gradients (+ losses, log α, and the update when world_size == 1)
  WgTable* wtab[1];
  float* act_part;      // sacf_policy_act head partials [2][H/32][act_cap]
  int64_t act_cap;
  unsigned* bar;        // step_kernel 1: grid barrier [arrive, generation] + error flag (int) after them
  int grid;             // step_kernel 1: co-resident blocks of the persistent kernel
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
  if (O < 1 || O + 1 > kXLd || H < 32 || H > SACF_MAX_HIDDEN || H % 32 || B < kTile2 || B % kTile2 || B > SACF_MAX_BATCH ||
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
  const int64_t CB = H / kTile2;
  const int64_t n_scr = 4 * BH + B * kXLd + 2 * B + 2 * (4 * BH + B * kXLd + B) + 5 * B +
                        2 * B * kXLd + 5 * B + BH + 12 * B + 6 * BH + 2 * BH +
                        2 * CB * 2 * B + 4 * CB * 2 * B + 2 * CB * B;
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
  ms.hpart = s; s += 2 * CB * 2 * B;
  ms.qpart = s; s += 4 * CB * 2 * B;
  ms.apart = s; s += 2 * CB * B;
  e = hipMalloc(&h->T, sizeof(float) * 5 * (size_t)H * H);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "hipMalloc(T): %s", hipGetErrorString(e));
  }
  // weight-gradient matrices: the H x H ones on MFMA tiles, the rest one element per thread (one launch;
  // a fork of the critics' part onto a second stream beside actor_bwd measured slower, and the critics'
  // log α update would race with actor_bwd's read of α)
  for (int part = 0; part < 1; ++part) {
    WgArgs& wg = h->wg[part];
    memset(&wg, 0, sizeof(wg));
    WgTable tab;
    memset(&tab, 0, sizeof(tab));
    int nm = 0, nb = 0;
    auto add = [&](const float* dY, int ldY, const float* X, int ldX, int M, int N, int64_t off, int slot) {
      if (M == H && N == H && X) {
        tab.big[nb] = nm;
        tab.big_slot[nb++] = slot;
      } else {
        tab.small_mat[tab.n_small_mats] = nm;
        tab.small_start[tab.n_small_mats + 1] = tab.small_start[tab.n_small_mats] + (int64_t)M * N;
        tab.n_small_mats++;
      }
      tab.mats[nm++] = GMat{dY, X, ldY, ldX, M, N, off};
    };
    {
      add(sc.a_dh1, H, sc.a_x, kXLd, H, O, L.p_w1, -1);
      add(sc.a_dh1, H, nullptr, 0, H, 1, L.p_b1, -1);
      add(sc.a_dh2, H, sc.a_h1, H, H, H, L.p_w2, 0);
      add(sc.a_dh2, H, nullptr, 0, H, 1, L.p_b2, -1);
      add(sc.a_dhead, 2, sc.a_h2, H, 1, H, L.p_wm, -1);
      add(sc.a_dhead, 2, nullptr, 0, 1, 1, L.p_bm, -1);
      add(sc.a_dhead + 1, 2, sc.a_h2, H, 1, H, L.p_ws, -1);
      add(sc.a_dhead + 1, 2, nullptr, 0, 1, 1, L.p_bs, -1);
      for (int k = 0; k < 2; ++k) {
        const int64_t b = L.q_base[k];
        add(sc.q_dg1[k], H, sc.q_x[k], kXLd, H, O + 1, b + L.c_w1, -1);
        add(sc.q_dg1[k], H, nullptr, 0, H, 1, b + L.c_b1, -1);
        add(sc.q_dg2[k], H, sc.q_g1[k], H, H, H, b + L.c_w2, 1 + k);
        add(sc.q_dg2[k], H, nullptr, 0, H, 1, b + L.c_b2, -1);
        add(sc.q_dq[k], 1, sc.q_g2[k], H, 1, H, b + L.c_w3, -1);
        add(sc.q_dq[k], 1, nullptr, 0, 1, 1, b + L.c_b3, -1);
      }
      tab.has_scalar = 1;
    }
    tab.n_mats = nm;
    wg.n_small = (int)tab.small_start[tab.n_small_mats];
    e = hipMalloc(&h->wtab[part], sizeof(WgTable));
    if (e == hipSuccess) e = hipMemcpy(h->wtab[part], &tab, sizeof(WgTable), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      *out = h;
      return sfail(h, SACF_EHIP, "wgrad table: %s", hipGetErrorString(e));
    }
    wg.tab = h->wtab[part];
    wg.n_mfma = nb * (H / kTile2) * (H / kTile2);
    wg.n_blocks = wg.n_mfma + (wg.n_small + 63) / 64 + tab.has_scalar;
    wg.B = B;
    wg.sc = sc;
    wg.hp = h->hp;
  }
  if (cfg->step_kernel == 1) {  // persistent single-launch step: barrier state and a co-resident grid
    // [0, kBarWords) barrier words (zeroed before every launch), [kBarWords] error flag, [kBarWords + 8 + r]
    // the XCD of block residue r mod 8 (+1, 0 = not seen yet)
    e = hipMalloc(&h->bar, (kBarWords + 16) * sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(h->bar, 0, (kBarWords + 16) * sizeof(unsigned));
    int per_cu = 0, cus = 0;
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = persistent_occupancy(H, &per_cu);
    if (e != hipSuccess) {
      *out = h;
      return sfail(h, SACF_EHIP, "persistent step kernel: %s", hipGetErrorString(e));
    }
    h->grid = (per_cu >= 2 ? 2 : per_cu) * cus / 8 * 8;  // a multiple of 8: tile t stays on XCD t % 8
    if (h->grid < 8) {
      *out = h;
      return sfail(h, SACF_EINVAL, "persistent step kernel: %d blocks per CU", per_cu);
    }
  }
  *out = h;
  return SACF_OK;
}

int sacf_destroy(sacf_handle* h) {
  if (!h) return SACF_OK;
  SDev g(h->device);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->T) (void)hipFree(h->T);
  if (h->wtab[0]) (void)hipFree(h->wtab[0]);
  if (h->act_part) (void)hipFree(h->act_part);
  if (h->bar) (void)hipFree(h->bar);
  delete h;
  return SACF_OK;
}

#ifdef SACF_PHASE_TIMING
int sacf_debug_reset(void) {
  unsigned long long init[64];
  for (int i = 0; i < 64; ++i) init[i] = i % 12 == 9 ? ~0ull : 0ull;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sac_stamp), init, sizeof(init)) == hipSuccess ? 0 : -1;
}
int sacf_debug_stamps(unsigned long long* out64) {
  return hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_sac_stamp), sizeof(unsigned long long) * 64) == hipSuccess ? 0 : -1;
}
// weight-gradient pass, per block: start, end (wall clock), XCC id; and the pass's block classes; per MFMA-tile
// block and wave: operands loaded, MFMA chain issued, split-K sum read, done (each after the wave's memory drained)
int sacf_debug_wg_blocks(const sacf_handle* h, unsigned long long* out, int* n_mfma, int* n_blocks,
                         unsigned long long* waves) {
  *n_mfma = h->wg[0].n_mfma;
  *n_blocks = h->wg[0].n_blocks;
  if (hipMemcpyFromSymbol(waves, HIP_SYMBOL(g_wg_wave), sizeof(unsigned long long) * 1024 * 16) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_blk), sizeof(unsigned long long) * 3 * 1024) == hipSuccess ? 0 : -1;
}
#endif

const char* sacf_last_error(const sacf_handle* h) { return h ? h->err : "null handle"; }

int sacf_step_kernel_status(sacf_handle* h) {
  if (!h) return SACF_EINVAL;
  if (!h->bar) return SACF_OK;
  SDev g(h->device);
  int flag = 0;
  hipError_t e = hipMemcpy(&flag, h->bar + kBarWords, sizeof(int), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return sfail(h, SACF_EHIP, "sacf_step_kernel_status: %s", hipGetErrorString(e));
  if (!flag) return SACF_OK;
  return sfail(h, SACF_ESTATE, "persistent step kernel: %s (flag 0x%x; results invalid)",
               (flag & 1) ? "a grid barrier wait timed out" : "blocks congruent mod 8 ran on different XCDs", flag);
}
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

// the forward/backward passes for the handle's hidden width: part 0 = actor_fwd, critic_fwd, critic_bwd;
// part 1 = actor_bwd
static bool launch_hidden(int H, const MArgs& a, hipStream_t st, int part) {
  switch (H) {
    case 32: launch_passes<32>(a, st, part); return true;
    case 64: launch_passes<64>(a, st, part); return true;
    case 96: launch_passes<96>(a, st, part); return true;
    case 128: launch_passes<128>(a, st, part); return true;
    case 160: launch_passes<160>(a, st, part); return true;
    case 192: launch_passes<192>(a, st, part); return true;
    case 224: launch_passes<224>(a, st, part); return true;
    case 256: launch_passes<256>(a, st, part); return true;
    default: return false;
  }
}

static ApplyArgs apply_args(const sacf_handle* h) {
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
  a.n_tile_blocks = 3 * (h->L.H / kTile) * (h->L.H / kTile);
  return a;
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
  SDev g(h->device);
  WgArgs& w = h->wg[0];
  w.grads = h->grads;
  w.params = h->params;
  w.step = h->step;
  w.stats = h->stats;
  w.fuse = h->cfg.world_size == 1 && !h->cfg.split_update;  // no all-reduce in between: apply in the same kernel
  w.ap = apply_args(h);
  if (h->cfg.step_kernel == 1) {  // the whole step in one launch
    PArgs p;
    p.m = a;
    p.w = w;
    p.bar = h->bar;
    p.err = reinterpret_cast<int*>(h->bar + kBarWords);
    // the barrier words from 0 for this launch (a memset node under graph capture; 2,304 bytes from the
    // allocation's start, a multiple of 16)
    hipError_t me = hipMemsetAsync(h->bar, 0, kBarWords * sizeof(unsigned), h->stream);
    if (me != hipSuccess) return sfail(h, SACF_EHIP, "sacf_grads: %s", hipGetErrorString(me));
    switch (h->L.H) {
      case 32: launch_persistent<32>(p, h->grid, h->stream); break;
      case 64: launch_persistent<64>(p, h->grid, h->stream); break;
      case 96: launch_persistent<96>(p, h->grid, h->stream); break;
      case 128: launch_persistent<128>(p, h->grid, h->stream); break;
      case 160: launch_persistent<160>(p, h->grid, h->stream); break;
      case 192: launch_persistent<192>(p, h->grid, h->stream); break;
      case 224: launch_persistent<224>(p, h->grid, h->stream); break;
      case 256: launch_persistent<256>(p, h->grid, h->stream); break;
      default: return sfail(h, SACF_EINVAL, "sacf_grads: hidden %d", h->L.H);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_grads: %s", hipGetErrorString(e));
  }
  if (!launch_hidden(h->L.H, a, h->stream, 0)) return sfail(h, SACF_EINVAL, "sacf_grads: hidden %d", h->L.H);
  launch_hidden(h->L.H, a, h->stream, 1);
  static const int wg_mode = getenv("SACF_WG_MODE") ? atoi(getenv("SACF_WG_MODE")) : 0;  // timing experiments
  if (wg_mode == 1) {  // two launches: the MFMA tiles, then the VALU elements and the scalars
    WgArgs w1 = w;
    w1.blk0 = 0;
    hipLaunchKernelGGL(sac_wgrad_mfma_kernel, dim3(w.n_mfma), dim3(256), 0, h->stream, w1);
    w1.blk0 = w.n_mfma;
    hipLaunchKernelGGL(sac_wgrad_mfma_kernel, dim3(w.n_blocks - w.n_mfma), dim3(256), 0, h->stream, w1);
  } else {
    WgArgs w1 = w;
    w1.blk0 = wg_mode == 2 ? w.n_mfma : 0;  // 2: the VALU / scalar blocks dispatched first
    hipLaunchKernelGGL(sac_wgrad_mfma_kernel, dim3(w.n_blocks), dim3(256), 0, h->stream, w1);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_grads: %s", hipGetErrorString(e));
}

int sacf_apply(sacf_handle* h) {
  if (!h || !h->params) return sfail(h, SACF_ESTATE, "sacf_apply: buffers not bound");
  if (h->cfg.world_size == 1 && !h->cfg.split_update) return SACF_OK;  // sacf_grads already applied the update
  ApplyArgs a = apply_args(h);
  const int64_t HH = (int64_t)h->L.H * h->L.H;
  const int64_t rest = h->L.n_params - 3 * HH;
  SDev g(h->device);
  hipLaunchKernelGGL(sac_apply_kernel, dim3((unsigned)(a.n_tile_blocks + (rest + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, h->stream, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_apply: %s", hipGetErrorString(e));
}

int sacf_policy_reserve(sacf_handle* h, int64_t n) {
  if (!h || n < 1) return sfail(h, SACF_EINVAL, "sacf_policy_reserve: bad argument");
  const int64_t n_pad = (n + kTile2 - 1) / kTile2 * kTile2;
  if (n_pad <= h->act_cap) return SACF_OK;
  SDev g(h->device);
  if (h->act_part) (void)hipFree(h->act_part);
  h->act_part = nullptr;
  h->act_cap = 0;
  hipError_t e = hipMalloc(&h->act_part, sizeof(float) * 2 * (size_t)(h->L.H / kTile2) * n_pad);
  if (e != hipSuccess) return sfail(h, SACF_EHIP, "sacf_policy_reserve: %s", hipGetErrorString(e));
  h->act_cap = n_pad;
  return SACF_OK;
}

int sacf_policy_act(sacf_handle* h, const float* obs, int64_t n, int32_t obs_stride, const uint8_t* mask,
                    int32_t deterministic, uint64_t seed, const int64_t* counter, float* act, float* eps_out) {
  if (!h || !h->params) return sfail(h, SACF_ESTATE, "sacf_policy_act: buffers not bound");
  if (!obs || !act || n < 1 || obs_stride < h->L.O) return sfail(h, SACF_EINVAL, "sacf_policy_act: bad argument");
  const int64_t n_pad = (n + kTile2 - 1) / kTile2 * kTile2;
  if (n_pad > h->act_cap)
    return sfail(h, SACF_ESTATE, "sacf_policy_act: %lld rows need sacf_policy_reserve first", (long long)n);
  ActArgs a;
  memset(&a, 0, sizeof(a));
  a.params = h->params; a.T = h->T; a.obs = obs; a.n = n; a.obs_stride = obs_stride; a.L = h->L;
  a.hpart = h->act_part; a.n_pad = n_pad; a.mask = mask; a.deterministic = deterministic;
  a.seed = seed; a.counter = counter; a.act = act; a.eps_out = eps_out;
  SDev g(h->device);
  switch (h->L.H) {
    case 32: launch_act<32>(a, h->stream); break;
    case 64: launch_act<64>(a, h->stream); break;
    case 96: launch_act<96>(a, h->stream); break;
    case 128: launch_act<128>(a, h->stream); break;
    case 160: launch_act<160>(a, h->stream); break;
    case 192: launch_act<192>(a, h->stream); break;
    case 224: launch_act<224>(a, h->stream); break;
    case 256: launch_act<256>(a, h->stream); break;
    default: return sfail(h, SACF_EINVAL, "sacf_policy_act: hidden %d", h->L.H);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_policy_act: %s", hipGetErrorString(e));
}

int sacf_policy_weights(const sacf_handle* h, const float** params, const float** w2t, int32_t* obs_dim,
                        int32_t* hidden) {
  if (!h || !h->params || !h->T) return SACF_ESTATE;
  if (params) *params = h->params + h->L.p_w1;
  if (w2t) *w2t = h->T;  // the actor's W2ᵀ leads the transposed copies (kept current by every update)
  if (obs_dim) *obs_dim = h->L.O;
  if (hidden) *hidden = h->L.H;
  return SACF_OK;
}

}  // extern "C"
