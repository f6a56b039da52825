// sac_kernels.hip — fused SAC update for gfx950 (C ABI: include/sac_fused.h) -> libsacfused.so
//
// One grad step of ast_sac/torch/sac/sac.py (compute_loss :156-270, train_from_torch :102-154,
// update_target_networks :160-166) for TanhGaussianPolicy + twin ConcatMlp critics with two hidden
// layers of width H and act_dim 1, as batched fp32 GEMMs on the matrix cores (v_mfma_f32_32x32x2_f32,
// exact fp32) in THREE dependent launches:
//
//   sac_fwd_kernel   (P1): replay gather; actor forward on [obs; next_obs] rows (h1, h2 and the per-column-
//                          block parts of the mean / log_std heads); critic forward on the (obs, a) data rows
//                          (g1, g2 and the parts of Q1 / Q2).
//   sac_mid_kernel   (P2): per row the actor head and its TanhNormal sample ã (ã' on next_obs); the critics on
//                          (obs, ã) TOGETHER WITH the forward-mode tangent of Q along the action (act_dim 1, so
//                          ∂Q/∂ã is one more chain on the same W2 operand, no backward pass); the target critics
//                          on (next_obs, ã'); and the backward factors that need only forward masks:
//                            U_m = ((wm ⊙ [h2>0]) W2) ⊙ [h1>0],  U_s = ((ws ⊙ [h2>0]) W2) ⊙ [h1>0]   (actor)
//                            U_q = ((w3 ⊙ [g2>0]) W2) ⊙ [g1>0]                                      (critics, data rows)
//                          The true input gradients are per-row scalings of these: dh1 = dmean·U_m + dls·U_s,
//                          dg1 = dq·U_q (the backward pass is linear in the head gradient).
//   sac_wgrad_kernel (P3): every per-row scalar (dq1, dq2 from the Q / target parts; dmean, dls from ∂Q/∂ã and
//                          the head) recomputed where it is needed, then every weight gradient Σ_rows dYᵀ X (the
//                          three H x H ones on MFMA, the rest on the VALU) with Adam, the soft target update and
//                          the transposed-weight refresh fused in (world_size 1), plus losses, d(log α), stats.
//   sac_apply_kernel     : world_size > 1 / split_update: Adam + soft update after the caller's all-reduce.
//
// The four gradients the reference keeps are formed (the π-loss gradient w.r.t. the critics, discarded by
// qf*_optimizer.zero_grad() at sac.py:123-133, is not); α is a constant inside the π- and Q-losses as after
// alpha_optimizer.step(). Every sum runs in a fixed order: results are deterministic (graph == eager bitwise).
// Batches of any size up to SACF_MAX_BATCH: rows are padded to Bp = ⌈B / 32⌉·32, padding rows carry zero
// gradient scalars and are left out of every loss.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <type_traits>

#include "sac_fused.h"

// Translation-unit role (the library is built from two objects of this file, ast_sac_amd/build_hash.py):
//   SACF_TU 1: every hidden width but the two widest, with the C ABI; the two widest go to the other object
//   SACF_TU 2: the kernels of the two widest widths (448, 512) and their two launch forwarders only
//   SACF_TU 0: everything in one object (diagnostics builds)
// so the narrow widths can use the max-ILP machine scheduler while the wide ones keep the default (max-ILP spills
// SGPRs there).
#ifndef SACF_TU
#define SACF_TU 0
#endif
#if SACF_TU == 1
bool sacf_wide_launch_step(int H, const void* m, const void* w, hipStream_t st);
bool sacf_wide_launch_act(int H, const void* a, hipStream_t st);
#endif

namespace {

constexpr int kThreads = 256;
constexpr int kXLd = 16;   // leading dim of the per-row input rows (obs | act), obs_dim <= 15
constexpr int kTile2 = 32; // output tile edge of the MFMA kernels
constexpr int kMaxN2 = 32; // MFMAs per wave per operand chunk
constexpr float kLog2 = 0.69314718055994530942f;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;

// hidden widths with compiled kernels: every multiple of 32 up to 256, multiples of 64 above
__host__ __device__ constexpr bool hidden_ok(int H) {
  return H >= 32 && H <= SACF_MAX_HIDDEN && (H <= 256 ? H % 32 == 0 : H % 64 == 0);
}

struct Layout {
  int O, H, B, Bp;  // obs_dim, hidden, batch, batch padded to a multiple of 32
  int64_t p_w1, p_b1, p_w2, p_b2, p_wm, p_bm, p_ws, p_bs;  // policy (params)
  int64_t q_base[2];                                      // start of qf1 / qf2 in params
  int64_t q_size;                                         // floats of one critic
  int64_t c_w1, c_b1, c_w2, c_b2, c_w3, c_b3;             // offsets inside one critic block
  int64_t n_params, n_targets;
};

struct Hyper {
  float gamma, rscale, tau, areg, clip, tent, lr_pi, lr_q, beta1, beta2, eps;
  int auto_ent;
  float inv_world;
};

// per-row parts (one per 32-column block, in block order) of the head dot products, in the row-tile word layout
// (rw_at below: [Bp / 32][set][CB][32])
enum { PS_Q1D, PS_Q2D, PS_T1, PS_T2, PS_Q1A, PS_Q2A, PS_D1, PS_D2, PS_N };
// The row-tile word layout of the per-row words (parts, head parts, activation masks): the words of one 32-row tile
// for one (set, column block) are contiguous, so the block that produced them writes them as runs (row_words_out)
// and a reader whose lanes hold consecutive rows reads them coalesced. (Row-major [row][set][CB], every epilogue
// store of these words was 4 bytes into a different row: P1 / P2 took 0.3 / 0.4 µs longer at B = 256 than
// without them, profiles/round6/r6y_*.)
__host__ __device__ __forceinline__ int64_t rw_at(int r, int set, int nsets, int CB, int by) {
  return ((((int64_t)(r >> 5) * nsets + set) * CB + by) << 5) + (r & 31);
}
// the per-row record, kRec words per row in the row-tile layout (rec_at below): the obs row's actor head (HD_*: mean,
// ls_raw, std, z, a, logp), its two reparameterisation normals, the replayed reward / terminal / action and
// log π(ã'|s') of the next_obs row
enum { HD_MEAN, HD_LSRAW, HD_STD, HD_Z, HD_A, HD_LOGP, R_EPS, R_EPSN, R_REW, R_TERM, R_ACT, R_LOGPN };
constexpr int kRec = 16;
// word f of row r's record
__host__ __device__ __forceinline__ int64_t rec_at(int r, int f) { return rw_at(r, f, kRec, 1, 0); }

// library-owned activations, all [Bp][...] (row pitch H unless stated)
struct Scr {
  float *x;                  // gathered obs rows [Bp][kXLd]
  float *qx;                 // critic data rows (obs | a) [Bp][kXLd]
  float *h1, *h2;            // actor on the obs rows
  float *g1[2], *g2[2];      // Q1 / Q2 on the (obs, a) rows
  float *um, *us;            // actor backward factors
  float *uq[2];              // critic backward factors (data rows)
  float *rec;                // per-row record (HD_* / R_*), Bp rows (rec_at)
  float *hpart;              // actor head parts (mean | log_std) of the obs and next_obs rows, 2Bp rows (rw_at, 2 sets)
  // fc0 of a critic up to (not including) its action term — b1 + Σ_{m < O} W1[:, m] x_m, the fmaf chain in input
  // order — on the obs rows (Q1, Q2: from P1's data tiles) and the next_obs rows (T1, T2: P1's target tiles), and
  // fc0's action column W1[:, O] of Q1, Q2, T1, T2 [4][H]: P2's critic tiles on (obs, ã) / (next_obs, ã') add the
  // action term themselves (the same chain, so the same bits as fc0 on the whole row)
  float *pre[4];             // [Bp][H] each: Q1, Q2 (obs rows), T1, T2 (next_obs rows)
  float *w1a;                // [4][H]
  float *part;               // Bp rows (rw_at, PS_N sets)
  // [h2 > 0] and [g2 > 0] of Q1 / Q2 as bit masks, Bp x CB words (rw_at, 1 set; bit c of word (r, b): column 32b + c
  // of row r):
  // the backward factors (P2) and the MFMA weight-gradient tiles (P3) use the layer-2 activations only through this
  // mask, so they read 1 bit per element instead of the float
  uint32_t *h2m, *g2m[2];
  // the parameters P3 reads, as they were before this step's update (P3 updates them in place with fused Adam,
  // so its blocks must not read the live values): [log α, b3 Q1, b3 Q2, b3 T1, b3 T2, -, -, -] then
  // wm [H], ws [H], w3 Q1 [H], w3 Q2 [H]
  float *snap;
  // the next step's batch, staged by P3 of a chained step (sacf_grads_chain): obs / next_obs rows [Bp][kXLd] and
  // [Bp][kAux] (act, rew, term, the two reparameterisation normals)
  float *sx, *sxn, *saux;
};
enum { AUX_ACT, AUX_REW, AUX_TERM, AUX_E0, AUX_E1, kAux = 8 };
enum { SN_LOGA, SN_BQ1, SN_BQ2, SN_BT1, SN_BT2, SN_HEAD = 8 };

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
  int64_t* step;
  float* stats;
  int chain;  // SACF_CHAIN_* of this step
  int wt;     // write-through mask of this launch (WT_*, wt_mask_for)
  Scr s;
  Layout L;
  Hyper hp;
};

// Diagnostics build only (-DSACF_PHASE_TIMING, scripts/sac_phase_timing.py): wave 0 of every block of the three
// step kernels stamps the device wall clock (100 MHz) at entry (0), operands ready (1), products done (2) and exit
// (3), and at up to four points inside the prologue (4..7; SAC_STAMP_ON: after the value `dep` has landed); the
// product build compiles the stamps out.
#ifdef SACF_PHASE_TIMING
constexpr int kStampBlocks = 8192, kStamps = 8;
__device__ unsigned long long g_sac_stamps[3][kStampBlocks][kStamps];
#define SAC_STAMP(K, P)                                                                               \
  do {                                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) g_sac_stamps[K][blockIdx.x][P] = wall_clock64(); \
  } while (0)
#define SAC_STAMP_ON(K, P, dep)                                                                          \
  do {                                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks && __float_as_uint((float)(dep)) != 0x7FBADBADu) \
      g_sac_stamps[K][blockIdx.x][P] = wall_clock64();                                                   \
  } while (0)
#else
#define SAC_STAMP(K, P) \
  do {                  \
  } while (0)
#define SAC_STAMP_ON(K, P, dep) \
  do {                          \
  } while (0)
#endif

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
// small helpers
// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based; one 4-word draw per batch row and step)
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

// block-wide sum of N (<= 32) per-thread partials; result in out[0..N) (LDS), visible after return
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

// Publication stores. Every value one launch of the step writes for a later launch (activations, parts, the row
// record, the step counter, the updated parameters, optimizer state and transposed copies) is stored write-through
// (`sc1`): the line leaves the XCD's L2 as it is written instead of waiting, dirty, for the end-of-kernel release,
// which otherwise writes back every dirty byte before the next launch may start (MI355X_MICROARCH.md "boundary":
// + B ÷ 6 TB/s for B dirty bytes; "publish-large": write-through wins for tens of KB per workgroup). The readers
// are other launches, so no store here is read back through the writer's L2. SACF_WT selects which stores publish
// write-through (a bit mask, for A/Bs): 1 the row inputs, parts, records and first-layer slices P1 / P2 hand on;
// 4 the split-K epilogues' activation and factor matrices (one word per lane and output); 2 what P3 (and the apply
// kernel) writes: gradients, Adam state, parameters, targets and the transposed copies. 0: plain stores. The launch
// chooses within that mask at run time (MArgs / ApplyArgs::wt, wt_mask_for below): the split-K epilogues' matrices
// are written through from 128 batch rows up — at B = 256 write-through takes 28.7 µs per step against 29.8 µs, at
// B = 64 the same stores cost more than the smaller dirty set's write-back (25.6 against 25.0 µs; without the
// row / part bits 24.6 µs): profiles/round6/r6b_*
#ifndef SACF_WT
#define SACF_WT 7
#endif
enum { WT_ACT = 1, WT_OPT = 2, WT_EPI = 4 };
// (not a store class: set in the weight-gradient kernel's mask, its launch does not write the flat gradient —
// SACF_CHAIN_NO_GRADS with the update fused; a compile-time choice: a run-time test around the stores cost 0.5 µs)
constexpr int WT_NOG = 8;
// the two masks the step kernels are instantiated with (the launch picks by batch: wt_mask_for)
constexpr int kWtLarge = WT_ACT | WT_OPT | WT_EPI, kWtSmall = WT_OPT | WT_EPI;
// (wt: the launch's mask — a template argument of every kernel that stores, so the test folds at compile time: a
// run-time test per store cost 2 µs per grad step)
template <int KIND>
__device__ __forceinline__ bool wt_on(int wt) {
  return (SACF_WT & KIND) != 0 && (wt & KIND) != 0;
}
template <int KIND, class T>
__device__ __forceinline__ void pub(int wt, T* p, T v) {
  if (wt_on<KIND>(wt)) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <int KIND>
__device__ __forceinline__ void pub4(int wt, float* p, float x, float y, float z, float w) {
  if (wt_on<KIND>(wt)) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const f32x4 v = {x, y, z, w};
    // (the compiler's hazard recognizer does not see an asm store: a store of more than 8 bytes needs a wait state
    // before a VALU instruction may overwrite its data registers, hence the s_nop)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(x, y, z, w);
  }
}

__device__ __forceinline__ float relu(float x) { return fmaxf(x, 0.0f); }
__device__ __forceinline__ float softplus(float x) { return x > 20.0f ? x : log1pf(expf(x)); }

// a pointer read from LDS has no address space for the compiler (flat loads, which also count on the LDS
// counter and get conservative waits): the operand matrices are all device memory
typedef const float __attribute__((address_space(1)))* gptr;
__device__ __forceinline__ gptr as_global(const float* p) { return (gptr)p; }

// n (compile-time) contiguous floats from p, 16-byte aligned when n % 4 == 0: float4 loads then
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

// Σ of n column-block parts in block order (a left fold: the consumer's sum is the same for every reader)
template <int N>
__device__ __forceinline__ float fold(const float (&v)[N]) {
  float s = v[0];
#pragma unroll
  for (int i = 1; i < N; ++i) s += v[i];
  return s;
}

// ---------------------------------------------------------------------------------------------
// MFMA tiles. Every GEMM runs in 32-row x 32-column output tiles, one 256-thread block (4 waves) per
// tile, the K dimension split over the 4 waves and the 4 partial tiles summed in LDS in a fixed order.
// Operand maps (cdna_hip_programming.md §3): lane l holds A[l & 31][k] and B[k][l & 31]; the lane's K
// slice is k = kb + i, kb = w·H/4 + (l >> 5)·H/8 (a permuted k order: the sum is the same, the loads stay
// contiguous per lane / per half wave), processed in chunks of CS MFMAs. C/D: col = l & 31,
// row = (reg & 3) + 8·(reg >> 2) + 4·(l >> 5).
// ---------------------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int H>
struct KSlice {
  static constexpr int N2 = H / 8;                    // K values per lane
  static constexpr int CS = N2 <= 32 ? N2 : N2 / 2;   // per chunk (H > 256: two chunks)
  static constexpr int NCH = N2 / CS;
  static constexpr int CB = H / kTile2;               // 32-column blocks
  static_assert(hidden_ok(H), "hidden width without kernels");
  static_assert(CS <= kMaxN2 && CS % 4 == 0, "chunk");
};

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int g = 0; g < 16; ++g) z[g] = 0.0f;
  return z;
}

// acc += Σ_i A_i ⊗ B_i over n MFMAs (compile-time n)
template <int N>
__device__ __forceinline__ void mfma_n(f32x16& acc, const float (&a)[N], const float (&b)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[i], acc, 0, 0, 0);
}
// ... over the first n of kMaxN2 (run-time n)
__device__ __forceinline__ void mfma_chain(f32x16& acc, const float (&a)[kMaxN2], const float (&b)[kMaxN2], int n) {
#pragma unroll
  for (int i = 0; i < kMaxN2; ++i)
    if (i < n) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[i], acc, 0, 0, 0);
}

// Sum of the 4 waves' partial tiles (wave 0 + 1 + 2 + 3, in that order) through lds (4·16·64 floats),
// then epi(q, row, col, v) on the 1024 outputs: wave w finishes accumulator registers 4w .. 4w + 3
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
    epi(q, (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5), lane & 31, v);
  }
}
// the same for two accumulators (two split regions of lds) behind one barrier: epi(q, row, col, v0, v1)
template <class EPI>
__device__ __forceinline__ void splitk_finish2(const f32x16& acc0, const f32x16& acc1, float* lds0, float* lds1,
                                               EPI&& epi) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    lds0[(w * 16 + g) * 64 + lane] = acc0[g];
    lds1[(w * 16 + g) * 64 + lane] = acc1[g];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int g = 4 * w + q;
    float v0 = lds0[(0 * 16 + g) * 64 + lane], v1 = lds1[(0 * 16 + g) * 64 + lane];
    v0 += lds0[(1 * 16 + g) * 64 + lane];
    v1 += lds1[(1 * 16 + g) * 64 + lane];
    v0 += lds0[(2 * 16 + g) * 64 + lane];
    v1 += lds1[(2 * 16 + g) * 64 + lane];
    v0 += lds0[(3 * 16 + g) * 64 + lane];
    v1 += lds1[(3 * 16 + g) * 64 + lane];
    epi(q, (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5), lane & 31, v0, v1);
  }
}
// A 32 x 32 epilogue tile staged in LDS (stage[row · kStageLd + col], written by splitk_finish's epilogue: one value
// per lane and output register, a word store each) out to dst[row · ld + col] as 16-byte stores: thread t writes row
// t / 8, columns 4 (t mod 8) .. 4 (t mod 8) + 3 (dst 16-byte aligned, ld a multiple of 4)
constexpr int kStageLd = kTile2 + 4;
template <int WTM>
__device__ __forceinline__ void tile_out(const float* stage, float* dst, int ld) {
  __syncthreads();
  const int row = (int)threadIdx.x >> 3, c4 = ((int)threadIdx.x & 7) * 4;
  const float4 v = *reinterpret_cast<const float4*>(stage + row * kStageLd + c4);
  pub4<WT_EPI>(WTM, dst + (int64_t)row * ld + c4, v.x, v.y, v.z, v.w);
}

// per-row words of a 32-row tile that splitk_finish's epilogue left in LDS (rwl[set · 32 + row], by its cc == 0
// lanes) out to the row-tile layout, dst[set] the run of the tile's 32 rows: wave w writes rows 8w .. 8w + 7, the
// rows splitk_finish gives it, so the LDS round trip stays inside the wave (no block barrier)
template <int WTM, int NS, class T>
__device__ __forceinline__ void row_words_out(const T* rwl, T* const (&dst)[NS]) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
  if (lane < 8 * NS) {
    const int st = lane >> 3, row = 8 * w + (lane & 7);
    pub<WT_ACT>(WTM, dst[st] + row, rwl[st * 32 + row]);
  }
}

// the row of output register q (0..3) of this lane in splitk_finish's order (defined below)
__device__ __forceinline__ int finish_row(int q);

// The same for up to two tiles whose values the epilogue kept in registers (v[q] at row finish_row(q), column lane & 31):
// staged into the split-K regions once their last reads are done (one more barrier), then out as 16-byte stores
template <int WTM, int NT>
__device__ __forceinline__ void tiles_out(const float (&v)[NT][4], float* const (&stage)[NT], float* const (&dst)[NT],
                                          int ld) {
  __syncthreads();  // (every wave's reads of the split regions are done)
  const int col = (int)threadIdx.x & 31;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) stage[t][finish_row(q) * kStageLd + col] = v[t][q];
  __syncthreads();
  const int row = (int)threadIdx.x >> 3, c4 = ((int)threadIdx.x & 7) * 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float4 x = *reinterpret_cast<const float4*>(stage[t] + row * kStageLd + c4);
    pub4<WT_EPI>(WTM, dst[t] + (int64_t)row * ld + c4, x.x, x.y, x.z, x.w);
  }
}

// the row of output register q (0..3) of this lane in splitk_finish's order
__device__ __forceinline__ int finish_row(int q) {
  const int g = 4 * (threadIdx.x >> 6) + q;
  return (g & 3) + 8 * (g >> 2) + 4 * ((threadIdx.x & 63) >> 5);
}

// Σ of x over the 32 lanes of this half wave (the 32 columns of one output row), every lane ending with the same
// bits: a pairwise tree in registers — lane ^ 1, lane ^ 2 (quad permutes), the two quads of each 8 (half-row
// mirror), the two halves of each 16 (row mirror), then the two rows of the half wave (v_permlane16_swap) — each
// step adds a pair of equal values in either order, so the partners' sums are equal (no LDS round trip per step)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float halfwave_sum(float x) {
  x += dpp_f<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp_f<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp_f<0x141>(x);  // row_half_mirror
  x += dpp_f<0x140>(x);  // row_mirror
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // (rows 2k, 2k + 1: the same order in both)
}

// B operand chunk: bv[i] = base[(k0 + i)·H + col] (W2ᵀ for a forward product, W2 for a backward factor)
template <int CS>
__device__ __forceinline__ void load_b(float (&bv)[CS], const float* base, int H, int k0, int col) {
#pragma unroll
  for (int i = 0; i < CS; ++i) bv[i] = base[(int64_t)(k0 + i) * H + col];
}

// W1 [H][nin] (row-major in the parameters) into LDS as W1ᵀ [nin][H], and b1 [H] after it, in two halves: load()
// issues this thread's loads into registers, store() writes LDS (and so waits for them) — the caller places other
// loads in between by what its critical chain needs first (vmcnt counts loads in issue order)
template <int H>
struct W1Stage {
  static constexpr int kIt = (H * kXLd + kThreads - 1) / kThreads, kB = (H + kThreads - 1) / kThreads;
  float v[kIt], bb[kB];
  __device__ __forceinline__ void load(const float* w1, const float* b1, int nin) {
    const int n = H * nin, tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < kIt; ++i) v[i] = tid + i * kThreads < n ? w1[tid + i * kThreads] : 0.0f;
#pragma unroll
    for (int i = 0; i < kB; ++i) bb[i] = tid + i * kThreads < H ? b1[tid + i * kThreads] : 0.0f;
  }
  __device__ __forceinline__ void store(float* dst, int nin) const;
};
template <int H>
__device__ __forceinline__ void W1Stage<H>::store(float* dst, int nin) const {
  const int n = H * nin, tid = threadIdx.x;
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
#pragma unroll
  for (int i = 0; i < kB; ++i)
    if (tid + i * kThreads < H) dst[nin * H + tid + i * kThreads] = bb[i];
}

// av[i] = relu(b1[k] + Σ_{m < nin} W1[k][m] · in[m]) for k = k0 + i: an fmaf chain from the bias in input
// order, as fc0 computes one output
template <int H, int CS>
__device__ __forceinline__ void first_layer(const float* lw1t, const float* xin, int nin, int k0, float (&av)[CS]) {
#pragma unroll
  for (int i = 0; i < CS; ++i) av[i] = lw1t[nin * H + k0 + i];
  for (int m = 0; m < nin; ++m) {
    const float xm = xin[m];
#pragma unroll
    for (int i = 0; i < CS; ++i) av[i] = fmaf(lw1t[m * H + k0 + i], xm, av[i]);
  }
#pragma unroll
  for (int i = 0; i < CS; ++i) av[i] = relu(av[i]);
}

// the same chain, also returning its value before the last input's term (the critics' pre-activation without the
// action: fmaf(W1[k][nin - 1], x[nin - 1], pre) is exactly the chain's last step)
template <int H, int CS>
__device__ __forceinline__ void first_layer_pre(const float* lw1t, const float* xin, int nin, int k0, float (&pre)[CS],
                                                float (&av)[CS]) {
#pragma unroll
  for (int i = 0; i < CS; ++i) pre[i] = lw1t[nin * H + k0 + i];
  for (int m = 0; m < nin - 1; ++m) {
    const float xm = xin[m];
#pragma unroll
    for (int i = 0; i < CS; ++i) pre[i] = fmaf(lw1t[m * H + k0 + i], xm, pre[i]);
  }
  const float xl = xin[nin - 1];
#pragma unroll
  for (int i = 0; i < CS; ++i) av[i] = relu(fmaf(lw1t[(nin - 1) * H + k0 + i], xl, pre[i]));
}

// this lane's first-layer chunk (row lane & 31, columns k0 .. k0 + CS) out to its row of the matrix by the block that
// owns column block k0 / 32 (every block computes the same values). A chunk of exactly one column block (CS = 32: H =
// 256, 512) goes through the half wave's own 32 x 32 tile in LDS (st) and out as whole 128-byte row segments, four
// rows per store instruction, still inside the product loop; other chunks straight from registers as 16-byte
// pieces. (Each 16-byte store instruction of the direct form wrote 32 rows' pieces: P1 0.85 µs longer at B = 256 than
// without these stores; staged to the block's end they moved the cost into the launch boundary, profiles/round6/r6s_*.)
template <int H, int CS, int WTM>
__device__ __forceinline__ void slice_out(float* st, float* base, int r0, int by, const float (&av)[CS], int k0) {
  if (k0 / kTile2 != by) return;
  const int rl = (int)threadIdx.x & 31;
  if constexpr (CS == kTile2 && (WTM & WT_ACT) != 0) {  // (plain stores, the small-batch mask: direct)
    float* d = st + rl * kStageLd;
#pragma unroll
    for (int q = 0; q < CS / 4; ++q)
      *reinterpret_cast<float4*>(d + 4 * q) = make_float4(av[4 * q], av[4 * q + 1], av[4 * q + 2], av[4 * q + 3]);
    // (the lanes reading back are the writing half wave's own: in-order LDS, a compiler barrier only)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int lr = rl >> 3, c4 = (rl & 7) * 4;
    float* g = base + (int64_t)r0 * H + k0 + c4;
#pragma unroll
    for (int j = 0; j < kTile2 / 4; ++j) {
      const int row = 4 * j + lr;
      const float4 v = *reinterpret_cast<const float4*>(st + row * kStageLd + c4);
      pub4<WT_ACT>(WTM, g + (int64_t)row * H, v.x, v.y, v.z, v.w);
    }
  } else {
    float* d = base + (int64_t)(r0 + rl) * H + k0;
#pragma unroll
    for (int q = 0; q < CS / 4; ++q) pub4<WT_ACT>(WTM, d + 4 * q, av[4 * q], av[4 * q + 1], av[4 * q + 2], av[4 * q + 3]);
  }
}

// a batch row's O inputs, zero past O, branch-free: a clamped index and a compare against O held in a VGPR, so
// no per-input lane mask is kept live (at H > 256 those masks spilled)
__device__ __forceinline__ void load_obs_row(const float* src, int64_t idx, int O, float (&x)[kXLd]) {
  int Ov = O;
  asm volatile("" : "+v"(Ov));
  if ((O & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {  // (uniform) 16-byte rows: kXLd / 4 float4s
    const float4* p = reinterpret_cast<const float4*>(src + idx * O);
#pragma unroll
    for (int q = 0; q < kXLd / 4; ++q) {
      const float4 v = p[min(q, (Ov >> 2) - 1)];
      const bool in = 4 * q < Ov;
      x[4 * q] = in ? v.x : 0.0f;
      x[4 * q + 1] = in ? v.y : 0.0f;
      x[4 * q + 2] = in ? v.z : 0.0f;
      x[4 * q + 3] = in ? v.w : 0.0f;
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < kXLd; ++m) {
    const float v = src[idx * O + min(m, Ov - 1)];
    x[m] = m < Ov ? v : 0.0f;
  }
}

// LDS of the forward kernels (P1, P2, policy act): two split-K regions, W1ᵀ | b1, the tile's input rows
template <int H>
struct FwdLds {
  static constexpr int kSplit = 4 * 16 * 64;
  static constexpr int kW1 = H * kXLd + H;
  static constexpr int kX = 32 * (kXLd + 1);
  static constexpr int kFloats = 2 * kSplit + kW1 + kX;
  static constexpr int kW1Off = 2 * kSplit;
  static constexpr int kXOff = 2 * kSplit + kW1;
  static_assert(3 * kTile2 * kStageLd + 3 * 32 <= kSplit, "P1's staged tiles and row words share the second split region");
};

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

// one batch item (replay sample or given batch) and its two reparameterisation normals; padding rows
// (item >= B) read a valid row and draw zero noise
__device__ __forceinline__ int64_t batch_item(const MArgs& a, int item, float& e0, float& e1) {
  const int B = a.L.B;
  const bool pad = item >= B;
  int64_t idx = pad ? B - 1 : item;
  uint32_t c[4] = {(uint32_t)item, (uint32_t)*a.step, (uint32_t)((uint64_t)*a.step >> 32), 0x5AC0u};
  if (a.sampled || !a.eps) philox(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
  if (a.sampled) {
    const int64_t size = *a.size_dev > 0 ? *a.size_dev : 1;
    const double u = ((double)c[0] + 0.5) * (1.0 / 4294967296.0);
    idx = (int64_t)(u * (double)size);
    if (idx >= a.capacity) idx = a.capacity - 1;
  }
  if (a.eps) {
    e0 = pad ? 0.0f : a.eps[item];
    e1 = pad ? 0.0f : a.eps[B + item];
  } else {
    const float u1 = ((float)c[1] + 1.0f) * 2.3283064365386963e-10f;
    const float u2 = (float)c[2] * 2.3283064365386963e-10f;
    const float rad = sqrtf(-2.0f * logf(u1));
    e0 = rad * cosf(6.283185307179586f * u2);
    e1 = rad * sinf(6.283185307179586f * u2);
  }
  return idx;
}

// the obs row (next_obs with nx) of batch item `item` into x: gathered from the replay (batch_item's draw; e0 / e1
// its normals, idx its replay row), or (chain FROM_STAGED) the row the previous step's P3 staged — the same values
__device__ __forceinline__ int64_t batch_row(const MArgs& a, int item, bool nx, float (&x)[kXLd], float& e0, float& e1) {
  if (a.chain & SACF_CHAIN_FROM_STAGED) {
    load_run<kXLd>((nx ? a.s.sxn : a.s.sx) + (int64_t)item * kXLd, x);
    e0 = e1 = 0.0f;  // (read from the staged aux where needed)
    return -1;
  }
  const int64_t idx = batch_item(a, item, e0, e1);
  load_obs_row(nx ? a.nobs : a.obs, idx, a.L.O, x);
  return idx;
}
// (act, rew, term, e0, e1) of batch item `item` whose row batch_row returned idx / e0 / e1
__device__ __forceinline__ void batch_aux(const MArgs& a, int item, int64_t idx, float e0, float e1, float (&v)[5]) {
  if (a.chain & SACF_CHAIN_FROM_STAGED) {
    const float* q = a.s.saux + (int64_t)item * kAux;
    const float4 u = *reinterpret_cast<const float4*>(q);
    v[AUX_ACT] = u.x; v[AUX_REW] = u.y; v[AUX_TERM] = u.z; v[AUX_E0] = u.w; v[AUX_E1] = q[AUX_E1];
    return;
  }
  v[AUX_ACT] = a.act[idx]; v[AUX_REW] = a.rew[idx]; v[AUX_TERM] = a.term[idx]; v[AUX_E0] = e0; v[AUX_E1] = e1;
}

// linear block id -> (row tile bx, column tile by): column tile = id mod CB, so with CB a multiple of 8 every
// block of one column tile runs on one XCD (blocks are dealt round-robin over the 8 XCDs) and that XCD's L2
// holds the column's weight slice (any placement gives the same results)
template <int H>
__device__ __forceinline__ void tile_of(int& bx, int& by) {
  constexpr int CB = H / kTile2;
  by = (int)blockIdx.x % CB;
  bx = (int)blockIdx.x / CB;
}

// ---------------------------------------------------------------------------------------------
// P1 (sac_fwd_kernel): row tiles [obs (Bp/32) | next_obs (Bp/32) | Q1 data (Bp/32) | Q2 data (Bp/32)] x CB
// ---------------------------------------------------------------------------------------------
// the gathered batch for the later passes of the step — the obs row, act / rew / term and the two normals — of
// batch item `item` (its replay row idx and normals as batch_item drew them) by the eight threads of its row in the
// T1 fc0 tiles of column block 0 (short tiles: in the actor tiles this hand-on set P1's span): thread j < 4 a quarter
// of the obs row (16 bytes; a row tile's rows are one contiguous run), j = 4 .. 7 the record words (each a run of the
// row tile's rows in the record's layout). load() at the tile's start, store() at its end: stored at once, the
// loads' wait held the tile's own operand loads back (the T1 tiles of column block 0 ended P1 1 µs late,
// profiles/round6/r6z_*)
struct HandOn {
  float v[4];
  __device__ __forceinline__ void load(const MArgs& a, int item, int64_t idx, float e0, float e1, int j) {
    const bool staged = (a.chain & SACF_CHAIN_FROM_STAGED) != 0;
    if (j < 4) {
      if (staged) {
        const float4 u = *reinterpret_cast<const float4*>(a.s.sx + (int64_t)item * kXLd + 4 * j);
        v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
      } else {
        const int O = a.L.O;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = 4 * j + k;
          const float x = a.obs[idx * O + min(c, O - 1)];
          v[k] = c < O ? x : 0.0f;
        }
      }
      return;
    }
    const float* sa = a.s.saux + (int64_t)item * kAux;
    if (j == 4) v[0] = staged ? sa[AUX_E0] : e0;
    else if (j == 5) v[0] = staged ? sa[AUX_E1] : e1;
    else if (j == 6) v[0] = staged ? sa[AUX_REW] : a.rew[idx];
    else {
      v[0] = staged ? sa[AUX_TERM] : a.term[idx];
      v[1] = staged ? sa[AUX_ACT] : a.act[idx];
    }
  }
  template <int WTM>
  __device__ __forceinline__ void store(const MArgs& a, int item, int j) const {
    float* rc = a.s.rec;
    if (j < 4) pub4<WT_ACT>(WTM, a.s.x + (int64_t)item * kXLd + 4 * j, v[0], v[1], v[2], v[3]);
    else if (j == 4) pub<WT_ACT>(WTM, rc + rec_at(item, R_EPS), v[0]);
    else if (j == 5) pub<WT_ACT>(WTM, rc + rec_at(item, R_EPSN), v[0]);
    else if (j == 6) pub<WT_ACT>(WTM, rc + rec_at(item, R_REW), v[0]);
    else {
      pub<WT_ACT>(WTM, rc + rec_at(item, R_TERM), v[0]);
      pub<WT_ACT>(WTM, rc + rec_at(item, R_ACT), v[1]);
    }
  }
};

// actor forward (gaussian_policy.py:105-118 up to the heads, mlp.py:86-99): h1 = relu(W1 x + b1) on the VALU,
// h2 = relu(h1 W2ᵀ + b2) on MFMA, the mean / log_std head parts of this column block in the epilogue
template <int H, int WTM>
__device__ __forceinline__ void p1_actor_tile(const MArgs& a, int rt, int by, float* lds) {
  using KS = KSlice<H>;
  constexpr int CS = KS::CS, CB = KS::CB;
  const Layout& L = a.L;
  const int O = L.O, B = L.B, Bp = L.Bp;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
  const int r0 = rt * kTile2, c0 = by * kTile2;
  const int kb = w * (H / 4) + h * KS::N2;
  // the batch gather first: its chain (step / size -> Philox -> replay row) is the longest of the prologue
  const int row = r0 + rl;
  const bool nrow = row >= Bp, nrow_tile = r0 >= Bp;  // (next_obs rows: a whole row tile)
  const int item = nrow ? row - Bp : row;
  float e0, e1;
  float x[kXLd];
  const int64_t idx = batch_row(a, item, nrow, x, e0, e1);
  SAC_STAMP_ON(0, 4, idx);
  SAC_STAMP_ON(0, 5, x[0]);
  // then W1 (needed before the barrier), then the B operand and epilogue weights (needed after it): the LDS
  // stores below wait for W1 only
  W1Stage<H> w1s;
  w1s.load(P + L.p_w1, P + L.p_b1, O);
  float bv[CS];
  load_b<CS>(bv, a.T, H, kb, c0 + rl);  // actor W2ᵀ, chunk 0
  const float b2c = P[L.p_b2 + c0 + rl];
  const float wm = P[L.p_wm + c0 + rl], ws = P[L.p_ws + c0 + rl];
  float* lw1 = lds + FwdLds<H>::kW1Off;
  float* lx = lds + FwdLds<H>::kXOff;
  w1s.store(lw1, O);
  SAC_STAMP(0, 6);
  if (w == 0 && h == 0) {
#pragma unroll
    for (int m = 0; m < kXLd; ++m) lx[rl * (kXLd + 1) + m] = x[m];  // (zero past O: no per-m mask kept live)
  }
  (void)B;
  __syncthreads();
  SAC_STAMP(0, 1);
  float* stage = lds + FwdLds<H>::kSplit;  // (the second split region: free in P1) h2 | h1 tiles
  float* st_h1 = stage + kTile2 * kStageLd;
  f32x16 acc = zero16();
#pragma unroll
  for (int c = 0; c < KS::NCH; ++c) {
    const int k0 = kb + c * CS;
    if (c) load_b<CS>(bv, a.T, H, k0, c0 + rl);
    float av[CS];
    first_layer<H, CS>(lw1, lx + rl * (kXLd + 1), O, k0, av);
    if (!nrow) slice_out<H, CS, WTM>(st_h1, a.s.h1, r0, by, av, k0);
    mfma_n<CS>(acc, av, bv);
  }
  SAC_STAMP(0, 2);
  float* rwl = st_h1 + kTile2 * kStageLd;  // row words: head parts (mean | log_std) [2][32], mask words [32]
  uint32_t* rwm = reinterpret_cast<uint32_t*>(rwl + 2 * kTile2);
  splitk_finish(acc, lds, [&](int, int rr, int cc, float v) {
    const float y = relu(v + b2c);
    stage[rr * kStageLd + cc] = y;
    const uint64_t pos = __ballot(y > 0.0f);  // (rows of the two half waves: the low / high 32 bits)
    const float pm = halfwave_sum(y * wm), ps = halfwave_sum(y * ws);
    if (cc == 0) {
      rwm[rr] = (uint32_t)(lane < 32 ? pos : pos >> 32);
      rwl[rr] = pm;
      rwl[kTile2 + rr] = ps;
    }
  });
  {
    float* const dp[2] = {a.s.hpart + rw_at(r0, 0, 2, CB, by), a.s.hpart + rw_at(r0, 1, 2, CB, by)};
    row_words_out<WTM, 2>(rwl, dp);
    if (!nrow_tile) {
      uint32_t* const dm[1] = {a.s.h2m + rw_at(r0, 0, 1, CB, by)};
      row_words_out<WTM, 1>(rwm, dm);
    }
  }
  (void)Bp;
  if (!nrow_tile) tile_out<WTM>(stage, a.s.h2 + (int64_t)r0 * H + c0, H);
}

// critic forward on the (obs, a) data rows of one critic (mlp.py:127-136 ConcatMlp): the row's observation and
// replayed action straight from the batch source (the same Philox draw as the actor tile's gather)
template <int H, int WTM>
__device__ __forceinline__ void p1_data_tile(const MArgs& a, int net, int rt, int by, float* lds) {
  using KS = KSlice<H>;
  constexpr int CS = KS::CS, CB = KS::CB;
  const Layout& L = a.L;
  const int O = L.O, Bp = L.Bp;
  const float* P = a.params;
  const float* C = P + L.q_base[net];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
  const int r0 = rt * kTile2, c0 = by * kTile2;
  const int kb = w * (H / 4) + h * KS::N2;
  const int item = r0 + rl;
  float e0, e1;
  float xin[kXLd];
  const int64_t idx = batch_row(a, item, false, xin, e0, e1);
  const float act = (a.chain & SACF_CHAIN_FROM_STAGED) ? a.s.saux[(int64_t)item * kAux + AUX_ACT] : a.act[idx];
  W1Stage<H> w1s;
  w1s.load(C + L.c_w1, C + L.c_b1, O + 1);
  float bv[CS];
  const float* WT = a.T + (int64_t)(1 + net) * H * H;
  load_b<CS>(bv, WT, H, kb, c0 + rl);
  const float b2c = C[L.c_b2 + c0 + rl], w3 = C[L.c_w3 + c0 + rl];
  float* lw1 = lds + FwdLds<H>::kW1Off;
  float* lx = lds + FwdLds<H>::kXOff;
  w1s.store(lw1, O + 1);
  if (w == 0 && h == 0) {
#pragma unroll
    for (int m = 0; m < kXLd; ++m) lx[rl * (kXLd + 1) + m] = xin[m];  // (zero past O; the action goes at O)
    lx[rl * (kXLd + 1) + O] = act;
  }
  __syncthreads();
  if (net == 0 && by == 0 && threadIdx.x < kTile2 * 4) {  // the (obs | a) rows for P3: 16 bytes per thread, one run
    const int row = (int)threadIdx.x >> 2, q4 = ((int)threadIdx.x & 3) * 4;
    const float* l = lx + row * (kXLd + 1) + q4;
    pub4<WT_ACT>(WTM, a.s.qx + (int64_t)(r0 + row) * kXLd + q4, l[0], l[1], l[2], l[3]);
  }
  SAC_STAMP(0, 1);
  float* stage = lds + FwdLds<H>::kSplit;  // (the second split region: free in P1) g2 | g1 | pre tiles
  float* st_g1 = stage + kTile2 * kStageLd;
  float* st_pre = st_g1 + kTile2 * kStageLd;
  f32x16 acc = zero16();
#pragma unroll
  for (int c = 0; c < KS::NCH; ++c) {
    const int k0 = kb + c * CS;
    if (c) load_b<CS>(bv, WT, H, k0, c0 + rl);
    float av[CS], pre[CS];
    first_layer_pre<H, CS>(lw1, lx + rl * (kXLd + 1), O + 1, k0, pre, av);
    slice_out<H, CS, WTM>(st_g1, a.s.g1[net], r0, by, av, k0);
    slice_out<H, CS, WTM>(st_pre, a.s.pre[net], r0, by, pre, k0);
    mfma_n<CS>(acc, av, bv);
  }
  if (rt == 0 && by == 0)  // fc0's action column, contiguous, for P2
    for (int k = threadIdx.x; k < H; k += kThreads) pub<WT_ACT>(WTM, a.s.w1a + net * H + k, lw1[O * H + k]);
  SAC_STAMP(0, 2);
  float* rwl = st_pre + kTile2 * kStageLd;  // row words: parts [32], mask words [32]
  uint32_t* rwm = reinterpret_cast<uint32_t*>(rwl + kTile2);
  splitk_finish(acc, lds, [&](int, int rr, int cc, float v) {
    const float y = relu(v + b2c);
    stage[rr * kStageLd + cc] = y;
    const uint64_t pos = __ballot(y > 0.0f);
    const float pq = halfwave_sum(y * w3);  // this column block's part of g2 · w3 for row r0 + rr
    if (cc == 0) {
      rwm[rr] = (uint32_t)(lane < 32 ? pos : pos >> 32);
      rwl[rr] = pq;
    }
  });
  {
    float* const dp[1] = {a.s.part + rw_at(r0, PS_Q1D + net, PS_N, CB, by)};
    row_words_out<WTM, 1>(rwl, dp);
    uint32_t* const dm[1] = {a.s.g2m[net] + rw_at(r0, 0, 1, CB, by)};
    row_words_out<WTM, 1>(rwm, dm);
  }
  tile_out<WTM>(stage, a.s.g2[net] + (int64_t)r0 * H + c0, H);
}

// target critic `net`'s fc0 pre-activation (without the action term) on the next_obs rows of row tile rt, columns
// by·32 .. by·32 + 31: the block stages those 32 rows of W1 (and b1) in LDS with coalesced loads, then thread t takes
// row t / 8 and four columns, the fmaf chain from the bias in input order as first_layer; row tile 0 also writes
// fc0's action column of those columns
template <int H, int WTM>
__device__ __forceinline__ void p1_target_pre_tile(const MArgs& a, int net, int rt, int by, float* lds) {
  const Layout& L = a.L;
  const int O = L.O, nin = O + 1;
  const float* C = a.targets + (int64_t)net * L.q_size;
  const int tid = threadIdx.x, row = tid >> 3, cq = (tid & 7) * 4, c0 = by * kTile2;
  const int item = rt * kTile2 + row;
  float e0, e1;
  float x[kXLd];
  const int64_t idx = batch_row(a, item, true, x, e0, e1);
  const bool hand_on = net == 0 && by == 0;
  HandOn ho;
  if (hand_on) ho.load(a, item, idx, e0, e1, tid & 7);
  float* w1 = lds;                   // [32][kXLd + 1]: W1 rows c0 .. c0 + 31
  float* b1 = lds + kTile2 * (kXLd + 1);
  const float* src = C + L.c_w1 + (int64_t)c0 * nin;  // the 32 rows are contiguous: 32·nin floats
  for (int e = tid; e < kTile2 * nin; e += kThreads) {
    const int kk = e / nin;
    w1[kk * (kXLd + 1) + (e - kk * nin)] = src[e];
  }
  if (tid < kTile2) b1[tid] = C[L.c_b1 + c0 + tid];
  __syncthreads();
  float pre[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pre[j] = b1[cq + j];
#pragma unroll
  for (int m = 0; m < kXLd; ++m)  // (unrolled, the run-time bound a select)
#pragma unroll
    for (int j = 0; j < 4; ++j) pre[j] = m < O ? fmaf(w1[(cq + j) * (kXLd + 1) + m], x[m], pre[j]) : pre[j];
  pub4<WT_ACT>(WTM, a.s.pre[2 + net] + (int64_t)item * H + c0 + cq, pre[0], pre[1], pre[2], pre[3]);
  if (rt == 0 && tid < kTile2) pub<WT_ACT>(WTM, a.s.w1a + (2 + net) * H + c0 + tid, w1[tid * (kXLd + 1) + O]);
  if (hand_on) ho.store<WTM>(a, item, tid & 7);
}

template <int H, int WT>
__global__ __launch_bounds__(256) void sac_fwd_kernel(MArgs a) {
  __shared__ float lds[FwdLds<H>::kFloats];
  SAC_STAMP(0, 0);
  int bx, by;
  tile_of<H>(bx, by);
  const int bt = a.L.Bp / kTile2;
  if (bx < 2 * bt) p1_actor_tile<H, WT>(a, bx, by, lds);
  else if (bx < 4 * bt) p1_data_tile<H, WT>(a, (bx - 2 * bt) / bt, (bx - 2 * bt) % bt, by, lds);
  else p1_target_pre_tile<H, WT>(a, (bx - 4 * bt) / bt, (bx - 4 * bt) % bt, by, lds);
  SAC_STAMP(0, 3);
}

// ---------------------------------------------------------------------------------------------
// P2 (sac_mid_kernel): row tiles [Q1, Q2 on (obs, ã) (2Bt) | T1, T2 on (next_obs, ã') (2Bt) | Q1, Q2 data-row factors
// (2Bt) | actor factors U_m (Bt) | U_s (Bt)] x CB; the target tiles also advance the step counter and snapshot for P3
// ---------------------------------------------------------------------------------------------
// the actor head of a row from its column-block parts (summed in block order) and its TanhNormal sample
template <int CB>
struct RowHeadIn {
  float pm[CB], pl[CB], bm, bs;
  __device__ __forceinline__ void load(const MArgs& a, int hrow) {
#pragma unroll
    for (int b = 0; b < CB; ++b) {
      pm[b] = a.s.hpart[rw_at(hrow, 0, 2, CB, b)];
      pl[b] = a.s.hpart[rw_at(hrow, 1, 2, CB, b)];
    }
    bm = a.params[a.L.p_bm];
    bs = a.params[a.L.p_bs];
  }
  __device__ __forceinline__ void head(float ev, float hd[6]) const {
    tanh_normal(fold(pm) + bm, fold(pl) + bs, ev, hd);
  }
};

// Q(obs, ã) of critic `net` and its tangent along the action: with t1 = [g1 > 0] ⊙ W1[:, a] (fc0's action
// column), v = t1 W2ᵀ and ∂Q/∂ã = Σ_cols w3 ⊙ [g2 > 0] ⊙ v (forward mode: one more MFMA chain on the same W2ᵀ
// operand). Also target rows (kTarget: T1 / T2 on (next_obs, ã'), no tangent).
template <int H, bool kTarget, int WTM>
__device__ __forceinline__ void p2_critic_tile(const MArgs& a, int net, int rt, int by, float* lds) {
  using KS = KSlice<H>;
  constexpr int CS = KS::CS, CB = KS::CB;
  const Layout& L = a.L;
  const int O = L.O, Bp = L.Bp;
  const float* C = kTarget ? a.targets + (int64_t)net * L.q_size : a.params + L.q_base[net];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
  const int r0 = rt * kTile2, c0 = by * kTile2;
  const int kb = w * (H / 4) + h * KS::N2;
  const int item = r0 + rl;
  // fc0 from P1's pre-activation of this row (without the action term) plus the action term on ã — the same fmaf
  // chain as fc0 on (obs, ã), so no W1 staging and no block barrier before the products. Loads in the order their
  // consumers need them (vmcnt counts in issue order): the row's head parts (the head's transcendentals are the
  // prologue's longest chain), the pre-activation and action column of this lane's K slice, the B operand
  RowHeadIn<CB> rh;
  rh.load(a, (kTarget ? Bp : 0) + item);
  const float ev = a.s.rec[rec_at(item, kTarget ? R_EPSN : R_EPS)];
  const float* PRE = a.s.pre[(kTarget ? 2 : 0) + net] + (int64_t)item * H;
  const float* W1A = a.s.w1a + ((kTarget ? 2 : 0) + net) * H;
  float pre[CS], wa[CS];
  load_run<CS>(PRE + kb, pre);
  load_run<CS>(W1A + kb, wa);
  float bv[CS];
  const float* WT = a.T + (int64_t)((kTarget ? 3 : 1) + net) * H * H;
  load_b<CS>(bv, WT, H, kb, c0 + rl);
  const float b2c = C[L.c_b2 + c0 + rl], w3 = C[L.c_w3 + c0 + rl];
  float hd[6];
  rh.head(ev, hd);
  SAC_STAMP_ON(1, 4, hd[HD_A]);
  if (w == 0 && h == 0 && net == 0 && by == 0) {
    float* rc = a.s.rec;
    if (kTarget) {
      pub<WT_ACT>(WTM, rc + rec_at(item, R_LOGPN), hd[HD_LOGP]);
    } else {
#pragma unroll
      for (int q = 0; q < 6; ++q) pub<WT_ACT>(WTM, rc + rec_at(item, q), hd[q]);
    }
  }
  (void)O;
  SAC_STAMP(1, 1);
  const float ah = hd[HD_A];
  f32x16 acc = zero16(), act = zero16();
#pragma unroll
  for (int c = 0; c < KS::NCH; ++c) {
    const int k0 = kb + c * CS;
    if (c) {
      load_b<CS>(bv, WT, H, k0, c0 + rl);
      load_run<CS>(PRE + k0, pre);
      load_run<CS>(W1A + k0, wa);
    }
    float av[CS];
#pragma unroll
    for (int i = 0; i < CS; ++i) av[i] = relu(fmaf(wa[i], ah, pre[i]));
    mfma_n<CS>(acc, av, bv);
    if constexpr (!kTarget) {
      float tv[CS];  // the tangent's input: [g1 > 0] ⊙ W1[:, a]
#pragma unroll
      for (int i = 0; i < CS; ++i) tv[i] = av[i] > 0.0f ? wa[i] : 0.0f;
      mfma_n<CS>(act, tv, bv);
    }
  }
  SAC_STAMP(1, 2);
  float* rwl = lds + FwdLds<H>::kW1Off;  // row words (the W1 region: unused in P2)
  if constexpr (kTarget) {
    splitk_finish(acc, lds, [&](int, int rr, int cc, float v) {
      const float pq = halfwave_sum(relu(v + b2c) * w3);
      if (cc == 0) rwl[rr] = pq;
    });
    float* const dp[1] = {a.s.part + rw_at(r0, PS_T1 + net, PS_N, CB, by)};
    row_words_out<WTM, 1>(rwl, dp);
  } else {  // Q and its tangent reduced behind one barrier
    splitk_finish2(acc, act, lds, lds + FwdLds<H>::kSplit, [&](int, int rr, int cc, float v, float t) {
      const float y = relu(v + b2c);
      const float pq = halfwave_sum(y * w3);
      const float pd = halfwave_sum(y > 0.0f ? w3 * t : 0.0f);  // this column block's part of ∂Q/∂ã
      if (cc == 0) {
        rwl[rr] = pq;
        rwl[kTile2 + rr] = pd;
      }
    });
    float* const dp[2] = {a.s.part + rw_at(r0, PS_Q1A + net, PS_N, CB, by),
                          a.s.part + rw_at(r0, PS_D1 + net, PS_N, CB, by)};
    row_words_out<WTM, 2>(rwl, dp);
  }
}

// mask words a lane's K slice (kb = w·H/4 + h·H/8, H/8 columns) spans, the most over the lanes
__host__ __device__ constexpr int mask_words(int H) {
  int most = 1;
  for (int w = 0; w < 4; ++w)
    for (int h = 0; h < 2; ++h) {
      const int kb = w * (H / 4) + h * (H / 8), n = ((kb & 31) + H / 8 - 1) / 32 + 1;
      most = n > most ? n : most;
    }
  return most;
}

// backward factors (the backward pass of layer 2 for a unit head gradient): out[r][j] = [x1[r][j] > 0] ·
// Σ_c W2[c][j] · hw[c] · [x2[r][c] > 0], with (x1, x2, hw) = (h1, h2, wm) → U_m (FK 1) and (h1, h2, ws) → U_s (FK 2)
// for the actor, or (g1, g2, w3) → U_q of a critic on its data rows (FK 0). The B operand is W2 in its own (out, in)
// row-major layout: B[k = c][n = j] = W2[c][j]. One MFMA chain per tile (U_m and U_s are separate tiles: a two-chain tile
// beside another tile on its CU set P2's span).
enum { FK_CRITIC = 0, FK_UM = 1, FK_US = 2 };
template <int H, int FK, int WTM>
__device__ __forceinline__ void p2_factor_tile(const MArgs& a, int net, int rt, int by, float* lds) {
  using KS = KSlice<H>;
  constexpr int CS = KS::CS, N2 = KS::N2;
  constexpr bool kActor = FK != FK_CRITIC;
  const Layout& L = a.L;
  const float* P = a.params;
  const float* C = P + L.q_base[net];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
  const int r0 = rt * kTile2, j0 = by * kTile2;
  const int kb = w * (H / 4) + h * N2;
  const float* X1 = kActor ? a.s.h1 : a.s.g1[net];
  const uint32_t* X2M = kActor ? a.s.h2m : a.s.g2m[net];
  const float* W2 = kActor ? P + L.p_w2 : C + L.c_w2;
  const float* HW = FK == FK_UM ? P + L.p_wm : FK == FK_US ? P + L.p_ws : C + L.c_w3;
  // [x2 > 0] of this lane's K slice (row r0 + rl, columns kb .. kb + N2 - 1): the mask words covering it, and the
  // head weights of those columns
  constexpr int CB = KS::CB, NW = mask_words(H);
  uint32_t mw[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) mw[q] = X2M[rw_at(r0 + rl, 0, 1, CB, min(kb / 32 + q, CB - 1))];
  auto pos2 = [&](int i) __attribute__((always_inline)) {  // bit kb + i (compile-time i)
    const int b = (kb & 31) + i;
    return ((mw[b >> 5] >> (b & 31)) & 1u) != 0u;
  };
  float bv[CS];
  load_b<CS>(bv, W2, H, kb, j0 + rl);
  float m1[4];  // [x1 > 0] of the four outputs this lane finishes
#pragma unroll
  for (int q = 0; q < 4; ++q) m1[q] = X1[(int64_t)(r0 + finish_row(q)) * H + j0 + rl];
  float hw[N2];  // (parameter offsets are not 16-byte aligned: element loads)
#pragma unroll
  for (int i = 0; i < N2; ++i) hw[i] = HW[kb + i];
  SAC_STAMP(1, 1);
  f32x16 acc = zero16();
#pragma unroll
  for (int c = 0; c < KS::NCH; ++c) {
    if (c) load_b<CS>(bv, W2, H, kb + c * CS, j0 + rl);
    float av[CS];
#pragma unroll
    for (int i = 0; i < CS; ++i) av[i] = pos2(c * CS + i) ? hw[c * CS + i] : 0.0f;
    mfma_n<CS>(acc, av, bv);
  }
  SAC_STAMP(1, 2);
  float* o1 = FK == FK_UM ? a.s.um : FK == FK_US ? a.s.us : a.s.uq[net];
  // (out through LDS as 16-byte stores: tiles_out)
  float v[1][4];
  splitk_finish(acc, lds, [&](int q, int, int, float x) { v[0][q] = m1[q] > 0.0f ? x : 0.0f; });
  float* const st[1] = {lds};
  float* const dst[1] = {o1 + (int64_t)r0 * H + j0};
  tiles_out<WTM, 1>(v, st, dst, H);
}

template <int H, int WT>
__global__ __launch_bounds__(256) void sac_mid_kernel(MArgs a) {
  __shared__ float lds[FwdLds<H>::kFloats];
  SAC_STAMP(1, 0);
  // Block order (block i and block i + 256 share a CU): the critic tiles (heavy prologue: the pre-activation rows and
  // the W2ᵀ slice) take the first block of every CU, the backward-factor tiles (a mask word per row) the second, the
  // one-chain critic factors beside the two-chain Q / tangent tiles and the U_m / U_s tiles beside the target tiles.
  // (With the T2 target tiles in second slots their prologue waited 2.5 µs behind the first block's loads, and
  // two-chain tiles sharing a CU stretched each other's products: per-block stamps profiles/round6/r6i_*, r6j_*.)
  // The target tiles, the first to end, also advance the step and snapshot what P3 reads, after their tile: in front
  // of a tile that serial work (a dependent load, the double-precision bias corrections, 4·H stores) held the tile
  // 3 µs, and as an extra block past the 2 × 256 slots it waited for a slot and ended the launch 1.6 µs late.
  const int bt = a.L.Bp / kTile2;
  int bx, by;
  tile_of<H>(bx, by);
  if (bx < 2 * bt) p2_critic_tile<H, false, WT>(a, bx / bt, bx % bt, by, lds);
  else if (bx < 4 * bt) {
    constexpr int CB = H / kTile2;
    const int nt = 2 * bt * CB, part = (int)blockIdx.x - nt, tid = threadIdx.x;
    const Layout& L = a.L;
    const float* P = a.params;
    // the parameters P3 reads (it updates them in place), before this step's update: element e of [5 scalars | 4·H]
    const int e = part * kThreads + tid;
    float sv = 0.0f;
    if (e < 5) sv = e == 0 ? P[0] : e < 3 ? P[L.q_base[e - 1] + L.c_b3] : a.targets[(int64_t)(e - 3) * L.q_size + L.c_b3];
    else if (e < 5 + 4 * H) {
      const int k = e - 5, m = k / H, j = k % H;
      sv = P[(m == 0 ? L.p_wm : m == 1 ? L.p_ws : L.q_base[m - 2] + L.c_w3) + j];
    }
    const bool stepper = part == nt - 1 && tid == 0;
    const int64_t t = stepper ? *a.step + 1 : 0;  // P1 read the old value
    p2_critic_tile<H, true, WT>(a, (bx - 2 * bt) / bt, (bx - 2 * bt) % bt, by, lds);
    if (e < 5) pub<WT_ACT>(WT, a.s.snap + e, sv);
    else if (e < 5 + 4 * H) pub<WT_ACT>(WT, a.s.snap + SN_HEAD + (e - 5), sv);
    if (stepper) {  // step t and Adam's bias corrections
      pub<WT_ACT>(WT, a.step, t);
      const AdamStep st = adam_step(a.hp, t);
      pub<WT_ACT>(WT, a.stats + 5, st.step_pi);
      pub<WT_ACT>(WT, a.stats + 6, st.step_q);
      pub<WT_ACT>(WT, a.stats + 7, st.bc2_sqrt);
    }
  } else if (bx < 6 * bt) p2_factor_tile<H, FK_CRITIC, WT>(a, (bx - 4 * bt) / bt, (bx - 4 * bt) % bt, by, lds);
  else if (bx < 7 * bt) p2_factor_tile<H, FK_UM, WT>(a, 0, bx - 6 * bt, by, lds);
  else p2_factor_tile<H, FK_US, WT>(a, 0, bx - 7 * bt, by, lds);
  SAC_STAMP(1, 3);
}

// ---------------------------------------------------------------------------------------------
// per-row scalars (P3): everything the losses and the weight gradients need of one batch row, from the parts
// the forward passes left (each reader sums them in block order, so every reader gets the same bits)
// ---------------------------------------------------------------------------------------------
// one row's inputs to its scalars: four consecutive part sets (critic: Q1, Q2 on the data rows and the two
// targets; actor: Q1, Q2 on ã and the two tangents) and the row's record. load() only issues the loads, so a caller
// can issue its other loads behind them before the scalars wait for these
template <int CB>
struct RowIn {
  float p[4 * CB], rc[kRec];
  __device__ __forceinline__ void load(const MArgs& a, int r, bool actor) {
    const float* pp = a.s.part + rw_at(r, actor ? PS_Q1A : PS_Q1D, PS_N, CB, 0);  // (set k, block b: + (k·CB + b)·32)
#pragma unroll
    for (int i = 0; i < 4 * CB; ++i) p[i] = pp[(int64_t)i << 5];
    const float* rp = a.s.rec + rec_at(r, 0);  // (word f: + f·32)
#pragma unroll
    for (int f = 0; f < kRec; ++f) rc[f] = rp[f << 5];
  }
  // Σ of set k's column-block parts in block order (a left fold: every reader gets the same bits)
  __device__ __forceinline__ float sum(int k) const {
    float s = p[k * CB];
#pragma unroll
    for (int i = 1; i < CB; ++i) s += p[k * CB + i];
    return s;
  }
};

struct CriticRow {
  float q1, q2, y;  // Q1 / Q2 predictions on (obs, a), the clamped target (sac.py:232-247)
};
template <int CB>
__device__ __forceinline__ CriticRow critic_row(const MArgs& a, const RowIn<CB>& in, float alpha) {
  const float* sn = a.s.snap;  // (the pre-update biases: P3 updates the live ones)
  const float logpn = in.rc[R_LOGPN], rw = in.rc[R_REW], tm = in.rc[R_TERM];
  CriticRow o;
  o.q1 = in.sum(0) + sn[SN_BQ1];
  o.q2 = in.sum(1) + sn[SN_BQ2];
  const float t1 = in.sum(2) + sn[SN_BT1], t2 = in.sum(3) + sn[SN_BT2];
  const float tq = fminf(t1, t2) - alpha * logpn;
  float y = a.hp.rscale * rw + ((1.0f - tm) * a.hp.gamma) * tq;
  o.y = fminf(fmaxf(y, -a.hp.clip), a.hp.clip);
  return o;
}

struct ActorRow {
  float dmean, dls;     // ∂(π-loss)/∂ mean, ∂/∂ log_std (raw, before the clamp's mask)
  float pl, la, ga;     // per-row π-loss, α-loss, ∂α-loss/∂ log α terms
  float logp, mean, std;
};
// π-loss through min(Q1, Q2)(obs, ã) (sac.py:185-205): dA = ∂/∂ã from the tangent parts, then TanhNormal's
// reparameterised backward to (mean, log_std)
template <int CB>
__device__ __forceinline__ ActorRow actor_row(const MArgs& a, const RowIn<CB>& in, float alpha, float log_alpha) {
  const Layout& L = a.L;
  const float* rc = in.rc;
  const float mean = rc[HD_MEAN], ls_raw = rc[HD_LSRAW], std = rc[HD_STD];
  const float z = rc[HD_Z], act = rc[HD_A], logp = rc[HD_LOGP];
  const float eps_i = rc[R_EPS];
  const float* sn = a.s.snap;
  const float q1a = in.sum(0) + sn[SN_BQ1];
  const float q2a = in.sum(1) + sn[SN_BQ2];
  const float invB = 1.0f / (float)L.B;
  // d min(Q1, Q2): all to the smaller, split evenly on a tie (torch.min's backward)
  const float w1 = (q1a < q2a) ? 1.0f : ((q1a == q2a) ? 0.5f : 0.0f);
  float dA = (-w1 * invB) * in.sum(2) + (-(1.0f - w1) * invB) * in.sum(3);
  if (a.hp.areg != 0.0f) dA += (a.hp.areg * invB) * (2.0f * act);
  const float ainv = alpha * invB;
  const float d = z - mean, var = std * std;
  const float sig = 1.0f / (1.0f + expf(2.0f * z));  // sigmoid(-2z)
  const float gz = dA * (1.0f - act * act) + ainv * (-(d / var) + (2.0f - 4.0f * sig));
  ActorRow o;
  o.dmean = gz + ainv * (d / var);
  const float dstd = gz * eps_i + ainv * ((d * d) / (var * std) - 1.0f / std);
  o.dls = (ls_raw >= -20.0f && ls_raw <= 2.0f) ? dstd * std : 0.0f;
  o.pl = alpha * logp - fminf(q1a, q2a) + (a.hp.areg != 0.0f ? a.hp.areg * (act * act) : 0.0f);
  o.la = -(log_alpha * (logp + a.hp.tent));
  o.ga = -(logp + a.hp.tent);
  o.logp = logp;
  o.mean = mean;
  o.std = std;
  return o;
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
  float* T;
  const float* stats;
  Layout L;
  Hyper hp;
  int n_tile_blocks;  // blocks [0, n_tile_blocks) take 32x32 tiles of the three H x H W2 matrices
  int wt;             // write-through mask (WT_*)
};

// one element: loads (ld) and update/stores (st) split so several elements' loads are in flight first. q: the
// element is a critic's (lr_q, and a soft-updated target) — the caller knows it (a block's elements share it)
struct AdamElem {
  float g, m, v, p, t;
};
__device__ __forceinline__ AdamElem adam_ld(const ApplyArgs& a, int64_t e, bool q, bool with_g = true) {
  AdamElem x;
  x.g = with_g ? a.grads[e] : 0.0f;
  x.m = a.m[e];
  x.v = a.v[e];
  x.p = a.params[e];
  x.t = q ? a.targets[e - a.L.q_base[0]] : 0.0f;
  return x;
}
__device__ __forceinline__ void adam_st(const ApplyArgs& a, const AdamStep& st, int64_t e, AdamElem& x, bool q, int wt) {
  const float g = x.g * a.hp.inv_world;
  const float m = x.m + (1.0f - a.hp.beta1) * (g - x.m);              // exp_avg.lerp_(grad, 1 - beta1)
  const float v = x.v * a.hp.beta2 + (1.0f - a.hp.beta2) * (g * g);   // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / st.bc2_sqrt + a.hp.eps;
  const float p = x.p + (-(q ? st.step_q : st.step_pi)) * (m / denom);
  pub<WT_OPT>(wt, a.m + e, m);
  pub<WT_OPT>(wt, a.v + e, v);
  pub<WT_OPT>(wt, a.params + e, p);
  x.p = p;
  if (q) {
    x.t = x.t * (1.0f - a.hp.tau) + p * a.hp.tau;
    pub<WT_OPT>(wt, a.targets + (e - a.L.q_base[0]), x.t);
  }
}

// ---------------------------------------------------------------------------------------------
// P3 (sac_wgrad_kernel): [3·CB² MFMA tiles of the H x H gradients | VALU blocks (3 nets x H/16 units) | scalars]
// ---------------------------------------------------------------------------------------------
struct WArgs {
  MArgs m;
  float* grads;
  int fuse;   // single process: each block also applies Adam / soft update / W2ᵀ to the elements it finished
  int pub_grads;  // write the flat gradient (always without fuse; chain SACF_CHAIN_NO_GRADS clears it): the host's
                  // choice of kernel (WT_NOG)
  int n_mfma, n_valu;
  int n_stage;  // chain STAGE_NEXT: blocks staging the next step's batch (after the scalar block), else 0
  ApplyArgs ap;
  // per H x H matrix (0 actor, 1 / 2 Q1 / Q2): the MFMA tiles' operands and output offset, indexed (one scalar
  // load) rather than selected between fields (a live mask and both candidates across the GEMM loop)
  const uint32_t* dy_mask[3];  // [h2 > 0] | [g2 > 0] Q1 | Q2 (Scr::h2m / g2m)
  const float* x_src[3];   // h1 | g1 Q1 | g1 Q2
  int64_t w2_off[3];       // the W2 block in params (and grads, Adam state)
  int hw_off[3];           // the first head-weight row in snap's SN_HEAD block: wm | w3 Q1 | w3 Q2
};

constexpr int kRowChunk = 256;  // rows whose scalars a block holds at once (one per thread)
constexpr int kValuAcc = kXLd + 4;

struct WLds {
  union {
    struct {
      float split[4 * 16 * 64];
      float tt[2][kTile2][kTile2 + 1];
    } mm;
    float vred[kThreads / 16][kValuAcc][16];  // VALU blocks: [row stream][accumulator][unit]
  } u;
  alignas(16) float s0[kRowChunk];
  alignas(16) float s1[kRowChunk];
  float xs[kRowChunk][kXLd + 1];
  float red[4][32];
  float sum[32];
};

// this step's Adam bias corrections (the mid kernel wrote them): read by every block at its start, into registers,
// for its epilogue (no block barrier on the load)
__device__ __forceinline__ AdamStep adam_step_of(const MArgs& m) {
  return AdamStep{m.stats[5], m.stats[6], m.stats[7]};
}

__device__ __forceinline__ float alpha_of(const MArgs& a) {
  return a.hp.auto_ent ? expf(a.s.snap[SN_LOGA]) : 1.0f;
}

// MFMA tile of dW2 for matrix mat (0 actor, 1 / 2 Q1 / Q2): out[j][k] = Σ_r dY[r][j] X[r][k] with
//   actor  dY = [h2 > 0] ⊙ (wm dmean + ws dls), X = h1;   critic  dY = [g2 > 0] ⊙ w3 dq, X = g1
template <int H>
__device__ __forceinline__ void mfma_tile_of(int bx, int& mat, int& j0, int& k0) {
  constexpr int CB = H / kTile2, tiles = CB * CB;
  mat = bx / tiles;
  int t = bx % tiles;
  if constexpr (CB == 8) {
    // XCD-aware (64 tiles per matrix, 24 per XCD): XCD x = bx mod 8 takes, of each matrix, the 2 x 4 tiles of row
    // blocks 2(x / 2) + {0, 1} and column blocks 4(x mod 2) + {0..3}, so its L2 fetches a quarter of dYᵀ's
    // columns and half of X's
    const int x = bx & 7, sl = bx >> 3, tt = sl & 7;
    mat = sl >> 3;
    t = ((x >> 1) * 2 + (tt >> 2)) * 8 + (x & 1) * 4 + (tt & 3);
  }
  j0 = (t / CB) * kTile2;
  k0 = (t % CB) * kTile2;
}

template <int H, int WT>
__device__ __forceinline__ void p3_mfma_tile_wt(const WArgs& a, int bx, WLds& S) {
  constexpr int CB = H / kTile2;
  const MArgs& m = a.m;
  const AdamStep sst = adam_step_of(m);
  const Layout& L = m.L;
  const int B = L.B, Bp = L.Bp;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane >> 5, rl = lane & 31;
  int mat, j0, k0;
  mfma_tile_of<H>(bx, mat, j0, k0);
  const bool actor = mat == 0;
  const int net = actor ? 0 : mat - 1;
  const float* hw = m.s.snap + SN_HEAD;  // pre-update head weights: wm | ws | w3 Q1 | w3 Q2
  const uint32_t __attribute__((address_space(1)))* Y = (const uint32_t __attribute__((address_space(1)))*)a.dy_mask[mat];
  const gptr X = as_global(a.x_src[mat]);
  const int jc = j0 + rl;
  const float c1 = hw[a.hw_off[mat] + jc];
  const float c2 = actor ? hw[H + jc] : 0.0f;
  const float alpha = alpha_of(m), log_alpha = m.s.snap[SN_LOGA];
  const int64_t out_off = a.w2_off[mat];
  AdamElem xe[4];  // the optimizer state of the four outputs this lane finishes, in flight during the GEMM
  f32x16 acc = zero16();
  for (int rc = 0; rc < Bp; rc += kRowChunk) {
    const int nrow = min(kRowChunk, Bp - rc);
    const int rows_w = nrow / 4, n2 = rows_w / 2, rl0 = w * rows_w + h * n2;
    // loads in the order they are consumed (vmcnt counts in issue order): the inputs of row rc + tid's scalars
    // (every thread computes one), the chunk's operands, then (first chunk) the Adam state
    const int r = min(rc + tid, Bp - 1);
    RowIn<CB> rin;
    rin.load(m, r, actor);
    // the chunk's operands as one straight-line batch of loads (a run-time guard per load would make a chain of
    // branches with a wait after every load): n2 = 32 for full chunks, 16 / 8 / 4 for Bp = 128 / 64 / 32
    // (Y: the [dY-side activation > 0] mask word of column block j0 / 32 per row; this lane's column is bit rl)
    uint32_t yv[kMaxN2];
    float xv[kMaxN2];
    const int rb = rc + rl0, jw = j0 >> 5;
    auto load_chunk = [&](auto n_tag) __attribute__((always_inline)) {
      constexpr int N = decltype(n_tag)::value;
      // (N rows from rb, a multiple of N: inside one 32-row tile, so their mask words are one 16-byte aligned run)
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      typedef const u32x4 __attribute__((address_space(1))) * gu4;
      const gu4 yq = reinterpret_cast<gu4>(Y + ((((int64_t)(rb >> 5) * CB + jw) << 5) + (rb & 31)));
#pragma unroll
      for (int i4 = 0; i4 < N / 4; ++i4) {
        const u32x4 u = yq[i4];
        yv[4 * i4] = u[0]; yv[4 * i4 + 1] = u[1]; yv[4 * i4 + 2] = u[2]; yv[4 * i4 + 3] = u[3];
      }
#pragma unroll
      for (int i = 0; i < N; ++i) xv[i] = X[(int64_t)(rb + i) * H + k0 + rl];
    };
    if (n2 == 32) load_chunk(std::integral_constant<int, 32>{});
    else if (n2 == 16) load_chunk(std::integral_constant<int, 16>{});
    else if (n2 == 8) load_chunk(std::integral_constant<int, 8>{});
    else if (n2 == 4) load_chunk(std::integral_constant<int, 4>{});
    else {
#pragma unroll
      for (int i = 0; i < kMaxN2; ++i) {
        yv[i] = 0u;
        xv[i] = 0.0f;
        if (i >= n2) continue;  // (continue, not break: the constant trip count keeps the loop unrolled)
        yv[i] = Y[rw_at(rb + i, 0, 1, CB, jw)];
        xv[i] = X[(int64_t)(rb + i) * H + k0 + rl];
      }
    }
    if (rc == 0 && a.fuse)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        xe[q] = adam_ld(a.ap, out_off + (int64_t)(j0 + finish_row(q)) * H + k0 + rl, !actor, false);
    float s0, s1 = 0.0f;
    if (actor) {
      const ActorRow ar = actor_row<CB>(m, rin, alpha, log_alpha);
      s0 = ar.dmean;
      s1 = ar.dls;
    } else {
      const CriticRow cr = critic_row<CB>(m, rin, alpha);
      s0 = (2.0f / (float)B) * ((net == 0 ? cr.q1 : cr.q2) - cr.y);
    }
    if (rc + tid >= B) s0 = s1 = 0.0f;
    SAC_STAMP_ON(2, 4, s0);
    SAC_STAMP_ON(2, 5, (float)yv[kMaxN2 - 1] + xv[kMaxN2 - 1]);
    S.s0[tid] = s0;
    S.s1[tid] = s1;
    __syncthreads();
    SAC_STAMP(2, 1);
    // (every LDS read unconditional — rl0 + i < 256 for every chunk shape — and the actor / critic choice a select
    // of values: a guard or branch per read compiles into a wait per read)
    // (rl0 is a multiple of 4 for every chunk shape — rows per wave a multiple of 8 — so the row scalars are read four at
    // a time: 16 LDS reads per array instead of 32)
    float av[kMaxN2];
#pragma unroll
    for (int i4 = 0; i4 < kMaxN2; i4 += 4) {
      const float4 s0q = *reinterpret_cast<const float4*>(&S.s0[rl0 + i4]);
      const float4 s1q = *reinterpret_cast<const float4*>(&S.s1[rl0 + i4]);
      const float s0a[4] = {s0q.x, s0q.y, s0q.z, s0q.w}, s1a[4] = {s1q.x, s1q.y, s1q.z, s1q.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float d = actor ? c1 * s0a[u] + c2 * s1a[u] : c1 * s0a[u];
        av[i4 + u] = ((yv[i4 + u] >> rl) & 1u) ? d : 0.0f;
      }
    }
    if (n2 == kMaxN2) mfma_n<kMaxN2>(acc, av, xv);  // (full chunks: one straight chain)
    else mfma_chain(acc, av, xv, n2);
    if (rc + kRowChunk < Bp) __syncthreads();  // S.s0 / s1 reused
  }
  SAC_STAMP(2, 2);
  auto& tt = S.u.mm.tt;
  {
  // the tile's coordinates again, from an opaque block id: recomputed here rather than held across the loop
  int bxe = (int)blockIdx.x;
  asm volatile("" : "+s"(bxe));
  mfma_tile_of<H>(bxe, mat, j0, k0);
  const int64_t out_off = a.w2_off[mat];
  splitk_finish(acc, S.u.mm.split, [&](int q, int rr, int cc, float v) {
    const int64_t e = out_off + (int64_t)(j0 + rr) * H + k0 + cc;
    if constexpr ((WT & WT_NOG) == 0) pub<WT_OPT>(WT, a.grads + e, v);
    if (a.fuse) {
      xe[q].g = v;
      adam_st(a.ap, sst, e, xe[q], mat > 0, WT);
      tt[0][cc][rr] = xe[q].p;
      tt[1][cc][rr] = xe[q].t;
    }
  });
  SAC_STAMP_ON(2, 6, xe[3].p);
  if (a.fuse) {  // W2ᵀ (and the target's) for the next step's forward passes: T[col][row]
    __syncthreads();
    SAC_STAMP(2, 7);
    // (thread t: T row k0 + t / 8, the four columns j0 + 4 (t mod 8) ..: one 16-byte store per copy)
    const int64_t HH = (int64_t)H * H;
    const int cc = tid >> 3, j4 = (tid & 7) * 4;
    const int64_t o = (int64_t)(k0 + cc) * H + j0 + j4;
    pub4<WT_OPT>(WT, a.ap.T + (size_t)mat * HH + o, tt[0][cc][j4], tt[0][cc][j4 + 1], tt[0][cc][j4 + 2], tt[0][cc][j4 + 3]);
    if (mat > 0)
      pub4<WT_OPT>(WT, a.ap.T + (size_t)(2 + mat) * HH + o, tt[1][cc][j4], tt[1][cc][j4 + 1], tt[1][cc][j4 + 2],
                   tt[1][cc][j4 + 3]);
  }
  }
}

// VALU block: hidden units j = jb .. jb + 15 of net (0 actor, 1 / 2 Q1 / Q2). Lane l of wave w serves unit l % 16
// on row stream 4w + l / 16: the 16 streams split the rows (16 per stream at B = 256, two batches of 8 in flight),
// and their partials are added in stream order. Per j: fc0 row (Σ dh1·x), fc0 bias (Σ dh1), fc1 bias (Σ dh2), head
// weight(s) (Σ dmean·h2, Σ dls·h2 / Σ dq·g2), with
//   actor  dh1 = dmean U_m + dls U_s, dh2 = [h2 > 0] (wm dmean + ws dls);  critic  dg1 = dq U_q, dg2 = [g2 > 0] w3 dq
constexpr int kValuUnits = 16, kValuStreams = kThreads / kValuUnits;
template <int H, int WT>
__device__ __forceinline__ void p3_valu_block_wt(const WArgs& a, int vb, WLds& S) {
  constexpr int CB = H / kTile2, NB = H / kValuUnits;
  static_assert(H % kValuUnits == 0, "units per VALU block");
  const MArgs& m = a.m;
  const AdamStep sst = adam_step_of(m);
  const Layout& L = m.L;
  const int B = L.B, Bp = L.Bp;
  const int tid = threadIdx.x;
  const int net = vb / NB, j0 = (vb % NB) * kValuUnits;
  const int u = tid % kValuUnits, strm = tid / kValuUnits, j = j0 + u;
  const bool actor = net == 0;
  const int cn = actor ? 0 : net - 1;
  const float* hw = m.s.snap + SN_HEAD;  // pre-update head weights: wm | ws | w3 Q1 | w3 Q2
  const int nin = actor ? L.O : L.O + 1;
  const float* U1 = actor ? m.s.um : m.s.uq[cn];
  const float* U2 = m.s.us;
  const float* A2 = actor ? m.s.h2 : m.s.g2[cn];
  const float* XR = actor ? m.s.x : m.s.qx;
  const float c1 = actor ? hw[j] : hw[(2 + cn) * H + j];
  const float c2 = actor ? hw[H + j] : 0.0f;
  const float alpha = alpha_of(m), log_alpha = m.s.snap[SN_LOGA];
  // the block's outputs: per unit its fc0 row (nin), fc0 bias, fc1 bias, head weight(s); thread t finishes output
  // t / 16 (and t / 16 + 16) of unit t % 16, their optimizer state in flight during the row pass
  const int n_el = nin + (actor ? 4 : 3);
  const int64_t base = actor ? 0 : L.q_base[cn];
  auto el_off = [&](int k) -> int64_t {
    if (k < nin) return base + (actor ? L.p_w1 : L.c_w1) + (int64_t)j * nin + k;
    if (k == nin) return base + (actor ? L.p_b1 : L.c_b1) + j;
    if (k == nin + 1) return base + (actor ? L.p_b2 : L.c_b2) + j;
    if (k == nin + 2) return base + (actor ? L.p_wm : L.c_w3) + j;
    return L.p_ws + j;
  };
  AdamElem xe[2];
  if (a.fuse)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (strm + kValuStreams * q < n_el) xe[q] = adam_ld(a.ap, el_off(strm + kValuStreams * q), !actor, false);
  float w1a[kXLd], b1a = 0.0f, b2a = 0.0f, ha1 = 0.0f, ha2 = 0.0f;
#pragma unroll
  for (int i = 0; i < kXLd; ++i) w1a[i] = 0.0f;
  for (int rc = 0; rc < Bp; rc += kRowChunk) {
    const int nrow = min(kRowChunk, Bp - rc);
    const int r = min(rc + tid, Bp - 1);
    RowIn<CB> rin;
    rin.load(m, r, actor);
    float xr[kXLd];
    load_run<kXLd>(XR + (int64_t)r * kXLd, xr);
    float s0, s1 = 0.0f;
    if (actor) {
      const ActorRow ar = actor_row<CB>(m, rin, alpha, log_alpha);
      s0 = ar.dmean;
      s1 = ar.dls;
    } else {
      const CriticRow cr = critic_row<CB>(m, rin, alpha);
      s0 = (2.0f / (float)B) * ((cn == 0 ? cr.q1 : cr.q2) - cr.y);
    }
    if (rc + tid >= B) s0 = s1 = 0.0f;
    S.s0[tid] = s0;
    S.s1[tid] = s1;
#pragma unroll
    for (int i = 0; i < kXLd; ++i) S.xs[tid][i] = xr[i];
    __syncthreads();
    SAC_STAMP(2, 1);
    // this stream's rows (nrow / 16: even, a multiple of 8 from 128 rows up) in batches of R with every load of a
    // batch in flight together; every load and LDS read unconditional (U2 is a valid buffer for a critic too, the
    // input rows are zero past nin) and the actor / critic choice a select of values — a guard per read compiles
    // into a wait per read
    const int rows_s = nrow / kValuStreams;
    auto run = [&](auto r_tag) __attribute__((always_inline)) {
      constexpr int R = decltype(r_tag)::value;
      for (int q0 = strm * rows_s; q0 < (strm + 1) * rows_s; q0 += R) {
        float u1[R], u2[R], x2[R];
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const int64_t o = (int64_t)(rc + q0 + t) * H + j;
          u1[t] = U1[o];
          u2[t] = U2[o];
          x2[t] = A2[o];
        }
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const float a0 = S.s0[q0 + t], a1 = S.s1[q0 + t];
          const float d1 = actor ? a0 * u1[t] + a1 * u2[t] : a0 * u1[t];
          const float d2 = x2[t] > 0.0f ? (actor ? c1 * a0 + c2 * a1 : c1 * a0) : 0.0f;
#pragma unroll
          for (int i = 0; i < kXLd; ++i) w1a[i] = fmaf(d1, S.xs[q0 + t][i], w1a[i]);
          b1a += d1;
          b2a += d2;
          ha1 = fmaf(a0, x2[t], ha1);
          ha2 = fmaf(a1, x2[t], ha2);
        }
      }
    };
    if (rows_s % 8 == 0) run(std::integral_constant<int, 8>{});
    else run(std::integral_constant<int, 2>{});
    __syncthreads();
  }
  SAC_STAMP(2, 2);
  auto& vr = S.u.vred;  // [stream][accumulator][unit]
#pragma unroll
  for (int i = 0; i < kXLd; ++i) vr[strm][i][u] = w1a[i];
  vr[strm][kXLd][u] = b1a;
  vr[strm][kXLd + 1][u] = b2a;
  vr[strm][kXLd + 2][u] = ha1;
  vr[strm][kXLd + 3][u] = ha2;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = strm + kValuStreams * q;
    if (k >= n_el) break;
    const int i = k < nin ? k : kXLd + (k - nin);
    float g = vr[0][i][u];
#pragma unroll
    for (int st = 1; st < kValuStreams; ++st) g += vr[st][i][u];
    const int64_t e = el_off(k);
    if constexpr ((WT & WT_NOG) == 0) pub<WT_OPT>(WT, a.grads + e, g);
    if (a.fuse) {
      xe[q].g = g;
      adam_st(a.ap, sst, e, xe[q], !actor, WT);
    }
  }
}

// scalar block: per-row losses and diagnostics, the loss means, the bias gradients of the scalar heads
// (Σ dmean, Σ dls, Σ dq1, Σ dq2), d(log α) (sac.py:174-180) and α
template <int H, int WT>
__device__ __forceinline__ void p3_scalar_block_wt(const WArgs& a, WLds& S) {
  constexpr int CB = H / kTile2;
  const MArgs& m = a.m;
  const AdamStep sst = adam_step_of(m);
  const Layout& L = m.L;
  const int B = L.B, Bp = L.Bp, tid = threadIdx.x;
  const float alpha = alpha_of(m), log_alpha = m.s.snap[SN_LOGA];
  const float invB = 1.0f / (float)B;
  // the five scalar parameters (log α, b_mean, b_log_std, b3 Q1, b3 Q2): thread i < 5 finishes parameter i, its
  // optimizer state in flight during the row pass
  const int64_t off = tid == 0 ? 0 : tid == 1 ? L.p_bm : tid == 2 ? L.p_bs : L.q_base[tid >= 4 ? 1 : 0] + L.c_b3;
  AdamElem xs;
  if (a.fuse && tid < 5) xs = adam_ld(a.ap, off, tid >= 3, false);
  float v[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) v[i] = 0.0f;
  float* st = m.stats + 8;
  for (int rc = 0; rc < Bp; rc += kRowChunk) {
    const int r = rc + tid;
    if (r >= B) continue;
    RowIn<CB> rq, ra;
    rq.load(m, r, false);
    ra.load(m, r, true);
    const CriticRow cr = critic_row<CB>(m, rq, alpha);
    const ActorRow ar = actor_row<CB>(m, ra, alpha, log_alpha);
    const float d1 = cr.q1 - cr.y, d2 = cr.q2 - cr.y;
    v[0] += ar.pl;
    v[1] += d1 * d1;
    v[2] += d2 * d2;
    v[3] += ar.la;
    v[4] += ar.ga;
    v[5] += ar.dmean;
    v[6] += ar.dls;
    v[7] += (2.0f * invB) * d1;
    v[8] += (2.0f * invB) * d2;
    st[r] = cr.q1;
    st[B + r] = cr.q2;
    st[2 * B + r] = cr.y;
    st[3 * B + r] = ar.logp;
    st[4 * B + r] = tanhf(ar.mean);
    st[5 * B + r] = ar.std;
  }
  SAC_STAMP(2, 1);
  block_sum<9>(v, S.red, S.sum);
  SAC_STAMP(2, 2);
  const float* sum = S.sum;
  if (tid == 0) {
    m.stats[0] = sum[0] * invB;
    m.stats[1] = sum[1] * invB;
    m.stats[2] = sum[2] * invB;
    m.stats[3] = m.hp.auto_ent ? sum[3] * invB : 0.0f;
    m.stats[4] = alpha;
  }
  if (tid >= 5) return;
  const float g = tid == 0 ? (m.hp.auto_ent ? sum[4] * invB : 0.0f) : sum[4 + tid];
  if constexpr ((WT & WT_NOG) == 0) pub<WT_OPT>(WT, a.grads + off, g);
  if (a.fuse && (tid > 0 || m.hp.auto_ent)) {
    xs.g = g;
    adam_st(a.ap, sst, off, xs, tid >= 3, WT);
  }
}

// chain STAGE_NEXT: the next step's batch (P2 has advanced the step counter, so batch_item draws what the next
// P1 would): item sb·256 + thread — its replay row, both observation rows, act / rew / term and its two normals
template <int WT>
__device__ __forceinline__ void p3_stage_block(const WArgs& a, int sb) {
  const MArgs& m = a.m;
  const int item = sb * kThreads + (int)threadIdx.x;
  if (item >= m.L.Bp) return;
  float e0, e1;
  const int64_t idx = batch_item(m, item, e0, e1);
  float x[kXLd], xn[kXLd];
  load_obs_row(m.obs, idx, m.L.O, x);
  load_obs_row(m.nobs, idx, m.L.O, xn);
  const float act = m.act[idx], rew = m.rew[idx], term = m.term[idx];
  float* dx = m.s.sx + (int64_t)item * kXLd;
  float* dn = m.s.sxn + (int64_t)item * kXLd;
#pragma unroll
  for (int q = 0; q < kXLd / 4; ++q) {
    pub4<WT_ACT>(WT, dx + 4 * q, x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
    pub4<WT_ACT>(WT, dn + 4 * q, xn[4 * q], xn[4 * q + 1], xn[4 * q + 2], xn[4 * q + 3]);
  }
  float* q = m.s.saux + (int64_t)item * kAux;
  pub4<WT_ACT>(WT, q, act, rew, term, e0);
  pub<WT_ACT>(WT, q + AUX_E1, e1);
}

// the kernel's WArgs read through the kernarg segment pointer, laundered: a field is a scalar load where a block
// uses it instead of ~150 argument dwords held in SGPRs (which spilled) across the whole kernel
typedef const __attribute__((address_space(4))) WArgs* WArgsPtr;
__device__ __forceinline__ const WArgs& wargs() {
  WArgsPtr q = (WArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return *(const WArgs*)q;
}

template <int H, int WT>
__global__ __launch_bounds__(256) void sac_wgrad_kernel(WArgs a_arg) {
  (void)a_arg;  // read through wargs()
  __shared__ WLds S;
  const WArgs& a = wargs();
  SAC_STAMP(2, 0);
  const int bx = (int)blockIdx.x;
  if (bx < a.n_mfma) p3_mfma_tile_wt<H, WT>(a, bx, S);
  else if (bx < a.n_mfma + a.n_valu) p3_valu_block_wt<H, WT>(a, bx - a.n_mfma, S);
  else if (bx == a.n_mfma + a.n_valu) p3_scalar_block_wt<H, WT>(a, S);
  else p3_stage_block<WT>(a, bx - a.n_mfma - a.n_valu - 1);
  SAC_STAMP(2, 3);
}

// world_size > 1 / split_update: the update from the (all-reduced) flat gradient
template <int WT>
__global__ __launch_bounds__(kThreads) void sac_apply_kernel(ApplyArgs a) {
  __shared__ float tile[2][kTile2][kTile2 + 1];
  const AdamStep st{a.stats[5], a.stats[6], a.stats[7]};
  const Layout& L = a.L;
  const int H = L.H;
  const int64_t HH = (int64_t)H * H;
  const int64_t w2[3] = {L.p_w2, L.q_base[0] + L.c_w2, L.q_base[1] + L.c_w2};
  if ((int)blockIdx.x < a.n_tile_blocks) {
    // 32 x 32 tile of one W2: Adam on row-major elements, transposed copies written through LDS
    constexpr int kPer = kTile2 / (kThreads / kTile2);  // 4 rows per thread
    const int tpm = (H / kTile2) * (H / kTile2);
    const int mat = blockIdx.x / tpm, t = blockIdx.x % tpm;
    const int r0 = (t / (H / kTile2)) * kTile2, c0 = (t % (H / kTile2)) * kTile2;
    const int tc = threadIdx.x % kTile2, tr = threadIdx.x / kTile2;  // 8 rows per pass
    AdamElem x[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) x[u] = adam_ld(a, w2[mat] + (int64_t)(r0 + tr + u * 8) * H + c0 + tc, mat > 0);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int rr = tr + u * 8;
      adam_st(a, st, w2[mat] + (int64_t)(r0 + rr) * H + c0 + tc, x[u], mat > 0, WT);
      tile[0][tc][rr] = x[u].p;
      tile[1][tc][rr] = x[u].t;
    }
    __syncthreads();
    for (int cc = tr; cc < kTile2; cc += kThreads / kTile2) {
      const int64_t o = (int64_t)(c0 + cc) * H + r0 + tc;  // T[col][row]
      if (mat == 0) {
        pub<WT_OPT>(WT, a.T + o, tile[0][cc][tc]);
      } else {
        pub<WT_OPT>(WT, a.T + (size_t)mat * HH + o, tile[0][cc][tc]);
        pub<WT_OPT>(WT, a.T + (size_t)(2 + mat) * HH + o, tile[1][cc][tc]);
      }
    }
    return;
  }
  // every other element: flat index over the parameters outside the three W2 blocks
  const int64_t f = (int64_t)(blockIdx.x - a.n_tile_blocks) * kThreads + threadIdx.x;
  int64_t e = f;
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (e >= w2[k]) e += HH;
  if (e >= L.n_params) return;
  if (e == 0 && !a.hp.auto_ent) return;
  const bool q = e >= L.q_base[0];
  AdamElem x = adam_ld(a, e, q);
  adam_st(a, st, e, x, q, WT);
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
//   sac_act_fwd_kernel  : grid (n / 32) x (H / 32): h1 (VALU), h2 = relu(h1 W2ᵀ + b2) on MFMA, this column
//                         block's part of the mean / log_std heads of each row
//   sac_act_head_kernel : per row: the parts summed in block order + biases, log_std clamped, std = exp,
//                         a = tanh(mean + std·ε) (ε from Philox(seed, counter, row)) or tanh(mean); rows whose
//                         mask byte is 0 keep their previous action
// ---------------------------------------------------------------------------------------------
struct ActArgs {
  const float* params;
  const float* T;
  const float* obs;  // [n][obs_stride]
  int64_t n;
  int obs_stride;
  Layout L;
  float* hpart;      // [2][H/32][n_pad]
  int64_t n_pad;
  const uint8_t* mask;
  int deterministic;
  uint64_t seed;
  const int64_t* counter;
  float* act;        // [n]
  float* eps_out;    // [n] or null
};

template <int H>
__global__ __launch_bounds__(256) void sac_act_fwd_kernel(ActArgs a) {
  using KS = KSlice<H>;
  constexpr int CS = KS::CS;
  __shared__ float lds[FwdLds<H>::kFloats];
  const Layout& L = a.L;
  const int O = L.O;
  const float* P = a.params;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
  const int r0 = blockIdx.x * kTile2, c0 = blockIdx.y * kTile2;
  const int kb = w * (H / 4) + h * KS::N2;
  const int64_t row = r0 + rl;
  const int64_t rowc = row < a.n ? row : a.n - 1;  // rows past n (last tile) repeat the last row
  float x[kXLd];
#pragma unroll
  for (int m = 0; m < kXLd; ++m) x[m] = m < O ? a.obs[rowc * a.obs_stride + m] : 0.0f;
  W1Stage<H> w1s;
  w1s.load(P + L.p_w1, P + L.p_b1, O);
  float bv[CS];
  load_b<CS>(bv, a.T, H, kb, c0 + rl);
  const float b2c = P[L.p_b2 + c0 + rl];
  const float wm = P[L.p_wm + c0 + rl], ws = P[L.p_ws + c0 + rl];
  float* lw1 = lds + FwdLds<H>::kW1Off;
  float* lx = lds + FwdLds<H>::kXOff;
  w1s.store(lw1, O);
  if (w == 0 && h == 0)
    for (int m = 0; m < O; ++m) lx[rl * (kXLd + 1) + m] = x[m];
  __syncthreads();
  f32x16 acc = zero16();
#pragma unroll
  for (int c = 0; c < KS::NCH; ++c) {
    const int k0 = kb + c * CS;
    if (c) load_b<CS>(bv, a.T, H, k0, c0 + rl);
    float av[CS];
    first_layer<H, CS>(lw1, lx + rl * (kXLd + 1), O, k0, av);
    mfma_n<CS>(acc, av, bv);
  }
  constexpr int CB = KS::CB;
  splitk_finish(acc, lds, [&](int, int rr, int cc, float v) {
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
  float pm[CB], pl[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    pm[cb] = a.hpart[(int64_t)cb * a.n_pad + r];
    pl[cb] = a.hpart[(int64_t)(CB + cb) * a.n_pad + r];
  }
  const float mean = fold(pm) + P[a.L.p_bm];
  const float ls = fold(pl) + P[a.L.p_bs];
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

// ---------------------------------------------------------------------------------------------
// launches per hidden width (a compile-time tile count)
// ---------------------------------------------------------------------------------------------
template <int H>
void launch_step(const MArgs& m, const WArgs& w, hipStream_t st) {
  const unsigned bt = (unsigned)(m.L.Bp / kTile2), cb = H / kTile2;
  const dim3 g1(6 * bt * cb), g2p(8 * bt * cb), g3((unsigned)(w.n_mfma + w.n_valu + 1 + w.n_stage));
  if (m.wt == kWtLarge) {
    hipLaunchKernelGGL((sac_fwd_kernel<H, kWtLarge>), g1, dim3(256), 0, st, m);
    hipLaunchKernelGGL((sac_mid_kernel<H, kWtLarge>), g2p, dim3(256), 0, st, m);
    if (w.pub_grads) hipLaunchKernelGGL((sac_wgrad_kernel<H, kWtLarge>), g3, dim3(256), 0, st, w);
    else hipLaunchKernelGGL((sac_wgrad_kernel<H, kWtLarge | WT_NOG>), g3, dim3(256), 0, st, w);
  } else {
    hipLaunchKernelGGL((sac_fwd_kernel<H, kWtSmall>), g1, dim3(256), 0, st, m);
    hipLaunchKernelGGL((sac_mid_kernel<H, kWtSmall>), g2p, dim3(256), 0, st, m);
    if (w.pub_grads) hipLaunchKernelGGL((sac_wgrad_kernel<H, kWtSmall>), g3, dim3(256), 0, st, w);
    else hipLaunchKernelGGL((sac_wgrad_kernel<H, kWtSmall | WT_NOG>), g3, dim3(256), 0, st, w);
  }
}

template <int H>
void launch_act(const ActArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sac_act_fwd_kernel<H>, dim3((unsigned)(a.n_pad / kTile2), H / kTile2), dim3(256), 0, st, a);
  hipLaunchKernelGGL(sac_act_head_kernel<H>, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
}

// F(std::integral_constant<int, H>) for the handle's hidden width; false if none is compiled
template <class F>
bool with_hidden(int H, F&& f) {
#ifdef SACF_REGCHECK_H  // register-report builds of one width (scripts/regcheck.sh sac H)
  if (H != SACF_REGCHECK_H) return false;
  f(std::integral_constant<int, SACF_REGCHECK_H>{});
  return true;
#else
  switch (H) {
#define SACF_H(h) \
  case h: f(std::integral_constant<int, h>{}); return true;
#if SACF_TU != 2
    SACF_H(32) SACF_H(64) SACF_H(96) SACF_H(128) SACF_H(160) SACF_H(192) SACF_H(224) SACF_H(256)
    SACF_H(320) SACF_H(384)
#endif
#if SACF_TU != 1
    SACF_H(448) SACF_H(512)
#endif
#undef SACF_H
    default: return false;
  }
#endif
}

}  // namespace

#if SACF_TU == 2
// the wide widths' launches, called by the SACF_TU 1 object (the argument structs are this file's, identical there)
bool sacf_wide_launch_step(int H, const void* m, const void* w, hipStream_t st) {
  return with_hidden(H, [&](auto hc) {
    launch_step<decltype(hc)::value>(*static_cast<const MArgs*>(m), *static_cast<const WArgs*>(w), st);
  });
}
bool sacf_wide_launch_act(int H, const void* a, hipStream_t st) {
  return with_hidden(H, [&](auto hc) { launch_act<decltype(hc)::value>(*static_cast<const ActArgs*>(a), st); });
}
#else
namespace {
// a width this object does not hold: the other object's launches (SACF_TU 1), or none (SACF_TU 0)
bool wide_step(int H, const MArgs& m, const WArgs& w, hipStream_t st) {
#if SACF_TU == 1
  return sacf_wide_launch_step(H, &m, &w, st);
#else
  (void)H; (void)m; (void)w; (void)st;
  return false;
#endif
}
bool wide_act(int H, const ActArgs& a, hipStream_t st) {
#if SACF_TU == 1
  return sacf_wide_launch_act(H, &a, st);
#else
  (void)H; (void)a; (void)st;
  return false;
#endif
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
  bool staged;  // the last sacf_grads* call staged the next batch (SACF_CHAIN_STAGE_NEXT)
  float* T;
  float* scratch;
  Scr s;
  float* act_part;  // sacf_policy_act head partials [2][H/32][act_cap]
  int64_t act_cap;
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

#ifdef SACF_PHASE_TIMING
// diagnostics build: the last step's stamps, [3 kernels][kStampBlocks][kStamps] (not in include/sac_fused.h)
int sacf_debug_stamps(unsigned long long* out, int n) {
  const size_t bytes = sizeof(unsigned long long) * 3 * kStampBlocks * kStamps;
  if (!out || (size_t)n * sizeof(unsigned long long) < bytes) return kStampBlocks;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sac_stamps), bytes) == hipSuccess ? 0 : -1;
}
#endif

int sacf_hidden_supported(int32_t hidden) { return hidden_ok(hidden) ? 1 : 0; }

int sacf_create(const sacf_config* cfg, int device, void* stream, sacf_handle** out) {
  if (!out) return SACF_EINVAL;
  *out = nullptr;
  if (!cfg || cfg->abi_version != SACF_ABI_VERSION) return SACF_EINVAL;
  const int O = cfg->obs_dim, H = cfg->hidden, B = cfg->batch;
  if (O < 1 || O + 1 > kXLd || !hidden_ok(H) || B < 1 || B > SACF_MAX_BATCH || cfg->world_size < 1)
    return SACF_EINVAL;
  for (int i = 0; i < 5; ++i)
    if (cfg->reserved[i]) return SACF_EINVAL;
  sacf_handle* h = new (std::nothrow) sacf_handle();
  if (!h) return SACF_EINVAL;
  h->cfg = *cfg;
  h->device = device;
  h->stream = (hipStream_t)stream;
  Layout& L = h->L;
  L.O = O;
  L.H = H;
  L.B = B;
  L.Bp = (B + kTile2 - 1) / kTile2 * kTile2;
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
  const int64_t Bp = L.Bp, BH = Bp * H, CB = H / kTile2;
  // rows 2·16, activations 10·H, the row record, parts (2 + 8)·CB, the snapshot
  const int64_t n_scr = Bp * 2 * kXLd + 14 * BH + Bp * kRec + 2 * Bp * 2 * CB + PS_N * Bp * CB + SN_HEAD + 4 * H + 4 * H +
                        Bp * (2 * kXLd + kAux) + 3 * Bp * CB;
  hipError_t e = hipMalloc(&h->scratch, sizeof(float) * n_scr);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "hipMalloc(scratch): %s", hipGetErrorString(e));
  }
  (void)hipMemset(h->scratch, 0, sizeof(float) * n_scr);
  float* s = h->scratch;
  Scr& sc = h->s;
  sc.x = s; s += Bp * kXLd;
  sc.qx = s; s += Bp * kXLd;
  sc.h1 = s; s += BH;
  sc.h2 = s; s += BH;
  sc.um = s; s += BH;
  sc.us = s; s += BH;
  for (int k = 0; k < 2; ++k) {
    sc.g1[k] = s; s += BH;
    sc.g2[k] = s; s += BH;
    sc.uq[k] = s; s += BH;
  }
  sc.rec = s; s += Bp * kRec;
  sc.hpart = s; s += 2 * Bp * 2 * CB;
  for (int k = 0; k < 4; ++k) {
    sc.pre[k] = s;
    s += BH;
  }
  sc.w1a = s; s += 4 * H;
  sc.part = s; s += PS_N * Bp * CB;
  sc.snap = s; s += SN_HEAD + 4 * H;
  sc.sx = s; s += Bp * kXLd;
  sc.sxn = s; s += Bp * kXLd;
  sc.saux = s; s += Bp * kAux;
  sc.h2m = reinterpret_cast<uint32_t*>(s); s += Bp * CB;
  for (int k = 0; k < 2; ++k) {
    sc.g2m[k] = reinterpret_cast<uint32_t*>(s);
    s += Bp * CB;
  }
  e = hipMalloc(&h->T, sizeof(float) * 5 * (size_t)H * H);
  if (e != hipSuccess) {
    *out = h;
    return sfail(h, SACF_EHIP, "hipMalloc(T): %s", hipGetErrorString(e));
  }
  *out = h;
  return SACF_OK;
}

int sacf_destroy(sacf_handle* h) {
  if (!h) return SACF_OK;
  SDev g(h->device);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->T) (void)hipFree(h->T);
  if (h->act_part) (void)hipFree(h->act_part);
  delete h;
  return SACF_OK;
}

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
  h->staged = false;
  return SACF_OK;
}

// the write-through mask of a step's launches (see pub): everything from SACF_WT_ROWS padded rows up, below that not
// the row inputs / parts / records (WT_ACT). The threshold was 128 while those were 4- and 16-byte pieces of many
// rows; written as whole runs their write-through pays at every batch (0.3 µs less at B = 64 than plain stores,
// profiles/round6/r6wt_sac_ab.txt), so it is 32 now: every batch (the knob stays for A/B builds)
#ifndef SACF_WT_ROWS
#define SACF_WT_ROWS 32
#endif
static int wt_mask_for(const Layout& L) { return L.Bp >= SACF_WT_ROWS ? kWtLarge : kWtSmall; }

static ApplyArgs apply_args(const sacf_handle* h) {
  ApplyArgs a;
  a.wt = wt_mask_for(h->L);
  a.params = h->params;
  a.targets = h->targets;
  a.grads = h->grads;
  a.m = h->adam_m;
  a.v = h->adam_v;
  a.T = h->T;
  a.L = h->L;
  a.hp = h->hp;
  a.stats = h->stats;
  a.n_tile_blocks = 3 * (h->L.H / kTile2) * (h->L.H / kTile2);
  return a;
}

static int grads_impl(sacf_handle* h, const float* obs, const float* act, const float* rew, const float* term,
                      const float* next_obs, const float* eps, int chain) {
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
  a.chain = chain;
  a.wt = wt_mask_for(h->L);
  a.step = h->step;
  a.stats = h->stats;
  a.s = h->s;
  a.L = h->L;
  a.hp = h->hp;
  WArgs w;
  memset(&w, 0, sizeof(w));
  w.m = a;
  w.grads = h->grads;
  w.fuse = h->cfg.world_size == 1 && !h->cfg.split_update;  // no all-reduce in between: apply in the same kernel
  w.pub_grads = !(w.fuse && (chain & SACF_CHAIN_NO_GRADS));
  w.ap = apply_args(h);
  const int CB = h->L.H / kTile2;
  w.n_mfma = 3 * CB * CB;
  w.n_valu = 3 * (h->L.H / kValuUnits);
  w.n_stage = (chain & SACF_CHAIN_STAGE_NEXT) ? (int)((h->L.Bp + kThreads - 1) / kThreads) : 0;
  const Layout& L = h->L;
  for (int mat = 0; mat < 3; ++mat) {
    w.dy_mask[mat] = mat == 0 ? h->s.h2m : h->s.g2m[mat - 1];
    w.x_src[mat] = mat == 0 ? h->s.h1 : h->s.g1[mat - 1];
    w.w2_off[mat] = mat == 0 ? L.p_w2 : L.q_base[mat - 1] + L.c_w2;
    w.hw_off[mat] = mat == 0 ? 0 : (mat + 1) * L.H;
  }
  SDev g(h->device);
  if (!with_hidden(h->L.H, [&](auto hc) { launch_step<decltype(hc)::value>(a, w, h->stream); }) &&
      !wide_step(h->L.H, a, w, h->stream))
    return sfail(h, SACF_EINVAL, "sacf_grads: hidden %d", h->L.H);
  h->staged = (chain & SACF_CHAIN_STAGE_NEXT) != 0;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SACF_OK : sfail(h, SACF_EHIP, "sacf_grads: %s", hipGetErrorString(e));
}

int sacf_grads(sacf_handle* h, const float* obs, const float* act, const float* rew, const float* term,
               const float* next_obs, const float* eps) {
  return grads_impl(h, obs, act, rew, term, next_obs, eps, 0);
}

int sacf_grads_chain(sacf_handle* h, const float* eps, int32_t flags) {
  if (!h) return SACF_EINVAL;
  if (flags & ~(SACF_CHAIN_STAGE_NEXT | SACF_CHAIN_FROM_STAGED | SACF_CHAIN_NO_GRADS))
    return sfail(h, SACF_EINVAL, "sacf_grads_chain: flags");
  // a staged batch carries the normals of the call that staged it, so a chained step cannot take the caller's eps
  if ((flags & (SACF_CHAIN_STAGE_NEXT | SACF_CHAIN_FROM_STAGED)) && eps)
    return sfail(h, SACF_EINVAL, "sacf_grads_chain: STAGE_NEXT / FROM_STAGED need eps == NULL (in-kernel normals)");
  if (!h->r_obs) return sfail(h, SACF_ESTATE, "sacf_grads_chain: no replay bound");
  if ((flags & SACF_CHAIN_FROM_STAGED) && !h->staged)
    return sfail(h, SACF_ESTATE, "sacf_grads_chain: FROM_STAGED without a staging step before it");
  return grads_impl(h, nullptr, nullptr, nullptr, nullptr, nullptr, eps, flags);
}

int sacf_apply(sacf_handle* h) {
  if (!h || !h->params) return sfail(h, SACF_ESTATE, "sacf_apply: buffers not bound");
  if (h->cfg.world_size == 1 && !h->cfg.split_update) return SACF_OK;  // sacf_grads already applied the update
  ApplyArgs a = apply_args(h);
  const int64_t HH = (int64_t)h->L.H * h->L.H;
  const int64_t rest = h->L.n_params - 3 * HH;
  SDev g(h->device);
  const dim3 grid((unsigned)(a.n_tile_blocks + (rest + kThreads - 1) / kThreads));
  if (a.wt == kWtLarge) hipLaunchKernelGGL(sac_apply_kernel<kWtLarge>, grid, dim3(kThreads), 0, h->stream, a);
  else hipLaunchKernelGGL(sac_apply_kernel<kWtSmall>, grid, dim3(kThreads), 0, h->stream, a);
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
  if (!with_hidden(h->L.H, [&](auto hc) { launch_act<decltype(hc)::value>(a, h->stream); }) &&
      !wide_act(h->L.H, a, h->stream))
    return sfail(h, SACF_EINVAL, "sacf_policy_act: hidden %d", h->L.H);
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
#endif  // SACF_TU != 2
