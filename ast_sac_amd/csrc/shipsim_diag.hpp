// shipsim_diag.hpp — the diagnostics and ablation hooks of the env kernels, in one place. The product build
// (ast_sac_amd/build_hash.py flags) defines none of the SHIPSIM_* macros below, and every hook then compiles to
// nothing. Builds that define them are test or timing tools, never shipped:
//   -DSHIPSIM_LANECHECK      lane / index checks at every cross-lane exchange (scripts/build_abl.sh)
//   -DSHIPSIM_PHASE_TIMING   per-phase wall-clock stamps (scripts/build_timing.sh, scripts/phase_timing.py)
//   -DSHIPSIM_POISON_LDS=x   every LDS word preset to x before staging (stale-LDS check)
//   -DSHIPSIM_DEBUG_ENV=e    printf of env e's entry / exit state
//   -DSHIPSIM_ABL_*          ablations (scripts/build_ablations.sh; timing only, results intentionally differ):
//                            NO_WIND, NO_MAPDIST, NO_GROUND, NO_SBLOOP, SB_NEVER, SB_NONE
//   -DSHIPSIM_C2_ONE_WAVE    C2 simplified ticks on the one-wave single_tick_kernel (same results; timing A/B)
//   -DSHIPSIM_SB_STATS       multi-obstacle SBMPC counters (requests, passes, lone passes, obstacle evaluations),
//                            read back through shipsim_diag_lane_faults (words 16..31: eight u64)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shipsim {
namespace diag {

// ---- ablations -----------------------------------------------------------------------------------------------
#ifdef SHIPSIM_ABL_NO_WIND
constexpr bool kNoWind = true;      // wind force 0
#else
constexpr bool kNoWind = false;
#endif
#ifdef SHIPSIM_ABL_NO_MAPDIST
constexpr bool kNoMapDist = true;   // no coastline distance (+inf)
#else
constexpr bool kNoMapDist = false;
#endif
#ifdef SHIPSIM_ABL_NO_GROUND
constexpr bool kNoGround = true;    // no hull-corner grounding test
#else
constexpr bool kNoGround = false;
#endif
#ifdef SHIPSIM_ABL_NO_SBLOOP
constexpr bool kNoSbLoop = true;    // SBMPC horizon: sample 0 only
#else
constexpr bool kNoSbLoop = false;
#endif

#ifdef SHIPSIM_C2_ONE_WAVE
constexpr bool kC2OneWave = true;
#else
constexpr bool kC2OneWave = false;
#endif

// the test ship's SBMPC request as the tick loop makes it: SB_NEVER keeps the optimiser's code in the tick loop
// but never requests it (a run-time false the compiler cannot fold), SB_NONE compiles it out
__device__ __forceinline__ bool sb_request(bool need, int max_sampling) {
#if defined(SHIPSIM_ABL_SB_NEVER)
  return need && max_sampling < 0;
#elif defined(SHIPSIM_ABL_SB_NONE)
  (void)need; (void)max_sampling;
  return false;
#else
  (void)max_sampling;
  return need;
#endif
}

// ---- multi-obstacle SBMPC counters (SHIPSIM_SB_STATS) -----------------------------------------------------------
// [0] wave-ticks whose optimiser ran a pass, [1] passes, [2] lone-request passes, [3] requests served, [4] obstacle
// evaluations (scenario lanes with a horizon), [5] far-skipped obstacle evaluations (scenario lanes), [6] env-ticks
// with a request, [7] env-ticks (the test ship's sub-lane 0 ticking)
#ifdef SHIPSIM_SB_STATS
__device__ unsigned long long g_sb_stats[8];
// v summed over the wave's active lanes, one atomic per wave
__device__ __forceinline__ void sb_stat_lanes(int k, unsigned v) {
  const uint64_t ex = __builtin_amdgcn_read_exec();
  const unsigned long long t = __popcll(__ballot(v != 0));
  if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)ex) - 1 && t) atomicAdd(&g_sb_stats[k], t);
}
// v once per wave (a wave-uniform value)
__device__ __forceinline__ void sb_stat_wave(int k, unsigned v) {
  const uint64_t ex = __builtin_amdgcn_read_exec();
  if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)ex) - 1 && v) atomicAdd(&g_sb_stats[k], (unsigned long long)v);
}
#else
__device__ __forceinline__ void sb_stat_lanes(int, unsigned) {}
__device__ __forceinline__ void sb_stat_wave(int, unsigned) {}
#endif

// ---- lane / index checks ---------------------------------------------------------------------------------------
// Every cross-lane exchange checks that the lanes it reads are active (the env's LPE lanes for the DPP / shuffle
// helpers, a ship's lanes for its sub-lane pairs, the whole wave for the wave-cooperative SBMPC and policy passes),
// and the data-dependent indices of the decision path are range-checked. A violation is counted (first site and exec
// mask kept) and read back with shipsim_diag_lane_faults.
#ifdef SHIPSIM_LANECHECK
// [0] violations, [1] first site, [2] / [3] its exec mask lo / hi, [8 + site] violations per site
__device__ unsigned g_lane_diag[32];
__device__ __noinline__ void lane_fault(int site) {
  const uint64_t ex = __builtin_amdgcn_read_exec();
  atomicAdd(&g_lane_diag[8 + (site & 15)], 1u);
  if (atomicAdd(&g_lane_diag[0], 1u) == 0u) {
    atomicExch(&g_lane_diag[1], (unsigned)site);
    atomicExch(&g_lane_diag[2], (unsigned)ex);
    atomicExch(&g_lane_diag[3], (unsigned)(ex >> 32));
  }
}
template <int LPE>
__device__ __forceinline__ void lane_check(int site) {  // all LPE lanes of this lane's group active
  const int l0 = (int)(threadIdx.x & 63) & ~(LPE - 1);
  const uint64_t need = LPE >= 64 ? ~0ull : (((1ull << LPE) - 1) << l0);
  if ((__builtin_amdgcn_read_exec() & need) != need) lane_fault(site);
}
template <int LPE, int SLOTS>
__device__ __forceinline__ void ship_check(int site) {  // the lanes of this lane's ship within its env
  const int lane = (int)(threadIdx.x & 63), l0 = lane & ~(LPE - 1);
  uint64_t pat = 0;
  for (int k = lane % SLOTS; k < LPE; k += SLOTS) pat |= 1ull << k;
  const uint64_t need = pat << l0;
  if ((__builtin_amdgcn_read_exec() & need) != need) lane_fault(site);
}
#define SHIPSIM_LANE_CHECK(LPE_, site) ::shipsim::diag::lane_check<LPE_>(site)
#define SHIPSIM_SHIP_CHECK(LPE_, SLOTS_, site) ::shipsim::diag::ship_check<LPE_, SLOTS_>(site)
#define SHIPSIM_INDEX_CHECK(cond, site)           \
  do {                                            \
    if (!(cond)) ::shipsim::diag::lane_fault(site); \
  } while (0)
#else
#define SHIPSIM_LANE_CHECK(LPE_, site) ((void)0)
#define SHIPSIM_SHIP_CHECK(LPE_, SLOTS_, site) ((void)0)
#define SHIPSIM_INDEX_CHECK(cond, site) ((void)0)
#endif

// ---- phase timing ----------------------------------------------------------------------------------------------
// Per-phase wall-clock cycles summed over waves: [0..3] the tick loop's phases (PT_MARK), [4..7] the split of one
// SBMPC scenario evaluation (SB_MARK). The stamps serialise the wave, so the split is indicative only.
#ifdef SHIPSIM_PHASE_TIMING
__device__ unsigned long long g_phase_cycles[8];
struct PhaseTimer {
  unsigned long long acc[4] = {0, 0, 0, 0}, last;
  __device__ PhaseTimer() : last(wall_clock64()) {}
  __device__ void mark(int k) {
    const unsigned long long t = wall_clock64();
    acc[k] += t - last;
    last = t;
  }
  __device__ void flush(int base) {
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < 4; ++k) atomicAdd(&g_phase_cycles[base + k], acc[k]);
  }
};
struct SbTimer : PhaseTimer {
  __device__ ~SbTimer() {
    mark(3);
    if ((threadIdx.x & 31) == 0)
      for (int k = 0; k < 4; ++k) atomicAdd(&g_phase_cycles[4 + k], acc[k]);
  }
};
#define PT_DECL ::shipsim::diag::PhaseTimer pt_timer
#define PT_MARK(k) pt_timer.mark(k)
#define PT_FLUSH() pt_timer.flush(0)
#define SB_TIMER ::shipsim::diag::SbTimer sb_timer
#define SB_MARK(k) sb_timer.mark(k)
#else
#define PT_DECL \
  do {          \
  } while (0)
#define PT_MARK(k) \
  do {             \
  } while (0)
#define PT_FLUSH() \
  do {             \
  } while (0)
#define SB_TIMER \
  do {           \
  } while (0)
#define SB_MARK(k) \
  do {             \
  } while (0)
#endif

// ---- stale-LDS check -------------------------------------------------------------------------------------------
// every word of [p, p + bytes) set to SHIPSIM_POISON_LDS by the block, so a read of LDS the kernel did not write sees
// the pattern (a signalling NaN for fp64 state) instead of another kernel's leftovers
__device__ __forceinline__ void poison_lds(void* p, size_t bytes) {
#ifdef SHIPSIM_POISON_LDS
  for (size_t i = threadIdx.x; i < bytes / 4; i += blockDim.x) ((uint32_t*)p)[i] = SHIPSIM_POISON_LDS;
#else
  (void)p; (void)bytes;
#endif
}
constexpr bool kPoisonLds =
#ifdef SHIPSIM_POISON_LDS
    true;
#else
    false;
#endif

}  // namespace diag
}  // namespace shipsim

// ---- per-env printf -------------------------------------------------------------------------------------------
#ifdef SHIPSIM_DEBUG_ENV
#define SHIPSIM_DEBUG_PRINT(env_, ...)                   \
  do {                                                   \
    if ((env_) == SHIPSIM_DEBUG_ENV) printf(__VA_ARGS__); \
  } while (0)
#else
#define SHIPSIM_DEBUG_PRINT(env_, ...) \
  do {                                 \
  } while (0)
#endif
