// shipsim_kernels.hip — HIP kernels (gfx950) + C ABI (include/shipsim.h) of the batched
// ship-in-transit simulator -> ast_sac_amd/lib/libshipsim.so, linked from two objects of this file (SHIPSIM_TU below).
//
// Kernels
//   init_kernel    : state as constructed (ShipModelAST/SimpleShipModel.__init__, controllers,
//                    NavigationSystem, MultiShipRLEnv.__init__ :54-141)
//   reset_kernel   : MultiShipRLEnv.reset (env.py:238-295) incl. init_step (:297-342)
//   ast_step_kernel: MultiShipRLEnv.step (env.py:624-773) — event-driven: each env ticks
//                    (_step :563-622) until its decision point (RoA + 1 tick) or done
//   single_tick_kernel: C2 single-ship loop body (run_colav/run_simplified_model.py:248-249 shape)
//   single_tick_pipe_kernel: the same for the simplified machinery, three waves per 64 ships
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "shipsim.h"
#include "shipsim_device.hpp"

#include "shipsim_diag.hpp"  // diagnostics / ablation hooks (none in the product build)


using namespace shipsim;

// Translation-unit role (ast_sac_amd/build_hash.py OBJECTS):
//   SHIPSIM_TU 1: every kernel but single_tick_pipe_kernel, and the C ABI — built without machine-level LICM (the
//                 tick loops' constants are rematerialised rather than held in registers: DESIGN.md §7a)
//   SHIPSIM_TU 2: single_tick_pipe_kernel and its launch only — with LICM: its three short loops have registers to
//                 spare, and the fp64 constants of atan / sincos are hoisted out of the tick loop
//   SHIPSIM_TU 0: everything in one object (diagnostics and register-report builds)
#ifndef SHIPSIM_TU
#define SHIPSIM_TU 0
#endif
// (defined with single_tick_pipe_kernel, in the SHIPSIM_TU 2 object of the product build)
void shipsim_c2_pipe_launch(int blocks, hipStream_t st, const Params& P, const struct DevState& S,
                            const struct ConstBuf& K, int k);

// ---------------------------------------------------------------------------------------------
// device state (SoA). Ship arrays are indexed q = env * n_ships + ship (lane order).
// ---------------------------------------------------------------------------------------------
struct DevState {
  // One device block; every array lives at base + (index * stride). Keeping the table as one base
  // pointer + strides (instead of ~40 pointers) keeps it out of the SGPR budget of the big kernel.
  char* base;
  int64_t ship_stride;   // bytes of one [env][ship] array (doubles)
  int64_t route_stride;  // bytes of one [env][ship][kMaxRoute] route array
  int64_t env_stride;    // bytes of one per-env array (sized for the widest: 8 floats)
  int64_t env_off;       // start of the per-env arrays
  __host__ __device__ double* f(int k) const { return (double*)(base + k * ship_stride); }
  __host__ __device__ int32_t* next_wpt() const { return (int32_t*)(base + 19 * ship_stride); }
  __host__ __device__ int32_t* stop() const { return (int32_t*)(base + 20 * ship_stride); }
  __host__ __device__ int32_t* n_route() const { return (int32_t*)(base + 21 * ship_stride); }
  __host__ __device__ double* route_n() const { return (double*)(base + 22 * ship_stride); }
  __host__ __device__ double* route_e() const { return (double*)(base + 22 * ship_stride + route_stride); }
  __host__ __device__ char* ev(int k) const { return base + env_off + k * env_stride; }
  __host__ __device__ int32_t* sampling_count() const { return (int32_t*)ev(0); }
  __host__ __device__ double* travel_dist() const { return (double*)ev(1); }
  __host__ __device__ double* travel_time() const { return (double*)ev(2); }
  __host__ __device__ double* acc() const { return (double*)ev(3); }
  __host__ __device__ double* n_base() const { return (double*)ev(4); }
  __host__ __device__ double* e_base() const { return (double*)ev(5); }
  __host__ __device__ double* p_last() const { return (double*)ev(6); }
  __host__ __device__ double* chi_last() const { return (double*)ev(7); }
  __host__ __device__ double* mach_dt() const { return (double*)ev(8); }
  __host__ __device__ float* states4() const { return (float*)ev(9); }      // [env][4] self.states (simple collav)
  __host__ __device__ float* next_obs8() const { return (float*)ev(10); }   // [env][8] self.next_observations
  __host__ __device__ uint32_t* snap_bits() const { return (uint32_t*)ev(11); }
  __host__ __device__ int32_t* was_reset() const { return (int32_t*)ev(12); }
  __host__ __device__ int32_t* dec_flags() const { return (int32_t*)ev(13); }  // DF_* (sliced stepping)
  __host__ __device__ double* legacy_states() const { return (double*)ev(14); }  // [env][4] legacy self.states
  __host__ __device__ int32_t* legacy_flags() const { return (int32_t*)ev(15); }  // 1: still the f32 initial_states
  __host__ __device__ int32_t* dec_ticks() const { return (int32_t*)ev(16); }  // ticks of the decision in progress
  // the decision in progress as the stream logs it (SHIPSIM_DL_ACTION / _OBS0): its action, the observation it
  // was chosen from
  __host__ __device__ float* dec_action() const { return (float*)ev(17); }
  __host__ __device__ float* dec_obs0() const { return (float*)ev(18); }  // [env][8]
  int32_t* nonfinite;  // device counter: envs flagged SHIPSIM_EV_NONFINITE (read by shipsim_synchronize)
  static constexpr int kEnvArrays = 19;
  static constexpr int kShipArrays = 22;
};
// dec_flags bits (per env, persistent across calls)
#define DF_AWAITING 1
#define DF_HAVE_IW 2
#define DF_PHASE_SHIFT 2

enum { SF_N = 0, SF_E, SF_YAW, SF_U, SF_V, SF_R, SF_OMEGA, SF_TIME, SF_ECT, SF_ECT_INT, SF_HDG_EI, SF_HDG_PREV,
       SF_SPD_A, SF_SPD_B, SF_RUDDER, SF_THRUST, SF_LOG_ECT, SF_LOG_N, SF_LOG_E };

struct ConstBuf {
  // edges [SHIPSIM_MAX_VERTS] | boxes [SHIPSIM_MAX_POLYS] | config routes n/e [MAX_SHIPS][kMaxRoute] each
  // | ShipConst [MAX_SHIPS] | map grid: cell edge masks [gny][gnx] uint64 | cell containment flags [gny][gnx] uint8
  // | (8-B aligned) cell edge masks split by bit rank mod 8 [gny][gnx][8] uint64
  const char* base;
  int32_t n_edges;
  int32_t gnx, gny;            // grid cells (0 = no grid: every query runs over the full map)
  double gx0, gy0, ginv;       // grid origin (east, north) and 1 / cell size
  const uint64_t* grid_mask;   // edges whose distance to the (slightly enlarged) cell is <= kGroundReach
  const uint8_t* grid_flag;    // GRID_OUT: cell entirely outside every polygon, GRID_IN: inside one, GRID_MIXED
  const uint64_t* grid_part;   // [cell][8]: the cell's mask split by bit rank mod 8 (sub-lane shares, no bit skipping)
  __host__ __device__ const Edge* edges() const { return (const Edge*)base; }
  __host__ __device__ const PolyBox* boxes() const { return (const PolyBox*)(base + sizeof(Edge) * SHIPSIM_MAX_VERTS); }
  __host__ __device__ const double* cfg_route_n() const {
    return (const double*)(base + sizeof(Edge) * SHIPSIM_MAX_VERTS + sizeof(PolyBox) * SHIPSIM_MAX_POLYS);
  }
  __host__ __device__ const double* cfg_route_e() const { return cfg_route_n() + SHIPSIM_MAX_SHIPS * kMaxRoute; }
  // per-ship constants (host make_ship_const), [ship] for the 1 + K ships of an env
  static constexpr size_t kShipsOff = sizeof(Edge) * SHIPSIM_MAX_VERTS + sizeof(PolyBox) * SHIPSIM_MAX_POLYS +
                                      sizeof(double) * 2 * SHIPSIM_MAX_SHIPS * kMaxRoute;
  __host__ __device__ const ShipConst* ships() const { return (const ShipConst*)(base + kShipsOff); }
  static constexpr size_t kBytes = kShipsOff + sizeof(ShipConst) * SHIPSIM_MAX_SHIPS;
  // grid cell of (north, east), or -1 outside the grid / no grid / non-finite position
  __device__ __forceinline__ int cell(double n, double e) const {
    const double fx = floor((e - gx0) * ginv), fy = floor((n - gy0) * ginv);
    if (!(fx >= 0.0 && fx < (double)gnx && fy >= 0.0 && fy < (double)gny)) return -1;
    return (int)fy * gnx + (int)fx;
  }
};
#define GRID_OUT 0
#define GRID_IN 1
#define GRID_MIXED 2

// The ground-distance reward terms only use the coastline distance when it is <= 1000 m
// (reward_function.py:109-117: test_ship_grounding_reward / obs_ship_grounding_reward clip at 1 km),
// so a cell only needs the edges that can come within 1000 m of it: the min over that subset equals
// the min over all edges whenever the true min is <= 1000 m, and is > 1000 m (or +inf) otherwise.
constexpr double kGroundReach = 1000.0;

// Trajectory record (shipsim_set_trajectory): simulation_results rows per ship, RewardTracker rows per
// env. Row t of a ship is its t-th store_simulation_data since reset (row 0 = init_step); env row t is
// the reward of tick t + 1 of the episode. Rows past `cap` are dropped; len keeps counting.
struct Traj {
  double* ship;   // [q][cap][SHIPSIM_TRAJ_SHIP_COLS]
  double* env;    // [env][cap][SHIPSIM_TRAJ_ENV_COLS] (may be null)
  double* fuel;   // [q][3] fuel accumulators (library-owned)
  int32_t* len;   // [env] ship rows recorded since reset
  int32_t cap;
  __device__ __forceinline__ double* ship_row(int q, int t) const {
    return (t >= 0 && t < cap) ? ship + ((size_t)q * cap + t) * SHIPSIM_TRAJ_SHIP_COLS : nullptr;
  }
  __device__ __forceinline__ double* env_row(int e, int t) const {
    return (env && t >= 0 && t < cap) ? env + ((size_t)e * cap + t) * SHIPSIM_TRAJ_ENV_COLS : nullptr;
  }
};

__device__ __forceinline__ void load_ship(const DevState& S, int q, Ship& s) {
  s.n = S.f(SF_N)[q]; s.e = S.f(SF_E)[q]; s.yaw = S.f(SF_YAW)[q];
  s.u = S.f(SF_U)[q]; s.v = S.f(SF_V)[q]; s.r = S.f(SF_R)[q];
  s.omega = S.f(SF_OMEGA)[q]; s.time = S.f(SF_TIME)[q];
  s.e_ct = S.f(SF_ECT)[q]; s.e_ct_int = S.f(SF_ECT_INT)[q];
  s.hdg_ei = S.f(SF_HDG_EI)[q]; s.hdg_prev = S.f(SF_HDG_PREV)[q];
  s.spd_a = S.f(SF_SPD_A)[q]; s.spd_b = S.f(SF_SPD_B)[q];
  s.log_rudder = S.f(SF_RUDDER)[q]; s.log_thrust = S.f(SF_THRUST)[q]; s.log_ect = S.f(SF_LOG_ECT)[q];
  s.log_n = S.f(SF_LOG_N)[q]; s.log_e = S.f(SF_LOG_E)[q];
  s.next_wpt = S.next_wpt()[q]; s.stop = S.stop()[q]; s.n_route = S.n_route()[q];
  load_segment(s, S.route_n() + (size_t)q * kMaxRoute, S.route_e() + (size_t)q * kMaxRoute);
}
__device__ __forceinline__ void store_ship(const DevState& S, int q, const Ship& s) {
  S.f(SF_N)[q] = s.n; S.f(SF_E)[q] = s.e; S.f(SF_YAW)[q] = s.yaw;
  S.f(SF_U)[q] = s.u; S.f(SF_V)[q] = s.v; S.f(SF_R)[q] = s.r;
  S.f(SF_OMEGA)[q] = s.omega; S.f(SF_TIME)[q] = s.time;
  S.f(SF_ECT)[q] = s.e_ct; S.f(SF_ECT_INT)[q] = s.e_ct_int;
  S.f(SF_HDG_EI)[q] = s.hdg_ei; S.f(SF_HDG_PREV)[q] = s.hdg_prev;
  S.f(SF_SPD_A)[q] = s.spd_a; S.f(SF_SPD_B)[q] = s.spd_b;
  S.f(SF_RUDDER)[q] = s.log_rudder; S.f(SF_THRUST)[q] = s.log_thrust; S.f(SF_LOG_ECT)[q] = s.log_ect;
  S.f(SF_LOG_N)[q] = s.log_n; S.f(SF_LOG_E)[q] = s.log_e;
  S.next_wpt()[q] = s.next_wpt; S.stop()[q] = s.stop; S.n_route()[q] = s.n_route;
}

// per-block LDS copy of the ships' ShipConst (lanes of one ship read one address)
// (and the reciprocals div_by uses, formed here on the device: the bits of the division sequence's own)
__device__ __forceinline__ const ShipConst* stage_consts(const ConstBuf& K, ShipConst* lds, int n_ships, double dt) {
  const int nwords = (int)(sizeof(ShipConst) * n_ships / sizeof(double));
  const double* src = reinterpret_cast<const double*>(K.ships());
  double* dst = reinterpret_cast<double*>(lds);
  for (int i = threadIdx.x; i < nwords; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  if ((int)threadIdx.x < n_ships) {
    ShipConst& c = lds[threadIdx.x];
    c.rcp_r_me = div_rcp(c.r_me); c.rcp_r_hsg = div_rcp(c.r_hsg); c.rcp_jp = div_rcp(c.jp); c.rcp_dt = div_rcp(dt);
  }
  __syncthreads();
  return lds;
}

#if SHIPSIM_TU != 2
// control half of one ship tick: autopilot -> speed control -> (simple collav) -> store
// (env.py test_step :389-433 / obs_step :481-512 / init_step :309-339); returns (ctrl, rudder)
// PRE: (pre_q, pre_e) = los_q at (s.n, s.e) on the current segment, evaluated earlier in the tick; used unless the
// waypoint index advances here
template <bool DETAILED, bool REC, bool PRE = false>
__device__ __forceinline__ void control_and_store(const ShipConst& c, const Params& P, Ship& s,
                                                  const double* __restrict__ rn, const double* __restrict__ re,
                                                  double offset, double speed_factor, double mach_dt,
                                                  int simple_collav_flag /*0 none, 1 rl(-15deg), 2 noniw(+15)*/,
                                                  bool imminent, double* row, double* fuel, double& ctrl_out,
                                                  double& rudder_out, double pre_q = 0.0, double pre_e = 0.0) {
  const double N = s.n, E = s.e, H = s.yaw, U = s.u;
  double href;
  if constexpr (PRE) {
    double q = pre_q, e_ct = pre_e;
    if (next_wpt_advance(c, s, N, E)) {
      s.next_wpt += 1;
      load_segment(s, rn, re);
      q = los_q(c, s, N, E, e_ct);
    }
    s.e_ct = e_ct;
    href = s.seg_alpha + atan(los_windup(c, s, q));
  } else {
    if (next_wpt_advance(c, s, N, E)) {
      s.next_wpt += 1;
      load_segment(s, rn, re);
    }
    href = los_guidance(c, s, N, E);
  }
  double rudder = heading_ctrl(c, s, href + offset, H, P.dt, c.rcp_dt);
  double ctrl = speed_ctrl(c, s, c.desired_speed * speed_factor, U, P.dt, DETAILED, c.rcp_dt);
  if (simple_collav_flag && imminent) {
    ctrl *= 0.5;
    ctrl = py_min(py_max(ctrl, 0.0), 1.1);
    rudder += (simple_collav_flag == 1 ? -15.0 : 15.0) * (kPi / 180.0);
    rudder = py_min(py_max(rudder, -c.max_rudder), c.max_rudder);
  }
  // store_simulation_data (the fields later read back through simulation_results[-1])
  s.log_rudder = rudder;
  s.log_ect = s.e_ct;
  s.log_n = N;
  s.log_e = E;
  s.log_thrust = DETAILED ? (c.thrust_coeff * s.omega * fabs(s.omega)) / 1000 : ctrl;
  if (REC) {  // the full store_simulation_data row (ship_model.py:903-942) + ShipAssets trackers
    if (DETAILED) fuel_consumption(c, ctrl, mach_dt, fuel);
    if (row) {
      row[SHIPSIM_TS_TIME] = s.time; row[SHIPSIM_TS_NORTH] = N; row[SHIPSIM_TS_EAST] = E;
      row[SHIPSIM_TS_YAW] = H; row[SHIPSIM_TS_RUDDER] = rudder; row[SHIPSIM_TS_U] = U;
      row[SHIPSIM_TS_V] = s.v; row[SHIPSIM_TS_R] = s.r; row[SHIPSIM_TS_OMEGA] = DETAILED ? s.omega : 0.0;
      row[SHIPSIM_TS_THRUST] = DETAILED ? c.thrust_coeff * s.omega * fabs(s.omega) : ctrl;
      row[SHIPSIM_TS_E_CT] = s.e_ct; row[SHIPSIM_TS_E_PSI] = fabs(H - href); row[SHIPSIM_TS_LOAD] = ctrl;
      row[SHIPSIM_TS_FUEL_ME] = DETAILED ? fuel[0] : 0.0; row[SHIPSIM_TS_FUEL_EL] = DETAILED ? fuel[1] : 0.0;
      row[SHIPSIM_TS_FUEL] = DETAILED ? fuel[2] : 0.0; row[SHIPSIM_TS_E_CT_INT] = s.e_ct_int;
      row[SHIPSIM_TS_NEXT_WPT] = (double)s.next_wpt; row[SHIPSIM_TS_REPEAT] = 0.0;
      row[SHIPSIM_TS_TIME_LIST] = s.time;
    }
  }
  ctrl_out = ctrl;
  rudder_out = rudder;
}

// one controlled ship tick: autopilot -> speed control -> store -> update -> integrate -> next_time
// with the reference's angle-form wind force (PAIRED: sub-lanes 2k / 2k+1 share the batched sincos
// calls, odd = this lane is 2k+1) or the algebraic one (ALGW, (wsin, wcos) = sin/cos(wind_direction)).
// The legacy per-tick kernel and the C2 single-ship kernel use this form.
template <bool DETAILED, bool REC = false, bool PAIRED = false, bool ALGW = false>
__device__ __forceinline__ void control_and_integrate(const ShipConst& c, const Params& P, Ship& s,
                                                      const double* __restrict__ rn, const double* __restrict__ re,
                                                      double offset, double speed_factor, double mach_dt,
                                                      int simple_collav_flag, bool imminent, double* row = nullptr,
                                                      double* fuel = nullptr, bool odd = false, double wsin = 0.0,
                                                      double wcos = 1.0) {
  double ctrl, rudder;
  control_and_store<DETAILED, REC>(c, P, s, rn, re, offset, speed_factor, mach_dt, simple_collav_flag, imminent, row,
                                   fuel, ctrl, rudder);
  Deriv d = differentials<PAIRED, ALGW>(c, P, s, ctrl, rudder, DETAILED, odd, wsin, wcos);
  integrate(s, d, P.dt, mach_dt, DETAILED);
}

// the same tick in the AST kernels (step, decision stream, reset / init_step): algebraic wind force
// and sin/cos(yaw) carried in (sy, cy) — valid for s.yaw on entry, refreshed after the integration
// step, so one sincos per ship-tick serves both the kinematics and the reward's encounter angle.
template <bool DETAILED, bool REC = false, bool PRE = false>
__device__ __forceinline__ void control_and_integrate_sc(const ShipConst& c, const Params& P, Ship& s,
                                                         const double* __restrict__ rn,
                                                         const double* __restrict__ re, double offset,
                                                         double speed_factor, double mach_dt, int simple_collav_flag,
                                                         bool imminent, double* row, double* fuel, double& sy,
                                                         double& cy, double pre_q = 0.0, double pre_e = 0.0) {
  double ctrl, rudder;
  control_and_store<DETAILED, REC, PRE>(c, P, s, rn, re, offset, speed_factor, mach_dt, simple_collav_flag, imminent,
                                        row, fuel, ctrl, rudder, pre_q, pre_e);
  Deriv d = differentials_sc(c, P, s, ctrl, rudder, DETAILED, sy, cy);
  integrate(s, d, P.dt, mach_dt, DETAILED);
  sincos(s.yaw, &sy, &cy);
}

// store_last_simulation_data (ship_model.py:946-957) of a stopped ship: the previous row repeated
// with the current time; ShipAssets.time_list gets the time after the first next_time (env.py:451-465)
__device__ __forceinline__ void record_last(const Traj& T, int q, int t, double time, double time_list) {
  double* row = T.ship_row(q, t);
  const double* prev = T.ship_row(q, t - 1);
  if (!row || !prev) return;
  for (int k = 0; k < SHIPSIM_TRAJ_SHIP_COLS; ++k) row[k] = prev[k];
  row[SHIPSIM_TS_TIME] = time;
  row[SHIPSIM_TS_REPEAT] = 1.0;
  row[SHIPSIM_TS_TIME_LIST] = time_list;
}

// ---------------------------------------------------------------------------------------------
// SBMPC (sbmpc.py:113-298), wave-cooperative: each requesting env's 7 x 4 scenarios are spread
// over 28 lanes of a half-wave; two envs are served per pass.
// ---------------------------------------------------------------------------------------------
struct SbIn {
  double u_d, chi_d, os_x, os_y, os_v, ob_x, ob_y, ob_psi, ob_u, ob_v, obs_l, obs_w, p_last, chi_last;
  double ob_so, ob_co;  // sin / cos(ob_psi): the AST kernels pass the obstacle ship's carried sin/cos(yaw)
};
// sin/cos(ob_psi) of a request built from its heading alone
__device__ __forceinline__ void sb_set_heading_trig(SbIn& q) { sincos(q.ob_psi, &q.ob_so, &q.ob_co); }

// a lane value the compiler must re-derive after this point (loads indexed by it cannot be hoisted)
__device__ __forceinline__ int opaque_v(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
// a wave-uniform value the compiler must re-derive after this point (comparisons on it cannot be hoisted)
__device__ __forceinline__ int opaque_s(int x) {
  asm volatile("" : "+s"(x));
  return x;
}
// opaque_v where OPQ (the kernels whose allocation otherwise spills the lane masks derived from x), x as is
// elsewhere (there the recomputation costs more than the held mask)
template <bool OPQ>
__device__ __forceinline__ int opaque_if(int x) {
  if constexpr (OPQ) return opaque_v(x);
  return x;
}

__device__ __forceinline__ double shfl_d(double x, int src) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  lo = __shfl(lo, src, 64);
  hi = __shfl(hi, src, 64);
  return __hiloint2double(hi, lo);
}

constexpr double kCosPhiAh = 0.36650122672429719;  // cos(68.5°) (only used against a 1e-9 band)
constexpr double kSinPhiAh = 0.93041756798202460;  // sin(68.5°)

// sqrt(a) < c and sqrt(a) <= c (c > 0) decided on a against c², except within a relative 1e-12 of
// it where the correctly rounded square root itself decides: the reference's boolean, without the
// ~20-instruction f64 sqrt on every tick (NaN compares false either way)
__device__ __forceinline__ bool sqrt_lt(double a, double c) {
  const double c2 = c * c;
  if (a < c2 * (1.0 - 1e-12)) return true;
  if (!(a <= c2 * (1.0 + 1e-12))) return false;
  return sqrt(a) < c;
}
__device__ __forceinline__ bool sqrt_le(double a, double c) {
  const double c2 = c * c;
  if (a < c2 * (1.0 - 1e-12)) return true;
  if (!(a <= c2 * (1.0 + 1e-12))) return false;
  return sqrt(a) <= c;
}

// (d_safe / dist) ** Q_ with Q_ = 4 (sbmpc.py:262): x² = h + l and h² = h2 + e exactly (fma), so
// h2 + (e + (2hl + l²)) carries ~100 bits into its one final rounding — the correctly rounded x⁴, which
// is glibc's pow(x, 4.0) except where that pow's last 0.02 ulp decides (85 per 10⁵ random d_safe / dist
// in (0.9, 1000]) — in 11 VALU instructions instead of the general pow's 214. An infinite x⁴ (dist -> 0)
// is returned as is.
__device__ __forceinline__ double pow4(double x) {
  const double h = x * x, l = fma(x, x, -h);
  const double h2 = h * h;
  if (!(h2 < INFINITY)) return h2;
  const double e = fma(h, h, -h2);
  return h2 + (e + (2.0 * h * l + l * l));
}

// Per-sample collision cost H0 = C·R of sbmpc.py:205-289 (KAPPA_ = 0) for one prediction sample with
// obstacle-minus-own-ship offset (d0, d1); (ss, cs, sv) are the own ship's sin/cos(psi_) and sway
// at that sample. R and C stay 0 unless dist < d_safe_i <= max_d_safe, so the sector geometry (atan2,
// wrap, norms) is only evaluated there; identical results to the reference's `dist < d_close` block.
__device__ __forceinline__ double sbmpc_sample_cost(const SbIn& in, double so, double co, double vo0, double vo1,
                                                    double no, double t, double d0, double d1, double d2s,
                                                    double ss, double cs, double ud, double sv, double max_d_safe,
                                                    double lim2, double cos_ot) {
  const double os_l = 25.0, d_safe = 1000.0, d_close = 2000.0;
  const double PHI_AH = 68.5 * (kPi / 180.0), PHI_OT = 68.5 * (kPi / 180.0);
  if (!(d2s < lim2)) return 0.0;  // d2s >= lim2 already implies sqrt(d2s) >= max_d_safe
  const double dist = sqrt(d2s);
  if (!(dist < d_close && dist < max_d_safe)) return 0.0;
  double vs0 = -ss * ud + cs * sv;
  double vs1 = cs * ud + ss * sv;
  // sector of phi_o = wrap(atan2(-d1, -d0) - psi_o + pi/2) against PHI_AH == PHI_OT = θ: e is
  // (-d0, -d1) rotated by pi/2 - psi_o, so phi_o = angle(e); phi_o > θ <=> sin(angle(e) - θ) >= 0
  // and e_y > 0. Within 1e-9 rad of a decision boundary the reference expression is evaluated.
  const double ex = so * (-d0) - co * (-d1), ey = co * (-d0) + so * (-d1);
  const double cr = kCosPhiAh * ey - kSinPhiAh * ex;
  int sector;  // 0: phi_o < PHI_AH, 1: phi_o > PHI_OT, 2: equal
  if (fabs(cr) > 1e-9 * dist && fabs(ey) > 1e-9 * dist) {
    sector = (cr >= 0 && ey > 0) ? 1 : 0;
  } else {
    const double phi_o = wrap_pmpi(atan2(-d1, -d0) - in.ob_psi + kPi / 2);
    sector = (phi_o < PHI_AH) ? 0 : ((phi_o > PHI_OT) ? 1 : 2);
  }
  double d_safe_i;
  if (sector == 0) d_safe_i = d_safe + in.obs_l / 2;
  else if (sector == 1) d_safe_i = 0.5 * d_safe + in.obs_l / 2;
  else d_safe_i = d_safe + in.obs_w / 2;
  double dot = vs0 * vo0 + vs1 * vo1;
  double ns = sqrt(vs0 * vs0 + vs1 * vs1);
  if (dot > cos_ot * ns * no && ns > no) d_safe_i = d_safe + os_l / 2 + in.obs_l / 2;
  if (!(dist < d_safe_i)) return 0.0;
  const double R = (1 / fabs(t - 0.0)) * pow4(d_safe / dist);  // pow(|t|, 1.0) == |t| exactly
  const double k_coll = 1e-6 * os_l * in.obs_l;
  const double w0 = vs0 - vo0, w1 = vs1 - vo1;
  const double nrm = sqrt(w0 * w0 + w1 * w1);
  const double C = k_coll * (nrm * nrm);
  return C * R + 0.0 * 0;
}

// sbmpc.py:190-298 cost_func for one (Chi_ca, P_ca) scenario, sample by sample as the reference.
// Kept as the exact fallback of sbmpc_scenario_cost (near-ties between samples).
__device__ __forceinline__ double sbmpc_scenario_cost_direct(const SbIn& in, int n_samp, double DT, double ud,
                                                          double sp, double cp, double sp0, double cp0, double so,
                                                          double co, double vo0, double vo1, double no,
                                                          double max_d_safe, double lim2, double cos_ot, double H2) {
  const double r11 = -so, r12 = co, r21 = co, r22 = so;
  const double q11 = -sp, q12 = cp, q21 = cp, q22 = sp;
  double ox = in.ob_x, oy = in.ob_y, sx = in.os_x, sy = in.os_y, sv = in.os_v;
  double H1 = 0, t = 0;
  for (int i = 0; i < n_samp; ++i) {
    if (i > 0) {
      ox = ox + (r11 * in.ob_u + r12 * in.ob_v) * DT;
      oy = oy + (r21 * in.ob_u + r22 * in.ob_v) * DT;
      sx = sx + DT * (q11 * ud + q12 * sv);
      sy = sy + DT * (q21 * ud + q22 * sv);
      sv = 0.0;
    }
    t += DT;
    const double d0 = ox - sx, d1 = oy - sy;
    const double H0 = sbmpc_sample_cost(in, so, co, vo0, vo1, no, t, d0, d1, d0 * d0 + d1 * d1, (i == 0) ? sp0 : sp,
                                        (i == 0) ? cp0 : cp, ud, sv, max_d_safe, lim2, cos_ot);
    if (H0 > H1) H1 = H0;
  }
  return H1 + H2;
}


// SBMPCParams.P_ca_ = [0.4, 0.6, 0.8, 1.0] (sbmpc.py:36) by selects: a per-lane indexed constant array would be
// a memory load on the scenario's critical path
__device__ __forceinline__ double p_ca_of(int jp) {
  return jp == 0 ? 0.4 : (jp == 1 ? 0.6 : (jp == 2 ? 0.8 : 1.0));
}

// the scenario's own terms of the cost (sbmpc.py:200-214: P_ca, Chi_ca and their changes); the whole
// cost when no obstacle sample comes within max_d_safe
__device__ __forceinline__ double sbmpc_h2(const SbIn& in, int ichi, int jp) {
  const double P_ca = p_ca_of(jp);
  const double Chi_ca = (-30.0 + 10.0 * ichi) * (kPi / 180.0);
  const double dChi0 = Chi_ca - in.chi_last;
  return 25 * (1 - P_ca) + 30 * (Chi_ca * Chi_ca) + 20 * fabs(in.p_last - P_ca) +
         ((dChi0 > 0) ? 20 * dChi0 * dChi0 : (dChi0 < 0 ? 30 * dChi0 * dChi0 : 0));
}

// No scenario can bring this obstacle within max_d_safe over the horizon: the distance now minus the
// most either ship can travel (own ship: sample 0 at its current sway, then straight at <= u_d; the
// obstacle: straight at its speed) stays beyond max_d_safe with a 1 m margin (the incremental
// predictions round at ~1e-12 relative). Then every scenario's cost for it is exactly sbmpc_h2.
__device__ __forceinline__ bool sbmpc_far(const SbIn& in, int n_samp, double DT) {
  const double os_l = 25.0, d_safe = 1000.0;
  const double max_d_safe = py_max(py_max(d_safe + in.obs_l / 2, 0.5 * d_safe + in.obs_l / 2),
                                   py_max(d_safe + in.obs_w / 2, d_safe + os_l / 2 + in.obs_l / 2));
  const double ex = in.ob_x - in.os_x, ey = in.ob_y - in.os_y;
  const double own = DT * sqrt(in.u_d * in.u_d + in.os_v * in.os_v) + (n_samp - 2 > 0 ? n_samp - 2 : 0) * DT * in.u_d;
  const double obs = (n_samp - 1) * DT * sqrt(in.ob_u * in.ob_u + in.ob_v * in.ob_v);
  const double lim = max_d_safe + 1.0 + own + obs;
  return ex * ex + ey * ey > lim * lim;
}

// running state of a scenario's horizon: best (s1 at time t1, squared distance q1) and runner-up s2 of the
// ranking t·d², and whether any in-range sample sat within a rounding band of a decision (unc)
struct HzBest {
  double s1, s2, t1, q1;
  bool unc;
};
struct HzConst {
  double so, co, ovr2, ot2, ah2, cl2;  // obstacle heading sin/cos, squared thresholds
  bool ovr;                            // the overtaking override of d_safe_i holds for every sample
};
// one horizon sample (time tt, offset (d0, d1), d2s = |.|²) into the running state; inr: the sample is within
// max_d_safe (one beyond it contributes nothing and flags nothing). Branch-free (& | on bools).
__device__ __forceinline__ void hz_sample(HzBest& h, const HzConst c, double tt, double d0, double d1, double d2s,
                                          bool inr) {
  constexpr double kEps = 1e-12;
  // sector of phi_o (see sbmpc_sample_cost): overtaking sector iff cr >= 0 and ey > 0
  const double ex = c.so * (-d0) - c.co * (-d1), ey = c.co * (-d0) + c.so * (-d1);
  const double cr = kCosPhiAh * ey - kSinPhiAh * ex;
  const bool sec_ok = (cr * cr > 1e-18 * d2s) & (ey * ey > 1e-18 * d2s);
  const double D2 = c.ovr ? c.ovr2 : (((cr >= 0) & (ey > 0)) ? c.ot2 : c.ah2);
  const bool member = inr & (d2s < D2 * (1.0 - kEps)) & (d2s < c.cl2 * (1.0 - kEps));
  h.unc = h.unc | (inr & (((!c.ovr) & (!sec_ok)) | (fabs(d2s - D2) <= kEps * D2) | (fabs(d2s - c.cl2) <= kEps * c.cl2)));
  const double sc = member ? tt * d2s * d2s : INFINITY;
  const bool lt1 = sc < h.s1;
  h.s2 = fmin(h.s2, fmax(h.s1, sc));  // runner-up: the old best if sc takes the lead, else min(s2, sc)
  h.t1 = lt1 ? tt : h.t1;
  h.q1 = lt1 ? d2s : h.q1;
  h.s1 = fmin(h.s1, sc);
}

// part -1: the whole horizon on this lane. part 0 / 1: this lane and its partner (lane ^ 32: the same scenario of the
// same request) split the horizon's sample loop — part 0 takes the samples before i_split, part 1 the rest — and merge
// their running bests (every other step is computed by both; the result is the same bits as part -1)
__device__ double sbmpc_scenario_cost(const SbIn& in, int n_samp, double DT, int ichi, int jp, int part = -1) {
  SB_TIMER;
  const double os_l = 25.0;  // ShipLinearModel default length (sbmpc_misc.py:86, Q7)
  const double d_safe = 1000.0, d_close = 2000.0;
  // np.cos(np.deg2rad(PHI_OT_)) — PHI_OT_ is already in radians (sbmpc.py:248): a constant, taken
  // as the correctly rounded double of cos(68.5·(π/180)²) (NumPy and glibc agree on it)
  constexpr double cos_ot = 0.9997823068017366;
  const double max_d_safe = py_max(py_max(d_safe + in.obs_l / 2, 0.5 * d_safe + in.obs_l / 2),
                                   py_max(d_safe + in.obs_w / 2, d_safe + os_l / 2 + in.obs_l / 2));
  const double CHI_DEG = -30.0 + 10.0 * ichi;
  const double P_ca = p_ca_of(jp);
  const double Chi_ca = CHI_DEG * (kPi / 180.0);
  const double ud = in.u_d * P_ca;
  const double psi_d = in.chi_d + Chi_ca;
  // Obstacle trajectory (sbmpc_misc.py:65-83) and linear_pred (:103-123), advanced incrementally
  // the obstacle heading's sin/cos come with the request (ob_so, ob_co): the same values as
  // sincos(in.ob_psi) — in the AST kernels they are the obstacle ship's own carried sin/cos(yaw) with
  // ob_psi = -yaw, and the device sin is odd and cos even (both reduce |x|), so nothing is recomputed
  // per scenario
  const double so = in.ob_so, co = in.ob_co;
  const double r11 = -so, r12 = co, r21 = co, r22 = so;
  const double vo0 = -so * in.ob_u + co * in.ob_v;  // rot2d(obstacle.psi_, [u, v])
  const double vo1 = co * in.ob_u + so * in.ob_v;
  const double no = sqrt(vo0 * vo0 + vo1 * vo1);
  double sp, cp;
  sincos(psi_d, &sp, &cp);
  const double q11 = -sp, q12 = cp, q21 = cp, q22 = sp;
  double sp0 = sp, cp0 = cp;
  const double psi_w = wrap_pmpi(psi_d);
  if (psi_w != psi_d) sincos(psi_w, &sp0, &cp0);
  const double H2 = sbmpc_h2(in, ichi, jp);
  int i_last = n_samp - 1;  // (set by the skip test below)
  int i_first = 1;          // first sample that can be within range (ditto; only places the split)
  int i_past = n_samp + 1;  // first sample past the closest approach, with a one-sample margin (ditto)
  // Exact skip of the horizon loop: H0 can only be non-zero at samples with dist < max_d_safe.
  // After sample 0 both predictions are straight lines (the own ship's sway is zeroed after the
  // first step), so the relative position is P1 + k·W, k = 0..n_samp-2; if its continuous minimum
  // (and sample 0) stays above max_d_safe by a margin far beyond the rounding of the incremental
  // update below, every sample's H0 is 0 and the cost is H2 alone.
  {
    const double vox = r11 * in.ob_u + r12 * in.ob_v, voy = r21 * in.ob_u + r22 * in.ob_v;
    const double e0x = in.ob_x - in.os_x, e0y = in.ob_y - in.os_y;
    const double p1x = (in.ob_x + vox * DT) - (in.os_x + DT * (q11 * ud + q12 * in.os_v));
    const double p1y = (in.ob_y + voy * DT) - (in.os_y + DT * (q21 * ud + q22 * in.os_v));
    const double wx = (vox - q11 * ud) * DT, wy = (voy - q21 * ud) * DT;
    const double ww = wx * wx + wy * wy;
    const double iww = ww > 0 ? 1.0 / ww : 0.0;  // (k and j2 below only place bounds with margins)
    double k = ww > 0 ? -(p1x * wx + p1y * wy) * iww : 0.0;
    k = k < 0 ? 0 : (k > n_samp - 2 ? n_samp - 2 : k);
    const double mx = p1x + k * wx, my = p1y + k * wy;
    const double lim = max_d_safe + 1e-3;
    SB_MARK(0);
    if (e0x * e0x + e0y * e0y > lim * lim && mx * mx + my * my > lim * lim) return 0.0 + H2;
    // Last sample that can still be within max_d_safe: |P1 + j·W| is convex in j, so past the larger
    // root j2 of |P1 + j·W| = lim every later sample stays out of range (the incremental positions
    // below differ from this closed form by ~1e-10 m, far inside the 1e-3 m of lim). Sample i = j + 1.
    const double b = p1x * wx + p1y * wy, cq = p1x * p1x + p1y * p1y - lim * lim;
    const double disc = b * b - ww * cq;
    const double j2 = (ww > 0 && disc >= 0) ? (-b + sqrt(disc)) * iww : (double)n_samp;
    i_last = (j2 < (double)(n_samp - 2)) ? (int)floor(j2) + 2 : n_samp - 1;
    const double j1 = (ww > 0 && disc >= 0) ? (-b - sqrt(disc)) * iww : 0.0;
    i_first = (j1 > 1.0) ? (int)fmin(floor(j1), (double)(n_samp - 1)) : 1;
    // Past the continuous minimum k of |P1 + j·W| both t and the distance grow, so the ranking t·d⁴ grows
    // sample by sample: once a sample there ranks beyond the best so far by more than the runner-up band,
    // no later sample can win or tie (and a later sample's flags cannot change the result). Sample i = j + 1;
    // k is clamped to the horizon, so a minimum at its end never stops the loop.
    i_past = (int)ceil(k) + 3;
  }
  const double lim2 = (max_d_safe * (1.0 + 1e-9)) * (max_d_safe * (1.0 + 1e-9));
  // Sample 0 (own ship at wrap(psi_d) with its current sway) exactly as the reference.
  const double e0x = in.ob_x - in.os_x, e0y = in.ob_y - in.os_y;
  double H1 = 0;
  {
    const double H0 = sbmpc_sample_cost(in, so, co, vo0, vo1, no, DT, e0x, e0y, e0x * e0x + e0y * e0y, sp0, cp0, ud,
                                        in.os_v, max_d_safe, lim2, cos_ot);
    if (H0 > H1) H1 = H0;
  }
  SB_MARK(1);
  // Samples 1..n-1: the own ship's velocity is constant (sway zeroed), so C and the overtaking
  // override of d_safe_i are sample-independent, and H0 = C·R with R = d_safe^4 / (t·dist^4).
  // max_i fl(C·R_i) = fl(C·max_i R_i) (rounding is monotone), so only the sample with the largest
  // R needs the exact pow: members are ranked by s = t·d2s² (within ~1e-14 of the exact ordering);
  // a runner-up within 1e-10 of the best sends the scenario to the sample-by-sample evaluation.
  const double vs0 = -sp * ud + cp * 0.0, vs1 = cp * ud + sp * 0.0;
  const double dot1 = vs0 * vo0 + vs1 * vo1;
  const double ns1 = sqrt(vs0 * vs0 + vs1 * vs1);
  const bool ovr = dot1 > cos_ot * ns1 * no && ns1 > no;
  const double ds_ah = d_safe + in.obs_l / 2, ds_ot = 0.5 * d_safe + in.obs_l / 2;  // :239-242
  const double ds_ovr = d_safe + os_l / 2 + in.obs_l / 2;
  // Branch-free horizon: membership dist < d_safe_i (and < d_close) is decided on d2s against the
  // squared thresholds; a sample within 1e-12 of a threshold, or whose sector is within 1e-9 of
  // the PHI_AH / PHI_OT boundary, marks the scenario `unc` and it is re-evaluated sample by sample.
  constexpr double kEps = 1e-12;
  const double ah2 = ds_ah * ds_ah, ot2 = ds_ot * ds_ot, ovr2 = ds_ovr * ds_ovr, cl2 = d_close * d_close;
  // position increments: the obstacle's are constant, the own ship's use its sway at sample 1
  // only (linear_pred zeroes v after the first step)
  const double dox = (r11 * in.ob_u + r12 * in.ob_v) * DT, doy = (r21 * in.ob_u + r22 * in.ob_v) * DT;
  const double dsx = DT * (q11 * ud + q12 * 0.0), dsy = DT * (q21 * ud + q22 * 0.0);
  double ox = in.ob_x, oy = in.ob_y;
  double sx = in.os_x + DT * (q11 * ud + q12 * in.os_v), sy = in.os_y + DT * (q21 * ud + q22 * in.os_v);
  double t = DT;
  if constexpr (diag::kNoSbLoop) n_samp = 1;  // (ablation build only: no horizon samples after sample 0)
  HzBest hb{INFINITY, INFINITY, 0.0, 0.0, false};
  const HzConst hc{so, co, ovr2, ot2, ah2, cl2, ovr};
  auto sample = [&](double tt, double d0, double d1, double d2s, bool inr) __attribute__((always_inline)) {
    hz_sample(hb, hc, tt, d0, d1, d2s, inr);
  };
  // two samples per iteration (i, i + 1): their bodies are independent chains the one wave of the SIMD
  // can interleave; the positions are the same incremental sums as one per iteration, and the samples
  // enter the running best in order (ties keep the earlier sample).
  // Split (part 0 / 1): the window of samples that can be in range, [i_first, min(i_last, i_past + 2)], is cut at
  // its middle; part 1 first advances its positions to the cut by the loop's own sums (a uniform loop, the other
  // lanes predicated off), then both parts run the loop side by side on their own sample indices.
  int i_stop = n_samp, i = 1;
  if (part >= 0) {
    const int w0 = max(i_first, 1), w1 = max(w0, min(i_last, i_past + 2));
    const int i_split = min(w0 + (w1 - w0 + 1) / 2, n_samp);
    if (part == 0) i_stop = i_split;
    const int i_start = part == 1 ? i_split : 1;
    for (int c = 1; __any(c < i_start); ++c) {
      const bool adv = c < i_start, adv_s = adv & (c > 1);
      ox = adv ? ox + dox : ox;
      oy = adv ? oy + doy : oy;
      sx = adv_s ? sx + dsx : sx;
      sy = adv_s ? sy + dsy : sy;
      t = adv ? t + DT : t;
    }
    i = i_start;
  }
  bool done = false;  // past the minimum and beyond the best (see i_past)
  for (;; i += 2) {
    // (per lane: a split part has its own sample index; unsplit every lane has the same one)
    if (!__any((i + 1 < n_samp) & (i <= i_last) & !done & (i < i_stop))) break;  // every lane past its useful samples
    const double oxa = ox + dox, oya = oy + doy;
    const double sxa = (i > 1) ? sx + dsx : sx, sya = (i > 1) ? sy + dsy : sy;
    const double ta = t + DT;
    ox = oxa + dox;
    oy = oya + doy;
    sx = sxa + dsx;
    sy = sya + dsy;
    t = ta + DT;
    const double d0a = oxa - sxa, d1a = oya - sya, d0b = ox - sx, d1b = oy - sy;
    const double d2a = d0a * d0a + d1a * d1a, d2b = d0b * d0b + d1b * d1b;
    const bool ia = (d2a < lim2) & (i + 1 < n_samp) & (i < i_stop);
    const bool ib = (d2b < lim2) & (i + 1 < n_samp) & (i + 1 < i_stop);
    if (ia | ib) {
      sample(ta, d0a, d1a, d2a, ia);
      sample(t, d0b, d1b, d2b, ib);
    }
    done = done | ((i + 1 >= i_past) & (hb.s1 < INFINITY) & (t * d2b * d2b > hb.s1 * (1.0 + 2e-10)));
  }
  {
    const bool lo = (i < n_samp) & (i < i_stop);
    if (__any(lo & (i <= i_last) & !done)) {  // the last sample of an odd count
      ox = ox + dox;
      oy = oy + doy;
      if (i > 1) {
        sx = sx + dsx;
        sy = sy + dsy;
      }
      t += DT;
      const double d0 = ox - sx, d1 = oy - sy;
      const double d2s = d0 * d0 + d1 * d1;
      if ((d2s < lim2) & lo) sample(t, d0, d1, d2s, true);
    }
  }
  if (part >= 0) {  // the two parts' running bests in sample order: part 0's samples come first
    // the partner lane (lane ^ 32) by v_permlane32_swap: after the swap of a value with itself the lower half holds
    // the upper half's value in the second result, the upper half the lower half's in the first
    const bool upper = part == 1;
    auto other_u = [&](unsigned x) __attribute__((always_inline)) {
      const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
      return upper ? r[0] : r[1];
    };
    auto other_d = [&](double x) __attribute__((always_inline)) {
      const unsigned lo = other_u((unsigned)__double2loint(x)), hi = other_u((unsigned)__double2hiint(x));
      return __hiloint2double((int)hi, (int)lo);
    };
    HzBest o;
    o.s1 = other_d(hb.s1);
    o.s2 = other_d(hb.s2);
    o.t1 = other_d(hb.t1);
    o.q1 = other_d(hb.q1);
    o.unc = other_u((unsigned)hb.unc) != 0u;
    const HzBest A = part == 0 ? hb : o, Bp = part == 0 ? o : hb;
    const bool bwin = Bp.s1 < A.s1;  // (ties keep the earlier sample)
    hb.s1 = fmin(A.s1, Bp.s1);
    hb.s2 = fmin(fmin(A.s2, Bp.s2), fmax(A.s1, Bp.s1));  // the second smallest of both
    hb.t1 = bwin ? Bp.t1 : A.t1;
    hb.q1 = bwin ? Bp.q1 : A.q1;
    hb.unc = A.unc | Bp.unc;
  }
  const double s1 = hb.s1, s2 = hb.s2, t1 = hb.t1, q1 = hb.q1;
  if (hb.unc)
    return sbmpc_scenario_cost_direct(in, n_samp, DT, ud, sp, cp, sp0, cp0, so, co, vo0, vo1, no, max_d_safe, lim2,
                                      cos_ot, H2);
  SB_MARK(2);
  if (s1 < INFINITY) {
    if (s2 <= s1 * (1.0 + 1e-10))
      return sbmpc_scenario_cost_direct(in, n_samp, DT, ud, sp, cp, sp0, cp0, so, co, vo0, vo1, no, max_d_safe, lim2,
                                        cos_ot, H2);
    const double R = (1 / fabs(t1 - 0.0)) * pow4(d_safe / sqrt(q1));
    const double k_coll = 1e-6 * os_l * in.obs_l;
    const double w0 = vs0 - vo0, w1 = vs1 - vo1;
    const double nrm = sqrt(w0 * w0 + w1 * w1);
    const double H0 = (k_coll * (nrm * nrm)) * R + 0.0 * 0;
    if (H0 > H1) H1 = H0;
  }
  return H1 + H2;
}

// Argmin of (cost, index) over each half-wave (its 32 scenario lanes), every lane of the half ending with the
// result; ties -> the lower index. The order (cost, then index) is a total order on non-NaN costs, so any pairing
// gives the same result: inside each 16-lane row by DPP (quad xor 1, quad xor 2, row_ror 4, row_ror 8: every lane
// then holds its row's minimum), then one LDS permute across the half-wave's two rows. Every lane of the wave
// must be active (the cooperative passes are called wave-uniformly).
// SHFL: the cross-row step by an LDS permute instead (the multi-obstacle and C1 kernels: the swap's lane-mask select
// costs them SGPRs they do not have; the same result)
template <bool SHFL = false>
__device__ __forceinline__ void scenario_argmin(double& cost, int& idx, int lane) {
  auto take = [&](double oc, int oi) __attribute__((always_inline)) {
    if (oc < cost || (oc == cost && oi < idx)) { cost = oc; idx = oi; }
  };
  take(dpp_d<kDppQuadXor1>(cost), dpp_i<kDppQuadXor1>(idx));
  take(dpp_d<kDppQuadXor2>(cost), dpp_i<kDppQuadXor2>(idx));
  take(dpp_d<kDppRowRor4>(cost), dpp_i<kDppRowRor4>(idx));
  take(dpp_d<kDppRowRor8>(cost), dpp_i<kDppRowRor8>(idx));
  // the other row of the half-wave (lane ^ 16) by v_permlane16_swap: after the swap of a value with itself the even
  // rows hold their partner row's value in the second result, the odd rows in the first
  if constexpr (SHFL) {
    take(shfl_d(cost, lane ^ 16), __shfl(idx, lane ^ 16, 64));
    return;
  }
  const bool odd_row = (lane >> 4) & 1;
  const auto sl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(cost), (unsigned)__double2loint(cost), false, false);
  const auto sh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(cost), (unsigned)__double2hiint(cost), false, false);
  const auto si = __builtin_amdgcn_permlane16_swap((unsigned)idx, (unsigned)idx, false, false);
  const double oc = __hiloint2double((int)(odd_row ? sh[0] : sh[1]), (int)(odd_row ? sl[0] : sl[1]));
  take(oc, (int)(odd_row ? si[0] : si[1]));
}

// Must be called by every lane of the wave (wave-uniform control flow). `need` marks lanes that
// request an optimisation with inputs `in`; they receive (P_best, Chi_best). SHIP_UNIFORM: u_d, obs_l and
// obs_w are the same for every request and set in every lane's `in` (the AST kernels: the ships'
// configured desired speed and obstacle size), so they are not gathered from the requesting lane.
template <bool SHIP_UNIFORM = false, bool SHFL_ARGMIN = false>
__device__ void sbmpc_cooperative(bool need, const SbIn& in, int n_samp, double DT, double& p_best,
                                  double& chi_best) {
  SHIPSIM_LANE_CHECK(64, 4);
  const int lane = opaque_v(threadIdx.x) & 63;  // (opaque: no lane masks held across the caller's loop)
  const int half = lane >> 5;
  const int scen = lane & 31;
  uint64_t req = __ballot(need);
  while (req) {
    int src0 = __ffsll((unsigned long long)req) - 1;
    req &= req - 1;
    int src1 = -1;
    if (req) {
      src1 = __ffsll((unsigned long long)req) - 1;
      req &= req - 1;
    }
    int src = half ? src1 : src0;
    int srcc = src < 0 ? src0 : src;
    SbIn g;
    if constexpr (SHIP_UNIFORM) {
      g.u_d = in.u_d; g.obs_l = in.obs_l; g.obs_w = in.obs_w;
    } else {
      g.u_d = shfl_d(in.u_d, srcc); g.obs_l = shfl_d(in.obs_l, srcc); g.obs_w = shfl_d(in.obs_w, srcc);
    }
    g.chi_d = shfl_d(in.chi_d, srcc);
    g.os_x = shfl_d(in.os_x, srcc); g.os_y = shfl_d(in.os_y, srcc); g.os_v = shfl_d(in.os_v, srcc);
    g.ob_x = shfl_d(in.ob_x, srcc); g.ob_y = shfl_d(in.ob_y, srcc); g.ob_psi = shfl_d(in.ob_psi, srcc);
    g.ob_u = shfl_d(in.ob_u, srcc); g.ob_v = shfl_d(in.ob_v, srcc);
    g.p_last = shfl_d(in.p_last, srcc); g.chi_last = shfl_d(in.chi_last, srcc);
    g.ob_so = shfl_d(in.ob_so, srcc); g.ob_co = shfl_d(in.ob_co, srcc);
    double cost = INFINITY;
    int idx = 64;
    const bool split = src1 < 0;  // (uniform) one request this pass: both halves take it, each half of every horizon
    if ((split || src >= 0) && scen < 28) {
      cost = sbmpc_scenario_cost(g, n_samp, DT, scen >> 2, scen & 3, split ? half : -1);
      idx = scen;
    }
    // argmin over the half-wave; ties -> lowest scenario index (first strict improvement in the
    // reference's i-major / j-minor loop)
    scenario_argmin<SHFL_ARGMIN>(cost, idx, lane);
    const int best0 = __builtin_amdgcn_readlane(idx, 0);
    const int best1 = __builtin_amdgcn_readlane(idx, 32);
    if (lane == src0) {
      p_best = p_ca_of(best0 & 3);
      chi_best = (-30.0 + 10.0 * (best0 >> 2)) * (kPi / 180.0);
    }
    if (src1 >= 0 && lane == src1) {
      p_best = p_ca_of(best1 & 3);
      chi_best = (-30.0 + 10.0 * (best1 >> 2)) * (kPi / 180.0);
    }
  }
}

// SBMPC over a do_list of NOB obstacles (sbmpc.py:150-183; env.py:366-370 passes every obstacle ship):
// per scenario the worst obstacle's cost (cost_i = -1, then every strictly larger cost_k: the max of the costs),
// the scenario with the least worst cost wins (lowest index on ties). Slots of an env that duplicate its last
// ship repeat an obstacle, which changes neither the max nor the D_INIT test, and are not evaluated.
// Lanes: scenario = lane & 31 (28 used). With two or more requests pending a pass serves two, one per half-wave,
// each lane taking its scenario's obstacles in turn; with one request both halves serve it and split its
// obstacles — half h takes obstacles h, h + 2, … — and the two halves' worst costs are merged (lane ^ 32) before
// the argmin, so a lone request costs ⌈K / 2⌉ scenario evaluations per lane instead of K (the max over the same
// set of costs: the same value in either order).
template <int NOB>
struct SbMulti {
  double u_d, chi_d, os_x, os_y, os_v, p_last, chi_last;
  double ob_x[NOB], ob_y[NOB], ob_psi[NOB], ob_u[NOB], ob_v[NOB], obs_l[NOB], obs_w[NOB];
};

template <int NOB>
__device__ __forceinline__ void sbmpc_cooperative_multi(bool need, const SbMulti<NOB>& in, int n_obs, int n_samp, double DT,
                                        double& p_best, double& chi_best) {
  SHIPSIM_LANE_CHECK(64, 4);
  const int lane = opaque_v(threadIdx.x) & 63;
  const int half = lane >> 5;
  const int scen = lane & 31;
  uint64_t req = __ballot(need);
  diag::sb_stat_wave(0, req ? 1u : 0u);
  while (req) {
    // the counts re-derived per pass: tests on them are not hoisted out of this loop and held across it
    const int n_obs_p = opaque_s(n_obs), n_samp_p = opaque_s(n_samp);
    int src0 = __ffsll((unsigned long long)req) - 1;
    req &= req - 1;
    int src1 = -1;
    if (req) {
      src1 = __ffsll((unsigned long long)req) - 1;
      req &= req - 1;
    }
    const bool split = src1 < 0;  // (uniform) one request this pass: the halves split its obstacles
    diag::sb_stat_wave(1, 1u);
    diag::sb_stat_wave(2, split ? 1u : 0u);
    diag::sb_stat_wave(3, split ? 1u : 2u);
    int src = half ? src1 : src0;
    const int srcc = src < 0 ? src0 : src;
    SbIn g;
    g.u_d = shfl_d(in.u_d, srcc); g.chi_d = shfl_d(in.chi_d, srcc);
    g.os_x = shfl_d(in.os_x, srcc); g.os_y = shfl_d(in.os_y, srcc); g.os_v = shfl_d(in.os_v, srcc);
    g.p_last = shfl_d(in.p_last, srcc); g.chi_last = shfl_d(in.chi_last, srcc);
    double cost = INFINITY;
    int idx = 64;
    double worst = -1.0;
    bool any_far = false;
    const bool act = (split || src >= 0) && scen < 28;
    // obstacles in pairs (2j, 2j + 1): split, half h takes obstacle 2j + h; otherwise each lane both, in order
#pragma unroll
    for (int j = 0; j < (NOB + 1) / 2; ++j) {
      const int ka = 2 * j, kb = 2 * j + 1 < NOB ? 2 * j + 1 : 2 * j;
      if (ka >= n_obs_p) break;  // (wave-uniform) slots past the env's K obstacles duplicate the last one
      const bool b_ok = 2 * j + 1 < NOB && 2 * j + 1 < n_obs_p;
      for (int t = 0; t < (split ? 1 : 2); ++t) {  // (uniform trip count)
        const bool use_b = split ? half == 1 : t == 1;
        // this lane's obstacle, field by field (both candidates gathered, one kept: short live ranges)
        auto pick = [&](const double (&f)[NOB]) __attribute__((always_inline)) {
          const double a = shfl_d(f[ka], srcc);
          const double b = shfl_d(f[kb], srcc);
          return use_b ? b : a;
        };
        SbIn q = g;
        q.ob_x = pick(in.ob_x); q.ob_y = pick(in.ob_y); q.ob_psi = pick(in.ob_psi);
        q.ob_u = pick(in.ob_u); q.ob_v = pick(in.ob_v); q.obs_l = pick(in.obs_l); q.obs_w = pick(in.obs_w);
        const bool ok = act && (use_b ? b_ok : true);
        // an obstacle out of reach costs exactly sbmpc_h2 in every scenario (added once below)
        const bool far = ok && sbmpc_far(q, n_samp_p, DT);
        any_far = any_far || far;
        diag::sb_stat_lanes(4, (ok && !far) ? 1u : 0u);
        diag::sb_stat_lanes(5, far ? 1u : 0u);
        if (ok && !far) {
          sb_set_heading_trig(q);
          const double ck = sbmpc_scenario_cost(q, opaque_s(n_samp_p), DT, scen >> 2, scen & 3);
          if (ck > worst) worst = ck;
        }
      }
    }
    if (act && any_far) {
      const double h2 = sbmpc_h2(g, scen >> 2, scen & 3);
      if (h2 > worst) worst = h2;
    }
    if (split) {  // (uniform) the other half's worst over its obstacles (lane ^ 32)
      const double ow = shfl_d(worst, lane ^ 32);
      if (ow > worst) worst = ow;
    }
    if (act) {
      cost = worst;
      idx = scen;
    }
    scenario_argmin<true>(cost, idx, lane);
    const int best0 = __builtin_amdgcn_readlane(idx, 0);
    const int best1 = __builtin_amdgcn_readlane(idx, 32);
    if (lane == src0) {
      p_best = p_ca_of(best0 & 3);
      chi_best = (-30.0 + 10.0 * (best0 >> 2)) * (kPi / 180.0);
    }
    if (src1 >= 0 && lane == src1) {
      p_best = p_ca_of(best1 & 3);
      chi_best = (-30.0 + 10.0 * (best1 >> 2)) * (kPi / 180.0);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
// fresh state as constructed; for AST also env-level fields of MultiShipRLEnv.__init__
__global__ void init_kernel(const Params P, DevState S, ConstBuf K) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int nq = P.n_envs * P.n_ships;
  if (q >= nq) return;
  const int ship = q % P.n_ships;
  const int env = q / P.n_ships;
  const ShipConst& c = K.ships()[ship];
  Ship s;
  s.n = c.init_n; s.e = c.init_e; s.yaw = c.init_yaw; s.u = c.init_u; s.v = c.init_v; s.r = c.init_r;
  s.omega = c.init_omega; s.time = 0.0;
  s.e_ct = 0; s.e_ct_int = 0; s.hdg_ei = 0; s.hdg_prev = 0;
  s.spd_a = 0; s.spd_b = (P.machinery == SHIPSIM_MACH_DETAILED) ? c.init_shaft_ei : 0.0;
  s.log_rudder = 0; s.log_thrust = 0; s.log_ect = 0; s.log_n = s.n; s.log_e = s.e;
  s.next_wpt = 1; s.stop = 0; s.n_route = c.n_route;
  double* rn = S.route_n() + (size_t)q * kMaxRoute;
  double* re = S.route_e() + (size_t)q * kMaxRoute;
  for (int i = 0; i < kMaxRoute; ++i) {
    rn[i] = K.cfg_route_n()[ship * kMaxRoute + i];
    re[i] = K.cfg_route_e()[ship * kMaxRoute + i];
  }
  store_ship(S, q, s);
  if (ship == 0) {
    S.sampling_count()[env] = 0;
    S.travel_dist()[env] = 0; S.travel_time()[env] = 0; S.acc()[env] = 0;
    S.n_base()[env] = P.n_base0; S.e_base()[env] = P.e_base0;
    S.p_last()[env] = 1.0; S.chi_last()[env] = 0.0;  // SBMPCParams defaults (sbmpc.py:28-29)
    S.mach_dt()[env] = P.mach_dt_init;
    for (int i = 0; i < 4; ++i) S.states4()[env * 4 + i] = P.initial_states[i < 2 ? i : i + 1];
    for (int i = 0; i < 8; ++i) S.next_obs8()[env * 8 + i] = P.initial_states[i];
    S.snap_bits()[env] = 0;
    S.was_reset()[env] = 0;
    S.dec_flags()[env] = DF_AWAITING;
    for (int i = 0; i < 4; ++i) S.legacy_states()[env * 4 + i] = 0.0;
    S.legacy_flags()[env] = 1;
  }
}

// MultiShipRLEnv.reset (env.py:238-295): reset assets + IW sampler + snapshot, then init_step
template <bool DETAILED, bool REC>
__global__ __launch_bounds__(256) void reset_kernel(const Params P, DevState S, ConstBuf K, Traj T,
                                                   const uint8_t* mask, float* obs_out) {
  __shared__ ShipConst lds_sc[SHIPSIM_MAX_SHIPS];
  const ShipConst* SC = stage_consts(K, lds_sc, P.n_ships, P.dt);
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int nq = P.n_envs * P.n_ships;
  if (q >= nq) return;
  const int ship = q % P.n_ships;
  const int env = q / P.n_ships;
  if (mask && !mask[env]) return;
  const ShipConst& c = SC[ship];
  Ship s;
  s.n = c.init_n; s.e = c.init_e; s.yaw = c.init_yaw; s.u = c.init_u; s.v = c.init_v; s.r = c.init_r;
  s.omega = c.init_omega; s.time = 0.0;
  s.e_ct = 0; s.e_ct_int = 0; s.hdg_ei = 0; s.hdg_prev = 0;
  s.spd_a = 0; s.spd_b = DETAILED ? c.init_shaft_ei : 0.0;
  s.next_wpt = 1; s.stop = 0; s.n_route = c.n_route;
  double* rn = S.route_n() + (size_t)q * kMaxRoute;
  double* re = S.route_e() + (size_t)q * kMaxRoute;
  for (int i = 0; i < c.n_route; ++i) {
    rn[i] = K.cfg_route_n()[ship * kMaxRoute + i];
    re[i] = K.cfg_route_e()[ship * kMaxRoute + i];
  }
  load_segment(s, rn, re);
  const double mach_dt = P.mach_dt_reset;
  // init_step (env.py:307-339): one control + integrate tick, no collision avoidance
  double fuel[3] = {0.0, 0.0, 0.0};  // machinery reset restores the fuel accumulators (ship_engine.py:468-481)
  double sy, cy;
  sincos(s.yaw, &sy, &cy);
  control_and_integrate_sc<DETAILED, REC>(c, P, s, rn, re, 0.0, 1.0, mach_dt, 0, false,
                                          REC ? T.ship_row(q, 0) : nullptr, fuel, sy, cy);
  store_ship(S, q, s);
  if (REC) {
    for (int k = 0; k < 3; ++k) T.fuel[(size_t)q * 3 + k] = fuel[k];
    if (ship == 0) T.len[env] = 1;
  }
  if (ship == 0) {
    S.sampling_count()[env] = 0;
    S.travel_dist()[env] = 0; S.travel_time()[env] = 0; S.acc()[env] = 0;
    S.n_base()[env] = P.n_base0; S.e_base()[env] = P.e_base0;
    S.mach_dt()[env] = mach_dt;
    for (int i = 0; i < 8; ++i) S.next_obs8()[env * 8 + i] = P.initial_states[i];
    S.snap_bits()[env] = 0;
    S.was_reset()[env] = 1;
    S.dec_flags()[env] = DF_AWAITING;
    if (obs_out)
      for (int i = 0; i < 8; ++i) obs_out[env * 8 + i] = P.initial_states[i];
  }
}

// Map edge table with the per-edge constants of GEOS pointToSegment, staged in LDS.
struct EdgeX {
  double ax, ay, bx, by, dx, dy, len2, inv_len2;
};

// min over this lane's share of the edges (i = sub, sub + nsub, ...) of the squared point-segment
// distance. Equivalent to GEOS Distance::pointToSegment up to rounding (sqrt taken once at the end).
__device__ __forceinline__ double map_dist2_part(const EdgeX* __restrict__ E, int n_edges, double n, double e,
                                                 int sub, int nsub) {
  const double px = e, py = n;
  double best = INFINITY;
  for (int i = sub; i < n_edges; i += nsub) {
    const EdgeX ed = E[i];
    const double qx = px - ed.ax, qy = py - ed.ay;
    const double t = qx * ed.dx + qy * ed.dy;
    const double da = qx * qx + qy * qy;
    const double rx = px - ed.bx, ry = py - ed.by;
    const double db = rx * rx + ry * ry;
    const double c = (ed.ay - py) * ed.dx - (ed.ax - px) * ed.dy;
    const double dp = c * c * ed.inv_len2;
    const double d2 = (t <= 0.0) ? da : ((t >= ed.len2) ? db : dp);
    best = py_min(best, d2);
  }
  return best;
}

// this sub-lane's share of grid cell c's candidate edges: the set bits of rank = sub (mod nsub), read from the
// host-split masks (rank mod 8; nsub divides 8) — the min over the shares is over the same edges either way
__device__ __forceinline__ uint64_t grid_share(const ConstBuf& K, int c, int sub, int nsub) {
  uint64_t m = 0;
  for (int q = sub; q < 8; q += nsub) m |= K.grid_part[(size_t)c * 8 + q];
  return m;
}

// map_dist2_part over the edges of mask m (a grid cell's share): the same value as map_dist2_part over every edge
// when the true distance is <= kGroundReach (see above)
__device__ __forceinline__ double map_dist2_mask(const EdgeX* __restrict__ E, uint64_t m, double n, double e) {
  const double px = e, py = n;
  double best = INFINITY;
  while (m) {
    const int i = __builtin_ctzll(m);
    m &= m - 1;
    const EdgeX ed = E[i];
    const double qx = px - ed.ax, qy = py - ed.ay;
    const double t = qx * ed.dx + qy * ed.dy;
    const double da = qx * qx + qy * qy;
    const double rx = px - ed.bx, ry = py - ed.by;
    const double db = rx * rx + ry * ry;
    const double cc = (ed.ay - py) * ed.dx - (ed.ax - px) * ed.dy;
    const double dp = cc * cc * ed.inv_len2;
    const double d2 = (t <= 0.0) ? da : ((t >= ed.len2) ? db : dp);
    best = py_min(best, d2);
  }
  return best;
}

// if_pos_inside_obstacles with the grid's exact cell classification (full test on mixed cells)
__device__ __forceinline__ bool corner_inside(const ConstBuf& K, const Edge* __restrict__ edges,
                                              const PolyBox* __restrict__ boxes, int n_polys, double n, double e) {
  const int c = K.cell(n, e);
  if (c >= 0) {
    const int f = K.grid_flag[c];
    if (f != GRID_MIXED) return f == GRID_IN;
  }
  return map_inside(edges, boxes, n_polys, n, e);
}

__device__ __forceinline__ double xor_shfl_d(double x, int mask) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  lo = __shfl_xor(lo, mask, 64);
  hi = __shfl_xor(hi, mask, 64);
  return __hiloint2double(hi, lo);
}


// Open-loop decision stream (shipsim_run_table, the C3 workload of SURVEY.md §8(d)): actions come
// from a device table, a completed decision is followed at once by the next one and an ended
// episode is reset in place, so an env never idles inside a launch while it has ticks left.
struct ChainArgs {
  const float* table;  // [n_eps][n_dec][n_envs] scoping angles
  int32_t n_eps, n_dec;
  int32_t* ep_idx;     // [env] episode counter (table row = ep % n_eps)
  int32_t* dec_idx;    // [env] decision index within the episode
  int32_t* decisions;  // [env] decisions completed in this call (may be null)
  double* log;         // [env][log_cap][SHIPSIM_DECLOG_COLS] per-decision record (may be null)
  int32_t* log_len;    // [env] records written (counts on past log_cap)
  int32_t log_cap;
  int32_t log_stop;    // an env whose log is full stops for the launch, its next decision pending
  // work-conserving launch tail (shipsim_set_stream_tail): a wave whose envs met max_ticks keeps ticking in chunks
  // of kTailChunk while tail_ctr (waves that met it, zeroed per launch) < the grid, up to tail_extra more ticks
  int32_t* tail_ctr;
  int32_t tail_extra;
  int32_t tail_waves;  // waves of the launch (the grid: one wave per block)
  // shipsim_run_policy: actions from the policy instead of the table (policy != null)
  const float* policy;  // TanhGaussianPolicy parameters, torch order (shipsim_policy.params)
  const float* w2t;     // its fc1 weight transposed, [H][H] (shipsim_policy.w2t)
  int32_t pol_obs, pol_hidden, pol_det;
  uint64_t pol_seed;
  const int64_t* pol_counter;
};


// A copy of the state table whose base pointer the compiler cannot see through: addresses derived
// from it are recomputed where they are used (a few SALU) instead of being hoisted out of the tick
// loop and kept alive in SGPRs for the whole launch (the big kernels are at the SGPR limit).
__device__ __forceinline__ DevState opaque(const DevState& S) {
  DevState o = S;
  asm volatile("" : "+s"(o.base));
  return o;
}

// ---------------------------------------------------------------------------------------------
// The collector's policy inside the decision stream (shipsim_run_policy): TanhGaussianPolicy.forward
// + TanhNormal.sample (gaussian_policy.py:105-118, distributions.py:394-425) or MakeDeterministic's
// tanh(mean) (policies/base.py:54-64) on the observation of every env of the wave that needs its next
// action, evaluated by the whole wave (wave-uniform control flow): up to 8 envs per pass share every
// weight load; lane l computes hidden units l, l + 64, ... (fmaf chains from the bias in input order,
// h1 staged in LDS); the heads are reduced across the wave. fp32 as the policy.
// ---------------------------------------------------------------------------------------------
constexpr int kPolMaxRows = 8;
constexpr int kPolMaxHidden = 512;

__device__ inline void philox_env(uint32_t c[4], uint32_t k0, uint32_t k1) {  // Philox4x32-10
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

__device__ __forceinline__ float wave_sum_f(float x) {  // butterfly: every lane gets the same bits
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Must be called by every lane of the wave. want: this lane's env needs its next action (all lanes of an
// env agree); ns: its observation; seq: the env's decisions completed in this call (noise stream index).
// Returns the normalized action a in (-1, 1) for lanes whose env wanted one. The hidden units are taken in slices
// of 256 (one slice up to H = 256, two above): in slice c lane l owns the nj = min(4, (H - 256c) / 64) consecutive
// units [256c + l·nj, 256c + l·nj + nj), so one row of the transposed fc1 weight is one coalesced load per lane (a
// float4 in a full slice) and the h1 rows in LDS are read as broadcast float4s; the fc1 accumulators of one slice
// are live at a time (the register budget of H = 256 at every width), and each lane's head partials run on across
// the slices in unit order.
__device__ __forceinline__ float policy_actions(bool want, const float ns[8], int env, bool env_leader, int env_lane0,
                                                int seq, const ChainArgs& CH, float* lds_h1) {
  SHIPSIM_LANE_CHECK(64, 5);
  uint64_t req = __ballot(want && env_leader);
  float act = 0.0f;
  const int lane = threadIdx.x & 63;
  const int H = CH.pol_hidden, n_slices = (H + 255) / 256;
  const float* W1 = CH.policy;  // [H][8] (obs_dim 8: checked by the host)
  asm volatile("" : "+s"(W1));  // (the weight addresses below derived per call, not held across the tick loop)
  // the parameter blocks after W1 [H][8]: b1 [H], W2 [H][H], b2 [H], wm [H], bm, ws [H], bs — their addresses
  // derived where each is read, from a copy of W1 the compiler cannot hoist (no pointer pair live across the pass)
  auto blk = [&](int which) __attribute__((always_inline)) {
    const float* w = W1;
    asm volatile("" : "+s"(w));
    const size_t b1 = (size_t)H * 8, b2 = b1 + H + (size_t)H * H;
    return w + (which == 0 ? b1 : which == 1 ? b2 : which == 2 ? b2 + H : b2 + 2 * (size_t)H + 1);
  };
  constexpr int kJ = 4;  // units per lane per slice, at most
  while (req) {
    // the next (up to) kPolMaxRows requesting envs: the lowest set bits of req (no indexed arrays: row e's
    // source lane is recomputed from the mask, so nothing lands in scratch)
    const uint64_t rows = req;
    int E = 0;
    for (uint64_t m = req; m && E < kPolMaxRows; m &= m - 1) ++E;
    for (int e = 0; e < E; ++e) req &= req - 1;
    // fc0 + relu for every row, into LDS: unit u = b1[u] + sum_i W1[u][i] x[i], i ascending
    {
      uint64_t m = rows;
      for (int e = 0; e < E; ++e, m &= m - 1) {
        const int src = __ffsll((unsigned long long)m) - 1;
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __shfl(ns[i], src, 64);
#pragma nounroll
        for (int c = 0; c < n_slices; ++c) {
          const int nj = min(4, (H - 256 * c) >> 6), u0 = 256 * c + lane * nj;
#pragma unroll
          for (int j = 0; j < kJ; ++j) {
            if (j < nj) {
              const int u = u0 + j;
              float h = blk(0)[u];  // (the parameters are 4-byte aligned only: log α leads them)
#pragma unroll
              for (int i = 0; i < 8; ++i) h = fmaf(W1[(size_t)u * 8 + i], x[i], h);
              lds_h1[e * kPolMaxHidden + u] = fmaxf(h, 0.0f);
            }
          }
        }
      }
    }
    __syncthreads();  // (one wave per block)
    // per slice: fc1 + relu, acc[e][j] = b2[u] + sum_k W2[u][k] h1[e][k], k ascending (W2T row k is [H]
    // contiguous), folded into this lane's head partials pm / ps (fmaf chains over its units in order)
    float pm[kPolMaxRows], ps[kPolMaxRows];
#pragma unroll
    for (int e = 0; e < kPolMaxRows; ++e) pm[e] = ps[e] = 0.0f;
#pragma nounroll
    for (int c = 0; c < n_slices; ++c) {
      const int nj = min(4, (H - 256 * c) >> 6), u0 = 256 * c + lane * nj;
      float acc[kPolMaxRows][kJ];
      const float* b2 = blk(1);
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const float bj = j < nj ? b2[u0 + j] : 0.0f;
#pragma unroll
        for (int e = 0; e < kPolMaxRows; ++e) acc[e][j] = bj;
      }
      for (int k = 0; k < H; k += 4) {
        float w[4][kJ];
        if (nj == 4) {  // a full slice: one float4 per row
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const float4 v = *reinterpret_cast<const float4*>(CH.w2t + (size_t)(k + kk) * H + u0);
            w[kk][0] = v.x; w[kk][1] = v.y; w[kk][2] = v.z; w[kk][3] = v.w;
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int j = 0; j < kJ; ++j) w[kk][j] = j < nj ? CH.w2t[(size_t)(k + kk) * H + u0 + j] : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < kPolMaxRows; ++e) {
          if (e < E) {
            const float4 h4 = *reinterpret_cast<const float4*>(lds_h1 + e * kPolMaxHidden + k);
#pragma unroll
            for (int j = 0; j < kJ; ++j) {
              acc[e][j] = fmaf(w[0][j], h4.x, acc[e][j]);
              acc[e][j] = fmaf(w[1][j], h4.y, acc[e][j]);
              acc[e][j] = fmaf(w[2][j], h4.z, acc[e][j]);
              acc[e][j] = fmaf(w[3][j], h4.w, acc[e][j]);
            }
          }
        }
      }
      float wmj[kJ], wsj[kJ];
      const float *wm = blk(2), *ws = blk(3);
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        wmj[j] = j < nj ? wm[u0 + j] : 0.0f;
        wsj[j] = j < nj ? ws[u0 + j] : 0.0f;
      }
#pragma unroll
      for (int e = 0; e < kPolMaxRows; ++e) {
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
          const float y = fmaxf(acc[e][j], 0.0f);
          pm[e] = fmaf(wmj[j], y, pm[e]);
          ps[e] = fmaf(wsj[j], y, ps[e]);
        }
      }
    }
    // heads (mean, log_std) reduced across the wave, the sample, and the hand-over to the env's lanes
    const float bm = blk(2)[H], bs = blk(3)[H];
    const uint64_t ctr = CH.pol_counter ? (uint64_t)*CH.pol_counter : 0;
    uint64_t m = rows;
#pragma unroll
    for (int e = 0; e < kPolMaxRows; ++e) {
      if (e < E) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const float mean = wave_sum_f(pm[e]) + bm;
        const float log_std = fminf(fmaxf(wave_sum_f(ps[e]) + bs, -20.0f), 2.0f);
        float z = mean;
        if (!CH.pol_det) {
          const int e_env = __shfl(env, src, 64), e_seq = __shfl(seq, src, 64);
          uint32_t c[4] = {(uint32_t)e_env, (uint32_t)ctr, (uint32_t)(ctr >> 32), 0x5A100000u ^ (uint32_t)e_seq};
          philox_env(c, (uint32_t)CH.pol_seed, (uint32_t)(CH.pol_seed >> 32));
          const float u1 = ((float)c[0] + 1.0f) * 2.3283064365386963e-10f;
          const float u2 = (float)c[1] * 2.3283064365386963e-10f;
          z = mean + expf(log_std) * (sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2));
        }
        const float a = tanhf(z);
        if (env_lane0 == src) act = a;
      }
    }
    __syncthreads();  // lds_h1 free for the next pass
  }
  return act;
}

// NormalizedBoxEnv's float32 rule (normalized_box_env.py:48-51): lb + (a + 1) * 0.5 * (ub - lb), clipped
__device__ __forceinline__ float denormalize_f32(float a, float lb, float ub) {
  const float x = lb + ((a + 1.0f) * 0.5f) * (ub - lb);
  return fminf(fmaxf(x, lb), ub);
}

// lanes of the env: value of lane k of the env (LPE 16: the env is one DPP row)
template <int LPE, int K>
__device__ __forceinline__ double env_lane_d(double x, int env_lane0) {
  SHIPSIM_LANE_CHECK(LPE, 1);
  if constexpr (LPE == 16) return dpp_d<kDppRowBcast + K>(x);
  else return shfl_d(x, env_lane0 + K);
}
template <int LPE, int K>
__device__ __forceinline__ int env_lane_i(int x, int env_lane0) {
  SHIPSIM_LANE_CHECK(LPE, 2);
  if constexpr (LPE == 16) return dpp_i<kDppRowBcast + K>(x);
  else return __shfl(x, env_lane0 + K, 64);
}

// The env lane that evaluates each reward term's exp (LPE >= 8), and the term of env lane j < 5. Two-ship envs
// (lanes alternate test / obstacle ship, each computing from its own perspective): the obstacle ship's lanes 1 and 3
// take the terms of its own ground distance and cross-track error.
struct RewardTerm {
  double t, o, y, pad;  // target, scale, div_rcp(scale)
};
template <int SLOTS>
__host__ __device__ constexpr int reward_lane(int k) {
  return SLOTS != 2 ? k : k == 0 ? 0 : k == 1 ? 2 : k == 2 ? 4 : k == 3 ? 1 : 3;
}
template <int SLOTS>
__host__ __device__ constexpr int reward_term(int j) {
  return SLOTS != 2 ? j : j == 0 ? 0 : j == 1 ? 3 : j == 2 ? 1 : j == 3 ? 4 : 2;
}
// min of a double / OR of an int over the sub-lanes of one ship (same lane parity) of a 16-lane env:
// quad_perm [2,3,0,1], row_ror 4, row_ror 8 (parity-preserving) — DPP only, no LDS permute
template <int LPE, int SLOTS = 2>
__device__ __forceinline__ void ship_reduce(double& d2, int& gri) {
  SHIPSIM_LANE_CHECK(LPE, 3);
  if constexpr (LPE == 16) {  // sub-lanes of a ship are the lanes of equal index mod SLOTS
    if constexpr (SLOTS == 2) {
      d2 = py_min(d2, dpp_d<kDppQuadXor2>(d2));
      gri |= dpp_i<kDppQuadXor2>(gri);
    }
    if constexpr (SLOTS <= 4) {
      d2 = py_min(d2, dpp_d<kDppRowRor4>(d2));
      gri |= dpp_i<kDppRowRor4>(gri);
    }
    d2 = py_min(d2, dpp_d<kDppRowRor8>(d2));
    gri |= dpp_i<kDppRowRor8>(gri);
  } else {
#pragma unroll
    for (int m = SLOTS; m < LPE; m <<= 1) {
      d2 = py_min(d2, xor_shfl_d(d2, m));
      gri |= __shfl_xor(gri, m, 64);
    }
  }
}

// the OR of an int over the same sub-lanes (ship_reduce without the double)
template <int LPE, int SLOTS = 2>
__device__ __forceinline__ void ship_or(int& gri) {
  SHIPSIM_LANE_CHECK(LPE, 3);
  if constexpr (LPE == 16) {
    if constexpr (SLOTS == 2) gri |= dpp_i<kDppQuadXor2>(gri);
    if constexpr (SLOTS <= 4) gri |= dpp_i<kDppRowRor4>(gri);
    gri |= dpp_i<kDppRowRor8>(gri);
  } else {
#pragma unroll
    for (int m = SLOTS; m < LPE; m <<= 1) gri |= __shfl_xor(gri, m, 64);
  }
}

// |beta| > 165° of get_distance_and_encounter_type (compute_distance.py:16-40): beta =
// wrap(atan2(dy, dx) - heading) and cos(beta) = (dx cos h + dy sin h) / dist, so the overtaking
// sector is c < cos(165°)·dist with c = dx·cos h + dy·sin h (sin/cos(h) carried from the test ship's
// integration step). Within 1e-9·dist of the boundary (and at dist = 0) the reference expression
// itself decides, so the boolean equals the reference's.
__device__ __forceinline__ bool overtaking_sector(double dx, double dy, double dist, double sh, double ch, double h) {
  constexpr double kCos165 = -0.96592582628906831;  // cos(165°)
  const double c = dx * ch + dy * sh;
  const double m = c - kCos165 * dist;
  if (fabs(m) > 1e-9 * dist) return m < 0;
  const double beta = floor_mod((atan2(dy, dx) - h) + kPi, 2 * kPi) - kPi;
  return fabs(beta) > 165.0 * (kPi / 180.0);
}

// Everything ast_step_kernel is launched with, as its one by-value kernel argument. The kernel reads
// it through step_args(): the kernarg segment pointer laundered through an empty asm, so every read is
// a scalar load (constant cache) issued where the value is used. Read as ordinary kernel parameters
// these ~120 loop-invariant dwords were loaded at the entry and held in SGPRs for the whole launch,
// which put the kernel past the SGPR limit and spilled them to VGPR lanes.
struct StepArgs {
  Params P;
  DevState S;
  ConstBuf K;
  Traj T;
  const float* action;
  const uint8_t* active_mask;
  float* obs_out;
  double* reward_out;
  uint8_t* done_out;
  uint32_t* events_out;
  int32_t* ticks_out;
  uint8_t* ready_out;
  ChainArgs CH;
  int32_t max_ticks;
};
typedef const __attribute__((address_space(4))) StepArgs* StepArgsPtr;
__device__ __forceinline__ const StepArgs& step_args() {
  StepArgsPtr q = (StepArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();  // the kernel's first argument
  asm volatile("" : "+s"(q));
  return *(const StepArgs*)q;
}

// env flag bits exchanged between the two ships of an env every tick
#define XF_GROUND 1
#define XF_END 2
#define XF_OUTSIDE 4
#define XF_ROA 8
#define XF_NONFINITE 16

// MultiShipRLEnv.step (env.py:624-773), sliced: every env of the launch ticks (_step :563-622)
// until its decision point (RoA + one tick, or done) or until `max_ticks` ticks have run in this
// call; an env that paused resumes in the next call without consuming an action. Envs waiting
// for a decision consume action[env] first (IW sampling). LPE lanes per env: lane & 1 selects the
// ship, the LPE/2 sub-lanes of a ship hold identical state, run the control chain redundantly and
// split the map queries (edges for the coastline distance, hull corners for grounding).
// CHAIN (shipsim_run_table): decisions from the device table, chained and episodes reset in place.
// An env whose state goes non-finite completes its decision at once, done, with
// SHIPSIM_EV_NONFINITE | SHIPSIM_EV_TERMINAL, and is counted in S.nonfinite (shipsim_synchronize).
// SLOTS (2, 4, 8): ship slots per env. 2 is the reference's two-ship env (lane & 1 = ship); with
// K > 1 obstacle ships (shipsim_create) ship k sits on the lanes of index k mod SLOTS, and slots past
// the env's last ship repeat that ship (ghost lanes: same state and arithmetic, never stored).
template <bool DETAILED, int COLLAV, int LPE, bool REC, int CHAIN = 0, int SLOTS = 2>
__global__ __launch_bounds__(64) void ast_step_kernel(const StepArgs A_arg) {
  constexpr bool POLICY = CHAIN == 2;  // CHAIN: 0 shipsim_step, 1 shipsim_run_table, 2 shipsim_run_policy
  (void)A_arg;  // read through step_args() only (see StepArgs)
  const StepArgs& A0 = step_args();
  const Params& P = A0.P;
  const DevState& S = A0.S;
  const ConstBuf& K = A0.K;
  const Traj& T = A0.T;
  const int max_ticks = A0.max_ticks;
  static_assert(!(REC && CHAIN), "trajectory recording runs the per-decision step only");
  static_assert(SLOTS == 2 || (LPE == 16 && !REC && COLLAV != SHIPSIM_COLLAV_SIMPLE), "multi-obstacle layout");
  constexpr int NSUB = LPE / SLOTS;
  static_assert(NSUB >= 1 && 8 % NSUB == 0, "sub-lanes per ship must divide 8 (grid_part shares)");
  static_assert(LPE >= 2 && (LPE & (LPE - 1)) == 0 && LPE <= 16, "LPE must be a power of two in [2, 16]");
  constexpr bool SIMPLE = COLLAV == SHIPSIM_COLLAV_SIMPLE;
  constexpr bool OPQ = LPE != 16 || POLICY || SLOTS > 2;  // see opaque_if (measured: LPE-16 two-slot table kernels hold no spills without)
  __shared__ ShipConst lds_sc[SHIPSIM_MAX_SHIPS];
  __shared__ EdgeX lds_edges[SHIPSIM_MAX_VERTS];
  __shared__ Edge lds_edges_raw[SHIPSIM_MAX_VERTS];
  __shared__ PolyBox lds_boxes[SHIPSIM_MAX_POLYS];
  __shared__ float lds_pol[POLICY ? kPolMaxRows * kPolMaxHidden : 1];  // shipsim_run_policy: h1 rows
  __shared__ RewardTerm lds_rterm[8];  // the reward exp each lane of an env evaluates: its term's constants
  if constexpr (diag::kPoisonLds) {  // (stale-LDS diagnostics build only)
    diag::poison_lds(lds_sc, sizeof(lds_sc)); diag::poison_lds(lds_edges, sizeof(lds_edges));
    diag::poison_lds(lds_edges_raw, sizeof(lds_edges_raw)); diag::poison_lds(lds_boxes, sizeof(lds_boxes));
    __syncthreads();
  }
  const ShipConst* SC = stage_consts(K, lds_sc, P.n_ships, P.dt);
  for (int i = threadIdx.x; i < K.n_edges; i += blockDim.x) {
    const Edge ed = K.edges()[i];
    EdgeX x;
    x.ax = ed.ax; x.ay = ed.ay; x.bx = ed.bx; x.by = ed.by;
    x.dx = ed.bx - ed.ax; x.dy = ed.by - ed.ay;
    x.len2 = x.dx * x.dx + x.dy * x.dy;
    x.inv_len2 = x.len2 > 0 ? 1.0 / x.len2 : 0.0;
    lds_edges[i] = x;
    lds_edges_raw[i] = ed;
  }
  for (int i = threadIdx.x; i < P.n_polys; i += blockDim.x) lds_boxes[i] = K.boxes()[i];
  if (threadIdx.x < 8) {  // reward_designs.py:33-55 targets / scales, term reward_term(j) for env lane j
    const int j = threadIdx.x, t = j < 5 ? reward_term<SLOTS>(j) : 0;
    const double tg[5] = {0.0, 0.0, 3000.0, 0.0, 500.0};
    const double of[5] = {200000000.0, 175000.0, 1250000.0, 50000.0, 12500.0};
    const double o = j < 5 ? of[t] : 1.0;
    lds_rterm[j] = RewardTerm{j < 5 ? tg[t] : 0.0, o, div_rcp(o), 0.0};
  }
  __syncthreads();

  // one wave per block: envs [blockIdx.x * epw, + epw) on lanes [0, epw * LPE); lanes past them idle
  const int epw = P.epw > 0 && P.epw <= 64 / LPE ? P.epw : 64 / LPE;  // (as step_blocks)
  const int eslot = (int)(threadIdx.x & 63) / LPE;
  const int env = (int)blockIdx.x * epw + eslot;
  const int lie = (int)(threadIdx.x & 63) % LPE;
  const int ship = lie % SLOTS;
  const int sub = lie / SLOTS;
  const bool is_test = ship == 0;
  const int nsh = (SLOTS == 2) ? 2 : P.n_ships;
  const bool ghost = (SLOTS > 2) && ship >= nsh;
  const int shipc = ghost ? nsh - 1 : ship;  // the ship this lane simulates
  const bool is_obs1 = shipc == 1;            // "the" obstacle ship (sampling, decisions, observation)
  const int lane = threadIdx.x & 63;
  const int env_lane0 = lane - lie;
  const bool valid = eslot < epw && env < P.n_envs;
  const int envc = valid ? env : 0;
  const int qc = envc * nsh + shipc;
  const ShipConst& c = SC[shipc];
  double* rn = S.route_n() + (size_t)qc * kMaxRoute;
  double* re = S.route_e() + (size_t)qc * kMaxRoute;

  // (an int laundered where it is set, as have_iw: a bool here stayed a lane mask across the tick loop)
  int running = opaque_if<OPQ>((valid && (A0.active_mask == nullptr || A0.active_mask[envc]) && S.was_reset()[envc]) ? 1 : 0);
  // (ints in VGPRs read by the epilogue: not lane masks held in SGPRs for the whole launch)
  const int touched = opaque_v(running && valid ? 1 : 0);

  Ship s;
  load_ship(S, qc, s);
  double sy, cy;  // sin/cos(s.yaw), refreshed by every integration step
  sincos(s.yaw, &sy, &cy);
  int sampling_count = S.sampling_count()[envc];
  double travel_dist = S.travel_dist()[envc], travel_time = S.travel_time()[envc], acc = S.acc()[envc];
  double n_base = S.n_base()[envc], e_base = S.e_base()[envc];
  double p_last = S.p_last()[envc], chi_last = S.chi_last()[envc];
  double mach_dt = S.mach_dt()[envc];
  float st4[4] = {0.f, 0.f, 0.f, 0.f};  // self.states (read by the simple collision check only)
  if (SIMPLE)
    for (int i = 0; i < 4; ++i) st4[i] = S.states4()[envc * 4 + i];
  uint32_t snap_bits = S.snap_bits()[envc];
  int dflags = S.dec_flags()[envc];
  // (an int laundered where it is set and read: a bool here was kept as a lane mask across the tick loop and
  // spilled in the LPE-8 policy kernels)
  int have_iw = opaque_if<OPQ>((dflags & DF_HAVE_IW) ? 1 : 0);
  int phase = (dflags >> DF_PHASE_SHIFT) & 3;
  int dec_ticks = S.dec_ticks()[envc];  // ticks of the decision in progress (across calls)

  float ns[8];
  for (int i = 0; i < 8; ++i) ns[i] = S.next_obs8()[envc * 8 + i];
  int rec_t = 0;
  double fuel[3] = {0.0, 0.0, 0.0};
  if (REC) {
    rec_t = T.len[envc];
    for (int k = 0; k < 3; ++k) fuel[k] = T.fuel[(size_t)qc * 3 + k];
  }
  double out_r = 0.0;
  bool out_done = false, stalled = false;
  int ready = 0;  // (an int: OPQ kernels keep it in a VGPR, not a lane mask merged across the tick loop)
  uint32_t out_bits = 0;
  int out_ticks = 0;
  int ticks = 0;
  int budget = opaque_v(max_ticks);  // this launch's tick quota per env (CHAIN: extended in the launch tail; a VGPR)
  int tail_arrived = 0;  // this wave counted itself on the tail counter (an int: no lane mask held)
  int n_nonfinite = 0;

  SHIPSIM_DEBUG_PRINT(valid ? env : -1, "[dbg] env %d lie %d start: running %d dflags %d sc %d n_base %f phase %d\n", env,
                      lie, (int)running, dflags, sampling_count, n_base, phase);
  // ---- intermediate waypoint sampling (env.py:659-696) for an env that waits for a decision ----
  // CHAIN: episode / decision counters, decisions completed and records written in this call
  int ep_i = 0, dec_i = 0, n_decided = 0, log_n = 0;
  bool started_here = false;  // POLICY: the decision in progress started in this launch (its record row holds
                              // its action and observation-of-choice already)
  auto decision_prologue = [&](float sa, float a_log) __attribute__((always_inline)) {
    const StepArgs& A = step_args();
    const Params& P = A.P;
    const ConstBuf& K = A.K;
    if (POLICY && lie == 0) {  // what the decision record will report: the action and the observation it saw,
                               // into the record row it will complete in (stores only) and, for a decision
                               // that completes in a later launch, the state
      const DevState So = opaque(A.S);
      So.dec_action()[envc] = a_log;
      for (int i = 0; i < 8; ++i) So.dec_obs0()[envc * 8 + i] = ns[i];
      const ChainArgs& CH = A.CH;
      if (CH.log && log_n < CH.log_cap) {
        double* rec = CH.log + ((size_t)env * CH.log_cap + log_n) * SHIPSIM_DECLOG_COLS;
        rec[SHIPSIM_DL_ACTION] = (double)a_log;
        for (int i = 0; i < 8; ++i) rec[SHIPSIM_DL_OBS0 + i] = (double)ns[i];
      }
    }
    started_here = true;
    if (P.normalize_action) sa = (sa + 1.0f) / 2.0f * (P.action_high - P.action_low) + P.action_low;
    phase = 0;
    have_iw = opaque_if<OPQ>(0);
    dec_ticks = 0;
    if (sampling_count < P.max_sampling) {
      sampling_count += 1;
      float tn = (float)tan((double)sa);  // np.tan on the float32 scoping angle
      double l_s = fabs(P.AB_seg * (double)tn);
      double e_s = l_s * P.iw_cos;
      double n_s = l_s * P.iw_sin;
      if (sa > 0) e_s *= -1;
      else n_s *= -1;
      double iw_n = n_base + n_s, iw_e = e_base + e_s;
      n_base = iw_n + P.AB_seg_n;
      e_base = iw_e + P.AB_seg_e;
      if (opaque_if<OPQ>(shipc) == 1) {  // auto_pilot.update_route: list.insert(-1, IW); every sub-lane writes the same bytes
        int L = s.n_route;
        rn[L] = s.end_n; re[L] = s.end_e;
        rn[L - 1] = iw_n; re[L - 1] = iw_e;
        if (s.next_wpt == L - 1) {
          s.wp_n = iw_n;
          s.wp_e = iw_e;
          segment_changed(s);
        }
        s.n_route = L + 1;
      }
      travel_dist = 0;
      travel_time = 0;
      have_iw = opaque_if<OPQ>(1);
      bool fail = corner_inside(K, lds_edges_raw, lds_boxes, P.n_polys, iw_n, iw_e) ||
                  ((iw_n < P.min_north || iw_n > P.max_north) || (iw_e < P.min_east || iw_e > P.max_east));
      if (fail) {  // env.py:673-693 with obs_ship_IW_sampling_failure_reward (multiplier 2)
        out_r = (acc >= 0) ? -acc * 2.0 : acc * 2.0;
        snap_bits = (snap_bits | SHIPSIM_EV_SAMPLING_FAILURE | SHIPSIM_EV_TERMINAL) &
                    ~(uint32_t)(SHIPSIM_EV_TEST_STOP | SHIPSIM_EV_OBS_STOP);
        out_bits = snap_bits;
        out_done = true;
        out_ticks = 0;
        ready = opaque_if<OPQ>(1);
      } else {
        acc = 0;
      }
    }
  };

  // ---- CHAIN: in-place reset (env.py:238-342, as reset_kernel) and the next decision ----
  if (CHAIN) {
    const ChainArgs& CH = A0.CH;
    ep_i = CH.ep_idx[envc];
    dec_i = CH.dec_idx[envc];
    log_n = CH.log_len ? CH.log_len[envc] : 0;
    if (running && CH.log_stop && log_n >= CH.log_cap) {  // log already full: sit this launch out
      running = opaque_if<OPQ>(0);
      stalled = (dflags & DF_AWAITING) != 0;
    }
  }
  auto table_action = [&]() __attribute__((always_inline)) -> float {
    const StepArgs& A = step_args();
    const Params& P = A.P;
    const ChainArgs& CH = A.CH;
    SHIPSIM_INDEX_CHECK(ep_i >= 0 && dec_i >= 0 && dec_i < CH.n_dec && envc < P.n_envs, 10);
    return CH.table[((size_t)(ep_i % CH.n_eps) * CH.n_dec + dec_i) * P.n_envs + envc];
  };
  auto reset_env = [&]() __attribute__((always_inline)) {
    const StepArgs& A = step_args();
    const Params& P = A.P;
    const ConstBuf& K = A.K;
    const ShipConst& c = lds_sc[opaque_v(shipc)];
    SHIPSIM_INDEX_CHECK(c.n_route >= 2 && c.n_route <= kMaxRoute, 11);
    s.n = c.init_n; s.e = c.init_e; s.yaw = c.init_yaw; s.u = c.init_u; s.v = c.init_v; s.r = c.init_r;
    s.omega = c.init_omega; s.time = 0.0;
    s.e_ct = 0; s.e_ct_int = 0; s.hdg_ei = 0; s.hdg_prev = 0;
    s.spd_a = 0; s.spd_b = DETAILED ? c.init_shaft_ei : 0.0;
    s.next_wpt = 1; s.stop = 0; s.n_route = c.n_route;
    for (int i = 0; i < c.n_route; ++i) {
      rn[i] = K.cfg_route_n()[shipc * kMaxRoute + i];
      re[i] = K.cfg_route_e()[shipc * kMaxRoute + i];
    }
    load_segment(s, rn, re);
    mach_dt = P.mach_dt_reset;
    sincos(s.yaw, &sy, &cy);
    control_and_integrate_sc<DETAILED, false>(c, P, s, rn, re, 0.0, 1.0, mach_dt, 0, false, nullptr, nullptr, sy,
                                              cy);  // init_step
    sampling_count = 0;
    travel_dist = 0; travel_time = 0; acc = 0;
    n_base = P.n_base0; e_base = P.e_base0;
    for (int i = 0; i < 8; ++i) ns[i] = P.initial_states[i];
    snap_bits = 0;
    phase = 0;
    have_iw = opaque_if<OPQ>(0);
  };
  // A decision just completed (ready): record it, reset if the episode ended (done, or n_dec decisions
  // = the rollout's max_path_length), consume the next table action. A sampling failure completes the
  // new decision at once (no tick), hence the loop; after kChainBurst such back-to-back decisions (a
  // table whose actions all fail their sampling) the env stops for this launch with the last decision
  // recorded and the next one pending (DF_AWAITING): the wave keeps ticking its other envs and the
  // next launch resumes exactly there, so results do not depend on the burst bound.
  constexpr int kChainBurst = 8;
  constexpr int kTailChunk = 32;  // launch tail: ticks per extension
  // the next action of every env of the wave that needs one (want): the table entry, or the policy's
  // sample (wave-cooperative, shipsim_run_policy). Wave-uniform. sa: the scoping angle to run, a_log:
  // the action as the decision record reports it (the table's angle / the policy's normalized action).
  auto chain_action = [&](bool want, float& a_log) __attribute__((always_inline)) -> float {
    if constexpr (!POLICY) {
      a_log = want ? table_action() : 0.0f;
      return a_log;
    } else {
      const StepArgs& A = step_args();
      a_log = policy_actions(want, ns, envc, lie == 0, env_lane0, n_decided, A.CH, lds_pol);
      const Params& P = A.P;
      const float lb = P.normalize_action ? -1.0f : P.action_low, ub = P.normalize_action ? 1.0f : P.action_high;
      return denormalize_f32(a_log, lb, ub);  // NormalizedBoxEnv in front of the env
    }
  };
  // Decisions of the wave just completed (ready): record them, reset envs whose episode ended (done, or
  // n_dec decisions = the rollout's max_path_length), start each env's next decision. A sampling failure
  // completes the new decision at once (no tick), hence the loop; after kChainBurst such back-to-back
  // decisions (actions that all fail their sampling) the env stops for this launch with the last decision
  // recorded and the next one pending (DF_AWAITING): the wave keeps ticking its other envs and the next
  // launch resumes exactly there, so results do not depend on the burst bound. With the policy the loop is
  // wave-uniform (the policy is evaluated by the whole wave); with the table each env loops on its own.
  auto chain_next = [&]() __attribute__((always_inline)) {
    for (int burst = 0; POLICY ? __any(ready && running) : (ready && running); ++burst) {
      bool want = false;
      if (ready && running) {
        const ChainArgs& CH = step_args().CH;
        if (CH.log && opaque_if<OPQ>(lie) == 0 && log_n < CH.log_cap) {
          double* rec = CH.log + ((size_t)env * CH.log_cap + log_n) * SHIPSIM_DECLOG_COLS;
          rec[SHIPSIM_DL_REWARD] = out_r; rec[SHIPSIM_DL_EVENTS] = (double)out_bits;
          rec[SHIPSIM_DL_DONE] = out_done ? 1.0 : 0.0; rec[SHIPSIM_DL_EPISODE] = (double)ep_i;
          rec[SHIPSIM_DL_DECISION] = (double)dec_i; rec[SHIPSIM_DL_TICKS] = (double)out_ticks;
          for (int i = 0; i < 8; ++i) rec[SHIPSIM_DL_OBS + i] = (double)ns[i];
          if (POLICY && !started_here) {  // started in an earlier launch: from the state
            const DevState So = opaque(step_args().S);
            rec[SHIPSIM_DL_ACTION] = (double)So.dec_action()[envc];
            for (int i = 0; i < 8; ++i) rec[SHIPSIM_DL_OBS0 + i] = (double)So.dec_obs0()[envc * 8 + i];
          }
        }
        log_n += 1;
        n_decided += 1;
        started_here = false;
        if (out_done || dec_i + 1 >= CH.n_dec) {
          reset_env();
          ep_i += 1;
          dec_i = 0;
        } else {
          dec_i += 1;
        }
        if (opaque_if<OPQ>(lie) == 0) {
          const DevState So = opaque(step_args().S);
          for (int i = 0; i < 8; ++i) So.next_obs8()[envc * 8 + i] = ns[i];  // self.next_observations
        }
        ready = opaque_if<OPQ>(0);
        out_done = false;
        if (burst + 1 >= kChainBurst || (CH.log_stop && log_n >= CH.log_cap)) {
          stalled = true;  // next decision pending: resumed by the next launch
          running = opaque_if<OPQ>(0);
        } else {
          want = true;
        }
      }
      float a_log;
      const float sa = chain_action(want, a_log);
      if (want) decision_prologue(sa, a_log);
    }
  };

  {
    const bool want = running && (dflags & DF_AWAITING);
    if (CHAIN) {
      float a_log;
      const float sa = chain_action(want, a_log);
      if (want) decision_prologue(sa, a_log);
    } else if (want) {
      decision_prologue(A0.action[envc], A0.action[envc]);
    }
  }

  // The grid cell of the ship's position at its last map query, this sub-lane's share of the cell's candidate
  // edges and the cell's class: a ship moves a few metres per tick through 200 m cells, so the two dependent
  // global loads of a query are only issued when the cell changes (-2: none yet)
  int g_cell = -2, g_flag = GRID_MIXED;
  uint64_t g_mask = 0;
  // (an int: OPQ kernels hold it in a VGPR, not as a lane mask live across the whole tick loop)
  int going = opaque_if<OPQ>((running && !ready && (budget <= 0 || ticks < budget)) ? 1 : 0);
  PT_DECL;
  // CHAIN: the tick loop hands over to the (rare) chaining code below whenever a decision of the
  // wave completes, so the loop body itself is the per-decision kernel's.
  for (;;) {
  while (__any(opaque_if<OPQ>(going)) && !(CHAIN && __any(opaque_if<OPQ>(ready) && opaque_if<OPQ>(running)))) {
    // this tick's constants: re-read (scalar loads, LDS) rather than kept in registers across ticks
    const StepArgs& A = step_args();
    const Params& P = A.P;
    const ConstBuf& K = A.K;
    const Traj& T = A.T;
    // the lane's roles re-derived per tick where OPQ (shadowing the entry's): the run-time ship count and the
    // slot tests of the K > 1 kernels otherwise stay lane masks and scalars held across the loop, and spill
    const int lie_t = opaque_if<OPQ>(lie);
    const int ship = lie_t % SLOTS;
    const int sub = lie_t / SLOTS;
    const bool is_test = ship == 0;
    const int nsh = (SLOTS == 2) ? 2 : P.n_ships;
    const bool ghost = (SLOTS > 2) && ship >= nsh;
    const int shipc = ghost ? nsh - 1 : ship;
    const bool is_obs1 = shipc == 1;
    (void)ghost;
    // partner ship's pre-tick state (the test ship's SBMPC reads the obstacle ship before it moves)
    SHIPSIM_LANE_CHECK(LPE, 7);
    const double pn = pair_swap(s.n), pe = pair_swap(s.e);
    double sf = 1.0, off = 0.0;
    constexpr bool LOS_PRE = COLLAV == SHIPSIM_COLLAV_SBMPC && SLOTS == 2;  // the LOS term evaluated once per tick
    double los_pre_q = 0.0, los_pre_e = 0.0;
    bool sb_active = false;
    if (COLLAV == SHIPSIM_COLLAV_SBMPC && SLOTS > 2) {  // do_list of every obstacle ship (env.py:366-370)
      constexpr int NOB = SLOTS - 1 < SHIPSIM_MAX_OBS ? SLOTS - 1 : SHIPSIM_MAX_OBS;  // (slots past K duplicate a ship)
      SbMulti<NOB> in;
      double obn[NOB], obe[NOB];
#pragma unroll
      for (int k = 0; k < NOB; ++k) {
        double x = 0, y = 0, psi = 0, u = 0, v = 0;
        switch (k + 1) {  // slot k + 1's first lane of the env row (row broadcast)
#define SB_GATHER(M)                              \
  case M:                                         \
    if constexpr (M < SLOTS) {                    \
      x = env_lane_d<LPE, M>(s.e, env_lane0);     \
      y = env_lane_d<LPE, M>(s.n, env_lane0);     \
      psi = env_lane_d<LPE, M>(s.yaw, env_lane0); \
      u = env_lane_d<LPE, M>(s.u, env_lane0);     \
      v = env_lane_d<LPE, M>(s.v, env_lane0);     \
    }                                             \
    break;
          SB_GATHER(1) SB_GATHER(2) SB_GATHER(3) SB_GATHER(4) SB_GATHER(5) SB_GATHER(6) SB_GATHER(7)
#undef SB_GATHER
          default: break;
        }
        const ShipConst& ck = SC[(k + 1 < nsh) ? k + 1 : nsh - 1];
        in.ob_x[k] = x; in.ob_y[k] = y; in.ob_psi[k] = -psi; in.ob_u[k] = u; in.ob_v[k] = v;
        in.obs_l[k] = ck.obs_l_cfg; in.obs_w[k] = ck.obs_w_cfg;
        obn[k] = y; obe[k] = x;
      }
      bool need = false;
      in.u_d = 0; in.chi_d = 0; in.os_x = 0; in.os_y = 0; in.os_v = 0; in.p_last = 0; in.chi_last = 0;
      if (going && is_test) {
        const double los_arg = los_update(c, s, s.n, s.e);
#pragma unroll
        for (int k = 0; k < NOB; ++k) {  // sbmpc.py:150-156: active when any obstacle is within D_INIT
          const double d0 = obe[k] - s.e, d1 = obn[k] - s.n;
          need = need || sqrt_lt(d0 * d0 + d1 * d1, 2000.0);
        }
        if (need) in.chi_d = -(s.seg_alpha + atan(los_arg));
        in.u_d = c.desired_speed;
        in.os_x = s.e; in.os_y = s.n; in.os_v = s.v;
        in.p_last = p_last; in.chi_last = chi_last;
      }
      double pb = 1.0, cb = 0.0;
      need = diag::sb_request(need, P.max_sampling);  // (the product: need itself)
      diag::sb_stat_lanes(6, (need && sub == 0) ? 1u : 0u);
      diag::sb_stat_lanes(7, (going && is_test && sub == 0) ? 1u : 0u);
      sbmpc_cooperative_multi<NOB>(need && sub == 0, in, nsh - 1, P.sbmpc_nsamp, P.sbmpc_dt, pb, cb);
      pb = env_lane_d<LPE, 0>(pb, env_lane0);
      cb = env_lane_d<LPE, 0>(cb, env_lane0);
      const int need0 = env_lane_i<LPE, 0>((int)need, env_lane0);
      sb_active = need0;
      if (opaque_if<OPQ>(going)) {  // (tested here, not held as a lane mask across the optimiser's loop)
        if (need0) { p_last = pb; chi_last = cb; }
        else { p_last = 1; chi_last = 0; }
        if (opaque_if<OPQ>(is_test ? 1 : 0) && need0) { sf = pb; off = cb; }
      }
    } else if (COLLAV == SHIPSIM_COLLAV_SBMPC) {
      bool need = false;
      double los_arg = 0.0;
      if (going) {
        // the LOS cross-track term at this position, for every ship: its control below reuses it (its position
        // and segment are the same there unless the waypoint index advances)
        los_pre_q = los_q(c, s, s.n, s.e, los_pre_e);
      }
      if (going && is_test) {
        // env.py:362-363: next_wpt result discarded; los_guidance integrates e_ct_int (Q3). The
        // course (atan) only feeds the optimisation, so it is evaluated for requesting envs only.
        s.e_ct = los_pre_e;
        los_arg = los_windup(c, s, los_pre_q);
        double d0 = pe - s.e, d1 = pn - s.n;
        need = sqrt_lt(d0 * d0 + d1 * d1, 2000.0);  // D_INIT_
        need = diag::sb_request(need, P.max_sampling);  // (the product: need itself)
      }
      double pb = 1.0, cb = 0.0;
      int need0 = 0;
      // the optimiser's inputs, pass and hand-out only in a wave where some env requests it this tick (a
      // wave-uniform branch: every lane takes part in the exchanges inside)
      if (__any(need)) {
        const double pyaw = pair_swap(s.yaw), pu = pair_swap(s.u), pv = pair_swap(s.v);
        const double psy = pair_swap(sy), pcy = pair_swap(cy);  // sin/cos(pyaw), carried by the partner
        SbIn in = SbIn{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        in.u_d = SC[0].desired_speed;  // the same in every lane (sbmpc_cooperative<true>)
        in.obs_l = SC[1].obs_l_cfg; in.obs_w = SC[1].obs_w_cfg;
        if (going && is_test) {
          if (need) in.chi_d = -(s.seg_alpha + atan(los_arg));
          in.os_x = s.e; in.os_y = s.n; in.os_v = s.v;
          in.ob_x = pe; in.ob_y = pn; in.ob_psi = -pyaw; in.ob_u = pu; in.ob_v = pv;
          in.ob_so = -psy; in.ob_co = pcy;  // sin(-yaw) = -sin(yaw), cos(-yaw) = cos(yaw)
          in.p_last = p_last; in.chi_last = chi_last;
        }
        sbmpc_cooperative<true>(need && sub == 0, in, P.sbmpc_nsamp, P.sbmpc_dt, pb, cb);
        pb = env_lane_d<LPE, 0>(pb, env_lane0);
        cb = env_lane_d<LPE, 0>(cb, env_lane0);
        need0 = env_lane_i<LPE, 0>((int)need, env_lane0);
      }
      sb_active = need0;
      if (opaque_if<OPQ>(going)) {  // (tested here, not held as a lane mask across the optimiser's loop)
        if (need0) { p_last = pb; chi_last = cb; }
        else { p_last = 1; chi_last = 0; }
        if (opaque_if<OPQ>(is_test ? 1 : 0) && need0) { sf = pb; off = cb; }
      }
    }

    PT_MARK(0);
    // ---- ship ticks (test_step :345-445 / obs_step :447-536) ----
    double my_speed_out = 0.0, dtravel = 0.0, dtime = 0.0;
    if (going) {
      if (!is_test && s.stop) {
        // frozen obstacle ship: store_last_simulation_data + two next_time (Q9)
        if (REC && sub == 0) record_last(T, qc, rec_t, s.time, s.time + P.dt);
        s.time = s.time + P.dt;
        s.time = s.time + P.dt;
      } else {
        const double prev_log_n = s.log_n, prev_log_e = s.log_e;
        const double U = s.u;
        bool imminent = false;
        if (SIMPLE && is_test) {  // check_condition.py:130 on float32 self.states
          float dn = st4[0] - st4[2], de = st4[1] - st4[3];
          imminent = (dn * dn + de * de) < 9000000.0f;
        }
        SHIPSIM_SHIP_CHECK(LPE, SLOTS, 6);  // (its DPP exchanges pair sub-lanes of one ship)
        control_and_integrate_sc<DETAILED, REC, LOS_PRE>(c, P, s, rn, re, -off, sf, mach_dt,
                                                         (SIMPLE && is_test) ? 1 : 0, imminent,
                                                         (REC && sub == 0) ? T.ship_row(qc, rec_t) : nullptr, fuel, sy,
                                                         cy, los_pre_q, los_pre_e);
        my_speed_out = U;
        if (is_obs1) {  // travel tracker (env.py:527-534, Q6)
          double tn = s.log_n - prev_log_n, te = s.log_e - prev_log_e;
          dtravel = sqrt(tn * tn + te * te);
          dtime = P.dt;
        }
      }
    }
    PT_MARK(1);
    // ---- own-ship map queries, split over the ship's sub-lanes ----
    double d2 = INFINITY;
    bool gr = false;
    if (going) {
      const int cc = K.cell(s.n, s.e);
      if (cc != g_cell) {  // (rare) a new cell: its edge share and class
        g_cell = cc;
        g_mask = cc >= 0 ? grid_share(K, cc, sub, NSUB) : 0;
        g_flag = cc >= 0 ? (int)K.grid_flag[cc] : GRID_MIXED;
      }
      if constexpr (!diag::kNoMapDist)
        d2 = cc >= 0 ? map_dist2_mask(lds_edges, g_mask, s.n, s.e) : map_dist2_part(lds_edges, K.n_edges, s.n, s.e, sub, NSUB);
      const double margin = c.l_ship / 2;  // check_condition.py:50-78 hull hard points
      // Every hull corner is within margin·√2 of the centre. With no coastline edge that close (the
      // ship's min over its cell's candidate edges, which hold every edge within kGroundReach) and the
      // centre's cell entirely outside / inside the land, the segment centre → corner crosses no edge:
      // each corner has the centre cell's status, exactly what the four point-in-polygon tests return.
      double d2s = d2;
      int dummy = 0;
      ship_reduce<LPE, SLOTS>(d2s, dummy);
      const double lim = margin * 1.4142135623730951 + 1e-3;
      const int fcen = g_flag;
      const bool far_shore = d2s > lim * lim && fcen != GRID_MIXED && lim < kGroundReach;
      if constexpr (diag::kNoGround) {
      } else if (far_shore) {
        gr = fcen == GRID_IN;
      } else if constexpr (NSUB == 8) {
        // 8 sub-lanes for 4 corners: sub-lanes k and k + 4 split corner k's ring edges (every other
        // edge) and combine the crossing parity (XOR) and the boundary flag (OR) per polygon — the
        // same boolean as corner_inside (the partner lane is 4·SLOTS lanes away, same env and ship)
        const int sv = opaque_if<OPQ>(sub);  // (recomputed in the loop: no lane masks kept across it)
        const int k = sv & 3, half = sv >> 2;
        const double cn = (k < 2) ? s.n - margin : s.n + margin;
        const double ce = (k & 1) ? s.e + margin : s.e - margin;
        const int c = K.cell(cn, ce);
        const int f = c >= 0 ? (int)K.grid_flag[c] : GRID_MIXED;
        uint32_t par = 0, bnd = 0;
        if (f == GRID_MIXED) map_inside_half(lds_edges_raw, lds_boxes, P.n_polys, cn, ce, half, par, bnd);
        const uint32_t par_o = (uint32_t)__shfl_xor((int)par, 4 * SLOTS, 64);
        const uint32_t bnd_o = (uint32_t)__shfl_xor((int)bnd, 4 * SLOTS, 64);
        if (f == GRID_MIXED ? (((par ^ par_o) & ~(bnd | bnd_o)) != 0) : (f == GRID_IN)) gr = true;
      } else {
        for (int k = opaque_if<OPQ>(sub); k < 4; k += NSUB) {  // (opaque: no lane masks kept across the loop)
          const double cn = (k < 2) ? s.n - margin : s.n + margin;
          const double ce = (k & 1) ? s.e + margin : s.e - margin;
          if (corner_inside(K, lds_edges_raw, lds_boxes, P.n_polys, cn, ce)) gr = true;
        }
      }
      d2 = d2s;  // the ship's min over its sub-lanes' edge shares (reduced once, above)
    }
    int gri = gr ? XF_GROUND : 0;
    ship_or<LPE, SLOTS>(gri);
    const double my_ground = sqrt(d2);
    PT_MARK(2);
    bool my_end = false, my_outside = false, my_roa = false, my_nf = false;
    if (going) {
      my_end = sqrt_le((s.n - s.end_n) * (s.n - s.end_n) + (s.e - s.end_e) * (s.e - s.end_e), 200.0);
      double margin = c.l_ship / 2;
      my_outside = (s.n < P.min_north + margin || s.n > P.max_north - margin) ||
                   (s.e < P.min_east + margin || s.e > P.max_east - margin);
      double rdn = s.n - s.wp_n, rde = s.e - s.wp_e;  // is_reach_radius_of_acceptance (obstacle ship)
      my_roa = (rdn * rdn + rde * rde) < P.roa2;
      // a NaN / Inf anywhere in the dynamic state poisons this sum (boundary error contract)
      my_nf = !isfinite(((s.n + s.e) + (s.yaw + s.u)) + ((s.v + s.r) + (s.omega + s.e_ct_int)));
    }
    const int my_flags = gri | (my_end ? XF_END : 0) | (my_outside ? XF_OUTSIDE : 0) | (my_roa ? XF_ROA : 0) |
                         (my_nf ? XF_NONFINITE : 0);
    // env-level view of the tick: the ship under test (T), the obstacle ship (O) and the nearest
    // obstacle ship (C; = O with one obstacle ship)
    double Tn, Te, Th, Tsh, Tch, Tect, Tground, Ttime, On, Oe, Oyaw, Oect, Oground, Ospeed, Odtravel, Odtime, Cn, Ce;
    int Tf, Of;
    bool any_nf;
    if constexpr (SLOTS == 2) {
      // each lane's own perspective: T = its own ship, O = the partner lane's (lane ^ 1). That is the env's view
      // on the test ship's lanes; the env's outcome is the test ship's first lane's (its event bits, taken by every
      // lane of the env below), so the obstacle ship's lanes need no role selects
      SHIPSIM_LANE_CHECK(LPE, 8);
      Tn = s.n; Te = s.e; Th = s.yaw; Tsh = sy; Tch = cy; Tect = s.log_ect; Tground = my_ground; Ttime = s.time;
      Tf = my_flags;
      Of = pair_swap_i(my_flags);
      On = pair_swap(s.n); Oe = pair_swap(s.e); Oyaw = pair_swap(s.yaw);
      Oect = pair_swap(s.log_ect); Oground = pair_swap(my_ground);
      Ospeed = pair_swap(my_speed_out); Odtravel = pair_swap(dtravel); Odtime = pair_swap(dtime);
      Cn = On; Ce = Oe;
      any_nf = (my_flags | Of) & XF_NONFINITE;
    } else {  // slot k's first lane of the env row holds ship k
      Tn = env_lane_d<LPE, 0>(s.n, env_lane0); Te = env_lane_d<LPE, 0>(s.e, env_lane0);
      Th = env_lane_d<LPE, 0>(s.yaw, env_lane0); Tsh = env_lane_d<LPE, 0>(sy, env_lane0);
      Tch = env_lane_d<LPE, 0>(cy, env_lane0); Tect = env_lane_d<LPE, 0>(s.log_ect, env_lane0);
      Tground = env_lane_d<LPE, 0>(my_ground, env_lane0); Ttime = env_lane_d<LPE, 0>(s.time, env_lane0);
      Tf = env_lane_i<LPE, 0>(my_flags, env_lane0);
      On = env_lane_d<LPE, 1>(s.n, env_lane0); Oe = env_lane_d<LPE, 1>(s.e, env_lane0);
      Oyaw = env_lane_d<LPE, 1>(s.yaw, env_lane0); Oect = env_lane_d<LPE, 1>(s.log_ect, env_lane0);
      Oground = env_lane_d<LPE, 1>(my_ground, env_lane0); Ospeed = env_lane_d<LPE, 1>(my_speed_out, env_lane0);
      Odtravel = env_lane_d<LPE, 1>(dtravel, env_lane0); Odtime = env_lane_d<LPE, 1>(dtime, env_lane0);
      Of = env_lane_i<LPE, 1>(my_flags, env_lane0);
      int nf = Tf | Of;
      Cn = On; Ce = Oe;
      double cd = (Tn - On) * (Tn - On) + (Te - Oe) * (Te - Oe);
#define NEAREST(M)                                                                                  \
  if constexpr (M < SLOTS) {                                                                        \
    const double kn = env_lane_d<LPE, M>(s.n, env_lane0), ke = env_lane_d<LPE, M>(s.e, env_lane0); \
    nf |= env_lane_i<LPE, M>(my_flags, env_lane0);                                                  \
    const double kd = (Tn - kn) * (Tn - kn) + (Te - ke) * (Te - ke);                                \
    if (kd < cd) { cd = kd; Cn = kn; Ce = ke; }                                                     \
  }
      NEAREST(2) NEAREST(3) NEAREST(4) NEAREST(5) NEAREST(6) NEAREST(7)
#undef NEAREST
      any_nf = nf & XF_NONFINITE;
    }
    if (going) {
      travel_dist += Odtravel;
      travel_time += Odtime;
      // next_states (env.py:582-591) and self.states
      ns[0] = (float)Tn; ns[1] = (float)Te; ns[2] = (float)Tect;
      ns[3] = (float)On; ns[4] = (float)Oe; ns[5] = (float)Oyaw; ns[6] = (float)Ospeed; ns[7] = (float)Oect;
      if (SIMPLE) { st4[0] = ns[0]; st4[1] = ns[1]; st4[2] = ns[3]; st4[3] = ns[4]; }
      // get_reward_and_env_info (reward_function.py:59-270)
      const bool is_collision = ((Tn - Cn) * (Tn - Cn) + (Te - Ce) * (Te - Ce)) < 2500.0;
      const bool is_tg = Tf & XF_GROUND, is_og = Of & XF_GROUND;
      const bool is_tnav = fabs(Tect) > 3000;
      const bool is_onav = (travel_dist > P.AB_seg * 2) || (travel_time > INFINITY) || (fabs(Oect) > 500);
      double dx = Cn - Tn, dy = Ce - Te;
      double dist = sqrt(dx * dx + dy * dy);
      const bool enc_ok = !overtaking_sector(dx, dy, dist, Tsh, Tch, Th);  // head-on or crossing (Q5)
      // the five shaped terms of reward_designs.py:33-55 (RewardDesign4 / 3): one exp each,
      // evaluated by five lanes of the env in one call when LPE >= 8, then gathered
      const double xv[5] = {dist, Tground, fabs(Tect), Oground, fabs(Oect)};
      const double tg[5] = {0.0, 0.0, 3000.0, 0.0, 500.0};
      const double of[5] = {200000000.0, 175000.0, 1250000.0, 50000.0, 12500.0};
      double ex[5];
      if (LPE >= 8) {
        const int j = opaque_v(lie) & 7;  // (recomputed in the loop: no lane masks kept across it)
        double xj;
        if constexpr (SLOTS == 2)  // lanes 1 / 3 (obstacle ship): its own ground / |e_ct| (terms 3 / 4)
          xj = (j == 0) ? dist : (j < 3) ? Tground : fabs(Tect);
        else
          xj = (j == 0) ? xv[0] : (j == 1) ? xv[1] : (j == 2) ? xv[2] : (j == 3) ? xv[3] : xv[4];
        const RewardTerm to = lds_rterm[j];
        const double ej = exp(div_by(-((xj - to.t) * (xj - to.t)), to.o, to.y));
        ex[0] = env_lane_d<LPE, reward_lane<SLOTS>(0)>(ej, env_lane0);
        ex[1] = env_lane_d<LPE, reward_lane<SLOTS>(1)>(ej, env_lane0);
        ex[2] = env_lane_d<LPE, reward_lane<SLOTS>(2)>(ej, env_lane0);
        ex[3] = env_lane_d<LPE, reward_lane<SLOTS>(3)>(ej, env_lane0);
        ex[4] = env_lane_d<LPE, reward_lane<SLOTS>(4)>(ej, env_lane0);
      } else {
#pragma unroll
        for (int k = 0; k < 5; ++k) ex[k] = exp(-((xv[k] - tg[k]) * (xv[k] - tg[k])) / of[k]);
      }
      // rd4(t, off, v) = v < t ? 1 : exp(.), rd3(t, off, v) = v < t ? exp(.) : 1
      double r0 = (dist < 10000 && enc_ok) ? ((xv[0] < 0.0) ? 1.0 : ex[0]) : 0.0;
      double r1 = (Tground <= 1000) ? ((xv[1] < 0.0) ? 1.0 : ex[1]) : 0.0;
      double r2 = (xv[2] < 3000.0) ? ex[2] : 1.0;
      double r3 = (Oground <= 1000) ? -((xv[3] < 0.0) ? 1.0 : ex[3]) : 0.0;
      double r4 = -((xv[4] < 500.0) ? ex[4] : 1.0);
      double r = (r0 + ((((0.0 + r1) + r2) + r3) + r4)) / 5;  // np.sum(5 terms) / 5
      if (is_collision || is_tg || is_tnav || is_og || is_onav) {  // :272-314
        const double reward = r + acc;
        double o = 0;
        const bool cond[5] = {is_collision, is_tg, is_tnav, is_og, is_onav};
        const double mult[5] = {10.0, 5.0, 5.0, -2.5, -2.5};
        for (int i = 0; i < 5; ++i) {
          if (acc > 0 && cond[i]) o += reward * mult[i];
          else if (acc < 0 && cond[i]) o += reward * -mult[i];
        }
        r = o;
      }
      const bool t6 = Tf & XF_END, t7 = Tf & XF_OUTSIDE, t8 = Of & XF_END, t9 = Of & XF_OUTSIDE;
      const bool t10 = Ttime > P.sim_time;
      constexpr uint32_t kRoaBit = 1u << 31;  // (private: the obstacle ship reached its waypoint radius)
      uint32_t bits = (is_collision ? SHIPSIM_EV_COLLISION : 0) | (is_tg ? SHIPSIM_EV_TEST_GROUNDING : 0) |
                      (is_tnav ? SHIPSIM_EV_TEST_NAV_FAILURE : 0) | (is_og ? SHIPSIM_EV_OBS_GROUNDING : 0) |
                      (is_onav ? SHIPSIM_EV_OBS_NAV_FAILURE : 0) | (t6 ? SHIPSIM_EV_TEST_REACHES_END : 0) |
                      (t7 ? SHIPSIM_EV_TEST_OUTSIDE_MAP : 0) | (t8 ? SHIPSIM_EV_OBS_REACHES_END : 0) |
                      (t9 ? SHIPSIM_EV_OBS_OUTSIDE_MAP : 0) | (t10 ? SHIPSIM_EV_TIME_LIMIT : 0) |
                      ((Of & XF_ROA) ? kRoaBit : 0u);
      if constexpr (SLOTS == 2) bits = (uint32_t)env_lane_i<LPE, 0>((int)bits, env_lane0);  // the test ship's view
      const bool roa_o = bits & kRoaBit;
      bits &= ~kRoaBit;
      const bool terminal = bits & 0x1F;
      const bool test_stop = bits & (SHIPSIM_EV_COLLISION | SHIPSIM_EV_TEST_GROUNDING | SHIPSIM_EV_TEST_NAV_FAILURE |
                                     SHIPSIM_EV_TEST_REACHES_END | SHIPSIM_EV_TEST_OUTSIDE_MAP | SHIPSIM_EV_TIME_LIMIT);
      const bool obs_stop = bits & (SHIPSIM_EV_COLLISION | SHIPSIM_EV_OBS_GROUNDING | SHIPSIM_EV_OBS_NAV_FAILURE |
                                    SHIPSIM_EV_OBS_REACHES_END | SHIPSIM_EV_OBS_OUTSIDE_MAP | SHIPSIM_EV_TIME_LIMIT);
      if (terminal) bits |= SHIPSIM_EV_TERMINAL;
      if (test_stop) bits |= SHIPSIM_EV_TEST_STOP;
      if (obs_stop) bits |= SHIPSIM_EV_OBS_STOP;
      if (obs_stop && !terminal && is_obs1) s.stop = 1;
      if (SLOTS > 2 && shipc >= 2 && (my_flags & (XF_END | XF_OUTSIDE | XF_GROUND)))
        s.stop = 1;  // further obstacle ships freeze at their last waypoint / off the map / aground
      bool combined_done = terminal || (test_stop && !terminal);
      const bool nonfinite = any_nf;
      if (nonfinite) {  // not a reference outcome: the env ends its episode here, flagged
        bits |= SHIPSIM_EV_NONFINITE | SHIPSIM_EV_TERMINAL;
        combined_done = true;
        n_nonfinite += 1;
      }
      if (REC) {  // RewardTracker.update (reward_function.py:181-186) + env.py:613-620 animation lists
        double* er = (lie == 0) ? T.env_row(env, rec_t - 1) : nullptr;
        if (er) {
          er[SHIPSIM_TE_R_COLLISION] = r0 / 5; er[SHIPSIM_TE_R_TEST_GROUNDING] = r1 / 5;
          er[SHIPSIM_TE_R_TEST_NAV] = r2 / 5; er[SHIPSIM_TE_R_OBS_GROUNDING] = r3 / 5;
          er[SHIPSIM_TE_R_OBS_NAV] = r4 / 5; er[SHIPSIM_TE_R_TOTAL] = r; er[SHIPSIM_TE_BITS] = (double)bits;
          const bool imm = (COLLAV == SHIPSIM_COLLAV_SBMPC)
                               ? sb_active
                               : ((Tn - On) * (Tn - On) + (Te - Oe) * (Te - Oe)) < 9000000.0;
          er[SHIPSIM_TE_FLAGS] = (double)((is_collision ? SHIPSIM_TE_FLAG_COLLISION : 0) |
                                          (imm ? SHIPSIM_TE_FLAG_IMMINENT : 0));
        }
        rec_t += 1;
      }
      // ---- env.py:700-771 decision logic ----
      acc += r;
      ticks += 1;
      dec_ticks += 1;
      bool finish = nonfinite;
      if (phase == 0) {
        const bool roa = roa_o;
        if (combined_done) finish = true;
        else if (roa) {
          if (opaque_if<OPQ>(have_iw) != 0) phase = 1;
          else finish = true;
        }
      } else if (phase == 1) {
        if (sampling_count == P.max_sampling) {
          travel_dist = 0;
          travel_time = 0;
          if (combined_done) finish = true;
          else phase = 2;
        } else {
          finish = true;
        }
      } else {
        if (combined_done) finish = true;
      }
      if (finish) {
        out_r = acc;
        out_done = combined_done;
        out_bits = bits;
        out_ticks = dec_ticks;
        snap_bits = bits;
        ready = opaque_if<OPQ>(1);
      }
      const int mt = OPQ ? opaque_v(budget) : budget;  // (OPQ: its test not held across the loop)
      going = opaque_if<OPQ>((!ready && (mt <= 0 || ticks < mt)) ? 1 : 0);
    }
    PT_MARK(3);
  }
  if (!CHAIN) break;
  if (POLICY || (ready && running)) chain_next();  // (policy: wave-uniform, a no-op unless a decision completed)
  {
    const int mt = OPQ ? opaque_v(budget) : budget;
    going = opaque_if<OPQ>((running && !ready && (mt <= 0 || ticks < mt)) ? 1 : 0);
  }
  if (!__any(opaque_if<OPQ>(going))) {
    // Launch tail: this wave's envs met the quota. While any wave of the launch has not, keep ticking in chunks
    // instead of idling the SIMD until the slowest wave ends (an env's results do not depend on where a launch
    // ends: slicing is exact). Bounded by tail_extra, so a wave that is not co-resident delays nothing forever.
    // (One exit, every test wave-uniform: no flow masks held across the loop.)
    const ChainArgs& CT = step_args().CH;
    if (SLOTS == 2 && CT.tail_ctr && budget < step_args().max_ticks + CT.tail_extra) {  // (two-ship envs)
      const bool lead = (opaque_v(threadIdx.x) & 63) == 0;  // (re-derived here: no lane mask held across the loop)
      if (lead && opaque_v(tail_arrived) == 0)
        __hip_atomic_fetch_add(CT.tail_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tail_arrived = opaque_v(1);
      int n_met = 0;
      if (lead) n_met = __hip_atomic_load(CT.tail_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_readfirstlane(n_met) < CT.tail_waves) {
        budget += kTailChunk;
        going = opaque_if<OPQ>((running && !ready && ticks < budget) ? 1 : 0);
      }
    }
    if (!__any(opaque_if<OPQ>(going))) break;  // (quota met, or every env of the wave stalled)
  }
  }
  PT_FLUSH();

  if (touched == 0) return;  // (!valid || !touched)
  const StepArgs& AE = step_args();  // not the values loaded before the loop (no live range across it)
  const ChainArgs& CH = AE.CH;
  const Traj& TE = AE.T;
  SHIPSIM_DEBUG_PRINT(env, "[dbg] env %d lie %d end: ready %d ticks %d sc %d n_base %f phase %d have_iw %d\n", env, lie,
                      (int)ready, ticks, sampling_count, n_base, phase, (int)have_iw);
  const DevState So = opaque(AE.S);  // addresses recomputed here, not carried through the loop
  // the lane's role re-derived here (opaque), not lane masks carried through the loop
  const int lie_e = opaque_v(lie), sub_e = lie_e / SLOTS, ship_e = lie_e % SLOTS;
  const bool ghost_e = (SLOTS > 2) && ship_e >= nsh;
  if (sub_e == 0 && !ghost_e) store_ship(So, qc, s);
  if (REC) {
    if (sub_e == 0)
      for (int k = 0; k < 3; ++k) TE.fuel[(size_t)qc * 3 + k] = fuel[k];
    if (lie_e == 0) TE.len[env] = rec_t;
  }
  if (CHAIN && lie_e == 0) {
    CH.ep_idx[env] = ep_i;
    CH.dec_idx[env] = dec_i;
    if (CH.decisions) CH.decisions[env] = n_decided;
    if (CH.log_len) CH.log_len[env] = log_n;
    So.mach_dt()[env] = mach_dt;
  }
  if (lie_e == 0) {
    So.sampling_count()[env] = sampling_count;
    So.travel_dist()[env] = travel_dist; So.travel_time()[env] = travel_time; So.acc()[env] = acc;
    So.n_base()[env] = n_base; So.e_base()[env] = e_base;
    So.p_last()[env] = p_last; So.chi_last()[env] = chi_last;
    if (SIMPLE)
      for (int i = 0; i < 4; ++i) So.states4()[env * 4 + i] = st4[i];
    if (ready)
      for (int i = 0; i < 8; ++i) So.next_obs8()[env * 8 + i] = ns[i];
    So.snap_bits()[env] = snap_bits;
    So.dec_flags()[env] = ((ready || stalled) ? DF_AWAITING : 0) | (have_iw ? DF_HAVE_IW : 0) |
                          (phase << DF_PHASE_SHIFT);
    So.dec_ticks()[env] = dec_ticks;
    if (n_nonfinite) atomicAdd(So.nonfinite, n_nonfinite);
    if (ready) {
      if (AE.reward_out) AE.reward_out[env] = out_r;
      if (AE.done_out) AE.done_out[env] = out_done ? 1 : 0;
      if (AE.events_out) AE.events_out[env] = out_bits;
    }
    if (AE.ticks_out) AE.ticks_out[env] = ticks;
    if (AE.ready_out) AE.ready_out[env] = ready ? 1 : 0;
  }
  if (ready && AE.obs_out && lie_e == 0) {  // the test ship's first lane holds the env's observation
#pragma unroll
    for (int i = 0; i < 8; ++i) AE.obs_out[env * 8 + i] = ns[i];
  }
}

// C2 single-ship loop body, k ticks per launch (one lane per ship; algebraic wind force)
template <bool DETAILED>
__global__ __launch_bounds__(64) void single_tick_kernel(const Params P, DevState S, ConstBuf K, int k) {
  __shared__ ShipConst lds_sc[SHIPSIM_MAX_SHIPS];
  const ShipConst* SC = stage_consts(K, lds_sc, P.n_ships, P.dt);
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.n_envs) return;
  const ShipConst& c = SC[0];
  const double* rn = S.route_n() + (size_t)q * kMaxRoute;
  const double* re = S.route_e() + (size_t)q * kMaxRoute;
  Ship s;
  load_ship(S, q, s);
  const double mach_dt = S.mach_dt()[q];
  double wsin, wcos;
  sincos(P.wind_dir, &wsin, &wcos);
  for (int i = 0; i < k; ++i)
    control_and_integrate<DETAILED, false, false, true>(c, P, s, rn, re, 0.0, 1.0, mach_dt, 0, false, nullptr, nullptr,
                                                        false, wsin, wcos);
  store_ship(S, q, s);
}

#endif  // SHIPSIM_TU != 2

#if SHIPSIM_TU != 1
// C2 with the simplified machinery (the C2 configuration, SimpleShipModel + ThrustFromSpeedSetPoint): the same ticks
// as single_tick_kernel<false>, bit for bit, on THREE waves per 64 ships, software-pipelined so that one workgroup
// barrier per tick separates them. A tick t only needs, besides its own (u, v, r):
//   sin/cos ψ_t    — ψ_t = ψ_{t-1} + r_{t-1} dt is known one tick early;
//   the rudder_t   — waypoint switch, LOS guidance (sqrt, divide, atan) and heading PID on (n, e, ψ)_t, which follow
//                    from tick t - 1's state by the explicit Euler step before tick t - 1's kinetics matter.
// So in interval t
//   wave 0 (guidance): (n, e, ψ)_{t+1} from (u, v, r)_t and sin/cos ψ_t, then the rudder of tick t + 1;
//   wave 1 (heading):  ψ_{t+1} and sin/cos ψ_{t+1};
//   wave 2 (dynamics): tick t's thrust (speed PID), wind force and kinetics -> (u, v, r)_{t+1};
// each reading what the others wrote in interval t - 1 (LDS, double-buffered by tick parity). Every value is formed
// by the same expression as in the one-wave tick (control_and_store, differentials, integrate): the same bits.
template <bool POW2_DT>  // dt a power of two: the PIDs' derivative division as the exact multiplication (pid)
__global__ __launch_bounds__(192) void single_tick_pipe_kernel(const Params P, DevState S, ConstBuf K, int k) {
  __shared__ ShipConst lds_sc[SHIPSIM_MAX_SHIPS];
  __shared__ double x_uvr[2][3][64];  // (u, v, r) of a tick, by tick parity
  __shared__ double x_sc[2][2][64];   // sin / cos ψ of a tick
  __shared__ double x_rud[2][64];     // rudder of a tick
  const ShipConst* SC = stage_consts(K, lds_sc, P.n_ships, P.dt);
  const int lane = threadIdx.x & 63, role = threadIdx.x >> 6;  // (wave-uniform)
  const int q0 = blockIdx.x * 64 + lane, q = min(q0, P.n_envs - 1);  // (every lane takes part in the barriers)
  const bool live = q0 < P.n_envs;
  const ShipConst& c = SC[0];
  const double dt = P.dt, inv_dt = pow2_inverse(dt);  // (the PIDs' derivative terms: see pid)
  Ship s;
  load_ship(S, q, s);
  // the kinematic rates of integrate's Euler step (differentials_body's expressions)
  auto advance_pose = [&](double u, double v, double r, double sy, double cy) __attribute__((always_inline)) {
    // (the rotation's structural zero terms dropped: a ±0 addend leaves every non-zero rate's bits as they are)
    const double dn = cy * u + (-sy) * v;
    const double de = sy * u + cy * v;
    const double dyaw = r;
    s.n = s.n + dn * dt;
    s.e = s.e + de * dt;
    s.yaw = s.yaw + dyaw * dt;
  };
  if (role == 0) {
    // guidance: the rudder of tick j from (n, e, ψ)_j — control_and_store's route half (DETAILED false, no collav)
    const double* rn = S.route_n() + (size_t)q * kMaxRoute;
    const double* re = S.route_e() + (size_t)q * kMaxRoute;
    auto guide = [&]() __attribute__((always_inline)) {
      const double N = s.n, E = s.e, H = s.yaw;
      if (next_wpt_advance(c, s, N, E)) {
        s.next_wpt += 1;
        load_segment(s, rn, re);
      }
      const double href = los_guidance(c, s, N, E);
      const double rudder = heading_ctrl<POW2_DT>(c, s, href + 0.0, H, dt, POW2_DT ? inv_dt : c.rcp_dt);
      s.log_rudder = rudder;
      s.log_ect = s.e_ct;
      s.log_n = N;
      s.log_e = E;
      return rudder;
    };
    x_rud[0][lane] = guide();
    __syncthreads();
    for (int t = 0; t < k; ++t) {
      const int b = t & 1;
      advance_pose(x_uvr[b][0][lane], x_uvr[b][1][lane], x_uvr[b][2][lane], x_sc[b][0][lane], x_sc[b][1][lane]);
      if (t + 1 < k) x_rud[b ^ 1][lane] = guide();
      __syncthreads();
    }
    if (live) {
      S.f(SF_N)[q] = s.n; S.f(SF_E)[q] = s.e; S.f(SF_YAW)[q] = s.yaw;
      S.f(SF_ECT)[q] = s.e_ct; S.f(SF_ECT_INT)[q] = s.e_ct_int;
      S.f(SF_HDG_EI)[q] = s.hdg_ei; S.f(SF_HDG_PREV)[q] = s.hdg_prev;
      S.f(SF_RUDDER)[q] = s.log_rudder; S.f(SF_LOG_ECT)[q] = s.log_ect;
      S.f(SF_LOG_N)[q] = s.log_n; S.f(SF_LOG_E)[q] = s.log_e;
      S.next_wpt()[q] = s.next_wpt;
    }
  } else if (role == 1) {
    // heading: sin/cos ψ of the next tick (differentials' sincos(s.yaw))
    double sy, cy;
    sincos(s.yaw, &sy, &cy);
    x_sc[0][0][lane] = sy; x_sc[0][1][lane] = cy;
    __syncthreads();
    for (int t = 0; t < k; ++t) {
      const int b = t & 1;
      const double r = x_uvr[b][2][lane];
      s.yaw = s.yaw + r * dt;  // (advance_pose's ψ rate)
      if (t + 1 < k) {
        sincos(s.yaw, &sy, &cy);
        x_sc[b ^ 1][0][lane] = sy; x_sc[b ^ 1][1][lane] = cy;
      }
      __syncthreads();
    }
  } else {
    // dynamics: tick t's thrust, wind force and kinetics (control_and_store's speed half, differentials, integrate)
    double wsin, wcos;
    sincos(P.wind_dir, &wsin, &wcos);
    x_uvr[0][0][lane] = s.u; x_uvr[0][1][lane] = s.v; x_uvr[0][2][lane] = s.r;
    __syncthreads();
    for (int t = 0; t < k; ++t) {
      const int b = t & 1;
      const double sy = x_sc[b][0][lane], cy = x_sc[b][1][lane], rudder = x_rud[b][lane];
      const double thrust = speed_ctrl<POW2_DT>(c, s, c.desired_speed * 1.0, s.u, dt, false, POW2_DT ? inv_dt : c.rcp_dt);
      s.log_thrust = thrust;
      double tau[3];
      wind_force_alg(c, P, s, sy, cy, wsin, wcos, tau);
      const Deriv d = differentials_body(c, P, s, thrust, rudder, false, sy, cy, tau);
      s.u = s.u + d.du * dt;
      s.v = s.v + d.dv * dt;
      s.r = s.r + d.dr * dt;
      s.time = s.time + dt;
      x_uvr[b ^ 1][0][lane] = s.u; x_uvr[b ^ 1][1][lane] = s.v; x_uvr[b ^ 1][2][lane] = s.r;
      __syncthreads();
    }
    if (live) {
      S.f(SF_U)[q] = s.u; S.f(SF_V)[q] = s.v; S.f(SF_R)[q] = s.r; S.f(SF_TIME)[q] = s.time;
      S.f(SF_SPD_A)[q] = s.spd_a; S.f(SF_SPD_B)[q] = s.spd_b; S.f(SF_THRUST)[q] = s.log_thrust;
    }
  }
}

#endif  // SHIPSIM_TU != 1

#if SHIPSIM_TU != 1
void shipsim_c2_pipe_launch(int blocks, hipStream_t st, const Params& P, const DevState& S, const ConstBuf& K, int k) {
  if (pow2_inverse(P.dt) != 0.0)
    hipLaunchKernelGGL(single_tick_pipe_kernel<true>, dim3(blocks), dim3(192), 0, st, P, S, K, k);
  else
    hipLaunchKernelGGL(single_tick_pipe_kernel<false>, dim3(blocks), dim3(192), 0, st, P, S, K, k);
}
#endif

#if SHIPSIM_TU != 2
// Legacy per-tick MultiShipEnv.step (rl_env/ship_in_transit/env.py:1104-1173), k steps per launch.
// Two lanes per env (lane & 1 = ship); the termination flags of get_termination_status
// (termination_flags.py:5-70) are evaluated in fp64 on the next_states, as the reference does on
// its Python-float list.
// Arguments read through the kernarg segment pointer (as step_args): the Params block and the state base
// addresses are scalar loads where a tick uses them, not argument SGPRs held (and spilled) across the loop.
struct LegacyArgs {
  Params P;
  DevState S;
  ConstBuf K;
  int k;
  double* states_out;
  uint8_t* done_out;
  uint32_t* status_out;
};
typedef const __attribute__((address_space(4))) LegacyArgs* LegacyArgsPtr;
__device__ __forceinline__ const LegacyArgs& legacy_args() {
  LegacyArgsPtr q = (LegacyArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return *(const LegacyArgs*)q;
}

template <bool DETAILED, int COLLAV>
__global__ __launch_bounds__(64) void legacy_step_kernel(LegacyArgs a_arg) {
  (void)a_arg;  // read through legacy_args()
  __shared__ ShipConst lds_sc[SHIPSIM_MAX_SHIPS];
  __shared__ Edge lds_edges_raw[SHIPSIM_MAX_VERTS];
  __shared__ PolyBox lds_boxes[SHIPSIM_MAX_POLYS];
  const LegacyArgs& A0 = legacy_args();
  const ShipConst* SC = stage_consts(A0.K, lds_sc, A0.P.n_ships, A0.P.dt);
  for (int i = threadIdx.x; i < A0.K.n_edges; i += blockDim.x) lds_edges_raw[i] = A0.K.edges()[i];
  for (int i = threadIdx.x; i < A0.P.n_polys; i += blockDim.x) lds_boxes[i] = A0.K.boxes()[i];
  __syncthreads();

  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int env = gl >> 1;
  const int ship = gl & 1;
  const bool is_test = ship == 0;
  const bool valid = env < A0.P.n_envs;
  const int envc = valid ? env : 0;
  const int qc = envc * 2 + ship;
  const ShipConst& c = SC[ship];
  const double* rn = A0.S.route_n() + (size_t)qc * kMaxRoute;
  const double* re = A0.S.route_e() + (size_t)qc * kMaxRoute;
  Ship s;
  load_ship(A0.S, qc, s);
  double p_last = A0.S.p_last()[envc], chi_last = A0.S.chi_last()[envc];
  const double mach_dt = A0.S.mach_dt()[envc];
  const double* lst = A0.S.legacy_states() + (size_t)envc * 4;  // self.states [test n, e, obs n, e]
  double st[4] = {lst[0], lst[1], lst[2], lst[3]};
  bool st_f32 = A0.S.legacy_flags()[envc] & 1;
  const int n_samp = (int)(A0.P.sbmpc_tf / A0.P.sbmpc_dt);

  double out8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t status = 0;
  bool done = false, ticked = false;
  bool going = valid;
  for (int it = 0; it < legacy_args().k; ++it) {
    if (!__any(going)) break;
    // this tick's constants: re-read through the kernarg pointer rather than kept in registers across ticks
    const LegacyArgs& A = legacy_args();
    const Params& P = A.P;
    const ConstBuf& K = A.K;
    const double pn = pair_swap(s.n), pe = pair_swap(s.e), pyaw = pair_swap(s.yaw);
    const double pu = pair_swap(s.u), pv = pair_swap(s.v);
    double sf = 1.0, off = 0.0;
    if (COLLAV == SHIPSIM_COLLAV_SBMPC) {  // test_step :938-963 (obstacle ship before it moves)
      bool need = false;
      SbIn in = SbIn{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      in.u_d = SC[0].desired_speed;  // the same in every lane (sbmpc_cooperative<true>)
      in.obs_l = SC[1].obs_l_cfg; in.obs_w = SC[1].obs_w_cfg;
      if (going && is_test) {
        const double los_arg = los_update(c, s, s.n, s.e);
        const double d0 = pe - s.e, d1 = pn - s.n;
        need = sqrt_lt(d0 * d0 + d1 * d1, 2000.0);  // D_INIT_
        need = diag::sb_request(need, P.max_sampling);  // (the product: need itself)
        if (need) in.chi_d = -(s.seg_alpha + atan(los_arg));
        in.os_x = s.e; in.os_y = s.n; in.os_v = s.v;
        in.ob_x = pe; in.ob_y = pn; in.ob_psi = -pyaw; in.ob_u = pu; in.ob_v = pv;
        sb_set_heading_trig(in);
        in.p_last = p_last; in.chi_last = chi_last;
      }
      double pb = 1.0, cb = 0.0;
      sbmpc_cooperative<true>(need, in, n_samp, P.sbmpc_dt, pb, cb);
      if (going && is_test) {
        if (need) { p_last = pb; chi_last = cb; sf = pb; off = cb; }
        else { p_last = 1; chi_last = 0; }
      }
    }
    double speed_out = 0.0;
    if (going) {
      if (!is_test && s.stop) {  // obs_step :1029-1056: store_last + two next_time, speed reported 0
        s.time = s.time + P.dt;
        s.time = s.time + P.dt;
      } else {
        bool imminent = false;
        if (COLLAV == SHIPSIM_COLLAV_SIMPLE && is_test) {  // is_collision_imminent(self.states[0:2], [3:5])
          if (st_f32) {
            const float dn = P.initial_states[0] - P.initial_states[3], de = P.initial_states[1] - P.initial_states[4];
            imminent = (dn * dn + de * de) < 9000000.0f;
          } else {
            imminent = ((st[0] - st[2]) * (st[0] - st[2]) + (st[1] - st[3]) * (st[1] - st[3])) < 9000000.0;
          }
        }
        speed_out = s.u;
        control_and_integrate<DETAILED>(c, P, s, rn, re, -off, sf, mach_dt,
                                        (COLLAV == SHIPSIM_COLLAV_SIMPLE && is_test) ? 1 : 0, imminent);
      }
    }
    // own-ship flags on the post-tick state (check_condition.py)
    bool my_end = false, my_out = false, my_gr = false;
    if (going) {
      const double margin = c.l_ship / 2;
      my_end = sqrt_le((s.n - s.end_n) * (s.n - s.end_n) + (s.e - s.end_e) * (s.e - s.end_e), 200.0);
      my_out = (s.n < P.min_north + margin || s.n > P.max_north - margin) ||
               (s.e < P.min_east + margin || s.e > P.max_east - margin);
      for (int q = 0; q < 4; ++q) {
        const double cn = (q < 2) ? s.n - margin : s.n + margin;
        const double ce = (q & 1) ? s.e + margin : s.e - margin;
        if (corner_inside(K, lds_edges_raw, lds_boxes, P.n_polys, cn, ce)) my_gr = true;
      }
    }
    const bool my_nav = fabs(s.log_ect) > 500;  // is_ship_navigation_failure (e_tol 500, both ships)
    const int my_flags = (my_end ? 1 : 0) | (my_out ? 2 : 0) | (my_gr ? 4 : 0) | (my_nav ? 8 : 0);
    const int o_flags = pair_swap_i(my_flags);
    const double o_n = pair_swap(s.n), o_e = pair_swap(s.e), o_yaw = pair_swap(s.yaw);
    const double o_ect = pair_swap(s.log_ect), o_speed = pair_swap(speed_out);
    if (going) {
      const double Tn = is_test ? s.n : o_n, Te = is_test ? s.e : o_e;
      const double On = is_test ? o_n : s.n, Oe = is_test ? o_e : s.e;
      const int Tf = is_test ? my_flags : o_flags, Of = is_test ? o_flags : my_flags;
      out8[0] = Tn; out8[1] = Te; out8[2] = is_test ? s.log_ect : o_ect;
      out8[3] = On; out8[4] = Oe; out8[5] = is_test ? o_yaw : s.yaw;
      out8[6] = is_test ? o_speed : speed_out; out8[7] = is_test ? o_ect : s.log_ect;
      const double cd = (Tn - On) * (Tn - On) + (Te - Oe) * (Te - Oe);
      status = (uint32_t)(Tf & 15) | (cd < 9000000.0 ? SHIPSIM_LT_NEAR_COLLISION : 0u) |
               (cd < 2500.0 ? SHIPSIM_LT_COLLISION : 0u) | ((uint32_t)(Of & 15) << 6);
      done = (status & (SHIPSIM_LT_TEST_REACHED | SHIPSIM_LT_TEST_OUTSIDE | SHIPSIM_LT_TEST_GROUNDED |
                        SHIPSIM_LT_TEST_NAV_FAILURE | SHIPSIM_LT_COLLISION | SHIPSIM_LT_OBS_GROUNDED |
                        SHIPSIM_LT_OBS_NAV_FAILURE)) != 0;
      // stop_int_obs = obs_is_outside and obs_is_reached (:1168-1171)
      if (!is_test && (Of & 2) && (Of & 1)) s.stop = 1;
      st[0] = Tn; st[1] = Te; st[2] = On; st[3] = Oe;
      st_f32 = false;
      ticked = true;
      going = !done;
    }
  }
  if (!valid) return;
  const LegacyArgs& A = legacy_args();
  const DevState S = opaque(A.S);
  store_ship(S, qc, s);
  if (is_test) {
    S.p_last()[env] = p_last; S.chi_last()[env] = chi_last;
    double* lsto = S.legacy_states() + (size_t)env * 4;
    for (int i = 0; i < 4; ++i) lsto[i] = st[i];
    S.legacy_flags()[env] = st_f32 ? 1 : 0;
    if (ticked) {
      if (A.states_out)
        for (int i = 0; i < 8; ++i) A.states_out[(size_t)env * 8 + i] = out8[i];
      if (A.done_out) A.done_out[env] = done ? 1 : 0;
      if (A.status_out) A.status_out[env] = status;
    }
  }
}

// C1: MultiShipNonIWEnv._step (run_colav/env.py:613-676) inside the run_simplified_model.py:245-249 loop, k ticks per
// launch (shipsim_tick). Two lanes per env (lane & 1 = ship); both ships follow fixed routes. Per tick, in the
// reference's order: the test ship's step (test_step :326-455: the SBMPC block when collav is sbmpc, control with the
// simple collision avoidance's +15° when imminent, one ship tick), then the obstacle ship's (obs_step :457-586: the
// same SBMPC block — its own LOS course and desired speed, the test ship's state after its tick as the own ship, the
// obstacle ship itself as the obstacle — then control and tick), each frozen ship storing its last row and advancing
// its clock twice instead; then get_env_info (:53-225, the flags of reward_function.py without the rewards) on the
// post-tick states and the stop flags (:658-664). The env's SBMPC memory (P_ca_last, Chi_ca_last) is one object that
// both ships' blocks update in turn. Event bits of the last tick to events_out.
// (its arguments as one struct read through the laundered kernarg pointer, as ast_step_kernel's StepArgs: a field is
// a scalar load where it is used, not ~100 dwords held in SGPRs across the tick loop, which spilled)
struct NoniwArgs {
  Params P;
  DevState S;
  ConstBuf K;
  int k;
  uint32_t* events_out;
};
typedef const __attribute__((address_space(4))) NoniwArgs* NoniwArgsPtr;
__device__ __forceinline__ const NoniwArgs& noniw_args() {
  NoniwArgsPtr q = (NoniwArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return *(const NoniwArgs*)q;
}
template <int COLLAV>
__global__ __launch_bounds__(64) void noniw_tick_kernel(NoniwArgs A_arg) {
  (void)A_arg;  // read through noniw_args()
#define P (noniw_args().P)
#define S (noniw_args().S)
#define K (noniw_args().K)
  const int k = noniw_args().k;
  __shared__ ShipConst lds_sc[SHIPSIM_MAX_SHIPS];
  __shared__ Edge lds_edges_raw[SHIPSIM_MAX_VERTS];
  __shared__ PolyBox lds_boxes[SHIPSIM_MAX_POLYS];
  const ShipConst* SC = stage_consts(K, lds_sc, P.n_ships, P.dt);
  for (int i = threadIdx.x; i < K.n_edges; i += blockDim.x) lds_edges_raw[i] = K.edges()[i];
  for (int i = threadIdx.x; i < P.n_polys; i += blockDim.x) lds_boxes[i] = K.boxes()[i];
  __syncthreads();
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int env = gl >> 1, ship = gl & 1;
  const bool is_test = ship == 0;
  const bool valid = env < P.n_envs;  // (invalid lanes run along: every lane takes part in the exchanges)
  const int envc = valid ? env : 0, qc = envc * 2 + ship;
  const ShipConst& c = SC[ship];
  const double* rn = S.route_n() + (size_t)qc * kMaxRoute;
  const double* re = S.route_e() + (size_t)qc * kMaxRoute;
  Ship s;
  load_ship(S, qc, s);
  double sy, cy;
  sincos(s.yaw, &sy, &cy);
  double p_last = S.p_last()[envc], chi_last = S.chi_last()[envc];
  float st[4];  // self.states (float32): test (n, e), obstacle (n, e) as the previous tick left them
  for (int i = 0; i < 4; ++i) st[i] = S.states4()[envc * 4 + i];
  const int n_samp = (int)(P.sbmpc_tf / P.sbmpc_dt);
  constexpr int kFlag = COLLAV == SHIPSIM_COLLAV_SIMPLE ? 2 : 0;  // the +15° avoidance (control_and_store)
  uint32_t bits = 0;
  for (int it = 0; it < k; ++it) {
    const float dn = st[0] - st[2], de = st[1] - st[3];
    const bool imminent = (dn * dn + de * de) < 9000000.0f;  // is_collision_imminent on self.states
    // one ship's step: its SBMPC block (need: the own ship within D_INIT of the obstacle) and control + tick
    auto ship_step = [&](int who, double os_n, double os_e, double os_v, double ob_n, double ob_e, double ob_yaw,
                         double ob_u, double ob_v) __attribute__((always_inline)) {
      const bool mine = ship == who;
      double sf = 1.0, off = 0.0;
      if constexpr (COLLAV == SHIPSIM_COLLAV_SBMPC) {
        const bool act = valid && mine && !s.stop;
        bool need = false;
        double los_arg = 0.0;
        if (act) {  // next_wpt's result discarded; los_guidance integrates e_ct_int (Q3)
          los_arg = los_update(c, s, s.n, s.e);
          const double d0 = ob_e - os_e, d1 = ob_n - os_n;
          need = sqrt_lt(d0 * d0 + d1 * d1, 2000.0);  // D_INIT_
        }
        double pb = 1.0, cb = 0.0;
        if (__any(need)) {
          SbIn in = SbIn{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
          in.u_d = SC[who].desired_speed;  // (every request of this pass is ship `who`'s: the same in each lane)
          in.obs_l = SC[1].obs_l_cfg; in.obs_w = SC[1].obs_w_cfg;
          if (need) {
            in.chi_d = -(s.seg_alpha + atan(los_arg));
            in.os_x = os_e; in.os_y = os_n; in.os_v = os_v;
            in.ob_x = ob_e; in.ob_y = ob_n; in.ob_psi = -ob_yaw; in.ob_u = ob_u; in.ob_v = ob_v;
            sb_set_heading_trig(in);
            in.p_last = p_last; in.chi_last = chi_last;
          }
          sbmpc_cooperative<true, true>(need, in, n_samp, P.sbmpc_dt, pb, cb);
        }
        if (act) {
          if (need) { p_last = pb; chi_last = cb; sf = pb; off = cb; }
          else { p_last = 1; chi_last = 0; }
        }
      }
      if (valid && mine) {
        if (s.stop) {  // store_last_simulation_data + two next_time
          s.time = s.time + P.dt;
          s.time = s.time + P.dt;
        } else {
          control_and_integrate_sc<false, false>(c, P, s, rn, re, -off, sf, 0.0, kFlag, imminent, nullptr, nullptr, sy,
                                                 cy);
        }
      }
    };
    {  // the test ship: the obstacle ship before it moves
      const double pn = pair_swap(s.n), pe = pair_swap(s.e), pyaw = pair_swap(s.yaw);
      const double pu = pair_swap(s.u), pv = pair_swap(s.v);
      ship_step(0, s.n, s.e, s.v, pn, pe, pyaw, pu, pv);
    }
    {  // the obstacle ship: the test ship after its tick, the env's SBMPC memory as the test ship's block left it
      const double tn = pair_swap(s.n), te = pair_swap(s.e), tv = pair_swap(s.v);
      const double pl = pair_swap(p_last), cl = pair_swap(chi_last);
      if (!is_test) { p_last = pl; chi_last = cl; }
      ship_step(1, tn, te, tv, s.n, s.e, s.yaw, s.u, s.v);
      const double pl2 = pair_swap(p_last), cl2 = pair_swap(chi_last);
      if (is_test) { p_last = pl2; chi_last = cl2; }
    }
    // get_env_info on the post-tick states (check_condition.py), both ships' own flags exchanged
    const double margin = c.l_ship / 2;
    const bool my_end = sqrt_le((s.n - s.end_n) * (s.n - s.end_n) + (s.e - s.end_e) * (s.e - s.end_e), 200.0);
    const bool my_out = (s.n < P.min_north + margin || s.n > P.max_north - margin) ||
                        (s.e < P.min_east + margin || s.e > P.max_east - margin);
    bool my_gr = false;
    for (int q = 0; q < 4; ++q) {
      const double cn = (q < 2) ? s.n - margin : s.n + margin;
      const double ce = (q & 1) ? s.e + margin : s.e - margin;
      if (corner_inside(K, lds_edges_raw, lds_boxes, P.n_polys, cn, ce)) my_gr = true;
    }
    const bool my_nav = fabs(s.log_ect) > (is_test ? 3000.0 : 500.0);  // is_tnav / is_onav (no travel tracker)
    const int my_flags = (my_end ? 1 : 0) | (my_out ? 2 : 0) | (my_gr ? 4 : 0) | (my_nav ? 8 : 0);
    const int o_flags = pair_swap_i(my_flags);
    const double on = pair_swap(s.n), oe = pair_swap(s.e);
    const int Tf = is_test ? my_flags : o_flags, Of = is_test ? o_flags : my_flags;
    const double cd = (s.n - on) * (s.n - on) + (s.e - oe) * (s.e - oe);
    const bool t10 = pair_swap(s.time) > P.sim_time;  // (the test ship's clock: read on its partner lane too)
    const bool t10_t = s.time > P.sim_time;
    const bool f[10] = {cd < 2500.0, (Tf & 4) != 0, (Tf & 8) != 0, (Of & 4) != 0, (Of & 8) != 0,
                        (Tf & 1) != 0, (Tf & 2) != 0, (Of & 1) != 0, (Of & 2) != 0, is_test ? t10_t : t10};
    bits = 0;
    for (int i = 0; i < 10; ++i)
      if (f[i]) bits |= 1u << i;
    if (bits & 0x1Fu) bits |= SHIPSIM_EV_TERMINAL;
    if (bits & 0x267u) bits |= SHIPSIM_EV_TEST_STOP;  // collision, test grounding / nav, test end / outside, time
    if (bits & 0x399u) bits |= SHIPSIM_EV_OBS_STOP;   // collision, obs grounding / nav, obs end / outside, time
    const bool terminal = bits & SHIPSIM_EV_TERMINAL;
    if (valid && !terminal && (bits & (is_test ? SHIPSIM_EV_TEST_STOP : SHIPSIM_EV_OBS_STOP))) s.stop = 1;
    const double Tn = is_test ? s.n : on, Te = is_test ? s.e : oe, On = is_test ? on : s.n, Oe = is_test ? oe : s.e;
    st[0] = (float)Tn; st[1] = (float)Te; st[2] = (float)On; st[3] = (float)Oe;
  }
  if (!valid) return;
  store_ship(S, qc, s);
  if (is_test) {
    S.p_last()[env] = p_last; S.chi_last()[env] = chi_last;
    for (int i = 0; i < 4; ++i) S.states4()[env * 4 + i] = st[i];
    uint32_t* events_out = noniw_args().events_out;
    if (events_out && k > 0) events_out[env] = bits;
  }
#undef P
#undef S
#undef K
}

// SBMPC.get_optimal_ctrl_offset (sbmpc.py:113-185) for a batch of independent single-obstacle
// requests (shipsim_sbmpc_eval): one request per lane, optimisations served wave-cooperatively.
__global__ __launch_bounds__(64) void sbmpc_eval_kernel(int n, double tf, double dt, const double* __restrict__ in,
                                                        double* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const bool valid = i < n;
  const double* r = in + (size_t)(valid ? i : 0) * SHIPSIM_SBMPC_IN;
  SbIn q;
  q.p_last = r[0]; q.chi_last = r[1]; q.u_d = r[2]; q.chi_d = r[3];
  q.os_x = r[4]; q.os_y = r[5]; q.os_v = r[8];  // os_state (x, y, psi, u, v, r): linear_pred uses x, y, v
  q.ob_x = r[10]; q.ob_y = r[11]; q.ob_psi = r[12]; q.ob_u = r[13]; q.ob_v = r[14];
  sb_set_heading_trig(q);
  q.obs_l = r[15]; q.obs_w = r[16];
  const double d0 = q.ob_x - q.os_x, d1 = q.ob_y - q.os_y;
  const bool active = valid && sqrt_lt(d0 * d0 + d1 * d1, 2000.0);  // D_INIT_ (sbmpc.py:154-159)
  double pb = 1.0, cb = 0.0;
  sbmpc_cooperative(active, q, (int)(tf / dt), dt, pb, cb);
  if (valid) {
    out[(size_t)i * 3 + 0] = active ? pb : 1.0;
    out[(size_t)i * 3 + 1] = active ? cb : 0.0;
    out[(size_t)i * 3 + 2] = active ? 1.0 : 0.0;
  }
}

// SBMPC.get_optimal_ctrl_offset over a do_list of n_obs obstacles (sbmpc.py:113-185) for n independent requests
// (shipsim_sbmpc_eval_multi): one request per lane, the optimisations served wave-cooperatively by the optimiser the
// multi-obstacle env kernels run (sbmpc_cooperative_multi)
__global__ __launch_bounds__(64) void sbmpc_multi_eval_kernel(int n, int n_obs, int n_samp, double dt,
                                                              const double* __restrict__ in, double* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const bool valid = i < n;
  const double* r = in + (size_t)(valid ? i : 0) * SHIPSIM_SBMPC_MULTI_IN;
  SbMulti<SHIPSIM_MAX_OBS> q;
  q.p_last = r[0]; q.chi_last = r[1]; q.u_d = r[2]; q.chi_d = r[3];
  q.os_x = r[4]; q.os_y = r[5]; q.os_v = r[8];  // os_state (x, y, psi, u, v, r): linear_pred uses x, y, v
  bool active = false;
#pragma unroll
  for (int k = 0; k < SHIPSIM_MAX_OBS; ++k) {
    const double* o = r + 10 + 7 * k;
    q.ob_x[k] = o[0]; q.ob_y[k] = o[1]; q.ob_psi[k] = o[2]; q.ob_u[k] = o[3]; q.ob_v[k] = o[4];
    q.obs_l[k] = o[5]; q.obs_w[k] = o[6];
    const double d0 = o[0] - q.os_x, d1 = o[1] - q.os_y;
    if (k < n_obs) active = active || sqrt_lt(d0 * d0 + d1 * d1, 2000.0);  // D_INIT_ (sbmpc.py:153-159)
  }
  active = valid && active;
  double pb = 1.0, cb = 0.0;
  sbmpc_cooperative_multi<SHIPSIM_MAX_OBS>(active, q, n_obs, n_samp, dt, pb, cb);  // (n_samp: int(tf / dt))
  if (valid) {
    out[(size_t)i * 3 + 0] = active ? pb : 1.0;
    out[(size_t)i * 3 + 1] = active ? cb : 0.0;
    out[(size_t)i * 3 + 2] = active ? 1.0 : 0.0;
  }
}

// shipsim_div_check: div_by with div_rcp (the kernels' division by a reused divisor) beside the plain division
__global__ __launch_bounds__(256) void div_check_kernel(int n, const double* __restrict__ num,
                                                        const double* __restrict__ den, double* __restrict__ fast,
                                                        double* __restrict__ ref) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double a = num[i], d = den[i];
  fast[i] = div_by(a, d, div_rcp(d));
  ref[i] = a / d;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct shipsim_handle {
  shipsim_config cfg;
  Params P;
  DevState S;
  ConstBuf K;
  int device;
  hipStream_t stream;
  void* dev_block;
  void* const_block;
  void* fuel_block;  // trajectory fuel accumulators
  int32_t* nonfinite_dev;   // device counter (DevState::nonfinite)
  int32_t nonfinite_seen;   // its value at the last shipsim_synchronize
  Traj T;
  size_t dev_bytes;
  int ever_reset;
  int lpe;  // lanes per AST env of the step / stream kernels (lanes_per_env)
  int32_t tail_extra;  // shipsim_set_stream_tail (0: off)
  int32_t* tail_ctr;   // its device counter (one int, zeroed before every stream launch)
  char err[512];
};

// ---------------------------------------------------------------------------------------------
// map grid (host): exact, conservative cell classification used by corner_inside / map_dist2_mask
// ---------------------------------------------------------------------------------------------
static const double kGridCell = 200.0;     // m
static const double kGridPad = 2000.0;     // m of grid beyond the polygon bounding box
static const double kGridEps = 1e-3;       // m: cells are enlarged by this before classification

// segment vs closed axis-aligned rectangle (Liang-Barsky clip)
static bool seg_hits_rect(const Edge& ed, double x0, double y0, double x1, double y1) {
  double t0 = 0.0, t1 = 1.0;
  const double dx = ed.bx - ed.ax, dy = ed.by - ed.ay;
  const double p[4] = {-dx, dx, -dy, dy};
  const double q[4] = {ed.ax - x0, x1 - ed.ax, ed.ay - y0, y1 - ed.ay};
  for (int i = 0; i < 4; ++i) {
    if (p[i] == 0.0) {
      if (q[i] < 0.0) return false;
    } else {
      const double t = q[i] / p[i];
      if (p[i] < 0.0) { if (t > t1) return false; if (t > t0) t0 = t; }
      else { if (t < t0) return false; if (t < t1) t1 = t; }
    }
  }
  return true;
}
static double point_seg_dist(double px, double py, const Edge& ed) {
  const double dx = ed.bx - ed.ax, dy = ed.by - ed.ay, l2 = dx * dx + dy * dy;
  double t = l2 > 0 ? ((px - ed.ax) * dx + (py - ed.ay) * dy) / l2 : 0.0;
  t = t < 0 ? 0 : (t > 1 ? 1 : t);
  const double ex = ed.ax + t * dx - px, ey = ed.ay + t * dy - py;
  return sqrt(ex * ex + ey * ey);
}
static double point_rect_dist(double px, double py, double x0, double y0, double x1, double y1) {
  const double dx = px < x0 ? x0 - px : (px > x1 ? px - x1 : 0.0);
  const double dy = py < y0 ? y0 - py : (py > y1 ? py - y1 : 0.0);
  return sqrt(dx * dx + dy * dy);
}
static double seg_rect_dist(const Edge& ed, double x0, double y0, double x1, double y1) {
  if (seg_hits_rect(ed, x0, y0, x1, y1)) return 0.0;
  double d = point_rect_dist(ed.ax, ed.ay, x0, y0, x1, y1);
  d = py_min(d, point_rect_dist(ed.bx, ed.by, x0, y0, x1, y1));
  d = py_min(d, point_seg_dist(x0, y0, ed));
  d = py_min(d, point_seg_dist(x1, y0, ed));
  d = py_min(d, point_seg_dist(x0, y1, ed));
  d = py_min(d, point_seg_dist(x1, y1, ed));
  return d;
}
// Fills mask/flag for a gnx x gny grid. A cell no edge touches is uniformly inside or outside
// (the polygons' boundary is the union of their edges), so its center decides it; any cell an
// edge touches is MIXED and gets the full test. Edge masks keep every edge within kGroundReach of
// the enlarged cell (+1 mm slack on the reach for rounding).
static void build_grid(const Edge* E, int n_edges, const PolyBox* B, int n_polys, double gx0, double gy0, int gnx,
                       int gny, uint64_t* mask, uint8_t* flag) {
  for (int j = 0; j < gny; ++j)
    for (int i = 0; i < gnx; ++i) {
      const double x0 = gx0 + i * kGridCell - kGridEps, x1 = gx0 + (i + 1) * kGridCell + kGridEps;
      const double y0 = gy0 + j * kGridCell - kGridEps, y1 = gy0 + (j + 1) * kGridCell + kGridEps;
      uint64_t m = 0;
      bool touched = false;
      for (int k = 0; k < n_edges; ++k) {
        const double d = seg_rect_dist(E[k], x0, y0, x1, y1);
        if (d <= kGroundReach + kGridEps) m |= (uint64_t)1 << k;
        if (d == 0.0) touched = true;
      }
      mask[(size_t)j * gnx + i] = m;
      const double cx = 0.5 * (x0 + x1), cy = 0.5 * (y0 + y1);
      flag[(size_t)j * gnx + i] = touched ? GRID_MIXED : (map_inside(E, B, n_polys, cy, cx) ? GRID_IN : GRID_OUT);
    }
}

static int fail(shipsim_handle* h, int code, const char* fmt, ...) {
  if (h) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(h->err, sizeof(h->err), fmt, ap);
    va_end(ap);
  }
  return code;
}

#define HIPCHK(h, x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) return fail(h, SHIPSIM_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Lanes per AST env. The kernels hold ~350-450 registers per lane, so a SIMD runs one wave and the
// throughput is (envs per wave) / (per-tick wave latency): pick the fewest lanes per env that still
// put a wave on every SIMD of the device (n_envs * LPE / 64 >= SIMDs), in [4, 16]. Measured on
// MI355X (profiles/round2_lpe_sweep.md): 4096 envs -> 16, 8192 -> 8 (1.5-1.8x over 16), 65536 -> 4
// (2.2-3.1x). cfg->lanes_per_env (or $SHIPSIM_LPE) overrides; results are identical at every LPE.
static int lanes_per_env(const shipsim_config* cfg, int n_envs, int device) {
  int lpe = cfg->lanes_per_env;
  if (lpe <= 0) {
    const char* e = getenv("SHIPSIM_LPE");
    lpe = e ? atoi(e) : 0;
  }
  if (lpe == 2 || lpe == 4 || lpe == 8 || lpe == 16) return lpe;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  const long simds = 4L * cus;
  lpe = 4;
  while (lpe < 16 && (long)n_envs * lpe < 64L * simds) lpe *= 2;
  return lpe;
}

// blocks (one wave each) of an AST step / stream launch at lpe lanes per env
static int step_blocks(const shipsim_handle* h, int lpe) {
  const int epw = h->P.epw > 0 && h->P.epw <= 64 / lpe ? h->P.epw : 64 / lpe;
  return (h->P.n_envs + epw - 1) / epw;
}

static StepArgs step_args_of(const shipsim_handle* h, const float* action, const uint8_t* active, int32_t max_ticks,
                            float* obs_out, double* reward_out, uint8_t* done_out, uint32_t* events_out,
                            int32_t* ticks_out, uint8_t* ready_out, const ChainArgs& ch) {
  StepArgs a;
  memset(&a, 0, sizeof(a));
  a.P = h->P; a.S = h->S; a.K = h->K; a.T = h->T;
  a.action = action; a.active_mask = active; a.max_ticks = max_ticks;
  a.obs_out = obs_out; a.reward_out = reward_out; a.done_out = done_out; a.events_out = events_out;
  a.ticks_out = ticks_out; a.ready_out = ready_out; a.CH = ch;
  return a;
}

template <bool D, int CA>
static void launch_step(shipsim_handle* h, int lpe, const float* action, const uint8_t* active, int32_t max_ticks,
                        float* obs_out, double* reward_out, uint8_t* done_out, uint32_t* events_out,
                        int32_t* ticks_out, uint8_t* ready_out) {
  const int threads = 64;
  if (h->T.ship) lpe = 16;  // recording kernels are built for the default layout only
  const int blocks = step_blocks(h, lpe);
#define L(LPE, REC)                                                                                              \
  hipLaunchKernelGGL((ast_step_kernel<D, CA, LPE, REC>), dim3(blocks), dim3(threads), 0, h->stream,            \
                     step_args_of(h, action, active, max_ticks, obs_out, reward_out, done_out, events_out, ticks_out, \
                                  ready_out, ChainArgs{}))
  if (h->T.ship) {
    L(16, true);
    return;
  }
  switch (lpe) {
    case 2: L(2, false); break;
    case 4: L(4, false); break;
    case 8: L(8, false); break;
    default: L(16, false); break;
  }
#undef L
}

// K > 1 obstacle ships (detailed machinery, collav none / sbmpc): 16 lanes per env in 4 or 8 ship slots
static int ship_slots(const shipsim_handle* h) { return h->P.n_ships <= 2 ? 2 : (h->P.n_ships <= 4 ? 4 : 8); }

template <int CA, int CHAIN>
static void launch_multi(shipsim_handle* h, const float* action, const uint8_t* active, int32_t max_ticks,
                         float* obs_out, double* reward_out, uint8_t* done_out, uint32_t* events_out,
                         int32_t* ticks_out, uint8_t* ready_out, const ChainArgs& ch) {
  const int threads = 64, blocks = step_blocks(h, 16);
#define LM(SL)                                                                                                         \
  hipLaunchKernelGGL((ast_step_kernel<true, CA, 16, false, CHAIN, SL>), dim3(blocks), dim3(threads), 0, h->stream,  \
                     step_args_of(h, action, active, max_ticks, obs_out, reward_out, done_out, events_out, ticks_out, \
                                  ready_out, ch))
  if (ship_slots(h) == 4) LM(4);
  else LM(8);
#undef LM
}

extern "C" {

int32_t shipsim_abi_version(void) { return SHIPSIM_ABI_VERSION; }

#ifdef SHIPSIM_PHASE_TIMING
// timing builds only (not part of the ABI): read and clear the per-phase cycle sums
int shipsim_debug_phase_cycles(unsigned long long* out8) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(diag::g_phase_cycles), sizeof(unsigned long long) * 8) != hipSuccess) return -2;
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(diag::g_phase_cycles), z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif

#ifndef SHIPSIM_SRC_HASH
#define SHIPSIM_SRC_HASH "unknown"
#endif
const char* shipsim_build_info(void) {
  return "shipsim gfx950 HIP (fp64, lane-pair AST kernel, wave-cooperative SBMPC) src " SHIPSIM_SRC_HASH;
}

static void fill_ship_common(shipsim_ship_config* s, double n, double e, double yaw, double u) {
  memset(s, 0, sizeof(*s));
  s->coefficient_of_deadweight_to_displacement = 0.7;
  s->bunkers = 200000;
  s->ballast = 200000;
  s->length_of_ship = 80;
  s->width_of_ship = 16;
  s->added_mass_coefficient_in_surge = 0.4;
  s->added_mass_coefficient_in_sway = 0.4;
  s->added_mass_coefficient_in_yaw = 0.4;
  s->dead_weight_tonnage = 3850000;
  s->mass_over_linear_friction_coefficient_in_surge = 130;
  s->mass_over_linear_friction_coefficient_in_sway = 18;
  s->mass_over_linear_friction_coefficient_in_yaw = 90;
  s->nonlinear_friction_coefficient_in_surge = 2400;
  s->nonlinear_friction_coefficient_in_sway = 4000;
  s->nonlinear_friction_coefficient_in_yaw = 400;
  s->initial_north_position_m = n;
  s->initial_east_position_m = e;
  s->initial_yaw_angle_rad = yaw;
  s->initial_forward_speed_m_per_s = u;
  s->rudder_angle_to_sway_force_coefficient = 50e3;
  s->rudder_angle_to_yaw_force_coefficient = 500e3;
  s->max_rudder_angle_degrees = 30;
  s->hotel_load = 200000;
  s->main_engine_capacity = 0;
  s->electrical_capacity = 2 * 510e3;
  s->shaft_generator_state = SHIPSIM_SG_MOTOR;
  s->rated_speed_main_engine_rpm = 1000;
  s->linear_friction_main_engine = 68;
  s->linear_friction_hybrid_shaft_generator = 57;
  s->gear_ratio_between_main_engine_and_propeller = 0.6;
  s->gear_ratio_between_hybrid_shaft_generator_and_propeller = 0.6;
  s->propeller_inertia = 6000;
  s->propeller_diameter = 3.1;
  s->propeller_speed_to_torque_coefficient = 7.5;
  s->propeller_speed_to_thrust_force_coefficient = 1.7;
  s->kp_ship_speed = 205.25;
  s->ki_ship_speed = 0.0525;
  s->kp_shaft_speed = 50;
  s->ki_shaft_speed = 0.00025;
  s->initial_shaft_speed_integral_error = 114;
  s->max_thrust = INFINITY;
  s->radius_of_acceptance = 300;
  s->lookahead_distance = 1000;
  s->los_integral_gain = 0.002;
  s->los_integrator_windup_limit = 4000;
}

static void set_route(shipsim_ship_config* s, const double (*r)[2], int n) {
  s->n_route = n;
  for (int i = 0; i < n; ++i) {
    s->route_north[i] = r[i][0];
    s->route_east[i] = r[i][1];
  }
}

int shipsim_default_config(int32_t kind, int32_t machinery, int32_t collav, double time_step, shipsim_config* cfg) {
  if (!cfg || kind < 0 || kind > 2 || machinery < 0 || machinery > 1 || collav < 0 || collav > 2) return SHIPSIM_EINVAL;
  static const double map_e_n[][2] = {
      {0, 10000}, {10000, 10000}, {9200, 9000}, {7600, 8500}, {6700, 7300}, {4900, 6500}, {4300, 5400},
      {4700, 4500}, {6000, 4000}, {5800, 3600}, {4200, 3200}, {3200, 4100}, {2000, 4500}, {1000, 4000},
      {900, 3500}, {500, 2600}, {0, 2350},
      {10000, 0}, {11500, 750}, {12000, 2000}, {11700, 3000}, {11000, 3600}, {11250, 4250}, {12300, 4000},
      {13000, 3800}, {14000, 3000}, {14500, 2300}, {15000, 1700}, {16000, 800}, {17500, 0},
      {15500, 10000}, {16000, 9000}, {18000, 8000}, {19000, 7500}, {20000, 6000}, {20000, 10000},
      {5500, 5300}, {6000, 5000}, {6800, 4500}, {8000, 5000}, {8700, 5500}, {9200, 6700}, {8000, 7000},
      {6700, 6300}, {6000, 6000},
      {15000, 5000}, {14000, 5500}, {12500, 5000}, {14000, 4100}, {16000, 2000}, {15700, 3700},
      {11000, 2000}, {10300, 3200}, {9000, 1500}, {10000, 1000}};
  static const int poly_counts[6] = {17, 13, 6, 9, 6, 4};
  static const double test_route[7][2] = {{0, 0}, {2000, 4500}, {2500, 7500}, {7000, 12000}, {6500, 16000},
                                          {3000, 17500}, {0, 20000}};
  static const double obs_route[2][2] = {{10000, 15000}, {0, 5000}};
  static const double obs_route_noniw[11][2] = {{10000, 15000}, {9500, 13500}, {8000, 13000}, {6500, 12500},
                                                {6000, 11000}, {5500, 9500}, {4000, 9000}, {2500, 8500},
                                                {2000, 7000}, {1500, 5500}, {0, 5000}};
  memset(cfg, 0, sizeof(*cfg));
  cfg->abi_version = SHIPSIM_ABI_VERSION;
  cfg->kind = kind;
  cfg->machinery = machinery;
  cfg->collav = collav;
  cfg->max_sampling_frequency = 9;
  cfg->machinery_dt_quirk = 1;
  cfg->normalize_action = 0;
  cfg->n_ships = kind == SHIPSIM_KIND_SINGLE ? 1 : 2;
  cfg->time_step = time_step;
  cfg->simulation_time = 10000;
  cfg->env_radius_of_acceptance = 300;
  cfg->current_velocity_component_from_north = -1;
  cfg->current_velocity_component_from_east = -1;
  cfg->wind_speed = 2;
  cfg->wind_direction = -M_PI / 4;
  cfg->sbmpc_tf = 1000;
  cfg->sbmpc_dt = 20;
  shipsim_ship_config* t = &cfg->ship[0];
  shipsim_ship_config* o = &cfg->ship[1];
  fill_ship_common(t, 100, 100, 60 * M_PI / 180, 4.25);
  fill_ship_common(o, 9900, 14900, -135 * M_PI / 180, 3.5);
  set_route(t, test_route, 7);
  t->desired_forward_speed = 4.5;
  o->desired_forward_speed = 4.0;
  if (kind == SHIPSIM_KIND_AST) {  // run/env_setup.py
    t->initial_propeller_shaft_speed_rad_per_s = 420 * M_PI / 30;
    o->initial_propeller_shaft_speed_rad_per_s = 200 * M_PI / 30;
    for (int i = 0; i < 2; ++i) {
      cfg->ship[i].heading_kp = 1.65; cfg->ship[i].heading_kd = 75; cfg->ship[i].heading_ki = 0.001;
      cfg->ship[i].speed_kp = 150; cfg->ship[i].speed_ki = 150; cfg->ship[i].speed_kd = 75;
    }
    set_route(o, obs_route, 2);
    cfg->action_low = (float)(-(30 * (M_PI / 180.0)));
    cfg->action_high = (float)(30 * (M_PI / 180.0));
  } else {  // run_colav/run_simplified_model.py
    t->speed_kp = 150; t->speed_ki = 150; t->speed_kd = 75;
    o->speed_kp = .025; o->speed_ki = 700.5; o->speed_kd = 550.5;
    t->heading_kp = .5; t->heading_ki = 0.01; t->heading_kd = 84;
    o->heading_kp = .65; o->heading_ki = 0.001; o->heading_kd = 50;
    set_route(o, obs_route_noniw, 11);
    cfg->action_low = (float)(-M_PI / 6);
    cfg->action_high = (float)(M_PI / 6);
  }
  int k = 0, p = 0;
  for (p = 0; p < 6; ++p) {
    cfg->poly_start[p] = k;
    for (int i = 0; i < poly_counts[p]; ++i, ++k) {
      cfg->poly_east[k] = map_e_n[k][0];
      cfg->poly_north[k] = map_e_n[k][1];
    }
  }
  cfg->poly_start[6] = k;
  cfg->n_polys = 6;
  return SHIPSIM_OK;
}

// host restatement of the constructors' derived constants (ship_model.py:412-474,
// ship_engine.py:32-44, 341-401)
static void make_ship_const(const shipsim_config* cfg, const shipsim_ship_config* c, ShipConst* k) {
  memset(k, 0, sizeof(*k));
  double payload = 0.9 * (c->dead_weight_tonnage - c->bunkers);
  double lsw = c->dead_weight_tonnage / c->coefficient_of_deadweight_to_displacement - c->dead_weight_tonnage;
  k->mass = lsw + payload + c->bunkers + c->ballast;
  k->l_ship = c->length_of_ship;
  k->w_ship = c->width_of_ship;
  k->obs_l_cfg = c->length_of_ship;
  k->obs_w_cfg = c->width_of_ship;
  k->i_z = k->mass * (k->l_ship * k->l_ship + k->w_ship * k->w_ship) / 12;
  k->x_du = k->mass * c->added_mass_coefficient_in_surge;
  k->y_dv = k->mass * c->added_mass_coefficient_in_sway;
  k->n_dr = k->i_z * c->added_mass_coefficient_in_yaw;
  k->inv_m0 = 1.0 / (k->mass + k->x_du);
  k->inv_m1 = 1.0 / (k->mass + k->y_dv);
  k->inv_m2 = 1.0 / (k->i_z + k->n_dr);
  k->dlin0 = k->mass / c->mass_over_linear_friction_coefficient_in_surge;
  k->dlin1 = k->mass / c->mass_over_linear_friction_coefficient_in_sway;
  k->dlin2 = k->i_z / c->mass_over_linear_friction_coefficient_in_yaw;
  k->ku = c->nonlinear_friction_coefficient_in_surge;
  k->kv = c->nonlinear_friction_coefficient_in_sway;
  k->kr = c->nonlinear_friction_coefficient_in_yaw;
  k->rho_a = 1.2;
  k->proj_area_f = k->w_ship * 8.0;
  k->proj_area_l = k->l_ship * 8.0;
  k->cx = 0.5;
  k->cy = 0.7;
  k->cn = 0.08;
  k->c_rudder_v = c->rudder_angle_to_sway_force_coefficient;
  k->c_rudder_r = c->rudder_angle_to_yaw_force_coefficient;
  k->max_rudder = c->max_rudder_angle_degrees * M_PI / 180;
  double me = c->main_engine_capacity, el = c->electrical_capacity, hl = c->hotel_load;
  if (c->shaft_generator_state == SHIPSIM_SG_MOTOR) {
    k->avail_me = me;
    k->avail_el = el - hl;
  } else if (c->shaft_generator_state == SHIPSIM_SG_GEN) {
    k->avail_me = me - hl;
    k->avail_el = 0;
  } else {
    k->avail_me = me;
    k->avail_el = 0;
  }
  k->cap_me = k->avail_me / 5 * M_PI / 30;
  k->cap_el = k->avail_el / 5 * M_PI / 30;
  k->d_me = c->linear_friction_main_engine;
  k->d_hsg = c->linear_friction_hybrid_shaft_generator;
  k->r_me = c->gear_ratio_between_main_engine_and_propeller;
  k->r_hsg = c->gear_ratio_between_hybrid_shaft_generator_and_propeller;
  k->jp = c->propeller_inertia;
  k->kp_prop = c->propeller_speed_to_torque_coefficient;
  k->thrust_coeff = pow(c->propeller_diameter, 4) * c->propeller_speed_to_thrust_force_coefficient;
  k->shaft_speed_max = 1.1 * (c->rated_speed_main_engine_rpm * M_PI / 30) * k->r_me;
  k->init_omega = c->initial_propeller_shaft_speed_rad_per_s;
  k->mode_me = me;
  k->mode_el = el;
  k->hotel = hl;
  k->avail_prop = (c->shaft_generator_state == SHIPSIM_SG_MOTOR) ? me + el - hl
                  : (c->shaft_generator_state == SHIPSIM_SG_GEN) ? me - hl : me;  // :32-44
  k->sg_state = c->shaft_generator_state;
  // run/env_setup.py:85-104: SpecificFuelConsumptionWartila6L26 (ME) / Baudouin6M26Dot3 (DG),
  // ship_engine.py:88-112 (BaseMachineryModel.fuel_consumption uses these, not the
  // ShipMachineryModel.specific_fuel_coeffs_* literals)
  k->fa_me = 128.9; k->fb_me = -168.9; k->fc_me = 246.8;
  k->fa_dg = 108.7; k->fb_dg = -289.9; k->fc_dg = 324.9;
  k->kp_ship_speed = c->kp_ship_speed;
  k->ki_ship_speed = c->ki_ship_speed;
  k->kp_shaft_speed = c->kp_shaft_speed;
  k->ki_shaft_speed = c->ki_shaft_speed;
  k->init_shaft_ei = c->initial_shaft_speed_integral_error;
  k->spd_kp = c->speed_kp;
  k->spd_ki = c->speed_ki;
  k->spd_kd = c->speed_kd;
  k->max_thrust = c->max_thrust;
  k->hdg_kp = c->heading_kp;
  k->hdg_kd = c->heading_kd;
  k->hdg_ki = c->heading_ki;
  k->ra2 = c->radius_of_acceptance * c->radius_of_acceptance;
  k->los_r = c->lookahead_distance;
  k->los_r2 = c->lookahead_distance * c->lookahead_distance;
  k->los_ki = c->los_integral_gain;
  k->los_limit = c->los_integrator_windup_limit;
  k->desired_speed = c->desired_forward_speed;
  k->init_n = c->initial_north_position_m;
  k->init_e = c->initial_east_position_m;
  k->init_yaw = c->initial_yaw_angle_rad;
  k->init_u = c->initial_forward_speed_m_per_s;
  k->init_v = c->initial_sideways_speed_m_per_s;
  k->init_r = c->initial_yaw_rate_rad_per_s;
  k->n_route = c->n_route;
  (void)cfg;
}

static int validate(const shipsim_config* cfg, char* err, size_t n) {
  if (cfg->abi_version != SHIPSIM_ABI_VERSION) return snprintf(err, n, "abi_version %d != %d", cfg->abi_version, SHIPSIM_ABI_VERSION), 1;
  if (cfg->kind < 0 || cfg->kind > 2) return snprintf(err, n, "bad kind %d", cfg->kind), 1;
  if (cfg->machinery < 0 || cfg->machinery > 1) return snprintf(err, n, "bad machinery %d", cfg->machinery), 1;
  if (cfg->collav < 0 || cfg->collav > 2) return snprintf(err, n, "bad collav %d", cfg->collav), 1;
  int ns = cfg->kind == SHIPSIM_KIND_SINGLE ? 1 : 2;
  if (cfg->kind == SHIPSIM_KIND_AST) {
    ns = cfg->n_ships;
    if (ns < 2 || ns > SHIPSIM_MAX_SHIPS)
      return snprintf(err, n, "n_ships %d: 1 ship under test + 1..%d obstacle ships", ns, SHIPSIM_MAX_OBS), 1;
    if (ns > 2 && (cfg->machinery != SHIPSIM_MACH_DETAILED || cfg->collav == SHIPSIM_COLLAV_SIMPLE))
      return snprintf(err, n, "%d obstacle ships: detailed machinery and collav none / sbmpc only", ns - 1), 1;
  }
  if (cfg->n_ships != ns) return snprintf(err, n, "n_ships %d != %d for kind %d", cfg->n_ships, ns, cfg->kind), 1;
  if (!(cfg->time_step > 0)) return snprintf(err, n, "time_step must be > 0"), 1;
  if (cfg->max_sampling_frequency < 0 || cfg->max_sampling_frequency + 2 > SHIPSIM_MAX_ROUTE)
    return snprintf(err, n, "max_sampling_frequency %d out of range", cfg->max_sampling_frequency), 1;
  for (int i = 0; i < ns; ++i) {
    int nr = cfg->ship[i].n_route;
    if (nr < 2 || nr > SHIPSIM_MAX_ROUTE) return snprintf(err, n, "ship %d route length %d out of range", i, nr), 1;
    if (cfg->kind == SHIPSIM_KIND_AST && i == 1 && nr + cfg->max_sampling_frequency > SHIPSIM_MAX_ROUTE)
      return snprintf(err, n, "obstacle route %d + samplings %d exceeds %d", nr, cfg->max_sampling_frequency, SHIPSIM_MAX_ROUTE), 1;
  }
  if (cfg->n_polys < 0 || cfg->n_polys > SHIPSIM_MAX_POLYS) return snprintf(err, n, "n_polys %d out of range", cfg->n_polys), 1;
  if (cfg->poly_start[0] != 0 || cfg->poly_start[cfg->n_polys] > SHIPSIM_MAX_VERTS)
    return snprintf(err, n, "bad poly_start"), 1;
  for (int p = 0; p < cfg->n_polys; ++p)
    if (cfg->poly_start[p + 1] - cfg->poly_start[p] < 3) return snprintf(err, n, "polygon %d has < 3 vertices", p), 1;
  if (cfg->sbmpc_dt <= 0 || cfg->sbmpc_tf / cfg->sbmpc_dt > 4096) return snprintf(err, n, "bad sbmpc horizon"), 1;
  return 0;
}

// message of this thread's last failed shipsim_create (shipsim_last_error(NULL)); set on every failing path
static thread_local char g_create_err[512];

int shipsim_create(const shipsim_config* cfg_in, int32_t n_envs, int32_t n_obs_ships, int32_t device, void* stream,
                   shipsim_handle** out) {
  g_create_err[0] = 0;
  if (!cfg_in || !out || n_envs <= 0) {
    snprintf(g_create_err, sizeof(g_create_err), "shipsim_create: %s", !cfg_in ? "config is NULL" : !out ? "out is NULL"
             : "n_envs must be > 0");
    return SHIPSIM_EINVAL;
  }
  *out = nullptr;
  shipsim_handle* h = new (std::nothrow) shipsim_handle();
  if (!h) {
    snprintf(g_create_err, sizeof(g_create_err), "shipsim_create: out of host memory");
    return SHIPSIM_ENOMEM;
  }
  memset(h, 0, sizeof(*h));
  h->cfg = *cfg_in;
  if (n_obs_ships > 0 && h->cfg.kind == SHIPSIM_KIND_AST) h->cfg.n_ships = 1 + n_obs_ships;
  const shipsim_config* cfg = &h->cfg;
  if (validate(cfg, h->err, sizeof(h->err))) {
    snprintf(g_create_err, sizeof(g_create_err), "%s", h->err);
    delete h;
    return SHIPSIM_EINVAL;
  }
  h->device = device;
  h->stream = (hipStream_t)stream;
  DeviceGuard g(device);
  h->lpe = cfg->n_ships > 2 ? 16 : lanes_per_env(cfg, n_envs, device);  // K > 1: 16 lanes in ship slots
  Params& P = h->P;
  memset(&P, 0, sizeof(P));
  P.epw = cfg->envs_per_wave;  // performance knob (0 = full waves; results identical)
  const int ns = cfg->n_ships;
  ShipConst sc[SHIPSIM_MAX_SHIPS];
  memset(sc, 0, sizeof(sc));
  for (int i = 0; i < ns; ++i) make_ship_const(cfg, &cfg->ship[i], &sc[i]);
  P.kind = cfg->kind;
  P.machinery = cfg->machinery;
  P.collav = cfg->collav;
  P.n_ships = ns;
  P.max_sampling = cfg->max_sampling_frequency;
  P.n_envs = n_envs;
  P.n_polys = cfg->n_polys;
  P.dt = cfg->time_step;
  P.sim_time = cfg->simulation_time;
  P.mach_dt_init = cfg->time_step;
  P.mach_dt_reset = cfg->machinery_dt_quirk ? 0.01 : cfg->time_step;
  P.vc_n = cfg->current_velocity_component_from_north;
  P.vc_e = cfg->current_velocity_component_from_east;
  P.wind_dir = cfg->wind_direction;
  P.wind_speed = cfg->wind_speed;
  P.roa2 = cfg->env_radius_of_acceptance * cfg->env_radius_of_acceptance;
  P.sbmpc_tf = cfg->sbmpc_tf;
  P.sbmpc_nsamp = (int32_t)(cfg->sbmpc_tf / cfg->sbmpc_dt);
  P.sbmpc_dt = cfg->sbmpc_dt;
  P.wind_sin = sin(cfg->wind_direction);
  P.wind_cos = cos(cfg->wind_direction);
  P.action_low = cfg->action_low;
  P.action_high = cfg->action_high;
  P.normalize_action = cfg->normalize_action;
  if (ns >= 2) {  // init_get_intermediate_waypoints env.py:143-161 (ship 1 samples)
    const shipsim_ship_config* o = &cfg->ship[1];
    double ABn = o->route_north[o->n_route - 1] - o->route_north[0];
    double ABe = o->route_east[o->n_route - 1] - o->route_east[0];
    int msf = cfg->max_sampling_frequency;
    double AB_length = sqrt(ABn * ABn + ABe * ABe);
    P.AB_seg = AB_length / (msf + 1);
    P.AB_seg_n = ABn / (msf + 1);
    P.AB_seg_e = ABe / (msf + 1);
    double AB_alpha = atan2(ABe, ABn);
    double AB_beta = M_PI / 2 - AB_alpha;
    P.omega_iw = M_PI / 2 - AB_beta;
    P.iw_cos = cos(P.omega_iw);  // np.cos / np.sin of the scalar omega (env.py:226-227): glibc, as NumPy
    P.iw_sin = sin(P.omega_iw);
    P.n_base0 = P.AB_seg_n + o->route_north[0];
    P.e_base0 = P.AB_seg_e + o->route_east[0];
    P.initial_states[0] = (float)cfg->ship[0].initial_north_position_m;
    P.initial_states[1] = (float)cfg->ship[0].initial_east_position_m;
    P.initial_states[2] = 0.0f;
    P.initial_states[3] = (float)o->initial_north_position_m;
    P.initial_states[4] = (float)o->initial_east_position_m;
    P.initial_states[5] = (float)o->initial_yaw_angle_rad;
    P.initial_states[6] = 0.0f;
    P.initial_states[7] = (float)o->initial_forward_speed_m_per_s;
  }
  // map
  int nv = cfg->poly_start[cfg->n_polys];
  double mn_e = cfg->poly_east[0], mx_e = mn_e, mn_n = cfg->poly_north[0], mx_n = mn_n;
  for (int i = 0; i < nv; ++i) {
    if (cfg->poly_east[i] < mn_e) mn_e = cfg->poly_east[i];
    if (cfg->poly_east[i] > mx_e) mx_e = cfg->poly_east[i];
    if (cfg->poly_north[i] < mn_n) mn_n = cfg->poly_north[i];
    if (cfg->poly_north[i] > mx_n) mx_n = cfg->poly_north[i];
  }
  P.min_east = mn_e; P.max_east = mx_e; P.min_north = mn_n; P.max_north = mx_n;

  // constant block: edges | boxes | config routes | grid (ConstBuf layout)
  const bool use_grid = nv <= 64 && nv > 0 && cfg->map_query == SHIPSIM_MAP_GRID;
  const int gnx = use_grid ? (int)ceil((mx_e - mn_e + 2 * kGridPad) / kGridCell) : 0;
  const int gny = use_grid ? (int)ceil((mx_n - mn_n + 2 * kGridPad) / kGridCell) : 0;
  const size_t gcells = (size_t)gnx * gny;
  const size_t grid_off = (ConstBuf::kBytes + 255) & ~(size_t)255;
  const size_t part_off = (grid_off + gcells * (sizeof(uint64_t) + 1) + 7) & ~(size_t)7;
  size_t cbytes = part_off + gcells * 8 * sizeof(uint64_t);
  char* hostc = (char*)calloc(1, cbytes);
  Edge* E = (Edge*)hostc;
  PolyBox* B = (PolyBox*)(hostc + sizeof(Edge) * SHIPSIM_MAX_VERTS);
  double* R = (double*)(hostc + sizeof(Edge) * SHIPSIM_MAX_VERTS + sizeof(PolyBox) * SHIPSIM_MAX_POLYS);
  for (int p = 0; p < cfg->n_polys; ++p) {
    int s0 = cfg->poly_start[p], cnt = cfg->poly_start[p + 1] - s0;
    B[p].first = s0;
    B[p].count = cnt;
    B[p].minx = B[p].maxx = cfg->poly_east[s0];
    B[p].miny = B[p].maxy = cfg->poly_north[s0];
    for (int i = 0; i < cnt; ++i) {
      int j = (i + 1 == cnt) ? 0 : i + 1;
      E[s0 + i].ax = cfg->poly_east[s0 + i];
      E[s0 + i].ay = cfg->poly_north[s0 + i];
      E[s0 + i].bx = cfg->poly_east[s0 + j];
      E[s0 + i].by = cfg->poly_north[s0 + j];
      if (E[s0 + i].ax < B[p].minx) B[p].minx = E[s0 + i].ax;
      if (E[s0 + i].ax > B[p].maxx) B[p].maxx = E[s0 + i].ax;
      if (E[s0 + i].ay < B[p].miny) B[p].miny = E[s0 + i].ay;
      if (E[s0 + i].ay > B[p].maxy) B[p].maxy = E[s0 + i].ay;
    }
  }
  for (int s = 0; s < ns; ++s)
    for (int i = 0; i < cfg->ship[s].n_route; ++i) {
      R[s * kMaxRoute + i] = cfg->ship[s].route_north[i];
      R[SHIPSIM_MAX_SHIPS * kMaxRoute + s * kMaxRoute + i] = cfg->ship[s].route_east[i];
    }
  memcpy(hostc + ConstBuf::kShipsOff, sc, sizeof(ShipConst) * SHIPSIM_MAX_SHIPS);
  if (use_grid) {
    build_grid(E, nv, B, cfg->n_polys, mn_e - kGridPad, mn_n - kGridPad, gnx, gny, (uint64_t*)(hostc + grid_off),
               (uint8_t*)(hostc + grid_off + gcells * sizeof(uint64_t)));
    const uint64_t* gm = (const uint64_t*)(hostc + grid_off);
    uint64_t* gp = (uint64_t*)(hostc + part_off);
    for (size_t c = 0; c < gcells; ++c) {
      int rank = 0;
      for (int k = 0; k < 64; ++k)
        if (gm[c] >> k & 1) gp[c * 8 + (rank++ & 7)] |= (uint64_t)1 << k;
    }
  }
  hipError_t e = hipMalloc(&h->const_block, cbytes);
  if (e != hipSuccess) {
    free(hostc);
    int rc = fail(h, SHIPSIM_EHIP, "hipMalloc(const): %s", hipGetErrorString(e));
    *out = h;
    return rc;
  }
  e = hipMemcpy(h->const_block, hostc, cbytes, hipMemcpyHostToDevice);
  free(hostc);
  if (e != hipSuccess) {
    *out = h;
    return fail(h, SHIPSIM_EHIP, "hipMemcpy(const): %s", hipGetErrorString(e));
  }
  h->K.base = (const char*)h->const_block;
  h->K.n_edges = nv;
  h->K.gnx = gnx;
  h->K.gny = gny;
  h->K.gx0 = mn_e - kGridPad;
  h->K.gy0 = mn_n - kGridPad;
  h->K.ginv = 1.0 / kGridCell;
  h->K.grid_mask = use_grid ? (const uint64_t*)((const char*)h->const_block + grid_off) : nullptr;
  h->K.grid_flag = use_grid ? (const uint8_t*)((const char*)h->const_block + grid_off + gcells * sizeof(uint64_t))
                            : nullptr;
  h->K.grid_part = use_grid ? (const uint64_t*)((const char*)h->const_block + part_off) : nullptr;

  // state block (DevState layout: ship arrays | routes | env arrays)
  const size_t S = (size_t)n_envs * ns, N = (size_t)n_envs;
  auto r256 = [](size_t b) { return (b + 255) & ~(size_t)255; };
  h->S.ship_stride = (int64_t)r256(S * sizeof(double));
  h->S.route_stride = (int64_t)r256(S * kMaxRoute * sizeof(double));
  h->S.env_stride = (int64_t)r256(N * 8 * sizeof(float));
  h->S.env_off = DevState::kShipArrays * h->S.ship_stride + 2 * h->S.route_stride;
  size_t bytes = (size_t)(h->S.env_off + DevState::kEnvArrays * h->S.env_stride);
  e = hipMalloc(&h->dev_block, bytes);
  if (e != hipSuccess) {
    *out = h;
    return fail(h, SHIPSIM_EHIP, "hipMalloc(state %zu B): %s", bytes, hipGetErrorString(e));
  }
  h->dev_bytes = bytes;
  h->S.base = (char*)h->dev_block;
  e = hipMalloc(&h->nonfinite_dev, sizeof(int32_t));
  if (e != hipSuccess) {
    *out = h;
    return fail(h, SHIPSIM_EHIP, "hipMalloc(counter): %s", hipGetErrorString(e));
  }
  h->S.nonfinite = h->nonfinite_dev;
  (void)hipMemsetAsync(h->nonfinite_dev, 0, sizeof(int32_t), h->stream);
  e = hipMemsetAsync(h->dev_block, 0, bytes, h->stream);
  if (e != hipSuccess) {
    *out = h;
    return fail(h, SHIPSIM_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
  }
  int threads = 256, blocks = (int)((S + threads - 1) / threads);
  hipLaunchKernelGGL(init_kernel, dim3(blocks), dim3(threads), 0, h->stream, h->P, h->S, h->K);
  e = hipGetLastError();
  *out = h;
  if (e != hipSuccess) return fail(h, SHIPSIM_EHIP, "init_kernel: %s", hipGetErrorString(e));
  return SHIPSIM_OK;
}

int shipsim_destroy(shipsim_handle* h) {
  if (!h) return SHIPSIM_EINVAL;
  {
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    else (void)hipDeviceSynchronize();
    if (h->dev_block) (void)hipFree(h->dev_block);
    if (h->const_block) (void)hipFree(h->const_block);
    if (h->fuel_block) (void)hipFree(h->fuel_block);
    if (h->nonfinite_dev) (void)hipFree(h->nonfinite_dev);
    if (h->tail_ctr) (void)hipFree(h->tail_ctr);
  }
  delete h;
  return SHIPSIM_OK;
}

const char* shipsim_last_error(const shipsim_handle* h) { return h ? h->err : g_create_err; }

int shipsim_set_stream(shipsim_handle* h, void* stream) {
  if (!h) return SHIPSIM_EINVAL;
  h->stream = (hipStream_t)stream;
  return SHIPSIM_OK;
}
int32_t shipsim_num_envs(const shipsim_handle* h) { return h ? h->P.n_envs : -1; }
int32_t shipsim_lanes_per_env(const shipsim_handle* h) { return h ? h->lpe : -1; }

int shipsim_reset(shipsim_handle* h, const uint8_t* env_mask, float* obs_out) {
  if (!h || !h->dev_block) return SHIPSIM_EINVAL;
  if (h->P.kind < SHIPSIM_KIND_SINGLE || h->P.kind > SHIPSIM_KIND_AST)
    return fail(h, SHIPSIM_EINVAL, "reset: kind %d not supported on device", h->P.kind);
  DeviceGuard g(h->device);
  int S = h->P.n_envs * h->P.n_ships, threads = 256, blocks = (S + threads - 1) / threads;
  const bool rec = h->T.ship != nullptr;
#define RL(D, REC) \
  hipLaunchKernelGGL((reset_kernel<D, REC>), dim3(blocks), dim3(threads), 0, h->stream, h->P, h->S, h->K, h->T, env_mask, obs_out)
  if (h->P.machinery == SHIPSIM_MACH_DETAILED) {
    if (rec) RL(true, true); else RL(true, false);
  } else {
    if (rec) RL(false, true); else RL(false, false);
  }
#undef RL
  HIPCHK(h, hipGetLastError());
  h->ever_reset = 1;
  return SHIPSIM_OK;
}

int shipsim_step(shipsim_handle* h, const float* action, const uint8_t* active, int32_t max_ticks, float* obs_out,
                 double* reward_out, uint8_t* done_out, uint32_t* events_out, int32_t* ticks_out,
                 uint8_t* ready_out) {
  if (!h || !h->dev_block) return SHIPSIM_EINVAL;
  if (h->P.kind != SHIPSIM_KIND_AST) return fail(h, SHIPSIM_EINVAL, "step: only SHIPSIM_KIND_AST has decision steps");
  if (!action) return fail(h, SHIPSIM_EINVAL, "step: action is NULL");
  if (!h->ever_reset) return fail(h, SHIPSIM_ESTATE, "step before reset");
  DeviceGuard g(h->device);
  const int lpe = h->lpe;
  const bool det = h->P.machinery == SHIPSIM_MACH_DETAILED;
#define LAUNCH(D, CA) launch_step<D, CA>(h, lpe, action, active, max_ticks, obs_out, reward_out, done_out, events_out, ticks_out, ready_out)
#ifdef SHIPSIM_REGCHECK  // register-usage inspection builds (scripts/regcheck.sh): headline kernels only
  (void)lpe; (void)det;
#if SHIPSIM_REGCHECK == 3  // the multi-obstacle (K > 1) kernels
  if (h->P.collav == SHIPSIM_COLLAV_SBMPC)
    launch_multi<SHIPSIM_COLLAV_SBMPC, 0>(h, action, active, max_ticks, obs_out, reward_out, done_out, events_out,
                                          ticks_out, ready_out, ChainArgs{});
  else
    launch_multi<SHIPSIM_COLLAV_NONE, 0>(h, action, active, max_ticks, obs_out, reward_out, done_out, events_out,
                                         ticks_out, ready_out, ChainArgs{});
#endif
  return fail(h, SHIPSIM_EINVAL, "REGCHECK build");
#else
  if (ship_slots(h) > 2) {
    if (h->P.collav == SHIPSIM_COLLAV_SBMPC)
      launch_multi<SHIPSIM_COLLAV_SBMPC, 0>(h, action, active, max_ticks, obs_out, reward_out, done_out,
                                                events_out, ticks_out, ready_out, ChainArgs{});
    else
      launch_multi<SHIPSIM_COLLAV_NONE, 0>(h, action, active, max_ticks, obs_out, reward_out, done_out,
                                               events_out, ticks_out, ready_out, ChainArgs{});
    HIPCHK(h, hipGetLastError());
    return SHIPSIM_OK;
  }
  switch (h->P.collav) {
    case SHIPSIM_COLLAV_NONE: if (det) LAUNCH(true, 0); else LAUNCH(false, 0); break;
    case SHIPSIM_COLLAV_SIMPLE: if (det) LAUNCH(true, 1); else LAUNCH(false, 1); break;
    default: if (det) LAUNCH(true, 2); else LAUNCH(false, 2); break;
  }
#endif
#undef LAUNCH
  HIPCHK(h, hipGetLastError());
  return SHIPSIM_OK;
}

int shipsim_tick(shipsim_handle* h, int32_t k, uint32_t* events_out) {
  if (!h || !h->dev_block || k < 0) return SHIPSIM_EINVAL;
  if (h->P.kind != SHIPSIM_KIND_SINGLE && h->P.kind != SHIPSIM_KIND_NONIW)
    return fail(h, SHIPSIM_EINVAL, "tick: device raw ticks for SHIPSIM_KIND_SINGLE and SHIPSIM_KIND_NONIW");
  if (k == 0) return SHIPSIM_OK;
  DeviceGuard g(h->device);
  if (h->P.kind == SHIPSIM_KIND_NONIW) {  // two lanes per env
    if (h->P.machinery != SHIPSIM_MACH_SIMPLIFIED)
      return fail(h, SHIPSIM_EINVAL, "tick: KIND_NONIW runs the simplified machinery (run_colav SimpleShipModel)");
    const int blocks = (2 * h->P.n_envs + 63) / 64;
#define NT(CA) \
  hipLaunchKernelGGL(noniw_tick_kernel<CA>, dim3(blocks), dim3(64), 0, h->stream, NoniwArgs{h->P, h->S, h->K, k, events_out})
    if (h->P.collav == SHIPSIM_COLLAV_SBMPC) NT(SHIPSIM_COLLAV_SBMPC);
    else if (h->P.collav == SHIPSIM_COLLAV_SIMPLE) NT(SHIPSIM_COLLAV_SIMPLE);
    else NT(SHIPSIM_COLLAV_NONE);
#undef NT
    HIPCHK(h, hipGetLastError());
    return SHIPSIM_OK;
  }
  const int threads = 64, blocks = (h->P.n_envs + threads - 1) / threads;
  if (h->P.machinery == SHIPSIM_MACH_DETAILED)
    hipLaunchKernelGGL(single_tick_kernel<true>, dim3(blocks), dim3(threads), 0, h->stream, h->P, h->S, h->K, k);
  else if (diag::kC2OneWave)  // (comparison builds: the one-wave form)
    hipLaunchKernelGGL(single_tick_kernel<false>, dim3(blocks), dim3(threads), 0, h->stream, h->P, h->S, h->K, k);
  else
    shipsim_c2_pipe_launch(blocks, h->stream, h->P, h->S, h->K, k);
  HIPCHK(h, hipGetLastError());
  return SHIPSIM_OK;
}

}  // extern "C"

// the launch tail is used when it is on and every wave of the launch is resident at once (one 64-thread block per
// wave): a wave that is not resident yet would only start after the resident ones ran their whole extension
static bool tail_on(const shipsim_handle* h, const void* kern, int blocks) {
  if (h->tail_extra <= 0 || !h->tail_ctr) return false;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) return false;
  return (int64_t)blocks <= (int64_t)per_cu * cus;
}

// the decision-stream launch shared by shipsim_run_table (MODE 1) and shipsim_run_policy (MODE 2)
template <int MODE>
static int run_chain(shipsim_handle* h, const ChainArgs& ch, int32_t max_ticks, int32_t* ticks_out) {
  DeviceGuard g(h->device);
  // lanes per env: 16 (default) or 8 / 4 (more envs per wave when the handle holds more envs than
  // the chip has SIMD slots at 16; identical results)
  const int lpe = (h->lpe == 8 || h->lpe == 4) ? h->lpe : (h->lpe == 2 ? 4 : 16);
  const int threads = 64, blocks = step_blocks(h, lpe);
#define CHAINED_L(D, CA, LPE)                                                                                      \
  do {                                                                                                             \
    const void* kern_ = reinterpret_cast<const void*>(&ast_step_kernel<D, CA, LPE, false, MODE>);                 \
    ChainArgs c_ = ch;                                                                                             \
    if (tail_on(h, kern_, blocks)) {                                                                               \
      (void)hipMemsetAsync(h->tail_ctr, 0, sizeof(int32_t), h->stream);                                            \
      c_.tail_ctr = h->tail_ctr;                                                                                   \
      c_.tail_extra = h->tail_extra;                                                                               \
      c_.tail_waves = blocks;                                                                                      \
    }                                                                                                              \
    hipLaunchKernelGGL((ast_step_kernel<D, CA, LPE, false, MODE>), dim3(blocks), dim3(threads), 0, h->stream,    \
                       step_args_of(h, nullptr, nullptr, max_ticks, nullptr, nullptr, nullptr, nullptr, ticks_out, \
                                    nullptr, c_));                                                                 \
  } while (0)
#define CHAINED(D, CA)                              \
  do {                                              \
    if (lpe == 8) CHAINED_L(D, CA, 8);              \
    else if (lpe == 4) CHAINED_L(D, CA, 4);         \
    else CHAINED_L(D, CA, 16);                      \
  } while (0)
  const bool det = h->P.machinery == SHIPSIM_MACH_DETAILED;
#ifdef SHIPSIM_REGCHECK
#if SHIPSIM_REGCHECK == 2  // the LPE-8 stream kernels (the C4 shard's collector)
  if (det) CHAINED_L(true, SHIPSIM_COLLAV_SBMPC, 8);
  else CHAINED_L(false, SHIPSIM_COLLAV_SBMPC, 8);
#elif SHIPSIM_REGCHECK == 3  // the multi-obstacle decision stream
  (void)det;
  if (MODE == 1)
    launch_multi<SHIPSIM_COLLAV_SBMPC, 1>(h, nullptr, nullptr, max_ticks, nullptr, nullptr, nullptr, nullptr, ticks_out,
                                          nullptr, ch);
#else
  if (h->P.collav == SHIPSIM_COLLAV_SBMPC) CHAINED_L(true, SHIPSIM_COLLAV_SBMPC, 16);
  else CHAINED_L(true, SHIPSIM_COLLAV_NONE, 16);
  (void)det;
#endif
#else
  if (MODE == 1 && ship_slots(h) > 2) {  // (run_policy refuses K > 1 before it gets here)
    if (h->P.collav == SHIPSIM_COLLAV_SBMPC)
      launch_multi<SHIPSIM_COLLAV_SBMPC, 1>(h, nullptr, nullptr, max_ticks, nullptr, nullptr, nullptr, nullptr,
                                            ticks_out, nullptr, ch);
    else
      launch_multi<SHIPSIM_COLLAV_NONE, 1>(h, nullptr, nullptr, max_ticks, nullptr, nullptr, nullptr, nullptr,
                                           ticks_out, nullptr, ch);
    HIPCHK(h, hipGetLastError());
    return SHIPSIM_OK;
  }
  switch (h->P.collav) {
    case SHIPSIM_COLLAV_SBMPC: if (det) CHAINED(true, SHIPSIM_COLLAV_SBMPC); else CHAINED(false, SHIPSIM_COLLAV_SBMPC); break;
    case SHIPSIM_COLLAV_SIMPLE: if (det) CHAINED(true, SHIPSIM_COLLAV_SIMPLE); else CHAINED(false, SHIPSIM_COLLAV_SIMPLE); break;
    default: if (det) CHAINED(true, SHIPSIM_COLLAV_NONE); else CHAINED(false, SHIPSIM_COLLAV_NONE); break;
  }
#endif
#undef CHAINED
#undef CHAINED_L
  HIPCHK(h, hipGetLastError());
  return SHIPSIM_OK;
}

extern "C" {

int shipsim_run_table(shipsim_handle* h, const float* table, int32_t n_eps, int32_t n_dec, int32_t max_ticks,
                      int32_t* ep_idx, int32_t* dec_idx, int32_t* ticks_out, int32_t* decisions_out, double* log,
                      int32_t log_cap, int32_t* log_len) {
  if (!h || !h->dev_block || !table || !ep_idx || !dec_idx || n_eps < 1 || n_dec < 1 || max_ticks < 1 ||
      (log && (!log_len || log_cap < 1)))
    return SHIPSIM_EINVAL;
  if (h->P.kind != SHIPSIM_KIND_AST) return fail(h, SHIPSIM_EINVAL, "run_table: AST kind only");
  if (h->T.ship) return fail(h, SHIPSIM_EINVAL, "run_table: trajectory recording is on (use shipsim_step)");
  ChainArgs ch = {};
  ch.table = table; ch.n_eps = n_eps; ch.n_dec = n_dec; ch.ep_idx = ep_idx; ch.dec_idx = dec_idx;
  ch.decisions = decisions_out; ch.log = log; ch.log_len = log_len; ch.log_cap = log_cap;
  return run_chain<1>(h, ch, max_ticks, ticks_out);
}

int shipsim_run_policy(shipsim_handle* h, const float* policy, const float* w2t, int32_t obs_dim, int32_t hidden,
                       int32_t deterministic, uint64_t seed, const int64_t* counter, int32_t n_dec,
                       int32_t max_ticks, int32_t* ep_idx, int32_t* dec_idx, int32_t* ticks_out,
                       int32_t* decisions_out, double* log, int32_t log_cap, int32_t* log_len) {
  if (!h || !h->dev_block || !policy || !w2t || !ep_idx || !dec_idx || n_dec < 1 || max_ticks < 1 ||
      (log && (!log_len || log_cap < 1)) || (!deterministic && !counter))
    return SHIPSIM_EINVAL;
  if (h->P.kind != SHIPSIM_KIND_AST) return fail(h, SHIPSIM_EINVAL, "run_policy: AST kind only");
  if (h->T.ship) return fail(h, SHIPSIM_EINVAL, "run_policy: trajectory recording is on (use shipsim_step)");
  if (obs_dim != 8) return fail(h, SHIPSIM_EINVAL, "run_policy: observation dim %d (the AST observation has 8)", obs_dim);
  if (hidden < 64 || hidden > kPolMaxHidden || hidden % 64)
    return fail(h, SHIPSIM_EINVAL, "run_policy: hidden %d (a multiple of 64 up to 512)", hidden);
  if (ship_slots(h) > 2) return fail(h, SHIPSIM_EINVAL, "run_policy: one obstacle ship only");
  ChainArgs ch = {};
  ch.n_eps = 1; ch.n_dec = n_dec; ch.ep_idx = ep_idx; ch.dec_idx = dec_idx;
  ch.decisions = decisions_out; ch.log = log; ch.log_len = log_len; ch.log_cap = log_cap;
  ch.log_stop = log ? 1 : 0;
  ch.policy = policy; ch.w2t = w2t; ch.pol_obs = obs_dim; ch.pol_hidden = hidden; ch.pol_det = deterministic ? 1 : 0;
  ch.pol_seed = seed; ch.pol_counter = counter;
  return run_chain<2>(h, ch, max_ticks, ticks_out);
}

int shipsim_set_stream_tail(shipsim_handle* h, int32_t extra_ticks) {
  if (!h || extra_ticks < 0) return SHIPSIM_EINVAL;
  if (extra_ticks > 0 && !h->tail_ctr) {
    DeviceGuard g(h->device);
    HIPCHK(h, hipMalloc(&h->tail_ctr, sizeof(int32_t)));
  }
  h->tail_extra = extra_ticks;
  return SHIPSIM_OK;
}

int shipsim_legacy_step(shipsim_handle* h, int32_t k, double* states_out, uint8_t* done_out, uint32_t* status_out) {
  if (!h || !h->dev_block || k < 0) return SHIPSIM_EINVAL;
  if (h->P.kind != SHIPSIM_KIND_AST) return fail(h, SHIPSIM_EINVAL, "legacy_step: AST kind only");
  if (h->P.n_ships != 2) return fail(h, SHIPSIM_EINVAL, "legacy_step: the legacy MultiShipEnv has one obstacle ship");
  if (k == 0) return SHIPSIM_OK;
  DeviceGuard g(h->device);
  const int threads = 64, blocks = (2 * h->P.n_envs + threads - 1) / threads;
  const LegacyArgs la{h->P, h->S, h->K, k, states_out, done_out, status_out};
#define LEGACY(D, CA) hipLaunchKernelGGL((legacy_step_kernel<D, CA>), dim3(blocks), dim3(threads), 0, h->stream, la)
  const bool det = h->P.machinery == SHIPSIM_MACH_DETAILED;
#ifdef SHIPSIM_REGCHECK
  (void)det;
  return fail(h, SHIPSIM_EINVAL, "REGCHECK build");
#else
  switch (h->P.collav) {
    case SHIPSIM_COLLAV_SBMPC: if (det) LEGACY(true, SHIPSIM_COLLAV_SBMPC); else LEGACY(false, SHIPSIM_COLLAV_SBMPC); break;
    case SHIPSIM_COLLAV_SIMPLE: if (det) LEGACY(true, SHIPSIM_COLLAV_SIMPLE); else LEGACY(false, SHIPSIM_COLLAV_SIMPLE); break;
    default: if (det) LEGACY(true, SHIPSIM_COLLAV_NONE); else LEGACY(false, SHIPSIM_COLLAV_NONE); break;
  }
#endif
#undef LEGACY
  HIPCHK(h, hipGetLastError());
  return SHIPSIM_OK;
}

static int field_ptr(shipsim_handle* h, int32_t field, void** p, size_t* bytes) {
  const size_t S = (size_t)h->P.n_envs * h->P.n_ships, N = (size_t)h->P.n_envs;
  if (field >= 0 && field < SHIPSIM_N_SHIP_FIELDS) {
    if (field == SHIPSIM_F_NEXT_WPT) { *p = h->S.next_wpt(); *bytes = S * 4; return 0; }
    if (field == SHIPSIM_F_STOP) { *p = h->S.stop(); *bytes = S * 4; return 0; }
    *p = h->S.f(field); *bytes = S * 8;
    return 0;
  }
  switch (field) {
    case SHIPSIM_E_SAMPLING_COUNT: *p = h->S.sampling_count(); *bytes = N * 4; return 0;
    case SHIPSIM_E_TRAVEL_DIST: *p = h->S.travel_dist(); *bytes = N * 8; return 0;
    case SHIPSIM_E_TRAVEL_TIME: *p = h->S.travel_time(); *bytes = N * 8; return 0;
    case SHIPSIM_E_ACC_REWARD: *p = h->S.acc(); *bytes = N * 8; return 0;
    case SHIPSIM_E_N_BASE: *p = h->S.n_base(); *bytes = N * 8; return 0;
    case SHIPSIM_E_E_BASE: *p = h->S.e_base(); *bytes = N * 8; return 0;
    case SHIPSIM_E_SBMPC_P_LAST: *p = h->S.p_last(); *bytes = N * 8; return 0;
    case SHIPSIM_E_SBMPC_CHI_LAST: *p = h->S.chi_last(); *bytes = N * 8; return 0;
    case SHIPSIM_E_ROUTE_LEN: *p = h->S.n_route(); *bytes = S * 4; return 0;
    case SHIPSIM_E_ROUTE_NORTH: *p = h->S.route_n(); *bytes = S * kMaxRoute * 8; return 0;
    case SHIPSIM_E_ROUTE_EAST: *p = h->S.route_e(); *bytes = S * kMaxRoute * 8; return 0;
  }
  return 1;
}

int shipsim_get_state(shipsim_handle* h, int32_t field, void* dst) {
  if (!h || !dst) return SHIPSIM_EINVAL;
  void* p;
  size_t b;
  if (field_ptr(h, field, &p, &b)) return fail(h, SHIPSIM_EINVAL, "unknown field %d", field);
  DeviceGuard g(h->device);
  HIPCHK(h, hipMemcpyAsync(dst, p, b, hipMemcpyDefault, h->stream));
  return SHIPSIM_OK;
}

int shipsim_set_state(shipsim_handle* h, int32_t field, const void* src) {
  if (!h || !src) return SHIPSIM_EINVAL;
  void* p;
  size_t b;
  if (field_ptr(h, field, &p, &b)) return fail(h, SHIPSIM_EINVAL, "unknown field %d", field);
  DeviceGuard g(h->device);
  HIPCHK(h, hipMemcpyAsync(p, src, b, hipMemcpyDefault, h->stream));
  return SHIPSIM_OK;
}

int shipsim_set_trajectory(shipsim_handle* h, double* ship_rows, double* env_rows, int32_t capacity,
                           int32_t* lengths) {
  if (!h || !h->dev_block) return SHIPSIM_EINVAL;
  if (h->P.kind != SHIPSIM_KIND_AST) return fail(h, SHIPSIM_EINVAL, "set_trajectory: SHIPSIM_KIND_AST only");
  if (h->P.n_ships != 2 && ship_rows) return fail(h, SHIPSIM_EINVAL, "set_trajectory: one obstacle ship only");
  if (!ship_rows) {
    memset(&h->T, 0, sizeof(h->T));
    return SHIPSIM_OK;
  }
  if (capacity <= 0 || !lengths) return fail(h, SHIPSIM_EINVAL, "set_trajectory: capacity %d / lengths", capacity);
  DeviceGuard g(h->device);
  const size_t fb = (size_t)h->P.n_envs * h->P.n_ships * 3 * sizeof(double);
  if (!h->fuel_block) HIPCHK(h, hipMalloc(&h->fuel_block, fb));
  HIPCHK(h, hipMemsetAsync(h->fuel_block, 0, fb, h->stream));
  HIPCHK(h, hipMemsetAsync(lengths, 0, (size_t)h->P.n_envs * sizeof(int32_t), h->stream));
  h->T.ship = ship_rows;
  h->T.env = env_rows;
  h->T.fuel = (double*)h->fuel_block;
  h->T.len = lengths;
  h->T.cap = capacity;
  return SHIPSIM_OK;
}

int shipsim_sbmpc_eval(int32_t n, double tf, double dt, const double* in, double* out, void* stream) {
  if (n < 0 || (n > 0 && (!in || !out)) || !(dt > 0) || tf / dt > 4096) return SHIPSIM_EINVAL;
  if (n == 0) return SHIPSIM_OK;
  hipLaunchKernelGGL(sbmpc_eval_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, tf, dt, in, out);
  return hipGetLastError() == hipSuccess ? SHIPSIM_OK : SHIPSIM_EHIP;
}

int shipsim_sbmpc_eval_multi(int32_t n, int32_t n_obs, double tf, double dt, const double* in, double* out,
                             void* stream) {
  if (n < 0 || n_obs < 1 || n_obs > SHIPSIM_MAX_OBS || (n > 0 && (!in || !out)) || !(dt > 0) || tf / dt > 4096)
    return SHIPSIM_EINVAL;
  if (n == 0) return SHIPSIM_OK;
  hipLaunchKernelGGL(sbmpc_multi_eval_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, n_obs,
                     (int)(tf / dt), dt, in, out);
  return hipGetLastError() == hipSuccess ? SHIPSIM_OK : SHIPSIM_EHIP;
}

int shipsim_div_check(int32_t n, const double* num, const double* den, double* fast, double* ref, void* stream) {
  if (n < 0 || (n > 0 && (!num || !den || !fast || !ref))) return SHIPSIM_EINVAL;
  if (n == 0) return SHIPSIM_OK;
  hipLaunchKernelGGL(div_check_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, num, den, fast,
                     ref);
  return hipGetLastError() == hipSuccess ? SHIPSIM_OK : SHIPSIM_EHIP;
}

int shipsim_synchronize(shipsim_handle* h) {
  if (!h) return SHIPSIM_EINVAL;
  DeviceGuard g(h->device);
  if (h->stream) HIPCHK(h, hipStreamSynchronize(h->stream));
  else HIPCHK(h, hipDeviceSynchronize());
  if (h->nonfinite_dev) {
    int32_t n = 0;
    HIPCHK(h, hipMemcpy(&n, h->nonfinite_dev, sizeof(n), hipMemcpyDeviceToHost));
    if (n > h->nonfinite_seen) {
      const int32_t fresh = n - h->nonfinite_seen;
      h->nonfinite_seen = n;
      return fail(h, SHIPSIM_ENONFINITE,
                  "%d env decision(s) ended on a non-finite ship state since the last synchronize (%d in all): "
                  "flagged SHIPSIM_EV_NONFINITE, done", fresh, n);
    }
  }
  return SHIPSIM_OK;
}

int32_t shipsim_nonfinite_count(const shipsim_handle* h) { return h ? h->nonfinite_seen : -1; }

int shipsim_diag_lane_faults(uint32_t* out32) {
  if (!out32) return SHIPSIM_EINVAL;
  for (int i = 0; i < 32; ++i) out32[i] = 0;
#ifdef SHIPSIM_LANECHECK
  if (hipDeviceSynchronize() != hipSuccess) return SHIPSIM_EHIP;
  if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(diag::g_lane_diag), 32 * sizeof(uint32_t)) != hipSuccess) return SHIPSIM_EHIP;
  const uint32_t zero[32] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(diag::g_lane_diag), zero, sizeof(zero)) != hipSuccess) return SHIPSIM_EHIP;
  return SHIPSIM_OK;
#elif defined(SHIPSIM_SB_STATS)
  if (hipDeviceSynchronize() != hipSuccess) return SHIPSIM_EHIP;
  if (hipMemcpyFromSymbol(out32 + 16, HIP_SYMBOL(diag::g_sb_stats), 8 * sizeof(uint64_t)) != hipSuccess)
    return SHIPSIM_EHIP;
  const uint64_t zero[8] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(diag::g_sb_stats), zero, sizeof(zero)) != hipSuccess) return SHIPSIM_EHIP;
  return SHIPSIM_OK;
#else
  return SHIPSIM_EINVAL;  // not a diagnostics build
#endif
}

}  // extern "C"
#endif  // SHIPSIM_TU != 2
