// shipsim_device.hpp — CDNA4 (gfx950) device code of the batched ship-in-transit simulator.
//
// Lane mapping: one ship per lane. Two-ship envs (AST) occupy an adjacent lane pair
// (lane 2e = ship under test, lane 2e+1 = obstacle ship), so both ships of an env advance in
// the same VALU instructions and exchange what the reward / termination logic needs through
// one DPP quad-permute (no LDS). Single-ship envs (C2) use one lane per env.
// All state is fp64 (the reference is NumPy float64) and lives in registers for the whole
// launch; HBM sees one coalesced SoA read at launch start and one write at the end.
//
// Every function restates the reference function cited next to it (paths relative to the
// reference root, AndreasKing-Goks/ast-sac @ 2025-09-05). Operation order follows the
// reference expression by expression (compiled with -ffp-contract=off) so that results differ
// from the NumPy reference only through libm ulps.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "shipsim.h"
#include "shipsim_diag.hpp"

namespace shipsim {

constexpr double kPi = 3.141592653589793;
constexpr int kMaxRoute = SHIPSIM_MAX_ROUTE;

// ---------------------------------------------------------------------------------------------
// constants (computed once on the host, identical arithmetic to the reference constructors)
// ---------------------------------------------------------------------------------------------
struct ShipConst {
  // BaseShipModel.__init__ (ship_model.py:412-474)
  double mass, i_z, x_du, y_dv, n_dr;
  double inv_m0, inv_m1, inv_m2;    // inv(mass_matrix()) diagonal (x_g = 0)
  double dlin0, dlin1, dlin2;       // linear_damping_matrix diagonal: mass/t_surge, mass/t_sway, i_z/t_yaw
  double ku, kv, kr;
  double l_ship, w_ship, obs_l_cfg, obs_w_cfg;  // ship_config.length/width (SBMPC do_list)
  double rho_a, proj_area_f, proj_area_l, cx, cy, cn;
  double c_rudder_v, c_rudder_r, max_rudder;
  // ShipMachineryModel (ship_engine.py:341-443) with the active MachineryMode
  double avail_me, avail_el, cap_me, cap_el;   // available powers; torque caps avail/5*pi/30
  double d_me, d_hsg, r_me, r_hsg, jp, kp_prop, thrust_coeff, shaft_speed_max;
  double init_omega;
  // MachineryMode.distribute_load / BaseMachineryModel.fuel_consumption (ship_engine.py:46-76, 259-295):
  // logging only (trajectory recording); capacities of the active mode, hotel load, fuel coefficients
  double mode_me, mode_el, hotel, avail_prop;
  double fa_me, fb_me, fc_me, fa_dg, fb_dg, fc_dg;
  int32_t sg_state, pad_sg_;
  // controllers (controllers.py:45-209; run_colav ThrustFromSpeedSetPoint)
  double kp_ship_speed, ki_ship_speed, kp_shaft_speed, ki_shaft_speed, init_shaft_ei;
  double spd_kp, spd_ki, spd_kd, max_thrust;
  double hdg_kp, hdg_kd, hdg_ki;
  // NavigationSystem (LOS_guidance.py:38-58)
  double ra2, los_r, los_r2, los_ki, los_limit;
  double desired_speed;
  // SimulationConfiguration
  double init_n, init_e, init_yaw, init_u, init_v, init_r;
  int32_t n_route, pad_;
  // filled on the device by stage_consts (the host leaves them 0): div_rcp of r_me, r_hsg, jp and of the step dt
  double rcp_r_me, rcp_r_hsg, rcp_jp, rcp_dt;
};

// fp64 division with the divisor's reciprocal formed once. The compiler's n / d is
//   y = div_rcp(d) (v_rcp_f64 + two Newton steps on d), q0 = n·y, rem = fma(−d, q0, n), q = fma(rem, y, q0),
//   then v_div_fixup(q, d, n), with v_div_scale pre-scaling both operands only near the ends of the exponent range;
// div_by runs the same operations with y computed once for a divisor that is reused (a constant of the ship, or
// one denominator of two quotients). The same bits as n / d whenever v_div_scale leaves the operands unscaled:
// finite d with 2^-1021 < |d| < 2^1021 (so 1/d is normal), |n| > 2^-969 or n = 0, and |n / d| normal — every
// divisor and quotient of the ship model (scripts/div_check.hip checks the identity on the device).
__device__ __forceinline__ double div_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}
__device__ __forceinline__ double div_by(double n, double d, double y) {
  const double q0 = n * y;
  const double rem = fma(-d, q0, n);
  return __builtin_amdgcn_div_fixup(fma(rem, y, q0), d, n);
}

struct Params {
  int32_t kind, machinery, collav, n_ships;
  int32_t max_sampling, n_envs, n_polys;
  int32_t epw;  // envs per wave of the AST step / stream kernels (0: 64 / lanes per env; fewer leave lanes idle)
  double dt, sim_time, mach_dt_reset, mach_dt_init;
  double vc_n, vc_e, wind_dir, wind_speed;
  double roa2;                       // args.radius_of_acceptance ** 2
  double sbmpc_tf, sbmpc_dt;
  // IW sampler (env.py:143-161), identical for every env of a handle
  double AB_seg, AB_seg_n, AB_seg_e, omega_iw, n_base0, e_base0;
  double min_north, max_north, min_east, max_east;
  float action_low, action_high;
  int32_t normalize_action, sbmpc_nsamp;  // sbmpc_nsamp = int(sbmpc_tf / sbmpc_dt) (sbmpc.py:121), host-evaluated
  float initial_states[8];           // env.py:107-109
  // host-evaluated sin/cos of uniform angles: wind_direction (algebraic wind force of the AST
  // kernels) and the IW sampler's omega (env.py:151-161)
  double wind_sin, wind_cos, iw_cos, iw_sin;
};

// Map edges (obstacle.py PolygonObstacle). Stored as a flat read-only device table; every lane
// walks it with the same (wave-uniform) index, so loads are scalar/broadcast.
struct Edge {
  double ax, ay, bx, by;   // (east, north) of the edge endpoints
};
struct PolyBox {
  double minx, maxx, miny, maxy;
  int32_t first, count, pad0, pad1;
};

// ---------------------------------------------------------------------------------------------
// register-resident ship state
// ---------------------------------------------------------------------------------------------
struct Ship {
  double n, e, yaw, u, v, r, omega, time;
  double e_ct, e_ct_int;          // navigate
  double hdg_ei, hdg_prev;        // heading PID
  double spd_a, spd_b;            // ship-speed PI ei | thrust PID ei ; shaft PI ei | thrust PID prev
  double log_rudder, log_thrust, log_ect, log_n, log_e;  // simulation_results[-1]
  double wp_prev_n, wp_prev_e, wp_n, wp_e;  // navigate.north/east[k-1], [k] (register cache)
  double seg_alpha, seg_sin, seg_cos;        // atan2 / sincos of the cached segment (los_guidance)
  double end_n, end_e;            // navigate.north/east[-1]
  int32_t next_wpt, n_route, stop;
};

__device__ __forceinline__ double sel(bool c, double a, double b) { return c ? a : b; }

// Python min/max semantics: min(a, b) returns a unless b < a
__host__ __device__ __forceinline__ double py_min(double a, double b) { return (b < a) ? b : a; }
__host__ __device__ __forceinline__ double py_max(double a, double b) { return (b > a) ? b : a; }
__device__ __forceinline__ double sat(double v, double lo, double hi) { return py_max(lo, py_min(v, hi)); }

// np.remainder / Python float % (floored)
__device__ __forceinline__ double floor_mod(double a, double b) {
  // fmod is exact; for b > 0 and |a| < 2b it is a, a - b or a + b, each exact by Sterbenz' lemma
  // (b <= |a| <= 2b), so the library call is only needed for larger ratios.
  double m;
  if (b > 0 && a > -2 * b && a < 2 * b) {
    m = (a >= b) ? a - b : ((a <= -b) ? a + b : a);
  } else {
    m = fmod(a, b);
  }
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}
// sbmpc_misc.py:20-32
__device__ __forceinline__ double wrap_pmpi(double x) { return -kPi + floor_mod(x - (-kPi), kPi - (-kPi)); }

// DPP moves of a double / int inside a 16-lane row (an AST env at LPE 16 is exactly one row, and
// every lane of an env shares its control flow, so every source lane is active)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, false);
  hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false); }
constexpr int kDppRowBcast = 0x150;  // row_newbcast:k (0x150 + k): lane k of the row to the whole row
constexpr int kDppRowRor4 = 0x124;   // row_ror:4
constexpr int kDppRowRor8 = 0x128;   // row_ror:8
constexpr int kDppQuadXor2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int kDppQuadXor1 = 0xB1;   // quad_perm [1,0,3,2]

// swap a double with the partner lane (lane ^ 1) — DPP quad_perm [1,0,3,2]
__device__ __forceinline__ double pair_swap(double x) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
  hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int pair_swap_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }

// ---------------------------------------------------------------------------------------------
// ship model: ship_model.py BaseShipModel / ShipModelAST, run_colav SimpleShipModel
// ---------------------------------------------------------------------------------------------
struct Deriv {
  double dn, de, dyaw, du, dv, dr, domega;
};

// swap a double with the lane two below/above (lane ^ 2) — DPP quad_perm [2,3,0,1]: in the AST
// lane layout (lane = env*LPE + 2*sub + ship) this pairs sub-lanes 2k and 2k+1 of the same ship
__device__ __forceinline__ double sub_pair_swap(double x) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false);
  hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// sincos of two angles: with PAIRED, sub-lane pairs of a ship evaluate one each in a single call
// (`odd` = odd sub-lane) and exchange the results; the values are those of two separate calls.
template <bool PAIRED>
__device__ __forceinline__ void sincos2(double a, double b, bool odd, double& sa, double& ca, double& sb, double& cb) {
  if (PAIRED) {
    double s_, c_;
    sincos(odd ? b : a, &s_, &c_);
    const double so = sub_pair_swap(s_), co = sub_pair_swap(c_);
    sa = odd ? so : s_; ca = odd ? co : c_;
    sb = odd ? s_ : so; cb = odd ? c_ : co;
  } else {
    sincos(a, &sa, &ca);
    sincos(b, &sb, &cb);
  }
}

// get_wind_force :497-517 (sw, cw = sin/cos(wind_direction - yaw))
template <bool PAIRED>
__device__ __forceinline__ void wind_force(const ShipConst& c, const Params& P, const Ship& s, double sw, double cw,
                                           bool odd, double tau[3]) {
  if constexpr (diag::kNoWind) {  // (ablation build only)
    tau[0] = tau[1] = tau[2] = 0.0;
    return;
  }
  double uw = P.wind_speed * cw;
  double vw = P.wind_speed * sw;
  double u_rw = uw - s.u;
  double v_rw = vw - s.v;
  double gamma_rw = -atan2(v_rw, u_rw);
  double wind_rw2 = u_rw * u_rw + v_rw * v_rw;
  double sg, cg, s2g, c2g;
  sincos2<PAIRED>(gamma_rw, 2 * gamma_rw, odd, sg, cg, s2g, c2g);  // sin(2 * gamma_rw) as sincos(.).sin
  (void)c2g;
  double c_x = -c.cx * cg;
  double c_y = c.cy * sg;
  double c_n = c.cn * s2g;
  double tau_coeff = 0.5 * c.rho_a * wind_rw2;
  tau[0] = tau_coeff * c_x * c.proj_area_f;
  tau[1] = tau_coeff * c_y * c.proj_area_l;
  tau[2] = tau_coeff * c_n * c.proj_area_l * c.l_ship;
}

// get_wind_force with the reference's angles eliminated algebraically (the C2 single-ship kernel):
// sin/cos(wind_direction - yaw) by the difference formulas from (sy, cy) = sin/cos(yaw) and
// (wsin, wcos) = sin/cos(wind_direction); with gamma_rw = -atan2(v_rw, u_rw) and V = |V_rw|,
// cos(gamma) = u_rw / V, sin(gamma) = -v_rw / V, sin(2 gamma) = -2 u_rw v_rw / V^2, so
//   tau = (-0.5 rho cx A_f u_rw V, -0.5 rho cy A_l v_rw V, -rho cn A_l L u_rw v_rw):
// one sqrt instead of atan2 and three sincos; equal to wind_force up to rounding (V = 0 gives 0).
__device__ __forceinline__ void wind_force_alg(const ShipConst& c, const Params& P, const Ship& s, double sy,
                                               double cy, double wsin, double wcos, double tau[3]) {
  if constexpr (diag::kNoWind) {  // (ablation build only)
    tau[0] = tau[1] = tau[2] = 0.0;
    return;
  }
  const double cw = wcos * cy + wsin * sy;
  const double sw = wsin * cy - wcos * sy;
  const double u_rw = P.wind_speed * cw - s.u;
  const double v_rw = P.wind_speed * sw - s.v;
  const double V = sqrt(u_rw * u_rw + v_rw * v_rw);
  const double h = 0.5 * c.rho_a;
  tau[0] = -(h * c.cx * c.proj_area_f) * (u_rw * V);
  tau[1] = -(h * c.cy * c.proj_area_l) * (v_rw * V);
  tau[2] = -(c.rho_a * c.cn * c.proj_area_l * c.l_ship) * (u_rw * v_rw);
}

// update_differentials (ShipModelAST :882-888 / SimpleShipModel run_colav :399-404):
// three_dof_kinematics :519-528, shaft_eq + thrust (ship_engine.py:403-443), three_dof_kinetics
// :834-864 with rudder :866-880. `ctrl` is the engine throttle (detailed) or thrust force (simplified);
// (sy, cy) = sin/cos(yaw), tau = get_wind_force.
__device__ __forceinline__ Deriv differentials_body(const ShipConst& c, const Params& P, const Ship& s, double ctrl,
                                                    double delta, bool detailed, double sy, double cy,
                                                    const double tau[3]) {
  Deriv d;
  d.dn = cy * s.u + (-sy) * s.v + 0 * s.r;
  d.de = sy * s.u + cy * s.v + 0 * s.r;
  d.dyaw = 0 * s.u + 0 * s.v + 1 * s.r;
  double thrust = ctrl;
  d.domega = 0.0;
  if (detailed) {
    // main_engine_torque / hsg_torque :416-432
    // (the divisions by the ship's constants, and the two by one denominator, with the reciprocals formed once)
    const double den = s.omega + 0.1, y_den = div_rcp(den);
    double t_me = py_min(div_by(ctrl * c.avail_me, den, y_den), c.cap_me);
    double t_hsg = py_min(div_by(ctrl * c.avail_el, den, y_den), c.cap_el);
    double eq_me = div_by(t_me - c.d_me * s.omega, c.r_me, c.rcp_r_me);
    double eq_hsg = div_by(t_hsg - c.d_hsg * s.omega, c.r_hsg, c.rcp_r_hsg);
    d.domega = div_by(eq_me + eq_hsg - c.kp_prop * (s.omega * s.omega), c.jp, c.rcp_jp);
    thrust = c.thrust_coeff * s.omega * fabs(s.omega);
  }
  // inv(rotation()) @ vel_c
  double vc0 = cy * P.vc_n + sy * P.vc_e;
  double vc1 = -sy * P.vc_n + cy * P.vc_e;
  double fv = -c.c_rudder_v * delta * (s.u - vc0);
  double fr = -c.c_rudder_r * delta * (s.u - vc0);
  double u_r = s.u - vc0;
  double v_r = s.v - vc1;
  double x_g = 0.0;
  double vr0 = s.u - vc0, vr1 = s.v - vc1, vr2 = s.r - 0.0;
  double crb0 = 0 * s.u + 0 * s.v + (-c.mass * (x_g * s.r + s.v)) * s.r;
  double crb1 = 0 * s.u + 0 * s.v + (c.mass * s.u) * s.r;
  double crb2 = (c.mass * (x_g * s.r + s.v)) * s.u + (-c.mass * s.u) * s.v + 0 * s.r;
  double ca0 = 0 * vr0 + 0 * vr1 + (c.y_dv * v_r) * vr2;
  double ca1 = 0 * vr0 + 0 * vr1 + (-c.x_du * u_r) * vr2;
  double ca2 = (-c.y_dv * v_r) * vr0 + (c.x_du * u_r) * vr1 + 0 * vr2;
  double d0 = c.dlin0 + c.ku * s.u;
  double d1 = c.dlin1 + c.kv * s.v;
  double d2 = c.dlin2 + c.kr * s.r;
  double f0 = -crb0 - ca0 - d0 * vr0 + tau[0] + 0 + thrust;
  double f1 = -crb1 - ca1 - d1 * vr1 + tau[1] + 0 + fv;
  double f2 = -crb2 - ca2 - d2 * vr2 + tau[2] + 0 + fr;
  d.du = c.inv_m0 * f0;
  d.dv = c.inv_m1 * f1;
  d.dr = c.inv_m2 * f2;
  return d;
}

// differentials with the reference's angle-form wind force (PAIRED: sub-lane pairs share the
// sincos calls) or, with ALGW, the algebraic one ((wsin, wcos) = sin/cos(wind_direction)).
template <bool PAIRED = false, bool ALGW = false>
__device__ __forceinline__ Deriv differentials(const ShipConst& c, const Params& P, const Ship& s, double ctrl,
                                               double delta, bool detailed, bool odd = false, double wsin = 0.0,
                                               double wcos = 1.0) {
  double sy, cy, sw = 0.0, cw = 1.0;
  if (ALGW) sincos(s.yaw, &sy, &cy);
  else sincos2<PAIRED>(s.yaw, P.wind_dir - s.yaw, odd, sy, cy, sw, cw);
  double tau[3];
  if (ALGW) wind_force_alg(c, P, s, sy, cy, wsin, wcos, tau);
  else wind_force<PAIRED>(c, P, s, sw, cw, odd, tau);
  return differentials_body(c, P, s, ctrl, delta, detailed, sy, cy, tau);
}

// differentials of the AST kernels: (sy, cy) = sin/cos(yaw) carried from the previous integration
// step (the kernels evaluate it once per tick, after integrating, and reuse it for the encounter
// angle of the reward), algebraic wind force with the host-evaluated sin/cos(wind_direction).
__device__ __forceinline__ Deriv differentials_sc(const ShipConst& c, const Params& P, const Ship& s, double ctrl,
                                                  double delta, bool detailed, double sy, double cy) {
  double tau[3];
  wind_force_alg(c, P, s, sy, cy, P.wind_sin, P.wind_cos, tau);
  return differentials_body(c, P, s, ctrl, delta, detailed, sy, cy, tau);
}

// integrate_differentials :890-901 (EulerInt.integrate utils.py:50) + int.next_time :42
__device__ __forceinline__ void integrate(Ship& s, const Deriv& d, double dt, double mach_dt, bool detailed) {
  s.n = s.n + d.dn * dt;
  s.e = s.e + d.de * dt;
  s.yaw = s.yaw + d.dyaw * dt;
  s.u = s.u + d.du * dt;
  s.v = s.v + d.dv * dt;
  s.r = s.r + d.dr * dt;
  if (detailed) s.omega = s.omega + d.domega * mach_dt;
  s.time = s.time + dt;
}

// ---------------------------------------------------------------------------------------------
// guidance & control
// ---------------------------------------------------------------------------------------------
// LOS_guidance.py:100-117 (k = next_wpt; waypoints k-1, k are register-cached): the state update
// (e_ct, windup-limited e_ct_int) and the argument of the course correction atan
// split in its two halves: the cross-track term q = e_ct / delta at (x, y) (e_ct: the windup-clamped cross-track
// error the caller stores as s.e_ct), and the integrator update with the course correction's argument
__device__ __forceinline__ double los_q(const ShipConst& c, const Ship& s, double x, double y, double& e_ct_out) {
  // alpha_k = atan2(dy, dx) and its sin/cos depend on the segment only: cached by segment_changed()
  const double sa = s.seg_sin, ca = s.seg_cos;
  double e_ct = -(x - s.wp_prev_n) * sa + (y - s.wp_prev_e) * ca;
  if (e_ct * e_ct >= c.los_r2) e_ct = 0.99 * c.los_r;
  e_ct_out = e_ct;
  const double delta = py_max(1e-6, sqrt(c.los_r2 - e_ct * e_ct));
  return e_ct / delta;
}
__device__ __forceinline__ double los_windup(const ShipConst& c, Ship& s, double q) {
  if (fabs(s.e_ct_int + q) <= c.los_limit) s.e_ct_int += q;
  return -q - s.e_ct_int * c.los_ki;  // (-e_ct / delta is -(e_ct / delta) exactly)
}
__device__ __forceinline__ double los_update(const ShipConst& c, Ship& s, double x, double y) {
  double e_ct;
  const double q = los_q(c, s, x, y, e_ct);
  s.e_ct = e_ct;
  return los_windup(c, s, q);
}
__device__ __forceinline__ double los_guidance(const ShipConst& c, Ship& s, double x, double y) {
  const double arg = los_update(c, s, x, y);
  return s.seg_alpha + atan(arg);
}

// LOS_guidance.py:83-98: true when the index advances (caller reloads the segment cache)
__device__ __forceinline__ bool next_wpt_advance(const ShipConst& c, const Ship& s, double N, double E) {
  double dn = s.wp_n - N, de = s.wp_e - E;
  return (dn * dn + de * de <= c.ra2) && (s.n_route > s.next_wpt + 1);
}

// LOS_guidance.py:104-106 per-segment terms: recompute whenever wp_prev_* / wp_* change
__device__ __forceinline__ void segment_changed(Ship& s) {
  const double dx = s.wp_n - s.wp_prev_n;
  const double dy = s.wp_e - s.wp_prev_e;
  s.seg_alpha = atan2(dy, dx);
  sincos(s.seg_alpha, &s.seg_sin, &s.seg_cos);
}

// reload the cached LOS segment (k-1, k) from the route table
__device__ __forceinline__ void load_segment(Ship& s, const double* __restrict__ rn, const double* __restrict__ re) {
  s.wp_prev_n = rn[s.next_wpt - 1];
  s.wp_prev_e = re[s.next_wpt - 1];
  s.wp_n = rn[s.next_wpt];
  s.wp_e = re[s.next_wpt];
  s.end_n = rn[s.n_route - 1];
  s.end_e = re[s.n_route - 1];
  segment_changed(s);
}

// 1 / x when x is a power of two (then y · (1 / x) is y / x exactly: both are the correctly rounded y / x), else 0
__host__ __device__ __forceinline__ double pow2_inverse(double x) {
  int e;
  const double m = frexp(x, &e);
  return (m == 0.5 && e > -1000 && e < 1000) ? ldexp(1.0, 1 - e) : 0.0;
}

// PidController.pid_ctrl controllers.py:106-118; MUL: dt is a power of two and inv_dt = pow2_inverse(dt), the
// derivative term's division a multiplication (the same bits); else inv_dt = div_rcp(dt) (ShipConst::rcp_dt)
template <bool MUL = false>
__device__ __forceinline__ double pid(double& ei, double& prev, double kp, double kd, double ki, double dt,
                                      double setpoint, double meas, double inv_dt) {
  double error = setpoint - meas;
  double d_error = MUL ? (error - prev) * inv_dt : div_by(error - prev, dt, inv_dt);
  double error_i = ei + error * dt;
  prev = error;
  ei = error_i;
  return error * kp + d_error * kd + error_i * ki;
}
// PiController.pi_ctrl controllers.py:55-65
__device__ __forceinline__ double pi_ctrl(double& ei, double kp, double ki, double dt, double setpoint, double meas) {
  double error = setpoint - meas;
  double error_i = ei + error * dt;
  ei = error_i;
  return error * kp + error_i * ki;
}

// speed control: EngineThrottleFromSpeedSetPoint.throttle controllers.py:185-189 (Q2: shaft
// measurement = forward speed) | ThrustFromSpeedSetPoint.thrust run_colav controllers.py:183-185
template <bool MUL = false>
__device__ __forceinline__ double speed_ctrl(const ShipConst& c, Ship& s, double setpoint, double u, double dt,
                                             bool detailed, double inv_dt) {
  if (detailed) {
    double desired_shaft = pi_ctrl(s.spd_a, c.kp_ship_speed, c.ki_ship_speed, dt, setpoint, u);
    desired_shaft = sat(desired_shaft, 0, c.shaft_speed_max);
    double thr = pi_ctrl(s.spd_b, c.kp_shaft_speed, c.ki_shaft_speed, dt, desired_shaft, u);
    return sat(thr, 0, 1.1);
  }
  double t = pid<MUL>(s.spd_a, s.spd_b, c.spd_kp, c.spd_kd, c.spd_ki, dt, setpoint, u, inv_dt);
  return sat(t, -c.max_thrust, c.max_thrust);
}

// BaseMachineryModel.fuel_consumption (ship_engine.py:266-295) with MachineryMode.distribute_load
// (:46-76) and spec_fuel_cons (:259-264): f = {fuel_cons_me, fuel_cons_electrical, fuel_cons}
__device__ __forceinline__ void fuel_consumption(const ShipConst& c, double load, double dt, double f[3]) {
  const double total = load * c.avail_prop;
  double l_me, l_el, p_me, p_el;
  if (c.sg_state == SHIPSIM_SG_MOTOR) {
    l_me = py_min(total, c.mode_me);
    l_el = total + c.hotel - l_me;
    p_el = l_el / c.mode_el;
    p_me = (c.mode_me == 0) ? 0.0 : l_me / c.mode_me;
  } else if (c.sg_state == SHIPSIM_SG_GEN) {
    l_el = py_min(c.hotel, c.mode_el);
    l_me = total + c.hotel - l_el;
    p_me = l_me / c.mode_me;
    p_el = (c.mode_el == 0) ? 0.0 : l_el / c.mode_el;
  } else {
    l_me = total;
    l_el = c.hotel;
    p_me = l_me / c.mode_me;
    p_el = l_el / c.mode_el;
  }
  const double rate_me = (l_me == 0) ? 0.0 : l_me * ((c.fa_me * (p_me * p_me) + c.fb_me * p_me + c.fc_me) / 3.6e9);
  const double rate_el = (p_el == 0) ? 0.0 : l_el * ((c.fa_dg * (p_el * p_el) + c.fb_dg * p_el + c.fc_dg) / 3.6e9);
  f[0] = f[0] + rate_me * dt;
  f[1] = f[1] + rate_el * dt;
  f[2] = f[2] + (rate_me + rate_el) * dt;
}

// HeadingByReferenceController.rudder_angle_from_heading_setpoint :246-255
template <bool MUL = false>
__device__ __forceinline__ double heading_ctrl(const ShipConst& c, Ship& s, double heading_ref, double heading,
                                               double dt, double inv_dt) {
  double rudder = -pid<MUL>(s.hdg_ei, s.hdg_prev, c.hdg_kp, c.hdg_kd, c.hdg_ki, dt, heading_ref, heading, inv_dt);
  return sat(rudder, -c.max_rudder, c.max_rudder);
}

// ---------------------------------------------------------------------------------------------
// map queries (obstacle.py:126-141 over shapely/GEOS; restated GEOS semantics)
// ---------------------------------------------------------------------------------------------
// GEOS RayCrossingCounter for one polygon, boundary -> not contained
__host__ __device__ __forceinline__ bool poly_contains(const Edge* __restrict__ edges, int first, int count, double px,
                                              double py) {
  int crossings = 0;
  bool boundary = false;
  for (int i = 0; i < count; ++i) {
    const Edge ed = edges[first + i];
    double x1 = ed.ax, y1 = ed.ay, x2 = ed.bx, y2 = ed.by;
    if (x1 < px && x2 < px) continue;
    if (px == x2 && py == y2) boundary = true;
    if (y1 == py && y2 == py) {
      double mn = py_min(x1, x2), mx = py_max(x1, x2);
      if (mn <= px && px <= mx) boundary = true;
      continue;
    }
    if ((y1 > py && y2 <= py) || (y2 > py && y1 <= py)) {
      double det = (x2 - x1) * (py - y1) - (y2 - y1) * (px - x1);
      int sign = (det > 0) - (det < 0);
      if (sign == 0) boundary = true;
      if (y2 < y1) sign = -sign;
      if (sign > 0) crossings++;
    }
  }
  return !boundary && (crossings & 1);
}

// poly_contains over every other edge of the ring (edges half, half + 2, ...): the parity of this
// half's crossings and whether this half saw the point on the boundary. Two halves combine exactly:
// crossings parity = XOR of the halves' parities, boundary = OR (shapely/GEOS rule as poly_contains).
__device__ __forceinline__ void poly_contains_half(const Edge* __restrict__ edges, int first, int count, double px,
                                                   double py, int half, int& parity, bool& boundary) {
  int crossings = 0;
  boundary = false;
  for (int i = half; i < count; i += 2) {
    const Edge ed = edges[first + i];
    double x1 = ed.ax, y1 = ed.ay, x2 = ed.bx, y2 = ed.by;
    if (x1 < px && x2 < px) continue;
    if (px == x2 && py == y2) boundary = true;
    if (y1 == py && y2 == py) {
      double mn = py_min(x1, x2), mx = py_max(x1, x2);
      if (mn <= px && px <= mx) boundary = true;
      continue;
    }
    if ((y1 > py && y2 <= py) || (y2 > py && y1 <= py)) {
      double det = (x2 - x1) * (py - y1) - (y2 - y1) * (px - x1);
      int sign = (det > 0) - (det < 0);
      if (sign == 0) boundary = true;
      if (y2 < y1) sign = -sign;
      if (sign > 0) crossings++;
    }
  }
  parity = crossings & 1;
}

// map_inside's per-polygon halves as bit masks (bit p: polygon p): par = this half's crossing parity,
// bnd = this half saw the boundary; inside = ((par_a ^ par_b) & ~(bnd_a | bnd_b)) != 0
__device__ __forceinline__ void map_inside_half(const Edge* __restrict__ edges, const PolyBox* __restrict__ boxes,
                                                int n_polys, double n, double e, int half, uint32_t& par,
                                                uint32_t& bnd) {
  par = 0;
  bnd = 0;
  for (int p = 0; p < n_polys; ++p) {
    const PolyBox b = boxes[p];
    if (e < b.minx || e > b.maxx || n < b.miny || n > b.maxy) continue;
    int pa;
    bool bo;
    poly_contains_half(edges, b.first, b.count, e, n, half, pa, bo);
    par |= (uint32_t)pa << p;
    bnd |= (uint32_t)bo << p;
  }
}

// if_pos_inside_obstacles :126-129 (bbox rejection is exact for the crossing rule)
__host__ __device__ __forceinline__ bool map_inside(const Edge* __restrict__ edges, const PolyBox* __restrict__ boxes,
                                           int n_polys, double n, double e) {
  bool inside = false;
  for (int p = 0; p < n_polys; ++p) {
    const PolyBox b = boxes[p];
    if (e < b.minx || e > b.maxx || n < b.miny || n > b.maxy) continue;
    if (poly_contains(edges, b.first, b.count, e, n)) inside = true;
  }
  return inside;
}

// obstacles_distance :138-141, GEOS Distance::pointToSegment min over every ring edge
__device__ __forceinline__ double map_distance(const Edge* __restrict__ edges, int n_edges, double n, double e) {
  double best = INFINITY;
  const double px = e, py = n;
  for (int i = 0; i < n_edges; ++i) {
    const Edge ed = edges[i];
    double ax = ed.ax, ay = ed.ay, bx = ed.bx, by = ed.by;
    double d;
    if (ax == bx && ay == by) {
      d = hypot(px - ax, py - ay);
    } else {
      double dx = bx - ax, dy = by - ay;
      double len2 = dx * dx + dy * dy;
      double r = ((px - ax) * dx + (py - ay) * dy) / len2;
      if (r <= 0.0) {
        d = hypot(px - ax, py - ay);
      } else if (r >= 1.0) {
        d = hypot(px - bx, py - by);
      } else {
        double sv = ((ay - py) * dx - (ax - px) * dy) / len2;
        d = fabs(sv) * sqrt(len2);
      }
    }
    best = py_min(best, d);
  }
  return best;
}

// check_condition.py:50-78 four hull hard points
__device__ __forceinline__ bool pos_inside_obstacles(const Edge* __restrict__ edges,
                                                     const PolyBox* __restrict__ boxes, int n_polys, double n,
                                                     double e, double L) {
  double margin = L / 2;
  double mnn = n - margin, mne = e - margin, mxn = n + margin, mxe = e + margin;
  bool inside = false;
  if (map_inside(edges, boxes, n_polys, mnn, mne)) inside = true;
  if (map_inside(edges, boxes, n_polys, mnn, mxe)) inside = true;
  if (map_inside(edges, boxes, n_polys, mxn, mne)) inside = true;
  if (map_inside(edges, boxes, n_polys, mxn, mxe)) inside = true;
  return inside;
}

// reward_designs.py:33-55
__device__ __forceinline__ double rd3(double target, double off, double val) {
  return (val < target) ? exp(-((val - target) * (val - target)) / off) : 1.0;
}
__device__ __forceinline__ double rd4(double target, double off, double val) {
  return (val < target) ? 1.0 : exp(-((val - target) * (val - target)) / off);
}

}  // namespace shipsim
