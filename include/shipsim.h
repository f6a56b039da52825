/*
 * shipsim.h — C ABI of the MI355X-native batched ship-in-transit simulator.
 *
 * The reference (AndreasKing-Goks/ast-sac) has no FFI: its boundary is the Python object API of
 * MultiShipRLEnv (rl_env/ship_in_transit/env.py:41) — reset() (:238) / step(action) (:624) —
 * plus run_colav/env.py:MultiShipNonIWEnv._step (:613) for the C1 loop and the
 * SimpleShipModel/controller loop of run_colav/run_simplified_model.py:245-249 for single ships.
 * These entry points are what that object API lowers to when N environments are batched on one
 * device; the Python facade in ast_sac_amd/ re-exposes the reference's reset/step signatures on
 * top of them (INTEGRATION.md shows the ctypes binding).
 *
 * Conventions
 *   - every function returns 0 on success or a negative SHIPSIM_E* code; never aborts or throws;
 *     shipsim_last_error(h) gives the message of the last failure on that handle.
 *   - one handle <-> one device <-> one HIP stream; calls are asynchronous on that stream.
 *     A handle is not thread-safe; handles on different devices are independent.
 *   - the library owns all device state (SoA ship state, per-env route tables, map);
 *     every I/O buffer below is a caller-owned DEVICE pointer (e.g. a torch tensor's data_ptr()).
 *   - no host allocation or synchronisation inside reset/step/tick.
 */
#ifndef SHIPSIM_H
#define SHIPSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHIPSIM_ABI_VERSION 10

#define SHIPSIM_MAX_ROUTE 16   /* waypoints per ship route (obs ship: 2 + max_sampling_frequency) */
#define SHIPSIM_MAX_POLYS 16   /* land polygons in the map */
#define SHIPSIM_MAX_VERTS 128  /* total polygon vertices */
#define SHIPSIM_MAX_OBS 4      /* obstacle ships per AST env (configs[4] C5: K in {1, 2, 4}) */
#define SHIPSIM_MAX_SHIPS (1 + SHIPSIM_MAX_OBS)

/* status codes */
#define SHIPSIM_OK 0
#define SHIPSIM_EINVAL -1   /* bad argument / config */
#define SHIPSIM_EHIP -2     /* HIP runtime failure */
#define SHIPSIM_ESTATE -3   /* call not valid in the current state (e.g. step before reset) */
#define SHIPSIM_ENOMEM -4
#define SHIPSIM_ENONFINITE -5 /* shipsim_synchronize: an env's ship state went NaN/Inf (see SHIPSIM_EV_NONFINITE) */

/* environment kinds */
#define SHIPSIM_KIND_SINGLE 0  /* one ship per env, no termination (config C2; run_simplified_model loop) */
#define SHIPSIM_KIND_NONIW 1   /* two ships, fixed routes, env_info flags only (C1; run_colav/env.py:37) */
#define SHIPSIM_KIND_AST 2     /* two-ship AST env with IW sampling + reward (C3/C4/C5; rl_env/.../env.py:41) */

/* collision avoidance of the ship under test (env.py:53, args.collav_mode) */
#define SHIPSIM_COLLAV_NONE 0
#define SHIPSIM_COLLAV_SIMPLE 1
#define SHIPSIM_COLLAV_SBMPC 2

/* propulsion model */
#define SHIPSIM_MACH_SIMPLIFIED 0 /* SimpleShipModel + ThrustFromSpeedSetPoint (run_colav) */
#define SHIPSIM_MACH_DETAILED 1   /* ShipModelAST + ShipMachineryModel + EngineThrottleFromSpeedSetPoint */

/* MachineryMode.shaft_generator_state (ship_engine.py:32-76) */
#define SHIPSIM_SG_GEN 0   /* PTO */
#define SHIPSIM_SG_MOTOR 1 /* PTI */
#define SHIPSIM_SG_OFF 2   /* MEC */

/* event bits, in the order get_reward_and_env_info appends its strings (reward_function.py:204-262) */
#define SHIPSIM_EV_COLLISION (1u << 0)
#define SHIPSIM_EV_TEST_GROUNDING (1u << 1)
#define SHIPSIM_EV_TEST_NAV_FAILURE (1u << 2)
#define SHIPSIM_EV_OBS_GROUNDING (1u << 3)
#define SHIPSIM_EV_OBS_NAV_FAILURE (1u << 4)
#define SHIPSIM_EV_TEST_REACHES_END (1u << 5)
#define SHIPSIM_EV_TEST_OUTSIDE_MAP (1u << 6)
#define SHIPSIM_EV_OBS_REACHES_END (1u << 7)
#define SHIPSIM_EV_OBS_OUTSIDE_MAP (1u << 8)
#define SHIPSIM_EV_TIME_LIMIT (1u << 9)
#define SHIPSIM_EV_SAMPLING_FAILURE (1u << 10) /* env.py:684 */
#define SHIPSIM_EV_TERMINAL (1u << 16)          /* env_info['terminal'] */
#define SHIPSIM_EV_TEST_STOP (1u << 17)         /* env_info['test_ship_stop'] */
#define SHIPSIM_EV_OBS_STOP (1u << 18)          /* env_info['obs_ship_stop'] */
#define SHIPSIM_EV_NONFINITE (1u << 24)         /* build-only, not a reference outcome: a ship state went
                                                   NaN/Inf in this decision; the decision ends at once with
                                                   done = 1 and SHIPSIM_EV_TERMINAL (boundary error contract) */

/* One ship: ShipConfiguration (ship_model.py:20), SimulationConfiguration (:45), rudder / machinery
 * (ship_engine.py:121,160), controller gains (controllers.py:16-38), LOS (LOS_guidance.py:15) and
 * the route file contents. Field names follow the reference's NamedTuple fields. */
typedef struct shipsim_ship_config {
  double dead_weight_tonnage;
  double coefficient_of_deadweight_to_displacement;
  double bunkers;
  double ballast;
  double length_of_ship;
  double width_of_ship;
  double added_mass_coefficient_in_surge;
  double added_mass_coefficient_in_sway;
  double added_mass_coefficient_in_yaw;
  double mass_over_linear_friction_coefficient_in_surge;
  double mass_over_linear_friction_coefficient_in_sway;
  double mass_over_linear_friction_coefficient_in_yaw;
  double nonlinear_friction_coefficient_in_surge;
  double nonlinear_friction_coefficient_in_sway;
  double nonlinear_friction_coefficient_in_yaw;
  /* initial state (SimulationConfiguration) */
  double initial_north_position_m;
  double initial_east_position_m;
  double initial_yaw_angle_rad;
  double initial_forward_speed_m_per_s;
  double initial_sideways_speed_m_per_s;
  double initial_yaw_rate_rad_per_s;
  /* rudder */
  double rudder_angle_to_sway_force_coefficient;
  double rudder_angle_to_yaw_force_coefficient;
  double max_rudder_angle_degrees;
  /* detailed machinery (MachinerySystemConfiguration, one active MachineryMode) */
  double hotel_load;
  double main_engine_capacity;
  double electrical_capacity;
  double rated_speed_main_engine_rpm;
  double linear_friction_main_engine;
  double linear_friction_hybrid_shaft_generator;
  double gear_ratio_between_main_engine_and_propeller;
  double gear_ratio_between_hybrid_shaft_generator_and_propeller;
  double propeller_inertia;
  double propeller_speed_to_torque_coefficient;
  double propeller_diameter;
  double propeller_speed_to_thrust_force_coefficient;
  double initial_propeller_shaft_speed_rad_per_s;
  /* EngineThrottleFromSpeedSetPoint gains (detailed) */
  double kp_ship_speed;
  double ki_ship_speed;
  double kp_shaft_speed;
  double ki_shaft_speed;
  double initial_shaft_speed_integral_error;
  /* ThrustFromSpeedSetPoint PID (simplified); max_thrust may be +inf */
  double speed_kp;
  double speed_ki;
  double speed_kd;
  double max_thrust;
  /* heading autopilot PID */
  double heading_kp;
  double heading_kd;
  double heading_ki;
  /* LOS guidance */
  double radius_of_acceptance;
  double lookahead_distance;
  double los_integral_gain;
  double los_integrator_windup_limit;
  double desired_forward_speed;
  int32_t shaft_generator_state; /* SHIPSIM_SG_* */
  int32_t n_route;               /* waypoints in route_north/route_east */
  double route_north[SHIPSIM_MAX_ROUTE];
  double route_east[SHIPSIM_MAX_ROUTE];
} shipsim_ship_config;

typedef struct shipsim_config {
  int32_t abi_version;            /* = SHIPSIM_ABI_VERSION */
  int32_t kind;                   /* SHIPSIM_KIND_* */
  int32_t machinery;              /* SHIPSIM_MACH_* */
  int32_t collav;                 /* SHIPSIM_COLLAV_* */
  int32_t max_sampling_frequency; /* args.max_sampling_frequency (9) */
  int32_t machinery_dt_quirk;     /* 1: machinery integrates with dt 0.01 after reset */
  int32_t normalize_action;       /* args.normalize_action: env denormalizes [-1,1] itself */
  int32_t n_ships;                /* 1 (SINGLE), 2 (NONIW), 1 + K obstacle ships (AST, K <= SHIPSIM_MAX_OBS) */
  double time_step;               /* args.time_step */
  double simulation_time;         /* SimulationConfiguration.simulation_time */
  double env_radius_of_acceptance;/* args.radius_of_acceptance used by is_reach_radius_of_acceptance */
  /* EnvironmentConfiguration */
  double current_velocity_component_from_north;
  double current_velocity_component_from_east;
  double wind_speed;
  double wind_direction;
  /* SBMPC(tf, dt) (env.py:123) */
  double sbmpc_tf;
  double sbmpc_dt;
  /* action box of the wrapped env (env.py:93-104), float32 as in the reference */
  float action_low;
  float action_high;
  /* [0] ship under test, [1] the obstacle ship (intermediate-waypoint sampling, the decisions, the
   * observation), [2..K] further obstacle ships (AST with K > 1, see shipsim_create) */
  shipsim_ship_config ship[SHIPSIM_MAX_SHIPS];
  /* PolygonObstacle map: polygon p owns vertices [poly_start[p], poly_start[p+1]), (east, north) */
  int32_t n_polys;
  int32_t poly_start[SHIPSIM_MAX_POLYS + 1];
  double poly_east[SHIPSIM_MAX_VERTS];
  double poly_north[SHIPSIM_MAX_VERTS];
  /* performance knob (no effect on results): device lanes per AST env, 2/4/8/16 (the decision
   * stream runs 4/8/16); 0 = $SHIPSIM_LPE or automatic (shipsim_lanes_per_env) */
  int32_t lanes_per_env;
  /* performance knobs (no effect on results; ABI 8): envs per wave (0 = as many as the wave holds, 64 / LPE;
   * fewer leave idle lanes), and the coastline query (SHIPSIM_MAP_GRID: the candidate edges of the ship's
   * 200 m grid cell; SHIPSIM_MAP_ALL_EDGES: every edge, the reference's own loop) */
  int32_t envs_per_wave;
  int32_t map_query;
  int32_t reserved[5];
} shipsim_config;

#define SHIPSIM_MAP_GRID 0
#define SHIPSIM_MAP_ALL_EDGES 1

/* Per-ship state fields for get/set_state (SoA, double unless noted; [env][ship], n_ships = 1 + K) */
#define SHIPSIM_F_NORTH 0
#define SHIPSIM_F_EAST 1
#define SHIPSIM_F_YAW 2
#define SHIPSIM_F_U 3
#define SHIPSIM_F_V 4
#define SHIPSIM_F_R 5
#define SHIPSIM_F_OMEGA 6        /* propeller shaft speed (detailed) */
#define SHIPSIM_F_TIME 7         /* ship_model.int.time */
#define SHIPSIM_F_E_CT 8         /* navigate.e_ct */
#define SHIPSIM_F_E_CT_INT 9     /* navigate.e_ct_int */
#define SHIPSIM_F_HDG_EI 10      /* heading PID error_i */
#define SHIPSIM_F_HDG_PREV 11    /* heading PID prev_error */
#define SHIPSIM_F_SPD_A 12       /* ship-speed PI error_i (detailed) | thrust PID error_i (simplified) */
#define SHIPSIM_F_SPD_B 13       /* shaft-speed PI error_i (detailed) | thrust PID prev_error (simplified) */
#define SHIPSIM_F_RUDDER 14      /* last commanded rudder angle (logged) */
#define SHIPSIM_F_THRUST 15      /* last thrust force [N] (logged) */
#define SHIPSIM_F_LOG_ECT 16     /* last logged cross-track error */
#define SHIPSIM_F_NEXT_WPT 17    /* int32: auto_pilot.next_wpt */
#define SHIPSIM_F_STOP 18        /* int32: ShipAssets.stop_flag */
#define SHIPSIM_N_SHIP_FIELDS 19

/* Per-env fields (AST / NONIW) */
#define SHIPSIM_E_SAMPLING_COUNT 100 /* int32 */
#define SHIPSIM_E_TRAVEL_DIST 101
#define SHIPSIM_E_TRAVEL_TIME 102
#define SHIPSIM_E_ACC_REWARD 103
#define SHIPSIM_E_N_BASE 104
#define SHIPSIM_E_E_BASE 105
#define SHIPSIM_E_SBMPC_P_LAST 106
#define SHIPSIM_E_SBMPC_CHI_LAST 107
#define SHIPSIM_E_ROUTE_LEN 108      /* int32: obstacle-ship route length */
#define SHIPSIM_E_ROUTE_NORTH 109    /* double[SHIPSIM_MAX_ROUTE] per env, env-major */
#define SHIPSIM_E_ROUTE_EAST 110

typedef struct shipsim_handle shipsim_handle;

/* Build info / ABI version of the loaded library. */
int32_t shipsim_abi_version(void);
const char* shipsim_build_info(void);

/* Fill *cfg with the reference scenario of record:
 *   kind SHIPSIM_KIND_AST : run/env_setup.py:17-254 (two ShipModelAST, PTI machinery, time_step 4,
 *                           runner defaults run/ast-sac_runner.py:27-43), collav as given;
 *   kind SHIPSIM_KIND_NONIW / SINGLE : run_colav/run_simplified_model.py:55-233 (SimpleShipModel,
 *                           ThrustFromSpeedSetPoint, time_step 30).
 * Routes and the 6-polygon map are the reference data files' contents. */
int shipsim_default_config(int32_t kind, int32_t machinery, int32_t collav, double time_step,
                           shipsim_config* cfg);

/* Allocate device state for n_envs environments on `device`, bound to `stream` (hipStream_t;
 * NULL = default stream). The handle starts un-reset.
 * n_obs_ships (AST kind): obstacle ships per env, 1..SHIPSIM_MAX_OBS (<= 0: cfg->n_ships - 1), configured
 * in cfg->ship[1..K]. K = 1 is the reference env (rl_env/ship_in_transit/env.py:76 unpacks [test, obs]).
 * K > 1 generalises it the way the reference's own pieces already do — parity unpinned beyond them:
 *   - SBMPC of the ship under test sees every obstacle ship (env.py:366-370 builds do_list from
 *     assets[1::]; sbmpc.py:150-176: active when any is within D_INIT, worst obstacle per scenario);
 *   - ship 1 is "the" obstacle ship: it samples the intermediate waypoints from the action, its radius
 *     of acceptance ends a decision, its grounding / navigation failure terms enter the reward and the
 *     observation reports it (env.py:538-773, reward_function.py:59-270);
 *   - ships 2..K follow their own routes with the same autopilot / throttle controllers (obs_step
 *     without sampling) and freeze (obs_step's stop branch) once they reach their last waypoint, leave
 *     the map or ground;
 *   - the collision reward / termination and the encounter angle use the nearest obstacle ship.
 * K > 1 needs detailed machinery and collav none or sbmpc. */
int shipsim_create(const shipsim_config* cfg, int32_t n_envs, int32_t n_obs_ships, int32_t device, void* stream,
                   shipsim_handle** out);
int shipsim_destroy(shipsim_handle* h);
/* Message of the last failed call on h; with h == NULL, of the calling thread's last shipsim_create that
 * failed before it could hand out a handle (every such path sets it; it is per thread). */
const char* shipsim_last_error(const shipsim_handle* h);
/* Launches of this handle go to `stream` from now on (e.g. a graph-capturing stream; ABI 6). */
int shipsim_set_stream(shipsim_handle* h, void* stream);
int32_t shipsim_num_envs(const shipsim_handle* h);
/* Lanes per AST env the step / stream kernels run at (config lanes_per_env, or chosen at create from
 * n_envs and the device's SIMD count; a performance knob only, results are identical). */
int32_t shipsim_lanes_per_env(const shipsim_handle* h);

/* MultiShipRLEnv.reset(): every env with env_mask[i] != 0 (NULL = all) is reset and placed with
 * init_step (one control + integrate tick, env.py:297); obs_out (N x 8 float32, device, may be NULL)
 * receives the reference's constant initial_states row for reset envs (Q11). */
int shipsim_reset(shipsim_handle* h, const uint8_t* env_mask, float* obs_out);

/* MultiShipRLEnv.step(action) for all N envs at once (AST kind only), sliced.
 * Every active env ticks (_step, env.py:563) until its decision point (RoA + one tick, or done —
 * env.py:700-771) or until it has run `max_ticks` ticks in this call (<= 0: no limit). An env that
 * paused keeps its decision in progress and resumes in the next call WITHOUT consuming an action;
 * an env waiting for a decision (after reset or after its previous decision completed) first
 * consumes action[i] (intermediate-waypoint sampling, env.py:659-696).
 *   action     N float32 scoping angles in radians (already denormalized, i.e. what
 *              NormalizedBoxEnv passes to the wrapped env), device.
 *   active     optional N uint8 mask (NULL = all): envs with 0 are left untouched.
 * Outputs (device, each may be NULL):
 *   ready  N uint8: 1 if the env completed a decision in this call; then obs (N x 8 float32),
 *          reward (N double, un-scaled accumulated reward of the decision), done (N uint8,
 *          combined_done) and events (N uint32, SHIPSIM_EV_* bits) hold that decision's result;
 *          rows of envs that did not complete are left untouched.
 *   ticks  N int32: _step calls executed by the env in this call. */
int shipsim_step(shipsim_handle* h, const float* action, const uint8_t* active, int32_t max_ticks,
                 float* obs_out, double* reward_out, uint8_t* done_out, uint32_t* events_out,
                 int32_t* ticks_out, uint8_t* ready_out);

/* Raw ticks for the SINGLE and NONIW kinds: advance every env by k ticks of the reference loop body
 * (run_simplified_model.py:248-249; for NONIW MultiShipNonIWEnv._step, run_colav/env.py:613-676: both ships'
 * steps with their SBMPC blocks in the reference's order, get_env_info's flags and the stop flags; simplified
 * machinery only). events_out (N uint32, may be NULL) receives the env_info bits (SHIPSIM_EV_*) of the last tick
 * (NONIW). The C1 loop runs while the test ship's F_TIME < simulation_time. */
int shipsim_tick(shipsim_handle* h, int32_t k, uint32_t* events_out);

/* Read / write one state field for all envs (device pointer dst/src). Ship fields are laid out
 * env-major [env][ship] (the device lane order), env fields [env], routes [env][ship][SHIPSIM_MAX_ROUTE]. */
int shipsim_get_state(shipsim_handle* h, int32_t field, void* dst);
int shipsim_set_state(shipsim_handle* h, int32_t field, const void* src);

/* ---- trajectory recording (f1: simulation_results export) ----------------------------------
 * Per-tick rows of ShipModelAST/SimpleShipModel.store_simulation_data (ship_model.py:903-957,
 * run_colav/.../ship_model.py:418-444) for both ships, plus the RewardTracker entry of every tick
 * (reward_function.py:30-57, 181-186) and the animation lists of env.py:612-620. Row t of a ship is its
 * t-th store since the env's last reset (row 0 = init_step, env.py:329); env row t belongs to tick
 * t + 1. Values are raw (SI units, radians); the Python facade derives the reference's keys and units.
 * Ship row columns: */
#define SHIPSIM_TRAJ_SHIP_COLS 20
#define SHIPSIM_TS_TIME 0       /* int.time at the store */
#define SHIPSIM_TS_NORTH 1
#define SHIPSIM_TS_EAST 2
#define SHIPSIM_TS_YAW 3        /* rad */
#define SHIPSIM_TS_RUDDER 4     /* rad */
#define SHIPSIM_TS_U 5
#define SHIPSIM_TS_V 6
#define SHIPSIM_TS_R 7          /* rad/s */
#define SHIPSIM_TS_OMEGA 8      /* propeller shaft speed rad/s (detailed) */
#define SHIPSIM_TS_THRUST 9     /* N: propeller thrust (detailed) | commanded thrust force (simplified) */
#define SHIPSIM_TS_E_CT 10      /* auto_pilot.get_cross_track_error() */
#define SHIPSIM_TS_E_PSI 11     /* auto_pilot.get_heading_error() = |heading_mea - heading_ref| (rad, Q8) */
#define SHIPSIM_TS_LOAD 12      /* engine throttle = load_perc (detailed) | thrust command (simplified) */
#define SHIPSIM_TS_FUEL_ME 13   /* accumulated fuel kg (detailed; machinery int.dt, Q1) */
#define SHIPSIM_TS_FUEL_EL 14
#define SHIPSIM_TS_FUEL 15
#define SHIPSIM_TS_E_CT_INT 16  /* navigate.e_ct_int after the tick (ShipAssets.integrator_term) */
#define SHIPSIM_TS_NEXT_WPT 17
#define SHIPSIM_TS_REPEAT 18    /* 1: store_last_simulation_data row of a stopped ship */
#define SHIPSIM_TS_TIME_LIST 19 /* ShipAssets.time_list entry of the tick */
/* Env row columns: */
#define SHIPSIM_TRAJ_ENV_COLS 8
#define SHIPSIM_TE_R_COLLISION 0      /* RewardTracker.ship_collision (already / 5) */
#define SHIPSIM_TE_R_TEST_GROUNDING 1
#define SHIPSIM_TE_R_TEST_NAV 2
#define SHIPSIM_TE_R_OBS_GROUNDING 3
#define SHIPSIM_TE_R_OBS_NAV 4
#define SHIPSIM_TE_R_TOTAL 5          /* RewardTracker.total (after the termination multipliers) */
#define SHIPSIM_TE_BITS 6             /* SHIPSIM_EV_* bits of the tick */
#define SHIPSIM_TE_FLAGS 7            /* SHIPSIM_TE_FLAG_* */
#define SHIPSIM_TE_FLAG_COLLISION 1   /* is_collision_list entry */
#define SHIPSIM_TE_FLAG_IMMINENT 2    /* is_collision_imminent_list entry (simple: distance, sbmpc: active) */

/* Enable recording into caller-owned device buffers: ship_rows n_envs*n_ships x capacity x
 * SHIPSIM_TRAJ_SHIP_COLS doubles ([env][ship][row][col]), env_rows n_envs x capacity x
 * SHIPSIM_TRAJ_ENV_COLS doubles (may be NULL), lengths n_envs int32 (ship rows recorded since the env's
 * last reset; rows past capacity are dropped while the count goes on). Lengths are zeroed here and by
 * every reset; enable before the reset that starts the episodes to record. ship_rows NULL disables.
 * AST kind only; recording steps run the lanes_per_env = 16 kernels (identical results). */
int shipsim_set_trajectory(shipsim_handle* h, double* ship_rows, double* env_rows, int32_t capacity,
                           int32_t* lengths);

/* SBMPC.get_optimal_ctrl_offset (sbmpc.py:113-185) for n independent single-obstacle requests on the
 * device, stateless (P_ca_last_ / Chi_ca_last_ are inputs). in: n x SHIPSIM_SBMPC_IN doubles
 * [P_ca_last, Chi_ca_last, u_d, chi_d, os_state(6: x, y, psi, u, v, r), obstacle(5: x, y, psi, u, v),
 *  obstacle length, obstacle width]; out: n x 3 doubles [speed factor, course offset, active].
 * SBMPC(tf, dt) horizon; stream is a hipStream_t (NULL = default); device pointers. */
#define SHIPSIM_SBMPC_IN 17
int shipsim_sbmpc_eval(int32_t n, double tf, double dt, const double* in, double* out, void* stream);

/* SBMPC.get_optimal_ctrl_offset (sbmpc.py:113-185) over a do_list of n_obs dynamic obstacles (1 <= n_obs <=
 * SHIPSIM_MAX_OBS; active when any of them is within D_INIT, per scenario the worst obstacle's cost, the least worst
 * scenario: :149-178) for n independent requests, stateless like shipsim_sbmpc_eval (ABI 10). in: n x
 * SHIPSIM_SBMPC_MULTI_IN doubles [P_ca_last, Chi_ca_last, u_d, chi_d, os_state(6: x, y, psi, u, v, r), then per
 * obstacle slot k < SHIPSIM_MAX_OBS: x, y, psi, u, v, length, width (the do_list tuple's state and size; slots
 * k >= n_obs are ignored)]; out: n x 3 doubles [speed factor, course offset, active]. The optimiser is the one the
 * multi-obstacle env kernels (n_obs_ships > 1) run. Replaces, per request, one call of the reference method with a
 * do_list of n_obs entries. */
#define SHIPSIM_SBMPC_MULTI_IN (10 + 7 * SHIPSIM_MAX_OBS)
int shipsim_sbmpc_eval_multi(int32_t n, int32_t n_obs, double tf, double dt, const double* in, double* out,
                             void* stream);

/* Diagnostics: the kernels' division by a reused divisor (the divisor's refined reciprocal formed once, the rest of
 * the compiler's fp64 division sequence per quotient) next to the plain IEEE division, for n operand
 * pairs: fast[i] = num[i] / den[i] as the kernels form it, ref[i] = num[i] / den[i]. Device pointers (n doubles
 * each); stream a hipStream_t (NULL = default). The two agree bit for bit for operands away from the ends of the
 * exponent range (tests/test_gpu_div_identity.py). */
int shipsim_div_check(int32_t n, const double* num, const double* den, double* fast, double* ref, void* stream);

/* ---- open-loop decision stream (the C3 workload of SURVEY.md §8(d)) -------------------------
 * Every env draws the scoping angle (radians, already denormalised) of decision d of its episode e from
 * table[((e % n_eps) * n_dec + d) * n_envs + env] and runs decisions back to back inside the call: a
 * completed decision (MultiShipRLEnv.step, env.py:624-773) is followed at once by the next one, and an
 * episode that ends — done, or n_dec decisions (the rollout's max_path_length, rollout_functions.py:
 * 106-160) — is reset in place (reset + init_step, env.py:238-342) before its next decision. Each env
 * runs at most max_ticks (>= 1) _step ticks per call; an env paused mid-decision resumes in the next
 * call. Results are those of shipsim_step / shipsim_reset driven by the same table.
 *   ep_idx, dec_idx  N int32 (device, in/out): episode counter and decision index of every env
 *   ticks_out        N int32: _step ticks run in this call (may be NULL)
 *   decisions_out    N int32: decisions completed in this call (may be NULL)
 *   log              N x log_cap x SHIPSIM_DECLOG_COLS doubles: one record per completed decision
 *                    (may be NULL); log_len N int32 (in/out) counts records (past log_cap too). */
#define SHIPSIM_DECLOG_COLS 23
#define SHIPSIM_DL_REWARD 0   /* accumulated (un-scaled) reward of the decision */
#define SHIPSIM_DL_EVENTS 1   /* SHIPSIM_EV_* bits */
#define SHIPSIM_DL_DONE 2     /* combined_done */
#define SHIPSIM_DL_EPISODE 3  /* ep_idx of the decision */
#define SHIPSIM_DL_DECISION 4 /* dec_idx of the decision */
#define SHIPSIM_DL_TICKS 5    /* _step ticks of the decision (across launches; 0 for a sampling failure) */
#define SHIPSIM_DL_OBS 6      /* 8 columns: the observation returned */
#define SHIPSIM_DL_ACTION 14  /* shipsim_run_policy only: the policy's normalized action a */
#define SHIPSIM_DL_OBS0 15    /* shipsim_run_policy only, 8 columns: the observation a was chosen from */
/* (shipsim_run_table leaves columns 14..22 as they were: its actions are the caller's table) */
int shipsim_run_table(shipsim_handle* h, const float* table, int32_t n_eps, int32_t n_dec, int32_t max_ticks,
                      int32_t* ep_idx, int32_t* dec_idx, int32_t* ticks_out, int32_t* decisions_out, double* log,
                      int32_t log_cap, int32_t* log_len);

/* The same decision stream with the collector's policy in the loop (ABI 7; also new in 7: the 23-column decision record): every decision's action is
 * sampled inside the launch from the observation the env returned, by the TanhGaussianPolicy
 * (gaussian_policy.py:105-118: fc0, relu, fc1, relu, mean / clamped log_std heads) then TanhNormal.sample
 * (distributions.py:394-425: tanh(mean + std * eps), eps ~ N(0, 1)) or, deterministic != 0,
 * MakeDeterministic's tanh(mean) (policies/base.py:54-64), and denormalized as NormalizedBoxEnv does
 * (normalized_box_env.py:48-51) — the rollout loop of rollout_functions.py:53-91 for every env at once,
 * without a host round trip. fp32 as the policy; the env in fp64.
 *   policy   the policy's parameters in torch order (fcs[0].weight [H][obs_dim], .bias, fcs[1].weight
 *            [H][H], .bias, last_fc.weight [1][H], .bias, last_fc_log_std.weight, .bias), device
 *   w2t      fcs[1].weight transposed ([H][H], w2t[k][u] = W2[u][k]), device (sacf_policy_weights)
 *   obs_dim  8; hidden a multiple of 64 up to 512
 *   seed, counter  the noise: eps of env i's s-th decision of a call is Philox4x32-10 keyed by seed on
 *            {i, *counter (64 bits), 0x5A100000 ^ s} then Box-Muller; *counter is read, not changed —
 *            advance it between calls (ignored when deterministic; counter may then be NULL)
 *   n_dec    decisions per episode (max_path_length); other arguments as shipsim_run_table, and the
 *            decision record's SHIPSIM_DL_ACTION column holds the normalized action a in (-1, 1).
 *            With a log, an env stops for the launch once it holds log_cap records (log_len starts where
 *            the caller left it), its next decision pending for the next call: no record is lost.
 * One obstacle ship only (SHIPSIM_EINVAL otherwise, as for a bad obs_dim / hidden). */
int shipsim_run_policy(shipsim_handle* h, const float* policy, const float* w2t, int32_t obs_dim, int32_t hidden,
                       int32_t deterministic, uint64_t seed, const int64_t* counter, int32_t n_dec,
                       int32_t max_ticks, int32_t* ep_idx, int32_t* dec_idx, int32_t* ticks_out,
                       int32_t* decisions_out, double* log, int32_t log_cap, int32_t* log_len);

/* Work-conserving launch tail of the decision streams (shipsim_run_table / shipsim_run_policy; ABI 8): a wave
 * whose envs all met max_ticks keeps ticking, 32 ticks at a time, while any wave of the same launch has not, up to
 * extra_ticks more (0, the default: off). Per-env results do not change (a decision stream is exact whatever its
 * launch boundaries); ticks_out / decisions_out then exceed max_ticks by up to extra_ticks for the envs of the
 * faster waves. Used only when every wave of the launch is resident at once (otherwise the launch runs as with 0),
 * and for one obstacle ship per env (the K > 1 streams run as with 0). */
int shipsim_set_stream_tail(shipsim_handle* h, int32_t extra_ticks);

/* ---- legacy per-tick MultiShipEnv (rl_env/ship_in_transit/env.py:783-1181) ----
 * AST kind. Each of the k ticks is one MultiShipEnv.step() (:1104-1173) of every env: test_step
 * (:923-1023, SBMPC / simple collision avoidance as configured) + obs_step (:1025-1102) +
 * get_termination_status (evaluation/termination_flags.py:5-70). No intermediate waypoints, no reward.
 * Envs start from shipsim_reset (MultiShipEnv.reset/init_step, :855-921 — same placement as the RL
 * reset); the simple collision check reads the previous step's next_states (the float32
 * initial_states before the first step after create), which survive reset, as in the reference.
 * An env whose step reports done stops ticking for the rest of the call (k = 1: the reference's
 * per-call semantics). Outputs of the env's last tick (device, each may be NULL):
 *   states  N x 8 doubles: next_states [test n, e, e_ct, obs n, e, yaw, speed, e_ct]
 *   done    N uint8: test reached/outside/grounded/nav failure, collision, obs grounded/nav failure
 *   status  N uint32: bit i = termination_conditions[i] (SHIPSIM_LT_*) */
#define SHIPSIM_LT_TEST_REACHED (1u << 0)
#define SHIPSIM_LT_TEST_OUTSIDE (1u << 1)
#define SHIPSIM_LT_TEST_GROUNDED (1u << 2)
#define SHIPSIM_LT_TEST_NAV_FAILURE (1u << 3)  /* |e_ct| > 500 */
#define SHIPSIM_LT_NEAR_COLLISION (1u << 4)    /* distance < 3000 m */
#define SHIPSIM_LT_COLLISION (1u << 5)         /* distance < 50 m */
#define SHIPSIM_LT_OBS_REACHED (1u << 6)
#define SHIPSIM_LT_OBS_OUTSIDE (1u << 7)
#define SHIPSIM_LT_OBS_GROUNDED (1u << 8)
#define SHIPSIM_LT_OBS_NAV_FAILURE (1u << 9)
int shipsim_legacy_step(shipsim_handle* h, int32_t k, double* states_out, uint8_t* done_out, uint32_t* status_out);

/* Block until all work queued on the handle's stream is done. Returns SHIPSIM_ENONFINITE (message in
 * shipsim_last_error) when env decisions ended on a non-finite ship state since the previous call. */
int shipsim_synchronize(shipsim_handle* h);
/* Decisions flagged SHIPSIM_EV_NONFINITE since create, as of the last shipsim_synchronize. */
int32_t shipsim_nonfinite_count(const shipsim_handle* h);
/* Diagnostics builds only (-DSHIPSIM_LANECHECK): out32 = {violations, first site, its exec mask lo, hi,
 * 0 x 4, violations of site 0..15 x 16, 0 x 8} of the cross-lane / index checks since the last call (then
 * cleared; synchronizes the current device). SHIPSIM_EINVAL (out32 zeroed) in the default build, which
 * compiles the checks out. */
int shipsim_diag_lane_faults(uint32_t* out32);

#ifdef __cplusplus
}
#endif
#endif /* SHIPSIM_H */
