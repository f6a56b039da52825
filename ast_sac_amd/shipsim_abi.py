"""ctypes mirror of include/shipsim.h (structs, constants) and the scenario builders.

The scenario builders restate the literal configuration blocks of the reference:
  * `ast_config`  — run/env_setup.py:31-246 (+ runner defaults run/ast-sac_runner.py:27-43)
  * `c1_config`   — run_colav/run_simplified_model.py:55-233
  * `c2_config`   — the C2 single-ship unit: C1's test ship alone on
                    own_ship_route.txt with HeadingByRouteController.
Routes / map are the contents of the reference data files (rl_env/ship_in_transit/data/*.txt,
run_colav/ship_in_transit/data/*.txt, map_data in env_setup.py:145-152).
"""
import ctypes as C
import math

import numpy as np

ABI_VERSION = 10
MAP_GRID, MAP_ALL_EDGES = 0, 1  # shipsim_config.map_query (results identical)
ENONFINITE = -5  # shipsim_synchronize status (include/shipsim.h)
MAX_ROUTE = 16
MAX_POLYS = 16
MAX_VERTS = 128
MAX_OBS = 4
MAX_SHIPS = 1 + MAX_OBS

KIND_SINGLE, KIND_NONIW, KIND_AST = 0, 1, 2
COLLAV_NONE, COLLAV_SIMPLE, COLLAV_SBMPC = 0, 1, 2
COLLAV = {"none": COLLAV_NONE, None: COLLAV_NONE, "simple": COLLAV_SIMPLE, "sbmpc": COLLAV_SBMPC}
MACH_SIMPLIFIED, MACH_DETAILED = 0, 1
SG_GEN, SG_MOTOR, SG_OFF = 0, 1, 2

# shipsim_run_table per-decision record columns
DECLOG_COLS = 23
DL_REWARD, DL_EVENTS, DL_DONE, DL_EPISODE, DL_DECISION, DL_TICKS, DL_OBS = 0, 1, 2, 3, 4, 5, 6
DL_ACTION, DL_OBS0 = 14, 15

# legacy MultiShipEnv termination_conditions bits (shipsim_legacy_step, termination_flags.py:66-68)
LT_TEST_REACHED = 1 << 0
LT_TEST_OUTSIDE = 1 << 1
LT_TEST_GROUNDED = 1 << 2
LT_TEST_NAV_FAILURE = 1 << 3
LT_NEAR_COLLISION = 1 << 4
LT_COLLISION = 1 << 5
LT_OBS_REACHED = 1 << 6
LT_OBS_OUTSIDE = 1 << 7
LT_OBS_GROUNDED = 1 << 8
LT_OBS_NAV_FAILURE = 1 << 9
LT_DONE_MASK = (LT_TEST_REACHED | LT_TEST_OUTSIDE | LT_TEST_GROUNDED | LT_TEST_NAV_FAILURE | LT_COLLISION
                | LT_OBS_GROUNDED | LT_OBS_NAV_FAILURE)

EV_COLLISION = 1 << 0
EV_TEST_GROUNDING = 1 << 1
EV_TEST_NAV_FAILURE = 1 << 2
EV_OBS_GROUNDING = 1 << 3
EV_OBS_NAV_FAILURE = 1 << 4
EV_TEST_REACHES_END = 1 << 5
EV_TEST_OUTSIDE_MAP = 1 << 6
EV_OBS_REACHES_END = 1 << 7
EV_OBS_OUTSIDE_MAP = 1 << 8
EV_TIME_LIMIT = 1 << 9
EV_SAMPLING_FAILURE = 1 << 10
EV_TERMINAL = 1 << 16
EV_TEST_STOP = 1 << 17
EV_OBS_STOP = 1 << 18
EV_NONFINITE = 1 << 24
EVENT_MASK = (1 << 11) - 1

# env_info['events'] strings, in bit order (reward_function.py:204-262, env.py:684)
EVENT_STRINGS = (
    "Ships collision!",
    "|Ship under test experiences grounding!|",
    "|Ship under test suffers navigational failure!|",
    "|Obstacle ship experiences grounding!|",
    "|Obstacle ship suffers navigational failure!|",
    "|Ship under test reaches its final destination!|",
    "|Ship under test goes outside the map horizon!|",
    "|Obstacle ship reaches its final destination!|",
    "|Obstacle ship goes outside the map horizon!|",
    "|Simulation reaches its time limit|",
    "|Learning agent samples false intermediate waypoints!|",
)

# ship state fields (get/set_state)
F_NORTH, F_EAST, F_YAW, F_U, F_V, F_R, F_OMEGA, F_TIME, F_E_CT, F_E_CT_INT = range(10)
F_HDG_EI, F_HDG_PREV, F_SPD_A, F_SPD_B, F_RUDDER, F_THRUST, F_LOG_ECT, F_NEXT_WPT, F_STOP = range(10, 19)
N_SHIP_FIELDS = 19
E_SAMPLING_COUNT, E_TRAVEL_DIST, E_TRAVEL_TIME, E_ACC_REWARD, E_N_BASE, E_E_BASE = range(100, 106)
E_SBMPC_P_LAST, E_SBMPC_CHI_LAST, E_ROUTE_LEN, E_ROUTE_NORTH, E_ROUTE_EAST = range(106, 111)
INT_FIELDS = {F_NEXT_WPT, F_STOP, E_SAMPLING_COUNT, E_ROUTE_LEN}

# trajectory record columns (shipsim_set_trajectory)
TRAJ_SHIP_COLS = 20
(TS_TIME, TS_NORTH, TS_EAST, TS_YAW, TS_RUDDER, TS_U, TS_V, TS_R, TS_OMEGA, TS_THRUST, TS_E_CT, TS_E_PSI, TS_LOAD,
 TS_FUEL_ME, TS_FUEL_EL, TS_FUEL, TS_E_CT_INT, TS_NEXT_WPT, TS_REPEAT, TS_TIME_LIST) = range(20)
TRAJ_ENV_COLS = 8
(TE_R_COLLISION, TE_R_TEST_GROUNDING, TE_R_TEST_NAV, TE_R_OBS_GROUNDING, TE_R_OBS_NAV, TE_R_TOTAL, TE_BITS,
 TE_FLAGS) = range(8)
TE_FLAG_COLLISION, TE_FLAG_IMMINENT = 1, 2
SBMPC_IN = 17
SBMPC_MULTI_IN = 10 + 7 * MAX_OBS  # shipsim_sbmpc_eval_multi rows (include/shipsim.h)


def events_to_string(bits):
    """Rebuild env_info['events'] from the event bits (same concatenation order as the reference)."""
    return "".join(s for i, s in enumerate(EVENT_STRINGS) if bits & (1 << i))


class ShipConfig(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "dead_weight_tonnage", "coefficient_of_deadweight_to_displacement", "bunkers", "ballast",
        "length_of_ship", "width_of_ship", "added_mass_coefficient_in_surge", "added_mass_coefficient_in_sway",
        "added_mass_coefficient_in_yaw", "mass_over_linear_friction_coefficient_in_surge",
        "mass_over_linear_friction_coefficient_in_sway", "mass_over_linear_friction_coefficient_in_yaw",
        "nonlinear_friction_coefficient_in_surge", "nonlinear_friction_coefficient_in_sway",
        "nonlinear_friction_coefficient_in_yaw", "initial_north_position_m", "initial_east_position_m",
        "initial_yaw_angle_rad", "initial_forward_speed_m_per_s", "initial_sideways_speed_m_per_s",
        "initial_yaw_rate_rad_per_s", "rudder_angle_to_sway_force_coefficient",
        "rudder_angle_to_yaw_force_coefficient", "max_rudder_angle_degrees", "hotel_load",
        "main_engine_capacity", "electrical_capacity", "rated_speed_main_engine_rpm",
        "linear_friction_main_engine", "linear_friction_hybrid_shaft_generator",
        "gear_ratio_between_main_engine_and_propeller", "gear_ratio_between_hybrid_shaft_generator_and_propeller",
        "propeller_inertia", "propeller_speed_to_torque_coefficient", "propeller_diameter",
        "propeller_speed_to_thrust_force_coefficient", "initial_propeller_shaft_speed_rad_per_s",
        "kp_ship_speed", "ki_ship_speed", "kp_shaft_speed", "ki_shaft_speed", "initial_shaft_speed_integral_error",
        "speed_kp", "speed_ki", "speed_kd", "max_thrust", "heading_kp", "heading_kd", "heading_ki",
        "radius_of_acceptance", "lookahead_distance", "los_integral_gain", "los_integrator_windup_limit",
        "desired_forward_speed")] + [
        ("shaft_generator_state", C.c_int32), ("n_route", C.c_int32),
        ("route_north", C.c_double * MAX_ROUTE), ("route_east", C.c_double * MAX_ROUTE)]


class Config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("kind", C.c_int32), ("machinery", C.c_int32), ("collav", C.c_int32),
        ("max_sampling_frequency", C.c_int32), ("machinery_dt_quirk", C.c_int32), ("normalize_action", C.c_int32),
        ("n_ships", C.c_int32), ("time_step", C.c_double), ("simulation_time", C.c_double),
        ("env_radius_of_acceptance", C.c_double), ("current_velocity_component_from_north", C.c_double),
        ("current_velocity_component_from_east", C.c_double), ("wind_speed", C.c_double),
        ("wind_direction", C.c_double), ("sbmpc_tf", C.c_double), ("sbmpc_dt", C.c_double),
        ("action_low", C.c_float), ("action_high", C.c_float), ("ship", ShipConfig * MAX_SHIPS),
        ("n_polys", C.c_int32), ("poly_start", C.c_int32 * (MAX_POLYS + 1)),
        ("poly_east", C.c_double * MAX_VERTS), ("poly_north", C.c_double * MAX_VERTS),
        ("lanes_per_env", C.c_int32), ("envs_per_wave", C.c_int32), ("map_query", C.c_int32),
        ("reserved", C.c_int32 * 5)]


# ------------------------------------------------------------------------------------------
# reference scenario data
# ------------------------------------------------------------------------------------------
MAP_DATA = (  # run/env_setup.py:145-152 == run_colav/run_simplified_model.py:121-128, (east, north)
    ((0, 10000), (10000, 10000), (9200, 9000), (7600, 8500), (6700, 7300), (4900, 6500), (4300, 5400),
     (4700, 4500), (6000, 4000), (5800, 3600), (4200, 3200), (3200, 4100), (2000, 4500), (1000, 4000),
     (900, 3500), (500, 2600), (0, 2350)),
    ((10000, 0), (11500, 750), (12000, 2000), (11700, 3000), (11000, 3600), (11250, 4250), (12300, 4000),
     (13000, 3800), (14000, 3000), (14500, 2300), (15000, 1700), (16000, 800), (17500, 0)),
    ((15500, 10000), (16000, 9000), (18000, 8000), (19000, 7500), (20000, 6000), (20000, 10000)),
    ((5500, 5300), (6000, 5000), (6800, 4500), (8000, 5000), (8700, 5500), (9200, 6700), (8000, 7000),
     (6700, 6300), (6000, 6000)),
    ((15000, 5000), (14000, 5500), (12500, 5000), (14000, 4100), (16000, 2000), (15700, 3700)),
    ((11000, 2000), (10300, 3200), (9000, 1500), (10000, 1000)),
)
# (north, east) waypoints
TEST_SHIP_ROUTE = ((0, 0), (2000, 4500), (2500, 7500), (7000, 12000), (6500, 16000), (3000, 17500), (0, 20000))
OBS_SHIP_ROUTE = ((10000, 15000), (0, 5000))  # rl_env/.../data/obs_ship_route.txt
OBS_SHIP_ROUTE_NONIW = ((10000, 15000), (9500, 13500), (8000, 13000), (6500, 12500), (6000, 11000),
                        (5500, 9500), (4000, 9000), (2500, 8500), (2000, 7000), (1500, 5500), (0, 5000))


def _ship_common(s, north, east, yaw, u):
    # ShipConfiguration (env_setup.py:39-55)
    s.coefficient_of_deadweight_to_displacement = 0.7
    s.bunkers = 200000
    s.ballast = 200000
    s.length_of_ship = 80
    s.width_of_ship = 16
    s.added_mass_coefficient_in_surge = 0.4
    s.added_mass_coefficient_in_sway = 0.4
    s.added_mass_coefficient_in_yaw = 0.4
    s.dead_weight_tonnage = 3850000
    s.mass_over_linear_friction_coefficient_in_surge = 130
    s.mass_over_linear_friction_coefficient_in_sway = 18
    s.mass_over_linear_friction_coefficient_in_yaw = 90
    s.nonlinear_friction_coefficient_in_surge = 2400
    s.nonlinear_friction_coefficient_in_sway = 4000
    s.nonlinear_friction_coefficient_in_yaw = 400
    s.initial_north_position_m = north
    s.initial_east_position_m = east
    s.initial_yaw_angle_rad = yaw
    s.initial_forward_speed_m_per_s = u
    s.initial_sideways_speed_m_per_s = 0
    s.initial_yaw_rate_rad_per_s = 0
    s.rudder_angle_to_sway_force_coefficient = 50e3
    s.rudder_angle_to_yaw_force_coefficient = 500e3
    s.max_rudder_angle_degrees = 30
    # MachinerySystemConfiguration + PTI mode (env_setup.py:69-105)
    s.hotel_load = 200000
    s.main_engine_capacity = 0
    s.electrical_capacity = 2 * 510e3
    s.shaft_generator_state = SG_MOTOR
    s.rated_speed_main_engine_rpm = 1000
    s.linear_friction_main_engine = 68
    s.linear_friction_hybrid_shaft_generator = 57
    s.gear_ratio_between_main_engine_and_propeller = 0.6
    s.gear_ratio_between_hybrid_shaft_generator_and_propeller = 0.6
    s.propeller_inertia = 6000
    s.propeller_diameter = 3.1
    s.propeller_speed_to_torque_coefficient = 7.5
    s.propeller_speed_to_thrust_force_coefficient = 1.7
    # ThrottleControllerGains (env_setup.py:157-165)
    s.kp_ship_speed = 205.25
    s.ki_ship_speed = 0.0525
    s.kp_shaft_speed = 50
    s.ki_shaft_speed = 0.00025
    s.initial_shaft_speed_integral_error = 114
    s.max_thrust = math.inf
    # LOS (env_setup.py:170-175 with runner defaults)
    s.radius_of_acceptance = 300
    s.lookahead_distance = 1000
    s.los_integral_gain = 0.002
    s.los_integrator_windup_limit = 4000


def _set_route(s, route):
    s.n_route = len(route)
    for i, (n, e) in enumerate(route):
        s.route_north[i] = n
        s.route_east[i] = e


def _set_map(cfg, map_data=MAP_DATA):
    cfg.n_polys = len(map_data)
    k = 0
    for p, poly in enumerate(map_data):
        cfg.poly_start[p] = k
        for (e, n) in poly:
            cfg.poly_east[k] = e
            cfg.poly_north[k] = n
            k += 1
    cfg.poly_start[len(map_data)] = k


def _base(kind, collav, time_step, machinery):
    cfg = Config()
    cfg.abi_version = ABI_VERSION
    cfg.kind = kind
    cfg.machinery = machinery
    cfg.collav = COLLAV[collav] if not isinstance(collav, int) else collav
    cfg.max_sampling_frequency = 9
    cfg.machinery_dt_quirk = 1
    cfg.normalize_action = 0
    cfg.n_ships = 1 if kind == KIND_SINGLE else 2
    cfg.time_step = time_step
    cfg.simulation_time = 10000
    cfg.env_radius_of_acceptance = 300
    cfg.current_velocity_component_from_north = -1
    cfg.current_velocity_component_from_east = -1
    cfg.wind_speed = 2
    cfg.wind_direction = -np.pi / 4
    cfg.sbmpc_tf = 1000
    cfg.sbmpc_dt = 20
    cfg.action_low = np.float32(-np.deg2rad(30))
    cfg.action_high = np.float32(np.deg2rad(30))
    _set_map(cfg)
    return cfg


# Further obstacle ships of the multi-obstacle scenarios (configs[4] C5, K > 1; beyond the reference,
# which builds one obstacle ship): (initial north, east, yaw [deg], speed, desired speed, route (north, east)).
# Routes run over water of the reference map: ship 2 sails the obstacle route in the opposite
# direction, ship 3 the test ship's route from its far end (head-on traffic), ship 4 the obstacle
# route from half way along it.
TRAFFIC_SHIPS = (
    (100.0, 5100.0, 45.0, 3.5, 4.0, ((0, 5000), (10000, 15000))),
    (3000.0, 17500.0, -23.2, 4.0, 4.0, ((3000, 17500), (6500, 16000), (7000, 12000), (2500, 7500), (2000, 4500),
                                        (0, 0))),
    (5000.0, 10000.0, -135.0, 3.5, 4.0, ((5000, 10000), (0, 5000))),
)


def ast_config(collav="sbmpc", time_step=4, machinery=MACH_DETAILED, n_obs_ships=1):
    """run/env_setup.py:prepare_multiship_rl_env (runner defaults). With machinery=MACH_SIMPLIFIED
    the ships become run_colav SimpleShipModel + ThrustFromSpeedSetPoint(150, 150, 75).
    n_obs_ships > 1 adds TRAFFIC_SHIPS[:K-1] as ships 2..K (include/shipsim.h shipsim_create)."""
    if not 1 <= n_obs_ships <= MAX_OBS:
        raise ValueError(f"n_obs_ships must be in 1..{MAX_OBS}")
    cfg = _base(KIND_AST, collav, time_step, machinery)
    cfg.n_ships = 1 + n_obs_ships
    for k in range(n_obs_ships - 1):
        north, east, yaw, u, ud, route = TRAFFIC_SHIPS[k]
        s = cfg.ship[2 + k]
        _ship_common(s, north, east, np.deg2rad(yaw), u)
        s.initial_propeller_shaft_speed_rad_per_s = 200 * np.pi / 30
        s.heading_kp, s.heading_kd, s.heading_ki = 1.65, 75, 0.001
        s.speed_kp, s.speed_ki, s.speed_kd = 150, 150, 75
        s.desired_forward_speed = ud
        _set_route(s, route)
    t, o = cfg.ship[0], cfg.ship[1]
    _ship_common(t, 100, 100, 60 * np.pi / 180, 4.25)
    _ship_common(o, 9900, 14900, -135 * np.pi / 180, 3.5)
    t.initial_propeller_shaft_speed_rad_per_s = 420 * np.pi / 30
    o.initial_propeller_shaft_speed_rad_per_s = 200 * np.pi / 30
    for s in (t, o):
        s.heading_kp, s.heading_kd, s.heading_ki = 1.65, 75, 0.001
        s.speed_kp, s.speed_ki, s.speed_kd = 150, 150, 75
    t.desired_forward_speed = 4.5
    o.desired_forward_speed = 4.0
    _set_route(t, TEST_SHIP_ROUTE)
    _set_route(o, OBS_SHIP_ROUTE)
    return cfg


# MachineryModeParams of run/env_setup.py:62-81 (main_engine_capacity 2160 kW, diesel_gen_capacity 510 kW)
MACHINERY_MODES = {
    "PTO": (2160e3, 0.0, SG_GEN),         # pto_mode :62-67
    "PTI": (0.0, 2 * 510e3, SG_MOTOR),    # pti_mode :69-74 (the mode the runner uses, :82-84)
    "MEC": (2160e3, 510e3, SG_OFF),       # mec_mode :76-81
}


def set_machinery_mode(cfg, mode, ships=(0, 1)):
    """Select the active MachineryMode of the given ships (MachineryModes([mode]) with
    machinery_operating_mode=0): PTO / PTI / MEC with the env_setup capacities."""
    me, el, sg = MACHINERY_MODES[mode]
    for i in ships:
        s = cfg.ship[i]
        s.main_engine_capacity = me
        s.electrical_capacity = el
        s.shaft_generator_state = sg
    return cfg


def c1_config(collav="none", time_step=30):
    """run_colav/run_simplified_model.py:55-233 (MultiShipNonIWEnv)."""
    cfg = _base(KIND_NONIW, collav, time_step, MACH_SIMPLIFIED)
    t, o = cfg.ship[0], cfg.ship[1]
    _ship_common(t, 100, 100, 60 * np.pi / 180, 4.25)
    _ship_common(o, 9900, 14900, -135 * np.pi / 180, 3.5)
    t.speed_kp, t.speed_ki, t.speed_kd = 150, 150, 75
    o.speed_kp, o.speed_ki, o.speed_kd = .025, 700.5, 550.5
    t.heading_kp, t.heading_ki, t.heading_kd = .5, 0.01, 84
    o.heading_kp, o.heading_ki, o.heading_kd = .65, 0.001, 50
    t.desired_forward_speed = 4.5
    o.desired_forward_speed = 4.0
    _set_route(t, TEST_SHIP_ROUTE)  # own_ship_route.txt == test_ship_route.txt
    _set_route(o, OBS_SHIP_ROUTE_NONIW)
    cfg.action_low = np.float32(-np.pi / 6)
    cfg.action_high = np.float32(np.pi / 6)
    return cfg


def c2_config(time_step=30):
    """Single SimpleShipModel + ThrustFromSpeedSetPoint + HeadingByRouteController (C2 unit)."""
    cfg = c1_config("none", time_step)
    cfg.kind = KIND_SINGLE
    cfg.n_ships = 1
    return cfg


def c2_initial_states(n, seed=20251015):
    """SURVEY.md §8(d) C2 input: perturbations of C1's test ship from PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((n, 4))
    for k in range(n):
        out[k, 0] = 100 + rng.uniform(-200, 200)
        out[k, 1] = 100 + rng.uniform(-200, 200)
        out[k, 2] = 60 * np.pi / 180 + rng.uniform(-np.deg2rad(10), np.deg2rad(10))
        out[k, 3] = rng.uniform(3.5, 5.0)
    return out


def ast_action_table(n_envs, n_dec=9, seed=20251015):
    """SURVEY.md §8(d) C3 input: per-env normalized actions U(-1, 1) from PCG64(seed + env_id)."""
    out = np.empty((n_envs, n_dec), np.float32)
    for i in range(n_envs):
        out[i] = np.random.Generator(np.random.PCG64(seed + i)).uniform(-1, 1, n_dec).astype(np.float32)
    return out


def normalized_to_scoping(a_norm, low=np.float32(-np.deg2rad(30)), high=np.float32(np.deg2rad(30))):
    """NormalizedBoxEnv.step's float32 mapping (ast_sac/env_wrapper/normalized_box_env.py:48-51)."""
    a = np.asarray(a_norm, np.float32)
    lb, ub = np.float32(low), np.float32(high)
    return np.clip(lb + (a + np.float32(1.)) * np.float32(0.5) * (ub - lb), lb, ub).astype(np.float32)
