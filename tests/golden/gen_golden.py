"""Generate golden fixtures by running the reference (AndreasKing-Goks/ast-sac) in THIS container.

TEST INFRASTRUCTURE ONLY.  Never imported by the product, by bench.py or by the GPU tests;
it needs /root/reference, which does not exist on the GPU box.  The fixtures it writes
(tests/golden/*.npz, data only) are what travel.

Run:   python3 -B tests/golden/gen_golden.py          (from the repo root)

What runs is the reference's own code: ship_model / ship_engine / controllers / LOS_guidance /
sbmpc / check_condition / reward_function / env.py / run_colav/env.py / ast_sac SACTrainer.
Three third-party imports are absent from the image and are replaced here, in-process, by
stand-ins:

* gymnasium (pinned 1.1.1 in ast-sac.yml): only `Env`, `spaces.Box`, `utils.seeding` are used
  and none of them does arithmetic on the env path -> trivial containers.
* gtimer (1.0.0b5): timing stamps only -> no-ops.
* shapely (2.0.6 / GEOS 3.10.6): `Polygon.contains(Point)` and `Polygon.exterior.distance(Point)`
  ARE arithmetic.  The stand-in restates GEOS' published algorithms (RayCrossingCounter for
  point-in-ring with "boundary is not interior", Distance::pointToSegment for the ring
  distance).  The fixtures are therefore pinned to the reference everywhere except at exact
  polygon-boundary points, which the reference's own tests never pin either ("parity unpinned"
  there).
"""
import argparse
import copy
import math
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------------------
# stand-ins for the missing third-party packages
# ----------------------------------------------------------------------------------------------
def _install_stubs():
    gym = types.ModuleType("gymnasium")

    class Env:
        def __init__(self, *a, **k):
            pass

    gym.Env = Env
    spaces = types.ModuleType("gymnasium.spaces")

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            low = np.asarray(low)
            high = np.asarray(high)
            if shape is not None:
                low = np.full(shape, low)
                high = np.full(shape, high)
            self.low = low.astype(dtype)
            self.high = high.astype(dtype)
            self.shape = self.low.shape
            self.dtype = np.dtype(dtype)

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Tuple:
        def __init__(self, spaces_):
            self.spaces = spaces_

    spaces.Box, spaces.Discrete, spaces.Tuple = Box, Discrete, Tuple
    gym.spaces = spaces
    utils = types.ModuleType("gymnasium.utils")
    seeding = types.ModuleType("gymnasium.utils.seeding")
    seeding.np_random = lambda seed=None: (np.random.default_rng(seed), seed)
    utils.seeding = seeding
    gym.utils = utils
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces,
                        "gymnasium.utils": utils, "gymnasium.utils.seeding": seeding})

    gt = types.ModuleType("gtimer")
    gt.stamp = lambda *a, **k: None
    gt.blank_stamp = lambda *a, **k: None
    gt.timed_for = lambda it, **k: it
    gt.reset_root = lambda *a, **k: None
    gt.get_times = lambda *a, **k: None
    sys.modules["gtimer"] = gt

    shp = types.ModuleType("shapely")
    geom = types.ModuleType("shapely.geometry")

    class Point:
        def __init__(self, x, y):
            self.x = float(x)
            self.y = float(y)

    def _pt_seg(px, py, ax, ay, bx, by):
        # GEOS Distance::pointToSegment
        if ax == bx and ay == by:
            return math.hypot(px - ax, py - ay)
        dx, dy = bx - ax, by - ay
        len2 = dx * dx + dy * dy
        r = ((px - ax) * dx + (py - ay) * dy) / len2
        if r <= 0.0:
            return math.hypot(px - ax, py - ay)
        if r >= 1.0:
            return math.hypot(px - bx, py - by)
        s = ((ay - py) * dx - (ax - px) * dy) / len2
        return abs(s) * math.sqrt(len2)

    class _Ring:
        def __init__(self, verts):
            self.coords = list(verts) + [verts[0]]

        def distance(self, p):
            c = self.coords
            return min(_pt_seg(p.x, p.y, c[i][0], c[i][1], c[i + 1][0], c[i + 1][1])
                       for i in range(len(c) - 1))

    class Polygon:
        def __init__(self, verts):
            self.exterior = _Ring([(float(a), float(b)) for a, b in verts])

        def contains(self, p):
            # GEOS RayCrossingCounter; a point on the boundary is not contained
            c = self.exterior.coords
            crossings = 0
            for i in range(len(c) - 1):
                x1, y1 = c[i]
                x2, y2 = c[i + 1]
                if x1 < p.x and x2 < p.x:
                    continue
                if p.x == x2 and p.y == y2:
                    return False
                if y1 == p.y and y2 == p.y:
                    minx, maxx = min(x1, x2), max(x1, x2)
                    if minx <= p.x <= maxx:
                        return False
                    continue
                if (y1 > p.y and y2 <= p.y) or (y2 > p.y and y1 <= p.y):
                    det = (x2 - x1) * (p.y - y1) - (y2 - y1) * (p.x - x1)
                    sign = (det > 0) - (det < 0)
                    if sign == 0:
                        return False
                    if y2 < y1:
                        sign = -sign
                    if sign > 0:
                        crossings += 1
            return (crossings & 1) == 1

    geom.Point, geom.Polygon = Point, Polygon
    shp.geometry = geom
    sys.modules.update({"shapely": shp, "shapely.geometry": geom})

    import matplotlib
    matplotlib.use("Agg")


_install_stubs()
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

MAP_DATA = [
    [(0, 10000), (10000, 10000), (9200, 9000), (7600, 8500), (6700, 7300), (4900, 6500), (4300, 5400),
     (4700, 4500), (6000, 4000), (5800, 3600), (4200, 3200), (3200, 4100), (2000, 4500), (1000, 4000),
     (900, 3500), (500, 2600), (0, 2350)],
    [(10000, 0), (11500, 750), (12000, 2000), (11700, 3000), (11000, 3600), (11250, 4250), (12300, 4000),
     (13000, 3800), (14000, 3000), (14500, 2300), (15000, 1700), (16000, 800), (17500, 0)],
    [(15500, 10000), (16000, 9000), (18000, 8000), (19000, 7500), (20000, 6000), (20000, 10000)],
    [(5500, 5300), (6000, 5000), (6800, 4500), (8000, 5000), (8700, 5500), (9200, 6700), (8000, 7000),
     (6700, 6300), (6000, 6000)],
    [(15000, 5000), (14000, 5500), (12500, 5000), (14000, 4100), (16000, 2000), (15700, 3700)],
    [(11000, 2000), (10300, 3200), (9000, 1500), (10000, 1000)],
]

# Termination-flag bit order used by every fixture and by the build (reward_function.py:204-262)
EVENT_STRINGS = [
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
]


def events_to_bits(s):
    bits = 0
    rest = s
    for i, e in enumerate(EVENT_STRINGS):
        if e in rest:
            bits |= 1 << i
            rest = rest.replace(e, "", 1)
    assert rest == "", (s, rest)
    return bits


def ns(**kw):
    return argparse.Namespace(**kw)


# ----------------------------------------------------------------------------------------------
# F2: C2 unit — single SimpleShipModel + ThrustFromSpeedSetPoint + HeadingByRouteController
# ----------------------------------------------------------------------------------------------
def c1_configs(time_step):
    from run_colav.ship_in_transit.sub_systems.ship_model import (ShipConfiguration, EnvironmentConfiguration,
                                                                 SimulationConfiguration)
    from run_colav.ship_in_transit.sub_systems.ship_engine import RudderConfiguration
    ship_config = ShipConfiguration(
        coefficient_of_deadweight_to_displacement=0.7, bunkers=200000, ballast=200000, length_of_ship=80,
        width_of_ship=16, added_mass_coefficient_in_surge=0.4, added_mass_coefficient_in_sway=0.4,
        added_mass_coefficient_in_yaw=0.4, dead_weight_tonnage=3850000,
        mass_over_linear_friction_coefficient_in_surge=130, mass_over_linear_friction_coefficient_in_sway=18,
        mass_over_linear_friction_coefficient_in_yaw=90, nonlinear_friction_coefficient__in_surge=2400,
        nonlinear_friction_coefficient__in_sway=4000, nonlinear_friction_coefficient__in_yaw=400)
    env_config = EnvironmentConfiguration(current_velocity_component_from_north=-1,
                                          current_velocity_component_from_east=-1, wind_speed=2,
                                          wind_direction=-np.pi / 4)
    rudder_config = RudderConfiguration(rudder_angle_to_sway_force_coefficient=50e3,
                                        rudder_angle_to_yaw_force_coefficient=500e3, max_rudder_angle_degrees=30)

    def sim(n, e, psi, u):
        return SimulationConfiguration(initial_north_position_m=n, initial_east_position_m=e,
                                       initial_yaw_angle_rad=psi, initial_forward_speed_m_per_s=u,
                                       initial_sideways_speed_m_per_s=0, initial_yaw_rate_rad_per_s=0,
                                       integration_step=time_step, simulation_time=10000)
    return ship_config, env_config, rudder_config, sim


def gen_c2():
    from run_colav.ship_in_transit.sub_systems.ship_model import SimpleShipModel
    from run_colav.ship_in_transit.sub_systems.LOS_guidance import LosParameters
    from run_colav.ship_in_transit.sub_systems.controllers import (SpeedControllerGains, HeadingControllerGains,
                                                                  ThrustFromSpeedSetPoint, HeadingByRouteController)
    route = os.path.join(REF, "run_colav/ship_in_transit/data/own_ship_route.txt")
    out = {}
    rng = np.random.Generator(np.random.PCG64(20251015))
    for dt, m in ((30, 4), (4, 2)):
        ship_config, env_config, rudder_config, sim = c1_configs(dt)
        inits = []
        traces = []
        finals = []
        for k in range(m):
            n0 = 100 + rng.uniform(-200, 200)
            e0 = 100 + rng.uniform(-200, 200)
            p0 = 60 * np.pi / 180 + rng.uniform(-np.deg2rad(10), np.deg2rad(10))
            u0 = rng.uniform(3.5, 5.0)
            inits.append([n0, e0, p0, u0])
            ship = SimpleShipModel(ship_config=ship_config, rudder_config=rudder_config,
                                   environment_config=env_config, simulation_config=sim(n0, e0, p0, u0))
            ctrl = ThrustFromSpeedSetPoint(gains=SpeedControllerGains(kp=150, ki=150, kd=75), max_thrust=np.inf,
                                           time_step=dt)
            ap = HeadingByRouteController(route, heading_controller_gains=HeadingControllerGains(kp=.5, ki=0.01,
                                                                                                 kd=84),
                                          los_parameters=LosParameters(radius_of_acceptance=300,
                                                                       lookahead_distance=1000,
                                                                       integral_gain=0.002,
                                                                       integrator_windup_limit=4000),
                                          time_step=dt, max_rudder_angle=np.deg2rad(30))
            rows = []
            while ship.int.time < ship.int.sim_time:
                rudder = ap.rudder_angle_from_route(north_position=ship.north, east_position=ship.east,
                                                    heading=ship.yaw_angle)
                thrust = ctrl.thrust(speed_set_point=4.5, measured_speed=ship.forward_speed)
                rows.append([ship.int.time, ship.north, ship.east, ship.yaw_angle, ship.forward_speed,
                             ship.sideways_speed, ship.yaw_rate, rudder, thrust, ap.navigate.e_ct,
                             ap.navigate.e_ct_int, ap.next_wpt])
                ship.store_simulation_data(thrust, rudder, ap.navigate.e_ct, 0.0)
                ship.update_differentials(thrust_force=thrust, rudder_angle=rudder)
                ship.integrate_differentials()
                ship.int.next_time()
            traces.append(rows)
            finals.append([ship.int.time, ship.north, ship.east, ship.yaw_angle, ship.forward_speed,
                           ship.sideways_speed, ship.yaw_rate])
        out[f"dt{dt}_init"] = np.array(inits)
        out[f"dt{dt}_trace"] = np.array(traces)
        out[f"dt{dt}_final"] = np.array(finals)
    out["trace_cols"] = np.array(["time", "north", "east", "yaw", "u", "v", "r", "rudder", "thrust", "e_ct",
                                  "e_ct_int", "next_wpt"])
    np.savez_compressed(os.path.join(OUT, "c2_single_ship.npz"), **out)
    print("c2:", {k: v.shape for k, v in out.items()})


# ----------------------------------------------------------------------------------------------
# F1: C1 two-ship NonIW loop (run_colav/run_simplified_model.py:55-249)
# ----------------------------------------------------------------------------------------------
def build_c1_env(collav, time_step=30):
    from run_colav.env import MultiShipNonIWEnv, ShipAssets
    from run_colav.ship_in_transit.sub_systems.ship_model import SimpleShipModel
    from run_colav.ship_in_transit.sub_systems.LOS_guidance import LosParameters
    from run_colav.ship_in_transit.sub_systems.obstacle import PolygonObstacle
    from run_colav.ship_in_transit.sub_systems.controllers import (SpeedControllerGains, HeadingControllerGains,
                                                                  ThrustFromSpeedSetPoint,
                                                                  HeadingBySampledRouteController)
    ship_config, env_config, rudder_config, sim = c1_configs(time_step)
    test_ship = SimpleShipModel(ship_config=ship_config, rudder_config=rudder_config, environment_config=env_config,
                                simulation_config=sim(100, 100, 60 * np.pi / 180, 4.25))
    obs_ship = SimpleShipModel(ship_config=ship_config, rudder_config=rudder_config, environment_config=env_config,
                               simulation_config=sim(9900, 14900, -135 * np.pi / 180, 3.5))
    los = LosParameters(radius_of_acceptance=300, lookahead_distance=1000, integral_gain=0.002,
                        integrator_windup_limit=4000)
    d = os.path.join(REF, "run_colav/ship_in_transit/data")
    test = ShipAssets(ship_model=test_ship,
                      speed_controller=ThrustFromSpeedSetPoint(gains=SpeedControllerGains(kp=150, ki=150, kd=75),
                                                               max_thrust=np.inf, time_step=time_step),
                      auto_pilot=HeadingBySampledRouteController(
                          os.path.join(d, "own_ship_route.txt"),
                          heading_controller_gains=HeadingControllerGains(kp=.5, ki=0.01, kd=84),
                          los_parameters=los, time_step=time_step, max_rudder_angle=np.deg2rad(30),
                          num_of_samplings=2),
                      desired_forward_speed=4.5, integrator_term=[], time_list=[], stop_flag=False,
                      type_tag="test_ship")
    obs = ShipAssets(ship_model=obs_ship,
                     speed_controller=ThrustFromSpeedSetPoint(gains=SpeedControllerGains(kp=.025, ki=700.5,
                                                                                         kd=550.5),
                                                              max_thrust=np.inf, time_step=time_step),
                     auto_pilot=HeadingBySampledRouteController(
                         os.path.join(d, "obs_ship_route_nonIW.txt"),
                         heading_controller_gains=HeadingControllerGains(kp=.65, ki=0.001, kd=50),
                         los_parameters=los, time_step=time_step, max_rudder_angle=np.deg2rad(30),
                         num_of_samplings=2),
                     desired_forward_speed=4.0, integrator_term=[], time_list=[], stop_flag=False,
                     type_tag="obs_ship")
    args = ns(max_sampling_frequency=9, time_step=time_step, radius_of_acceptance=300, lookahead_distance=1000,
              collav_mode=collav, ship_draw=False, time_since_last_ship_drawing=30, normalize_action=False)
    env = MultiShipNonIWEnv(assets=[test, obs], map=PolygonObstacle(MAP_DATA), args=args)
    return env, test, obs


SR_KEYS = ["time [s]", "north position [m]", "east position [m]", "yaw angle [deg]", "rudder angle [deg]",
           "forward speed [m/s]", "sideways speed [m/s]", "yaw rate [deg/sec]", "thrust force [kN]",
           "cross track error [m]", "heading error [deg]"]


def sr_array(ship, keys=SR_KEYS):
    r = ship.simulation_results
    return np.array([r[k] for k in keys], dtype=np.float64).T


def gen_c1():
    out = {}
    for collav in ("none", "sbmpc", "simple"):
        env, test, obs = build_c1_env(collav)
        env.init_step()
        bits = []
        stops = []
        while test.ship_model.int.time < test.ship_model.int.sim_time:
            _, done, info = env._step()
            bits.append(events_to_bits(info["events"]))
            stops.append([test.stop_flag, obs.stop_flag, bool(done)])
        out[f"{collav}_test_log"] = sr_array(test.ship_model)
        out[f"{collav}_obs_log"] = sr_array(obs.ship_model)
        out[f"{collav}_event_bits"] = np.array(bits, dtype=np.int64)
        out[f"{collav}_stops"] = np.array(stops, dtype=np.int64)
        out[f"{collav}_final"] = np.array([[s.ship_model.int.time, s.ship_model.north, s.ship_model.east,
                                            s.ship_model.yaw_angle, s.ship_model.forward_speed,
                                            s.ship_model.sideways_speed, s.ship_model.yaw_rate]
                                           for s in (test, obs)])
        print("c1", collav, "ticks", len(bits), "final time", test.ship_model.int.time)
    out["log_cols"] = np.array(SR_KEYS)
    np.savez_compressed(os.path.join(OUT, "c1_noniw.npz"), **out)


# ----------------------------------------------------------------------------------------------
# F3 + F4: the RL env (run/env_setup.py) with ShipModelAST detailed PTI machinery
# ----------------------------------------------------------------------------------------------
AST_KEYS = ["time [s]", "north position [m]", "east position [m]", "yaw angle [deg]", "rudder angle [deg]",
            "forward speed [m/s]", "sideways speed [m/s]", "yaw rate [deg/sec]", "propeller shaft speed [rpm]",
            "thrust force [kN]", "cross track error [m]", "heading error [deg]", "fuel consumption [kg]"]


def rl_args(collav, time_step=4):
    return ns(max_sampling_frequency=9, time_step=time_step, radius_of_acceptance=300, lookahead_distance=1000,
              collav_mode=collav, ship_draw=False, time_since_last_ship_drawing=30, normalize_action=False)


def gen_ast_single():
    """ShipModelAST + EngineThrottleFromSpeedSetPoint + sampled-route autopilot; before/after reset (Q1)."""
    from run.env_setup import prepare_multiship_rl_env
    env, assets = prepare_multiship_rl_env(rl_args("none"))
    test = assets[0]
    out = {}
    for phase in ("fresh", "after_reset"):
        if phase == "after_reset":
            test.ship_model.reset()
            test.throttle_controller.reset()
            test.auto_pilot.reset()
        m = test.ship_model
        out[f"{phase}_mach_dt"] = np.array(m.ship_machinery_model.int.dt)
        for _ in range(500):
            rudder = test.auto_pilot.rudder_angle_from_sampled_route(north_position=m.north, east_position=m.east,
                                                                     heading=m.yaw_angle)
            thr = test.throttle_controller.throttle(speed_set_point=4.5, measured_speed=m.forward_speed,
                                                    measured_shaft_speed=m.forward_speed)
            m.store_simulation_data(thr, rudder, test.auto_pilot.get_cross_track_error(),
                                    test.auto_pilot.get_heading_error())
            m.update_differentials(engine_throttle=thr, rudder_angle=rudder)
            m.integrate_differentials()
            m.int.next_time()
        out[f"{phase}_log"] = np.array([m.simulation_results[k] for k in AST_KEYS], dtype=np.float64).T
        out[f"{phase}_final"] = np.array([m.north, m.east, m.yaw_angle, m.forward_speed, m.sideways_speed,
                                          m.yaw_rate, m.ship_machinery_model.omega])
    out["log_cols"] = np.array(AST_KEYS)
    np.savez_compressed(os.path.join(OUT, "ast_single_ship.npz"), **out)
    print("ast single: mach dt fresh", out["fresh_mach_dt"], "after reset", out["after_reset_mach_dt"])


def scaled_action(a_norm):
    """NormalizedBoxEnv.step's float32 mapping onto the wrapped env's +-30 deg box
    (ast_sac/env_wrapper/normalized_box_env.py:48-51)."""
    lb = np.array([-np.deg2rad(30)], dtype=np.float32)
    ub = np.array([np.deg2rad(30)], dtype=np.float32)
    a = np.asarray(a_norm, dtype=np.float32).reshape(1)
    s = lb + (a + 1.) * 0.5 * (ub - lb)
    return np.clip(s, lb, ub)


class SimplifiedThrustAdapter:
    """Throttle-controller shaped adapter so the rl_env reward env can drive run_colav's
    SimpleShipModel (no reference script composes them; SURVEY.md §8(d) C3 input)."""

    def __init__(self, ctrl):
        self.ctrl = ctrl

    def throttle(self, speed_set_point, measured_speed, measured_shaft_speed):
        return self.ctrl.thrust(speed_set_point=speed_set_point, measured_speed=measured_speed)

    def reset(self):
        self.ctrl.reset()


def make_simplified_rl_env(collav):
    from run.env_setup import prepare_multiship_rl_env
    from rl_env.ship_in_transit.env import MultiShipRLEnv, ShipAssets
    from run_colav.ship_in_transit.sub_systems.ship_model import SimpleShipModel
    from run_colav.ship_in_transit.sub_systems.controllers import SpeedControllerGains, ThrustFromSpeedSetPoint

    class SimpleShipModelRL(SimpleShipModel):
        def update_differentials(self, engine_throttle=None, rudder_angle=None, *a, **k):
            return super().update_differentials(thrust_force=engine_throttle, rudder_angle=rudder_angle)

    args = rl_args(collav)
    ref_env, assets = prepare_multiship_rl_env(args)
    ship_config, env_config, rudder_config, sim = c1_configs(args.time_step)
    test_ship = SimpleShipModelRL(ship_config=ship_config, rudder_config=rudder_config,
                                  environment_config=env_config,
                                  simulation_config=sim(100, 100, 60 * np.pi / 180, 4.25))
    obs_ship = SimpleShipModelRL(ship_config=ship_config, rudder_config=rudder_config,
                                 environment_config=env_config,
                                 simulation_config=sim(9900, 14900, -135 * np.pi / 180, 3.5))
    new_assets = []
    for old, ship, gains in ((assets[0], test_ship, (150, 150, 75)), (assets[1], obs_ship, (150, 150, 75))):
        ctrl = ThrustFromSpeedSetPoint(gains=SpeedControllerGains(kp=gains[0], ki=gains[1], kd=gains[2]),
                                       max_thrust=np.inf, time_step=args.time_step)
        ap = copy.deepcopy(old.init_copy.auto_pilot)
        new_assets.append(ShipAssets(ship_model=ship, throttle_controller=SimplifiedThrustAdapter(ctrl),
                                     auto_pilot=ap, desired_forward_speed=old.desired_forward_speed,
                                     integrator_term=[], time_list=[], stop_flag=False, type_tag=old.type_tag))
    return MultiShipRLEnv(assets=new_assets, map=ref_env.map, args=args)


def run_rl_episodes(env, action_tables):
    """Drive env.reset()/env.step() exactly as ast_sac_rollout does (max_path_length 9)."""
    test, obs = env.test, env.obs
    ep = []
    for table in action_tables:
        o0 = env.reset()
        n_log0 = 0
        dec = []
        ticks = []
        for a_norm in table:
            a = scaled_action(a_norm)
            before = len(test.ship_model.simulation_results["time [s]"])
            o, r, d, info = env.step(a.copy())
            after = len(test.ship_model.simulation_results["time [s]"])
            dec.append(dict(a_norm=np.float32(a_norm), a=a[0], obs=np.asarray(o, np.float32), r=float(r),
                            done=bool(d), bits=events_to_bits(info["events"]), terminal=bool(info["terminal"]),
                            test_stop=bool(info["test_ship_stop"]), obs_stop=bool(info["obs_ship_stop"]),
                            nticks=after - before, sampling_count=env.sampling_count,
                            state=[test.ship_model.north, test.ship_model.east, test.ship_model.yaw_angle,
                                   test.ship_model.forward_speed, test.ship_model.sideways_speed,
                                   test.ship_model.yaw_rate, obs.ship_model.north, obs.ship_model.east,
                                   obs.ship_model.yaw_angle, obs.ship_model.forward_speed,
                                   obs.ship_model.sideways_speed, obs.ship_model.yaw_rate]))
            if d:
                break
        keys = AST_KEYS if hasattr(test.ship_model, "ship_machinery_model") else SR_KEYS
        ep.append(dict(o0=np.asarray(o0, np.float32), dec=dec,
                       test_log=np.array([test.ship_model.simulation_results[k] for k in keys], np.float64).T,
                       obs_log=np.array([obs.ship_model.simulation_results[k] for k in keys], np.float64).T,
                       r_tick=np.array(env.reward_tracker.total, np.float64),
                       obs_route=np.array([obs.auto_pilot.navigate.north, obs.auto_pilot.navigate.east]).T,
                       n_log0=n_log0))
    return ep


def pack_episodes(prefix, eps, out):
    out[f"{prefix}_n_episodes"] = np.array(len(eps))
    for i, e in enumerate(eps):
        p = f"{prefix}_ep{i}"
        out[p + "_o0"] = e["o0"]
        out[p + "_a_norm"] = np.array([d["a_norm"] for d in e["dec"]], np.float32)
        out[p + "_a"] = np.array([d["a"] for d in e["dec"]], np.float32)
        out[p + "_obs"] = np.array([d["obs"] for d in e["dec"]], np.float32)
        out[p + "_reward"] = np.array([d["r"] for d in e["dec"]], np.float64)
        out[p + "_done"] = np.array([d["done"] for d in e["dec"]], np.int64)
        out[p + "_bits"] = np.array([d["bits"] for d in e["dec"]], np.int64)
        out[p + "_terminal"] = np.array([d["terminal"] for d in e["dec"]], np.int64)
        out[p + "_test_stop"] = np.array([d["test_stop"] for d in e["dec"]], np.int64)
        out[p + "_obs_stop"] = np.array([d["obs_stop"] for d in e["dec"]], np.int64)
        out[p + "_nticks"] = np.array([d["nticks"] for d in e["dec"]], np.int64)
        out[p + "_state"] = np.array([d["state"] for d in e["dec"]], np.float64)
        out[p + "_test_log"] = e["test_log"]
        out[p + "_obs_log"] = e["obs_log"]
        out[p + "_r_tick"] = e["r_tick"]
        out[p + "_obs_route"] = e["obs_route"]


def action_tables():
    tabs = [np.zeros(9, np.float32)]
    for k in range(2):
        rng = np.random.Generator(np.random.PCG64(20251015 + k))
        tabs.append(rng.uniform(-1, 1, 9).astype(np.float32))
    tabs.append(np.ones(9, np.float32))       # IW drift -> sampling failure
    tabs.append(-np.ones(9, np.float32))
    return tabs


def gen_rl():
    from run.env_setup import prepare_multiship_rl_env
    tabs = action_tables()
    out = {}
    for collav in ("none", "sbmpc", "simple"):
        env, _ = prepare_multiship_rl_env(rl_args(collav))
        eps = run_rl_episodes(env, tabs)
        pack_episodes(collav, eps, out)
        for i, e in enumerate(eps):
            print("rl", collav, "ep", i, "decisions", len(e["dec"]), "ticks", [d["nticks"] for d in e["dec"]],
                  "bits", [hex(d["bits"]) for d in e["dec"]][-1], "rewards",
                  np.round([d["r"] for d in e["dec"]], 4))
    out["log_cols"] = np.array(AST_KEYS)
    np.savez_compressed(os.path.join(OUT, "rl_env_detailed.npz"), **out)

    out = {}
    for collav in ("none", "sbmpc"):
        env = make_simplified_rl_env(collav)
        eps = run_rl_episodes(env, tabs[:3])
        pack_episodes(collav, eps, out)
        for i, e in enumerate(eps):
            print("rl-simplified", collav, "ep", i, "ticks", [d["nticks"] for d in e["dec"]],
                  "bits", hex(e["dec"][-1]["bits"]))
    out["log_cols"] = np.array(SR_KEYS)
    np.savez_compressed(os.path.join(OUT, "rl_env_simplified.npz"), **out)


class _machinery_mode:
    """Build run/env_setup.py's scenario with MachineryModes([<mode>]) instead of [pti_mode]
    (env_setup.py:62-84 constructs pto/pti/mec modes; the runner only uses PTI). The mode objects
    the reference creates are captured and the requested one is handed to MachineryModes."""

    def __init__(self, state):  # 'GEN' (PTO), 'MOTOR' (PTI), 'OFF' (MEC)
        self.state = state

    def __enter__(self):
        import run.env_setup as es
        from rl_env.ship_in_transit.sub_systems import ship_engine as se
        made = []
        state = self.state

        class RecMode(se.MachineryMode):
            def __init__(self, params):
                super().__init__(params)
                made.append(self)

        class PickModes(se.MachineryModes):
            def __init__(self, list_of_modes):
                super().__init__([m for m in made if m.shaft_generator_state == state])

        self._es, self._saved = es, (es.MachineryMode, es.MachineryModes)
        es.MachineryMode, es.MachineryModes = RecMode, PickModes
        return self

    def __exit__(self, *exc):
        self._es.MachineryMode, self._es.MachineryModes = self._saved


MODE_TAGS = {"GEN": "pto", "MOTOR": "pti", "OFF": "mec"}


def gen_modes():
    """C5 machinery modes PTO / MEC: decision-level episodes like gen_rl (F4) for collav none/sbmpc."""
    from run.env_setup import prepare_multiship_rl_env
    tabs = action_tables()[:3]
    out = {}
    for state in ("GEN", "OFF"):
        for collav in ("none", "sbmpc"):
            with _machinery_mode(state):
                env, _ = prepare_multiship_rl_env(rl_args(collav))
            eps = run_rl_episodes(env, tabs)
            pack_episodes(f"{MODE_TAGS[state]}_{collav}", eps, out)
            for i, e in enumerate(eps):
                print("modes", state, collav, "ep", i, "ticks", [d["nticks"] for d in e["dec"]],
                      "bits", hex(e["dec"][-1]["bits"]), "fuel", e["test_log"][-1, -1])
    out["log_cols"] = np.array(AST_KEYS)
    np.savez_compressed(os.path.join(OUT, "rl_env_modes.npz"), **out)


REWARD_TRACKER_FIELDS = ("ship_collision", "test_ship_grounding", "test_ship_nav_failure", "obs_ship_grounding",
                         "obs_ship_nav_failure", "from_test_ship", "from_obs_ship", "total")


def gen_traj():
    """f1: the full simulation_results dict (every key, reference order) of both ships, the
    RewardTracker lists, ShipAssets.time_list / integrator_term, waypoint_sampling_times and the
    animation lists, for a few episodes (machinery modes x collav, incl. a sampling failure)."""
    from run.env_setup import prepare_multiship_rl_env
    tabs = action_tables()
    cases = [("MOTOR", "none", (1, 3)), ("MOTOR", "sbmpc", (2,)), ("MOTOR", "simple", (1,)),
             ("GEN", "none", (2,)), ("OFF", "none", (1,))]
    out = {}
    for state, collav, tab_ids in cases:
        with _machinery_mode(state):
            env, _ = prepare_multiship_rl_env(rl_args(collav))
        for k, ti in enumerate(tab_ids):
            p = f"{MODE_TAGS[state]}_{collav}_ep{k}"
            env.reset()
            acts = []
            for a_norm in tabs[ti]:
                a = scaled_action(a_norm)
                acts.append(a[0])
                _, _, d, _ = env.step(a.copy())
                if d:
                    break
            out[p + "_a"] = np.array(acts, np.float32)
            for name, ship in (("test", env.test), ("obs", env.obs)):
                sr = ship.ship_model.simulation_results
                keys = list(sr.keys())
                out[p + f"_{name}_keys"] = np.array(keys)
                out[p + f"_{name}_sr"] = np.array([sr[key] for key in keys], np.float64).T
                out[p + f"_{name}_time_list"] = np.array(ship.time_list, np.float64)
                out[p + f"_{name}_integrator_term"] = np.array(ship.integrator_term, np.float64)
            for f in REWARD_TRACKER_FIELDS:
                out[p + f"_rt_{f}"] = np.array(getattr(env.reward_tracker, f), np.float64)
            out[p + "_wst"] = np.array(env.waypoint_sampling_times, np.float64)
            out[p + "_waypoint_samples"] = np.array(env.waypoint_samples, np.float64).reshape(-1, 2)
            out[p + "_is_collision"] = np.array(env.is_collision_list, np.int64)
            out[p + "_imminent"] = np.array(env.is_collision_imminent_list, np.int64)
            print("traj", p, "rows", out[p + "_test_sr"].shape, "keys", len(out[p + "_test_keys"]),
                  "rt", len(out[p + "_rt_total"]), "wst", out[p + "_wst"])
    np.savez_compressed(os.path.join(OUT, "rl_env_traj.npz"), **out)


def gen_draw():
    """f4: ShipDraw snapshots (env.py:573-579, ship_model.py:612-624) with ship_draw=True over
    consecutive episodes of one env object (the drawing timer is env-level and survives reset,
    the drawings do not), plus the per-ship stop tick so the frozen-state case is visible."""
    from run.env_setup import prepare_multiship_rl_env
    tabs = action_tables()
    out = {}
    for collav, tab_ids in (("none", (1, 3, 0)), ("sbmpc", (2, 4))):
        args = rl_args(collav)
        args.ship_draw = True
        env, _ = prepare_multiship_rl_env(args)
        for k, ti in enumerate(tab_ids):
            p = f"{collav}_ep{k}"
            env.reset()
            acts = []
            for a_norm in tabs[ti]:
                a = scaled_action(a_norm)
                acts.append(a[0])
                _, _, d, _ = env.step(a.copy())
                if d:
                    break
            out[p + "_a"] = np.array(acts, np.float32)
            out[p + "_timer"] = np.float64(env.time_since_last_ship_drawing)
            for name, ship in (("test", env.test), ("obs", env.obs)):
                dr = ship.ship_model.ship_drawings
                out[p + f"_{name}_draw"] = np.array([np.stack([x, y]) for x, y in zip(dr[0], dr[1])],
                                                    np.float64).reshape(-1, 2, 6)
                out[p + f"_{name}_rows"] = np.int64(len(ship.ship_model.simulation_results["time [s]"]))
            print("draw", p, "snapshots", out[p + "_test_draw"].shape[0], out[p + "_obs_draw"].shape[0],
                  "rows", out[p + "_test_rows"], "timer", out[p + "_timer"])
    np.savez_compressed(os.path.join(OUT, "rl_env_draw.npz"), **out)


def gen_legacy(max_ticks=3000):
    """f4: the legacy per-tick MultiShipEnv (env.py:783-1181) on the scenario of record: per tick the
    next_states list, the 10 get_termination_status flags and done, for two consecutive episodes of one
    env object (self.states and the SBMPC memory survive reset), plus the ShipDraw snapshots."""
    from run.env_setup import prepare_multiship_rl_env
    from rl_env.ship_in_transit.env import MultiShipEnv
    out = {}
    for collav in ("none", "simple", "sbmpc"):
        args = rl_args(collav)
        rl_env, assets = prepare_multiship_rl_env(args)
        env = MultiShipEnv(assets=assets, map=rl_env.map, ship_draw=True, collav=collav,
                           time_since_last_ship_drawing=30, args=args)
        for ep in range(2):
            p = f"{collav}_ep{ep}"
            env.reset()
            states, conds, dones = [], [], []
            for _ in range(max_ticks):
                ns, done, cond = env.step()
                states.append(ns)
                conds.append([bool(c) for c in cond])
                dones.append(bool(done))
                if done:
                    break
            out[p + "_states"] = np.array(states, np.float64)
            out[p + "_cond"] = np.array(conds, np.int8)
            out[p + "_done"] = np.array(dones, np.int8)
            out[p + "_obs_stop"] = np.int8(env.obs.stop_flag)
            for name, ship in (("test", env.test), ("obs", env.obs)):
                dr = ship.ship_model.ship_drawings
                out[p + f"_{name}_draw"] = np.array([np.stack([x, y]) for x, y in zip(dr[0], dr[1])],
                                                    np.float64).reshape(-1, 2, 6)
            print("legacy", p, "ticks", len(dones), "done", dones[-1], "cond", np.nonzero(conds[-1])[0],
                  "obs_stop", env.obs.stop_flag, "near", int(np.sum(out[p + "_cond"][:, 4])))
    np.savez_compressed(os.path.join(OUT, "rl_env_legacy.npz"), **out)


# ----------------------------------------------------------------------------------------------
# F5 SBMPC known answers, F6 geometry / reward pure functions
# ----------------------------------------------------------------------------------------------
def gen_sbmpc_geometry():
    from rl_env.ship_in_transit.sub_systems.sbmpc import SBMPC
    from rl_env.ship_in_transit.sub_systems.obstacle import PolygonObstacle
    from rl_env.ship_in_transit.utils.compute_distance import get_distance_and_encounter_type
    from rl_env.ship_in_transit.evaluation.reward_function import (get_reward_due_to_ships_termination,
                                                                   ships_collision_reward,
                                                                   test_ship_grounding_reward,
                                                                   test_ship_nav_failure_reward,
                                                                   obs_ship_grounding_reward,
                                                                   obs_ship_nav_failure_reward)
    rng = np.random.Generator(np.random.PCG64(7))
    out = {}
    # SBMPC: one persistent controller, a sequence of calls (last-offset state carries over, Q7)
    sb = SBMPC(tf=1000, dt=20)
    ins, outs = [], []
    for k in range(64):
        os_state = np.array([rng.uniform(0, 20000), rng.uniform(0, 10000), rng.uniform(-np.pi, np.pi),
                             rng.uniform(0, 6), rng.uniform(-0.5, 0.5), rng.uniform(-0.01, 0.01)])
        ang = rng.uniform(-np.pi, np.pi)
        rad = rng.uniform(50, 2600) if k % 8 else 5000.0
        ob = np.array([os_state[0] + rad * np.cos(ang), os_state[1] + rad * np.sin(ang),
                       rng.uniform(-np.pi, np.pi), rng.uniform(0, 6), rng.uniform(-0.5, 0.5)])
        u_d = rng.uniform(3, 5)
        chi_d = rng.uniform(-4, 4)
        p, c = sb.get_optimal_ctrl_offset(u_d=u_d, chi_d=chi_d, os_state=os_state,
                                          do_list=[(0, ob, None, 80, 16)])
        ins.append(np.concatenate([[u_d, chi_d], os_state, ob]))
        outs.append([p, c, float(sb.is_stephen_useful()), sb._params.P_ca_last_, sb._params.Chi_ca_last_])
    out["sbmpc_in"] = np.array(ins)
    out["sbmpc_out"] = np.array(outs)
    sb2 = SBMPC(tf=1000, dt=20)
    out["sbmpc_survey_ka"] = np.array(sb2.get_optimal_ctrl_offset(
        u_d=4.5, chi_d=-1.0, os_state=np.array([1000, 1000, -1, 4.5, 0, 0]),
        do_list=[(0, np.array([2000, 1500, 2, 4, 0]), None, 80, 16)]), dtype=np.float64)

    # polygons (stand-in == restated GEOS) on random and near-coastline points
    pm = PolygonObstacle(MAP_DATA)
    pts = np.concatenate([np.stack([rng.uniform(-500, 10500, 3000), rng.uniform(-500, 20500, 3000)], 1),
                          np.stack([rng.uniform(3000, 7000, 1000), rng.uniform(3000, 9000, 1000)], 1)])
    out["poly_pts_ne"] = pts
    out["poly_inside"] = np.array([pm.if_pos_inside_obstacles(n, e) for n, e in pts], np.int64)
    out["poly_dist"] = np.array([pm.obstacles_distance(n, e) for n, e in pts])
    out["map_bounds"] = np.array([pm.min_north, pm.max_north, pm.min_east, pm.max_east])

    # encounter classification + reward shaping terms
    enc_codes = {"head-on": 0, "crossing": 1, "overtaking": 2}
    rows = []
    for k in range(2000):
        a = [rng.uniform(0, 10000), rng.uniform(0, 20000)]
        b = [a[0] + rng.uniform(-12000, 12000), a[1] + rng.uniform(-12000, 12000)]
        h1 = rng.uniform(-8, 8)
        h2 = rng.uniform(-8, 8)
        dist, enc = get_distance_and_encounter_type(a, h1, b, h2)
        rc, _ = ships_collision_reward(dist, enc, dist < 50)
        rows.append([a[0], a[1], h1, b[0], b[1], h2, dist, enc_codes[enc], rc])
    out["encounter"] = np.array(rows)
    rows = []
    for k in range(2000):
        dg = rng.uniform(0, 1500)
        ect = rng.uniform(-4000, 4000)
        ect_o = rng.uniform(-700, 700)
        rows.append([dg, ect, ect_o, test_ship_grounding_reward(dg, False)[0],
                     test_ship_nav_failure_reward(ect, False)[0], obs_ship_grounding_reward(dg, False)[0],
                     obs_ship_nav_failure_reward(ect_o, False)[0]])
    out["reward_terms"] = np.array(rows)
    rows = []
    for k in range(512):
        r = rng.normal()
        acc = [rng.normal() * 5, 0.0, -1.0, 1.0][k % 4]
        conds = [bool(x) for x in rng.integers(0, 2, 5)] if k % 3 else [False] * 5
        rows.append([r, acc] + [float(c) for c in conds] + [get_reward_due_to_ships_termination(r, acc, *conds)])
    out["terminal_reward"] = np.array(rows)
    np.savez_compressed(os.path.join(OUT, "sbmpc_geometry_reward.npz"), **out)
    print("sbmpc/geometry: survey KA", out["sbmpc_survey_ka"])


def gen_sbmpc_multi():
    """F5b: get_optimal_ctrl_offset over a do_list of K = 2, 3, 4 dynamic obstacles (sbmpc.py:113-185: active when
    any obstacle is within D_INIT, per scenario the worst obstacle's cost, the least worst scenario). One persistent
    controller per K, so P_ca_last_ / Chi_ca_last_ carry from call to call (Q7). Per call (96 per K): the obstacles at mixed
    ranges (all beyond D_INIT every 8th call: inactive; some beyond reach of every scenario, some close), a repeated
    obstacle every 5th call, and per-obstacle sizes (the do_list's length / width) varied every 3rd call.
    Rows: in [u_d, chi_d, os_state(6), then per obstacle slot x, y, psi, u, v, l, w (4 slots, unused zero)], out
    [speed factor, course offset, active, P_ca_last_, Chi_ca_last_]."""
    from rl_env.ship_in_transit.sub_systems.sbmpc import SBMPC
    rng = np.random.Generator(np.random.PCG64(11))
    out = {}
    for K in (2, 3, 4):
        sb = SBMPC(tf=1000, dt=20)
        ins, outs = [], []
        for call in range(96):
            os_state = np.array([rng.uniform(0, 20000), rng.uniform(0, 10000), rng.uniform(-np.pi, np.pi),
                                 rng.uniform(0, 6), rng.uniform(-0.5, 0.5), rng.uniform(-0.01, 0.01)])
            u_d = rng.uniform(3, 5)
            chi_d = rng.uniform(-4, 4)
            obs, row = [], [u_d, chi_d] + list(os_state)
            for k in range(K):
                ang = rng.uniform(-np.pi, np.pi)
                if call % 8 == 0:
                    rad = rng.uniform(2100, 6000)
                elif k == 0:
                    rad = rng.uniform(50, 1900)
                else:
                    rad = rng.uniform(50, 6000)
                ob = np.array([os_state[0] + rad * np.cos(ang), os_state[1] + rad * np.sin(ang),
                               rng.uniform(-np.pi, np.pi), rng.uniform(0, 6), rng.uniform(-0.5, 0.5)])
                if call % 8 and rng.uniform() < 0.6:
                    # on a collision course: ahead of the own ship's nominal course (linear_pred moves along
                    # (-sin psi, cos psi)), heading back towards it
                    rad = rng.uniform(300, 1900)
                    ax = chi_d + rng.uniform(-0.6, 0.6)
                    ob = np.array([os_state[0] - rad * np.sin(ax), os_state[1] + rad * np.cos(ax),
                                   chi_d + np.pi + rng.uniform(-0.5, 0.5), rng.uniform(2, 6), rng.uniform(-0.3, 0.3)])
                l, w = (80.0, 16.0) if call % 3 else (float(rng.uniform(40, 140)), float(rng.uniform(8, 30)))
                if call % 5 == 1 and k == K - 1:  # a repeated obstacle (the env's duplicate slots)
                    ob, l, w = obs[0][1].copy(), obs[0][3], obs[0][4]
                obs.append((k, ob, None, l, w))
                row += list(ob) + [l, w]
            row += [0.0] * (7 * (4 - K))
            p, c = sb.get_optimal_ctrl_offset(u_d=u_d, chi_d=chi_d, os_state=os_state, do_list=obs)
            ins.append(row)
            outs.append([p, c, float(sb.is_stephen_useful()), sb._params.P_ca_last_, sb._params.Chi_ca_last_])
        out[f"k{K}_in"] = np.array(ins)
        out[f"k{K}_out"] = np.array(outs)
        print(f"sbmpc multi K={K}: active {int(out[f'k{K}_out'][:, 2].sum())} / 96, "
              f"non-default {int(((out[f'k{K}_out'][:, 0] != 1) | (out[f'k{K}_out'][:, 1] != 0)).sum())}")
    np.savez_compressed(os.path.join(OUT, "sbmpc_multi.npz"), **out)


# ----------------------------------------------------------------------------------------------
# F7 SAC grad steps (sac.py:102-154) with fixed weights, batch and reparameterisation noise
# ----------------------------------------------------------------------------------------------
def gen_sac():
    import torch
    import ast_sac.torch.utils.pytorch_util as ptu
    ptu.set_gpu_mode(False)
    from ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac.torch.sac.sac import SACTrainer
    from ast_sac.torch.core import distributions as D

    torch.manual_seed(0)
    H, B, OBS, ACT = 32, 64, 8, 1
    qf1, qf2, tq1, tq2 = [ConcatMlp(input_size=OBS + ACT, output_size=1, hidden_sizes=[H, H]) for _ in range(4)]
    policy = TanhGaussianPolicy(obs_dim=OBS, action_dim=ACT, hidden_sizes=[H, H])

    class E:
        class action_space:
            shape = (1,)

    tr = SACTrainer(env=E, policy=policy, qf1=qf1, qf2=qf2, target_qf1=tq1, target_qf2=tq2, discount=0.965,
                    soft_target_tau=1e-3, target_update_period=1, policy_lr=8e-5, qf_lr=8e-5, reward_scale=0.75,
                    use_automatic_entropy_tuning=True, action_reg_coeff=0.01, clip_val=100)
    nets = {"policy": policy, "qf1": qf1, "qf2": qf2, "target_qf1": tq1, "target_qf2": tq2}
    out = {}
    for name, net in nets.items():
        for pn, p in net.named_parameters():
            out[f"init/{name}/{pn}"] = p.detach().numpy().copy()
    rng = np.random.Generator(np.random.PCG64(11))
    n_steps = 3
    noise = rng.standard_normal((n_steps, 2, B, ACT)).astype(np.float32)
    queue = []
    orig = D.MultivariateDiagonalNormal.sample

    def fake_sample(self, *a, **k):
        return queue.pop(0)

    D.MultivariateDiagonalNormal.sample = fake_sample
    try:
        for s in range(n_steps):
            batch = dict(observations=rng.uniform(-1, 1, (B, OBS)) * 1000.0,
                         actions=rng.uniform(-1, 1, (B, ACT)),
                         rewards=rng.normal(size=(B, 1)) * 3.0,
                         terminals=(rng.uniform(size=(B, 1)) < 0.2).astype(np.uint8),
                         next_observations=rng.uniform(-1, 1, (B, OBS)) * 1000.0)
            for k, v in batch.items():
                out[f"step{s}/batch/{k}"] = v
            out[f"step{s}/noise"] = noise[s]
            queue[:] = [torch.from_numpy(noise[s, 0]), torch.from_numpy(noise[s, 1])]
            tb = {k: torch.from_numpy(np.asarray(v)).float() for k, v in batch.items()}
            losses, _ = tr.compute_loss(tb, skip_statistics=True)
            out[f"step{s}/losses"] = np.array([losses.policy_loss.item(), losses.qf1_loss.item(),
                                              losses.qf2_loss.item(), losses.alpha_loss.item()])
            queue[:] = [torch.from_numpy(noise[s, 0]), torch.from_numpy(noise[s, 1])]
            tr.train_from_torch(tb)
            out[f"step{s}/log_alpha"] = tr.log_alpha.detach().numpy().copy()
            for name, net in nets.items():
                for pn, p in net.named_parameters():
                    out[f"step{s}/{name}/{pn}"] = p.detach().numpy().copy()
    finally:
        D.MultivariateDiagonalNormal.sample = orig
    out["hparams"] = np.array([H, B, OBS, ACT, 0.965, 1e-3, 8e-5, 8e-5, 0.75, 0.01, 100.0])
    np.savez_compressed(os.path.join(OUT, "sac_step.npz"), **out)
    print("sac: losses", out["step0/losses"], out[f"step{n_steps - 1}/losses"])


def gen_replay():
    """EnvReplayBuffer / SimpleReplayBuffer (data_management/env_replay_buffer.py:8-50,
    simple_replay_buffer.py:44-103, replay_buffer.py:34-77): three paths shaped like ast_sac_rollout's
    (rollout_functions.py:161-181) added to a 7-row ring (it wraps), without and with env_info
    sizes, then random_batch(5) under np.random.seed(123). Inputs and the buffers' arrays are saved."""
    from ast_sac.data_management.env_replay_buffer import EnvReplayBuffer
    from gymnasium.spaces import Box
    rng = np.random.default_rng(5)
    out = {}
    paths = []
    for k, T in enumerate((4, 5, 3)):
        obs = rng.normal(size=(T, 8)).astype(np.float32) * 100
        nobs = rng.normal(size=(T, 8)).astype(np.float32) * 100
        act = rng.uniform(-1, 1, size=(T, 1)).astype(np.float32)
        rew = rng.normal(size=(T, 1))
        term = np.zeros((T, 1), dtype=bool)
        term[-1, 0] = k != 1  # path 1 ends by max_path_length, not terminal
        info = rng.normal(size=(T, 2))
        env_infos = [dict(x=info[t], terminal=bool(term[t, 0]), events="") for t in range(T)]
        paths.append(dict(observations=obs, actions=act, rewards=rew, next_observations=nobs, terminals=term,
                          agent_infos=[{} for _ in range(T)], env_infos=env_infos))
        for key, v in (("obs", obs), ("nobs", nobs), ("act", act), ("rew", rew), ("term", term), ("info", info)):
            out[f"path{k}/{key}"] = v

    class _Env:
        observation_space = Box(-np.inf, np.inf, shape=(8,))
        action_space = Box(-1.0, 1.0, shape=(1,))

    class _EnvInfo(_Env):
        info_sizes = {"x": 2}

    for tag, env in (("plain", _Env()), ("info", _EnvInfo())):
        rb = EnvReplayBuffer(7, env)
        rb.add_paths(paths)
        np.random.seed(123)
        b = rb.random_batch(5)
        for key in ("_observations", "_actions", "_rewards", "_terminals", "_next_obs"):
            out[f"{tag}/{key}"] = getattr(rb, key)
        out[f"{tag}/top_size"] = np.array([rb._top, rb._size])
        for key, v in b.items():
            out[f"{tag}/batch/{key}"] = v
        if tag == "info":
            out["info/env_info_x"] = rb._env_infos["x"]
    np.savez_compressed(os.path.join(OUT, "replay_buffer.npz"), **out)
    print("replay: top/size", out["plain/top_size"])


def gen_policy():
    """f3: run/ast-sac_run_trained_policy.py:50-66 — a deterministic TanhGaussianPolicy (as the runner
    snapshots it, 'evaluation/policy' = MakeDeterministic) rolled out with ast_sac_rollout on the
    NormalizedBoxEnv-wrapped env (no max_path_length, as the script), then the test/obs ships'
    simulation_results and the env's waypoint_sampling_times. The policy is a seeded random init with
    its first layer scaled down (raw observations are O(1e4): unscaled, every action saturates at +-1),
    and its parameters are saved (no pickled snapshot is read or written here)."""
    import torch
    import ast_sac.torch.utils.pytorch_util as ptu
    ptu.set_gpu_mode(False)
    from ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac.torch.sac.policies.base import MakeDeterministic
    from ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv
    from ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
    from run.env_setup import prepare_multiship_rl_env
    out = {}
    cases = [("none_a", "none", 4, 1e-4), ("sbmpc_a", "sbmpc", 5, 1e-3), ("sbmpc_b", "sbmpc", 2, 1e-4)]
    for tag, collav, seed, scale in cases:
        torch.manual_seed(seed)
        pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[64, 64], init_w=0.5)
        with torch.no_grad():
            pol.fcs[0].weight.mul_(scale)
        for pn, prm in pol.named_parameters():
            out[f"{tag}/param/{pn}"] = prm.detach().numpy().copy()
        out[f"{tag}/collav"] = np.array(collav)
        env, _ = prepare_multiship_rl_env(rl_args(collav))
        path = ast_sac_rollout(NormalizedBoxEnv(env), MakeDeterministic(pol))
        for k in ("observations", "actions", "rewards", "next_observations", "terminals", "dones"):
            out[f"{tag}/path/{k}"] = np.asarray(path[k])
        out[f"{tag}/events"] = np.array([i["events"] for i in path["env_infos"]])
        for name, ship in (("test", env.test), ("obs", env.obs)):
            sr = ship.ship_model.simulation_results
            keys = list(sr.keys())
            out[f"{tag}/{name}_keys"] = np.array(keys)
            out[f"{tag}/{name}_sr"] = np.array([sr[key] for key in keys], np.float64).T
        out[f"{tag}/wst"] = np.array(env.waypoint_sampling_times, np.float64)
        print("policy", tag, "decisions", len(path["actions"]), "rows", out[f"{tag}/test_sr"].shape,
              "return", float(np.sum(path["rewards"])), out[f"{tag}/events"][-1])
    np.savez_compressed(os.path.join(OUT, "trained_policy.npz"), **out)


def gen_progress():
    """f2: the progress.csv the reference's own training loop writes — TorchBatchRLAlgorithm
    (core/batch_rl_algorithm.py:58-106, rl_algorithm.py:57-150) with SACTrainer, MdpPathCollector,
    EnvReplayBuffer and the runner's NormalizedBoxEnv-wrapped MultiShipRLEnv (run/ast-sac_runner.py:110-205;
    expl and eval envs share one env object, as there), for two epochs of a few decisions, on the CPU.
    gtimer (1.0.0b5) is absent, so its published behaviour for these calls is restated: inside
    `timed_for(..., save_itrs=True)` every `stamp(name)` appends the time since the previous stamp (or
    the loop start) to `get_times().stamps.itrs[name]`, and `get_times().total` is the elapsed time.
    Only the header (its column names; the logger writes them sorted, logging.py:285-305) and the
    row count are kept: the values are timings and a random init's losses."""
    import csv
    import json
    import tempfile
    import time
    import torch
    import ast_sac.torch.utils.pytorch_util as ptu
    ptu.set_gpu_mode(False)

    class _Itrs(dict):
        pass

    class _Times:
        def __init__(self):
            self.stamps = types.SimpleNamespace(itrs=_Itrs())
            self.total = 0.0

    state = dict(t0=time.perf_counter(), last=time.perf_counter(), times=_Times())

    def stamp(name, unique=True, **k):
        now = time.perf_counter()
        state["times"].stamps.itrs.setdefault(name, []).append(now - state["last"])
        state["last"] = now

    def timed_for(it, save_itrs=True, **k):
        for x in it:
            state["last"] = time.perf_counter()
            yield x

    def get_times():
        state["times"].total = time.perf_counter() - state["t0"]
        return state["times"]

    gt = sys.modules["gtimer"]
    saved = (gt.stamp, gt.timed_for, gt.get_times)
    gt.stamp, gt.timed_for, gt.get_times = stamp, timed_for, get_times
    try:
        for m in [m for m in sys.modules if m.startswith("ast_sac.core") or m.startswith("ast_sac.torch.core")]:
            del sys.modules[m]  # re-import the algorithm modules against the recording stand-in
        from ast_sac.core.logging import logger
        from ast_sac.data_management.env_replay_buffer import EnvReplayBuffer
        from ast_sac.samplers.data_collector.path_collector import MdpPathCollector
        from ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
        from ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy, MakeDeterministic
        from ast_sac.torch.sac.sac import SACTrainer
        from ast_sac.torch.networks.mlp import ConcatMlp
        from ast_sac.torch.core.torch_rl_algorithm import TorchBatchRLAlgorithm
        from ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv
        from run.env_setup import prepare_multiship_rl_env
        torch.manual_seed(0)
        np.random.seed(0)
        env, _ = prepare_multiship_rl_env(rl_args("none"))
        expl_env, eval_env = NormalizedBoxEnv(env, reward_scale=0.75), NormalizedBoxEnv(env, reward_scale=0.75)
        M = 16
        qf = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[M, M]) for _ in range(4)]
        policy = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[M, M])
        eval_col = MdpPathCollector(eval_env, MakeDeterministic(policy), rollout_fn=ast_sac_rollout)
        expl_col = MdpPathCollector(expl_env, policy, rollout_fn=ast_sac_rollout)
        rb = EnvReplayBuffer(1000, expl_env)
        tr = SACTrainer(env=eval_env, policy=policy, qf1=qf[0], qf2=qf[1], target_qf1=qf[2], target_qf2=qf[3],
                        discount=0.965, soft_target_tau=1e-3, target_update_period=1, policy_lr=8e-5, qf_lr=8e-5,
                        reward_scale=0.75, use_automatic_entropy_tuning=True, action_reg_coeff=0.01, clip_val=100)
        algo = TorchBatchRLAlgorithm(trainer=tr, exploration_env=expl_env, evaluation_env=eval_env,
                                     exploration_data_collector=expl_col, evaluation_data_collector=eval_col,
                                     replay_buffer=rb, batch_size=8, max_path_length=2, num_epochs=2,
                                     num_eval_steps_per_epoch=3, num_expl_steps_per_train_loop=3,
                                     num_trains_per_train_loop=2, min_num_steps_before_training=4)
        d = tempfile.mkdtemp()
        f = os.path.join(d, "progress.csv")
        logger.add_tabular_output(f)
        try:
            algo.train()
        finally:
            logger.remove_tabular_output(f)
        with open(f) as fh:
            rows = list(csv.reader(fh))
    finally:
        gt.stamp, gt.timed_for, gt.get_times = saved
    res = dict(columns=rows[0], n_rows=len(rows) - 1,
               generator="tests/golden/gen_golden.py progress: reference TorchBatchRLAlgorithm, 2 epochs, "
                         "MultiShipRLEnv (collav none), SACTrainer 2x16, gtimer restated (see gen_progress)")
    with open(os.path.join(OUT, "progress_header.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print("progress:", len(rows[0]), "columns,", len(rows) - 1, "rows")


if __name__ == "__main__":
    what = sys.argv[1:] or ["c2", "c1", "ast", "rl", "sbmpc", "sac"]
    if "replay" in what:
        os.chdir(REF)
        gen_replay()
    os.chdir(REF)
    if "c2" in what:
        gen_c2()
    if "c1" in what:
        gen_c1()
    if "ast" in what:
        gen_ast_single()
    if "sbmpc" in what:
        gen_sbmpc_geometry()
    if "sbmpc_multi" in what:
        gen_sbmpc_multi()
    if "sac" in what:
        gen_sac()
    if "rl" in what:
        gen_rl()
    if "modes" in what:
        gen_modes()
    if "traj" in what:
        gen_traj()
    if "draw" in what:
        gen_draw()
    if "legacy" in what:
        gen_legacy()
    if "policy" in what:
        gen_policy()
    if "progress" in what:
        gen_progress()
