"""Reference-schema views of the device trajectory record (include/shipsim.h, shipsim_set_trajectory).

The kernels store raw per-tick rows (SI units, radians, accumulated fuel); this module derives the
reference's `simulation_results` dict (ShipModelAST.store_simulation_data, ship_model.py:903-942;
SimpleShipModel, run_colav/ship_in_transit/sub_systems/ship_model.py:418-429), its `RewardTracker`
(reward_function.py:30-57) and the animation lists of env.py:612-620. Every derived column restates the
reference expression element-wise in float64 (the same IEEE operations in the same order), so e.g.
'yaw angle [deg]' is `yaw * 180 / np.pi` of the stored yaw, and the stateless machinery columns
(load fractions, powers, fuel rates, motor torque) are recomputed from the stored load and shaft
speed exactly as MachineryMode.distribute_load / fuel_consumption / main_engine_torque do
(ship_engine.py:46-76, 259-295, 416-423). store_last_simulation_data rows (stopped ship) repeat the
previous row with the new time in the reference; their stored raw row is that copy, so the derived
values repeat too.
"""
from dataclasses import dataclass, field

import numpy as np

from ... import shipsim_abi as abi

# ShipModelAST.simulation_results keys in insertion order (ship_model.py:905-942)
AST_RESULT_KEYS = (
    "time [s]", "north position [m]", "east position [m]", "yaw angle [deg]", "rudder angle [deg]",
    "forward speed [m/s]", "sideways speed [m/s]", "yaw rate [deg/sec]", "propeller shaft speed [rpm]",
    "commanded load fraction me [-]", "commanded load fraction hsg [-]", "power me [kw]",
    "available power me [kw]", "power electrical [kw]", "available power electrical [kw]", "power [kw]",
    "propulsion power [kw]", "fuel rate me [kg/s]", "fuel rate hsg [kg/s]", "fuel rate [kg/s]",
    "fuel consumption me [kg]", "fuel consumption hsg [kg]", "fuel consumption [kg]", "motor torque [Nm]",
    "thrust force [kN]", "cross track error [m]", "heading error [deg]")
# SimpleShipModel.simulation_results keys (run_colav/.../ship_model.py:419-429)
SIMPLE_RESULT_KEYS = (
    "time [s]", "north position [m]", "east position [m]", "yaw angle [deg]", "rudder angle [deg]",
    "forward speed [m/s]", "sideways speed [m/s]", "yaw rate [deg/sec]", "thrust force [kN]",
    "cross track error [m]", "heading error [deg]")

# SpecificFuelConsumptionWartila6L26 / Baudouin6M26Dot3 (ship_engine.py:88-112, run/env_setup.py:85-86)
FUEL_ME = (128.9, -168.9, 246.8)
FUEL_DG = (108.7, -289.9, 324.9)


def _mode(ship_cfg):
    """MachineryMode + update_available_propulsion_power (ship_engine.py:23-44) of one ship config."""
    me, el, hl = ship_cfg.main_engine_capacity, ship_cfg.electrical_capacity, ship_cfg.hotel_load
    sg = ship_cfg.shaft_generator_state
    if sg == abi.SG_MOTOR:
        avail, avail_me = me + el - hl, me
    elif sg == abi.SG_GEN:
        avail, avail_me = me - hl, me - hl
    else:
        avail, avail_me = me, me
    return me, el, hl, sg, avail, avail_me


def distribute_load(load, ship_cfg):
    """MachineryMode.distribute_load (ship_engine.py:46-76), element-wise:
    (load on ME, load on electrical, load fraction ME, load fraction electrical)."""
    me, el, hl, sg, avail, _ = _mode(ship_cfg)
    load = np.asarray(load, np.float64)
    total = load * avail
    if sg == abi.SG_MOTOR:
        l_me = np.where(me < total, me, total)  # min(total, me): the first argument unless me < total
        l_el = total + hl - l_me
        p_el = l_el / el
        p_me = np.zeros_like(total) if me == 0 else l_me / me
    elif sg == abi.SG_GEN:
        l_el = np.full_like(total, min(hl, el))
        l_me = total + hl - l_el
        p_me = l_me / me
        p_el = np.zeros_like(total) if el == 0 else l_el / el
    else:
        l_me = total
        l_el = np.full_like(total, hl)
        p_me = l_me / me
        p_el = l_el / el
    return l_me, l_el, p_me, p_el


def _spec(p, c):
    # BaseMachineryModel.spec_fuel_cons (ship_engine.py:259-264): (a * p**2 + b * p + c) / 3.6e9
    return (c[0] * (p * p) + c[1] * p + c[2]) / 3.6e9


def fuel_rates(load, ship_cfg):
    """rate_me, rate_electrical of BaseMachineryModel.fuel_consumption (ship_engine.py:277-290)."""
    l_me, l_el, p_me, p_el = distribute_load(load, ship_cfg)
    with np.errstate(divide="ignore", invalid="ignore"):
        rate_me = np.where(l_me == 0, 0.0, l_me * _spec(p_me, FUEL_ME))
        rate_el = np.where(p_el == 0, 0.0, l_el * _spec(p_el, FUEL_DG))
    return rate_me, rate_el


def simulation_results(rows, ship_cfg, detailed=True, as_lists=True):
    """The reference's simulation_results dict for one ship from its raw rows (T, 20)."""
    r = np.asarray(rows, np.float64).reshape(-1, abi.TRAJ_SHIP_COLS)
    pi = np.pi
    out = {
        "time [s]": r[:, abi.TS_TIME],
        "north position [m]": r[:, abi.TS_NORTH],
        "east position [m]": r[:, abi.TS_EAST],
        "yaw angle [deg]": r[:, abi.TS_YAW] * 180 / pi,
        "rudder angle [deg]": r[:, abi.TS_RUDDER] * 180 / pi,
        "forward speed [m/s]": r[:, abi.TS_U],
        "sideways speed [m/s]": r[:, abi.TS_V],
        "yaw rate [deg/sec]": r[:, abi.TS_R] * 180 / pi,
    }
    if detailed:
        load, omega = r[:, abi.TS_LOAD], r[:, abi.TS_OMEGA]
        me, el, hl, sg, avail, avail_me = _mode(ship_cfg)
        l_me, l_el, p_me, p_el = distribute_load(load, ship_cfg)
        rate_me, rate_el = fuel_rates(load, ship_cfg)
        torque_cap = avail_me / 5 * pi / 30
        t_me = load * avail_me / (omega + 0.1)
        out.update({
            "propeller shaft speed [rpm]": omega * 30 / pi,
            "commanded load fraction me [-]": p_me,
            "commanded load fraction hsg [-]": p_el,
            "power me [kw]": l_me / 1000,
            "available power me [kw]": np.full_like(load, me / 1000),
            "power electrical [kw]": l_el / 1000,
            "available power electrical [kw]": np.full_like(load, el / 1000),
            "power [kw]": (l_el + l_me) / 1000,
            "propulsion power [kw]": (load * avail) / 1000,
            "fuel rate me [kg/s]": rate_me,
            "fuel rate hsg [kg/s]": rate_el,
            "fuel rate [kg/s]": rate_me + rate_el,
            "fuel consumption me [kg]": r[:, abi.TS_FUEL_ME],
            "fuel consumption hsg [kg]": r[:, abi.TS_FUEL_EL],
            "fuel consumption [kg]": r[:, abi.TS_FUEL],
            "motor torque [Nm]": np.where(torque_cap < t_me, torque_cap, t_me),  # main_engine_torque :416-423
            "thrust force [kN]": r[:, abi.TS_THRUST] / 1000,
        })
        keys = AST_RESULT_KEYS
    else:
        out["thrust force [kN]"] = r[:, abi.TS_THRUST]
        keys = SIMPLE_RESULT_KEYS
    out["cross track error [m]"] = r[:, abi.TS_E_CT]
    out["heading error [deg]"] = r[:, abi.TS_E_PSI]
    return {k: (out[k].tolist() if as_lists else out[k]) for k in keys}


@dataclass
class RewardTracker:
    """reward_function.py:29-57 (same fields, same meaning)."""
    ship_collision: list = field(default_factory=list)
    test_ship_grounding: list = field(default_factory=list)
    test_ship_nav_failure: list = field(default_factory=list)
    obs_ship_grounding: list = field(default_factory=list)
    obs_ship_nav_failure: list = field(default_factory=list)
    from_test_ship: list = field(default_factory=list)
    from_obs_ship: list = field(default_factory=list)
    total: list = field(default_factory=list)

    @classmethod
    def from_rows(cls, env_rows):
        e = np.asarray(env_rows, np.float64).reshape(-1, abi.TRAJ_ENV_COLS)
        rt = cls()
        rt.ship_collision = e[:, abi.TE_R_COLLISION].tolist()
        rt.test_ship_grounding = e[:, abi.TE_R_TEST_GROUNDING].tolist()
        rt.test_ship_nav_failure = e[:, abi.TE_R_TEST_NAV].tolist()
        rt.obs_ship_grounding = e[:, abi.TE_R_OBS_GROUNDING].tolist()
        rt.obs_ship_nav_failure = e[:, abi.TE_R_OBS_NAV].tolist()
        rt.from_test_ship = (e[:, abi.TE_R_TEST_GROUNDING] + e[:, abi.TE_R_TEST_NAV]).tolist()
        rt.from_obs_ship = (e[:, abi.TE_R_OBS_GROUNDING] + e[:, abi.TE_R_OBS_NAV]).tolist()
        rt.total = e[:, abi.TE_R_TOTAL].tolist()
        return rt

    def update_r_total_only(self, r_total):
        self.total.append(r_total)


class ShipDraw:
    """Map-view ship outline (utils/utils.py:56-101): an 80 m x 20 m pentagon, rotated by the yaw
    angle and translated to (north, east). Snapshots are x = north-frame, y = east-frame arrays of 6
    points (closed outline), as ship_model.ship_snap_shot (ship_model.py:612-624) stores them."""
    l = 80.0
    b = 20.0

    def local_coords(self):
        l, b = self.l, self.b
        x = np.array([-l / 2, l / 4, l / 2, l / 4, -l / 2, -l / 2])
        y = np.array([-b / 2, -b / 2, 0.0, b / 2, b / 2, -b / 2])
        return x, y

    def rotate_coords(self, x, y, psi):
        return np.cos(psi) * x - np.sin(psi) * y, np.sin(psi) * x + np.cos(psi) * y

    def translate_coords(self, x_ned, y_ned, north, east):
        return x_ned + north, y_ned + east

    def snapshot(self, north, east, yaw):
        x, y = self.local_coords()
        xr, yr = self.rotate_coords(x, y, yaw)
        return self.translate_coords(xr, yr, north, east)


def post_tick_state(ship_rows, tick, final_state):
    """(north, east, yaw) of one ship right after episode tick `tick` (1-based; row 0 is the
    init_step row, row j is stored by tick j before integrating). The next row holds it unless that
    row is a store_last_simulation_data repeat (ship stopped, state frozen) or not yet written, in
    which case the ship's state now (`final_state`) is it."""
    nxt = tick + 1
    if nxt < len(ship_rows) and ship_rows[nxt, abi.TS_REPEAT] == 0:
        r = ship_rows[nxt]
        return r[abi.TS_NORTH], r[abi.TS_EAST], r[abi.TS_YAW]
    return final_state


class ShipSnapshots:
    """The env-level drawing timer and both ships' `ship_drawings` (env.py:118-120, :573-579).
    The timer starts at args.time_since_last_ship_drawing, survives reset (only __init__ sets it);
    each _step: snapshot both ships if timer > 30, then timer += dt. Drawings are cleared by reset
    (ship_model.reset restores the empty lists)."""

    def __init__(self, dt, timer0=30.0, n_ships=2):
        self.dt = float(dt)
        self.timer = float(timer0)
        self.n_ships = n_ships
        self.drawer = ShipDraw()
        self.reset()

    def reset(self):
        self.drawings = [[[], []] for _ in range(self.n_ships)]
        self.ticks = 0

    def advance(self, n_ticks):
        """Runs the timer over the next n_ticks episode ticks; returns the ticks that snapshot."""
        fire = []
        for j in range(self.ticks + 1, self.ticks + n_ticks + 1):
            if self.timer > 30:
                fire.append(j)
                self.timer = 0
            self.timer += self.dt
        self.ticks += n_ticks
        return fire

    def draw(self, fire, ship_rows, now):
        """ship_rows[s]: the ship's trajectory rows this episode; now[s]: its (north, east, yaw) now."""
        for s in range(self.n_ships):
            for j in fire:
                x, y = self.drawer.snapshot(*post_tick_state(ship_rows[s], j, now[s]))
                self.drawings[s][0].append(x)
                self.drawings[s][1].append(y)


class EpisodeRecord:
    """One env's record since its last reset, read back from the device buffers."""

    def __init__(self, traj, env_index, cfg, n_ships=2):
        n = int(traj["len"][env_index].item())
        self.n_rows = n
        self.overflow = n > traj["cap"]
        k = min(n, traj["cap"])
        self.ship_rows = [traj["ship"][env_index * n_ships + s, :k].cpu().numpy() for s in range(n_ships)]
        self.env_rows = traj["env"][env_index, :max(k - 1, 0)].cpu().numpy() if traj["env"] is not None else None
        self.cfg = cfg

    def simulation_results(self, ship, as_lists=True):
        return simulation_results(self.ship_rows[ship], self.cfg.ship[ship],
                                  detailed=self.cfg.machinery == abi.MACH_DETAILED, as_lists=as_lists)

    def time_list(self, ship):
        return self.ship_rows[ship][1:, abi.TS_TIME_LIST].tolist()

    def integrator_term(self, ship):
        return self.ship_rows[ship][1:, abi.TS_E_CT_INT].tolist()

    def reward_tracker(self):
        return RewardTracker.from_rows(self.env_rows)

    def is_collision_list(self):
        return [bool(int(f) & abi.TE_FLAG_COLLISION) for f in self.env_rows[:, abi.TE_FLAGS]]

    def is_collision_imminent_list(self):
        return [bool(int(f) & abi.TE_FLAG_IMMINENT) for f in self.env_rows[:, abi.TE_FLAGS]]
