"""Gym-style environments over the HIP simulator (drop-in for rl_env/ship_in_transit/env.py).

* `BatchedMultiShipRLEnv` — N independent MultiShipRLEnv instances resident on one device;
  reset/step take and return torch tensors. `step` runs every active env to its decision point
  (env.py:624-773); `step_async` runs at most `max_ticks` ticks per env and reports which envs
  completed a decision (GPU-native collectors use this).
* `MultiShipRLEnv` — the reference's single-env object API (reset() -> np.ndarray(8,) float32,
  step(action) -> (obs, reward, done, env_info)) as a one-env view of the batched env, so that
  reference callers (NormalizedBoxEnv, ast_sac_rollout, MdpPathCollector, EnvReplayBuffer,
  SACTrainer) run unchanged.

Semantics, quirks included, are those of the reference MultiShipRLEnv; the
numerics run in ast_sac_amd/csrc (fp64) and are checked against the CPU oracle in tests/.
"""
import argparse

import numpy as np
import torch

from ... import shipsim_abi as abi
from ...shipsim import ShipSim
from ...spaces import Box
from .trajectory import EpisodeRecord, RewardTracker, ShipSnapshots

# observation_space / action_space of env.py:86-104
OBS_LOW = np.array([0, 0, -3000, 0, 0, -np.pi, -3000, 0], dtype=np.float32)
OBS_HIGH = np.array([10000, 20000, 3000, 10000, 20000, np.pi, 3000, 10], dtype=np.float32)


def default_args(**kw):
    """run/ast-sac_runner.py:27-43 defaults (environment group)."""
    a = dict(max_sampling_frequency=9, time_step=4, radius_of_acceptance=300, lookahead_distance=1000,
             collav_mode="sbmpc", ship_draw=False, time_since_last_ship_drawing=30, normalize_action=False)
    a.update(kw)
    return argparse.Namespace(**a)


def config_from_args(args, machinery="detailed"):
    """The scenario of record (run/env_setup.py) with the env arguments applied."""
    mach = abi.MACH_DETAILED if machinery in ("detailed", abi.MACH_DETAILED) else abi.MACH_SIMPLIFIED
    collav = getattr(args, "collav_mode", "sbmpc")
    cfg = abi.ast_config(collav if collav in abi.COLLAV else "none", time_step=float(args.time_step), machinery=mach)
    cfg.max_sampling_frequency = int(args.max_sampling_frequency)
    cfg.env_radius_of_acceptance = float(args.radius_of_acceptance)
    for s in cfg.ship:
        s.radius_of_acceptance = float(args.radius_of_acceptance)
        s.lookahead_distance = float(args.lookahead_distance)
    cfg.normalize_action = int(bool(getattr(args, "normalize_action", False)))
    return cfg


class BatchedMultiShipRLEnv:
    def __init__(self, args=None, n_envs=1, device=None, machinery="detailed", cfg=None, lanes_per_env=0):
        self.args = args if args is not None else default_args()
        self.cfg = cfg if cfg is not None else config_from_args(self.args, machinery)
        if lanes_per_env:
            self.cfg.lanes_per_env = lanes_per_env
        self.n_envs = int(n_envs)
        self.sim = ShipSim(self.cfg, self.n_envs, device=device)
        self.device = self.sim.device
        self.collav = getattr(self.args, "collav_mode", "sbmpc")
        self.observation_space = Box(low=OBS_LOW, high=OBS_HIGH, dtype=np.float32)
        if self.cfg.normalize_action:
            self.action_space = Box(low=np.array([-1.0], np.float32), high=np.array([1.0], np.float32),
                                    dtype=np.float32)
        else:
            self.action_space = Box(low=np.array([-np.deg2rad(30)], np.float32),
                                    high=np.array([np.deg2rad(30)], np.float32), dtype=np.float32)
        self.initial_states = np.array([self.cfg.ship[0].initial_north_position_m, self.cfg.ship[0].initial_east_position_m,
                                        0.0, self.cfg.ship[1].initial_north_position_m,
                                        self.cfg.ship[1].initial_east_position_m, self.cfg.ship[1].initial_yaw_angle_rad,
                                        0.0, self.cfg.ship[1].initial_forward_speed_m_per_s], dtype=np.float32)
        self._out = None

    # -- reference helpers (env.py:186-196) --
    def do_normalize_action(self, a_real):
        return 2.0 * (a_real - self.action_space.low) / (self.action_space.high - self.action_space.low) - 1.0

    def do_denormalize_action(self, a_norm):
        return (a_norm + 1.0) / 2.0 * (self.action_space.high - self.action_space.low) + self.action_space.low

    def reset(self, mask=None, obs_out=None):
        """MultiShipRLEnv.reset for the envs in `mask` (all if None); returns (N, 8) float32 —
        reset rows hold the constant initial_states (env.py:295, Q11); other rows are untouched."""
        return self.sim.reset(mask=mask, obs_out=obs_out)

    def _info(self, out):
        ev = out["events"]
        return dict(events=ev, terminal=(ev & abi.EV_TERMINAL) != 0, test_ship_stop=(ev & abi.EV_TEST_STOP) != 0,
                    obs_ship_stop=(ev & abi.EV_OBS_STOP) != 0, ticks=out["ticks"])

    def step(self, action, active=None):
        """MultiShipRLEnv.step for every active env: returns obs (N,8) float32, accumulated reward (N,)
        float64, combined_done (N,) bool and an info dict of tensors (event bits + flags)."""
        out = self.sim.step(action, active=active, max_ticks=0)
        return out["obs"], out["reward"], out["done"].bool(), self._info(out)

    def step_async(self, action, max_ticks=64, active=None, out=None):
        """Run at most max_ticks ticks per env; envs that reach their decision point have
        out['ready'] == 1 and their obs/reward/done/events rows are valid."""
        return self.sim.step(action, active=active, max_ticks=max_ticks, out=out)

    @staticmethod
    def events_strings(bits):
        return [abi.events_to_string(int(b)) for b in torch.as_tensor(bits).cpu().tolist()]

    @property
    def sampling_count(self):
        return self.sim.get(abi.E_SAMPLING_COUNT)

    def obstacle_routes(self):
        """(N, L, 2) obstacle-ship route (north, east) incl. sampled intermediate waypoints."""
        n = self.sim.get(abi.E_ROUTE_NORTH).view(self.n_envs, 2, abi.MAX_ROUTE)[:, 1]
        e = self.sim.get(abi.E_ROUTE_EAST).view(self.n_envs, 2, abi.MAX_ROUTE)[:, 1]
        L = self.sim.get(abi.E_ROUTE_LEN).view(self.n_envs, 2)[:, 1]
        return torch.stack([n, e], -1), L

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)

    # -- trajectory recording (simulation_results export) --
    def legacy_step(self, k=1, out=None):
        """k ticks of the legacy per-tick MultiShipEnv.step() (env.py:1104-1173) for every env:
        dict(states (N, 8) float64 next_states, done (N,) uint8, status (N,) int32 LT_* bits)."""
        return self.sim.legacy_step(k, out=out)

    def record_trajectories(self, capacity=None):
        """Record every tick of every env (both ships' simulation_results rows + RewardTracker rows)
        into device buffers; rows start at the next reset. capacity defaults to the longest episode
        (simulation_time / time_step + 2 rows)."""
        if capacity is None:
            capacity = int(np.ceil(self.cfg.simulation_time / self.cfg.time_step)) + 8
        return self.sim.set_trajectory(capacity)

    def episode_record(self, env_index=0):
        """EpisodeRecord of one env (host copy of its rows since its last reset)."""
        if getattr(self.sim, "traj", None) is None:
            raise RuntimeError("trajectory recording is off: call record_trajectories() before reset()")
        return EpisodeRecord(self.sim.traj, env_index, self.cfg, self.sim.n_ships)

    def close(self):
        self.sim.close()

    # snapshots (logger.save_itr_params pickles the collectors' env): keep the config, not the device state
    def __getstate__(self):
        return dict(args=self.args, cfg=bytes(self.cfg), n_envs=self.n_envs, device=str(self.device))

    def __setstate__(self, st):
        cfg = abi.Config.from_buffer_copy(st["cfg"])
        self.__init__(st["args"], st["n_envs"], device=st["device"], cfg=cfg)


class _Int:
    """EulerInt view (utils.py:27-53): dt / sim_time, time read from the device."""

    def __init__(self, env, ship):
        self._env, self._ship = env, ship
        self.dt = float(env._b.cfg.time_step)
        self.sim_time = float(env._b.cfg.simulation_time)

    @property
    def time(self):
        return float(self._env._b.sim.get(abi.F_TIME)[self._ship].item())


class _ShipModelView:
    """ShipModelAST / SimpleShipModel attributes the reference's post-processing reads."""

    def __init__(self, env, ship):
        self._env, self._ship = env, ship
        self.int = _Int(env, ship)
        c = env._b.cfg.ship[ship]
        self.l_ship, self.w_ship = c.length_of_ship, c.width_of_ship

    def _field(self, f):
        return float(self._env._b.sim.get(f)[self._ship].item())

    north = property(lambda self: self._field(abi.F_NORTH))
    east = property(lambda self: self._field(abi.F_EAST))
    yaw_angle = property(lambda self: self._field(abi.F_YAW))
    forward_speed = property(lambda self: self._field(abi.F_U))
    sideways_speed = property(lambda self: self._field(abi.F_V))
    yaw_rate = property(lambda self: self._field(abi.F_R))

    @property
    def simulation_results(self):
        return self._env._record().simulation_results(self._ship)

    @property
    def ship_drawings(self):
        """[[x arrays], [y arrays]] of the ShipDraw snapshots since the last reset (ship_draw=True)."""
        return self._env._ship_drawings(self._ship)


class _NavigateView:
    def __init__(self, env, ship):
        self._env, self._ship = env, ship

    def _route(self):
        return self._env._route(self._ship)

    north = property(lambda self: [float(x) for x in self._route()[:, 0]])
    east = property(lambda self: [float(x) for x in self._route()[:, 1]])
    e_ct = property(lambda self: float(self._env._b.sim.get(abi.F_E_CT)[self._ship].item()))
    e_ct_int = property(lambda self: float(self._env._b.sim.get(abi.F_E_CT_INT)[self._ship].item()))


class _AutoPilotView:
    def __init__(self, env, ship):
        self.navigate = _NavigateView(env, ship)
        self._env, self._ship = env, ship

    next_wpt = property(lambda self: int(self._env._b.sim.get(abi.F_NEXT_WPT)[self._ship].item()))


class ShipAssetView:
    """ShipAssets (env.py:29-39) of one ship of the N = 1 device env, for the reference's plotting /
    post-analysis code: ship_model.simulation_results (needs record_trajectory=True), ship_model.int,
    auto_pilot.navigate.north/east, time_list, integrator_term, stop_flag, desired_forward_speed."""

    def __init__(self, env, ship):
        self._env, self._ship = env, ship
        self.ship_model = _ShipModelView(env, ship)
        self.auto_pilot = _AutoPilotView(env, ship)
        self.desired_forward_speed = float(env._b.cfg.ship[ship].desired_forward_speed)
        self.type_tag = "test_ship" if ship == 0 else "obs_ship"

    time_list = property(lambda self: self._env._record().time_list(self._ship))
    integrator_term = property(lambda self: self._env._record().integrator_term(self._ship))
    stop_flag = property(lambda self: bool(self._env._b.sim.get(abi.F_STOP)[self._ship].item()))


class MultiShipRLEnv:
    """Single-env object API of rl_env/ship_in_transit/env.py:MultiShipRLEnv over the device env.
    With record_trajectory=True every tick is recorded on the device and the reference's
    post-processing surface is available: test/obs/assets (ShipAssetView), reward_tracker,
    waypoint_sampling_times, is_collision_list, is_collision_imminent_list."""

    def __init__(self, args=None, device=None, machinery="detailed", cfg=None, assets=None, map=None,
                 record_trajectory=False, trajectory_capacity=None):
        self.args = args if args is not None else default_args()
        self._b = BatchedMultiShipRLEnv(self.args, 1, device=device, machinery=machinery, cfg=cfg)
        self.record_trajectory = bool(record_trajectory)
        if self.record_trajectory:
            self._b.record_trajectories(trajectory_capacity)
        self.test, self.obs = ShipAssetView(self, 0), ShipAssetView(self, 1)
        self.assets = [self.test, self.obs]
        self.waypoint_sampling_times = []
        self._extra_totals = []
        self.collav = self._b.collav
        self.observation_space = self._b.observation_space
        self.action_space = self._b.action_space
        self.initial_states = self._b.initial_states
        self.states = self.initial_states
        self.next_observations = self.initial_states
        self.accumulated_rewards_list = []
        self.env_info = {"events": "", "terminal": False, "test_ship_stop": False, "obs_ship_stop": False}
        self._dev = self._b.device
        # ShipDraw snapshots (env.py:118-120, :573-579): the timer is env-level and survives reset
        self.ship_draw = bool(getattr(self.args, "ship_draw", False))
        self._snap = ShipSnapshots(self._b.cfg.time_step, float(getattr(self.args, "time_since_last_ship_drawing", 30)))

    do_normalize_action = BatchedMultiShipRLEnv.do_normalize_action
    do_denormalize_action = BatchedMultiShipRLEnv.do_denormalize_action

    @property
    def sampling_count(self):
        return int(self._b.sampling_count[0].item())

    @property
    def waypoint_samples(self):
        routes, L = self._b.obstacle_routes()
        L = int(L[0])
        r = routes[0, 1:L - 1].cpu().numpy()
        return [[float(n), float(e)] for n, e in r]

    def _record(self):
        if not self.record_trajectory:
            raise RuntimeError("construct MultiShipRLEnv(record_trajectory=True) to read simulation results")
        return self._b.episode_record(0)

    def _route(self, ship):
        routes = self._b.sim.get(abi.E_ROUTE_NORTH).view(2, abi.MAX_ROUTE)[ship].cpu().numpy()
        routes_e = self._b.sim.get(abi.E_ROUTE_EAST).view(2, abi.MAX_ROUTE)[ship].cpu().numpy()
        L = int(self._b.sim.get(abi.E_ROUTE_LEN)[ship].item())
        return np.stack([routes[:L], routes_e[:L]], 1)

    @property
    def reward_tracker(self):
        rt = self._record().reward_tracker()
        for r in self._extra_totals:  # update_r_total_only on sampling failures (env.py:690)
            rt.update_r_total_only(r)
        return rt

    @property
    def is_collision_list(self):
        return self._record().is_collision_list()

    @property
    def is_collision_imminent_list(self):
        if self.collav not in ("simple", "sbmpc"):
            return []
        return self._record().is_collision_imminent_list()

    def reset(self, action=None):
        obs = self._b.reset()
        self.waypoint_sampling_times = []
        self._extra_totals = []
        self.accumulated_rewards_list = []
        self.env_info = {"events": "", "terminal": False, "test_ship_stop": False, "obs_ship_stop": False}
        self._snap.reset()  # ship_model.reset() restores the empty drawings; the timer carries on
        return obs[0].cpu().numpy()

    @property
    def time_since_last_ship_drawing(self):
        return self._snap.timer

    def _ship_drawings(self, ship):
        self._record()
        return self._snap.drawings[ship]

    def _ship_snapshots(self, n_ticks):
        """ShipDraw snapshots of this call's ticks, at each firing tick's post-tick state read from
        the device trajectory rows (or the state now, for the last tick / a stopped ship)."""
        fire = self._snap.advance(n_ticks)
        if not fire or not self.record_trajectory:
            return
        rec, sim = self._record(), self._b.sim
        now = [tuple(float(sim.get(f)[s].item()) for f in (abi.F_NORTH, abi.F_EAST, abi.F_YAW)) for s in (0, 1)]
        self._snap.draw(fire, rec.ship_rows, now)

    def step(self, action):
        a = np.asarray(action, dtype=np.float32).reshape(-1)[:1]
        if self.sampling_count < self._b.cfg.max_sampling_frequency:  # env.py:663-665
            t_obs = float(self._b.sim.get(abi.F_TIME)[1].item())
            self.waypoint_sampling_times.append(t_obs - float(self._b.cfg.time_step))
        obs, r, done, info = self._b.step(torch.from_numpy(a))
        bits = int(info["events"][0].item())
        if self.ship_draw:
            self._ship_snapshots(int(info["ticks"][0].item()))
        if bits & abi.EV_SAMPLING_FAILURE:
            self._extra_totals.append(float(r[0].item()))
        env_info = {"events": abi.events_to_string(bits), "terminal": bool(bits & abi.EV_TERMINAL),
                    "test_ship_stop": bool(bits & abi.EV_TEST_STOP), "obs_ship_stop": bool(bits & abi.EV_OBS_STOP)}
        reward = float(r[0].item())
        self.accumulated_rewards_list.append(reward)
        self.next_observations = obs[0].cpu().numpy()
        self.env_info = env_info
        return self.next_observations, reward, bool(done[0].item()), env_info

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)

    def close(self):
        self._b.close()

    def __getstate__(self):
        return dict(args=self.args, cfg=bytes(self._b.cfg), device=str(self._dev), record=self.record_trajectory)

    def __setstate__(self, st):
        self.__init__(st["args"], device=st["device"], cfg=abi.Config.from_buffer_copy(st["cfg"]),
                      record_trajectory=st.get("record", False))


class MultiShipEnv:
    """The legacy per-tick env of rl_env/ship_in_transit/env.py:783-1181 over the device (N = 1 view):
    reset() -> initial_states; step() -> (next_states: list of 8 floats, done, termination_cond: list
    of the 10 get_termination_status flags). One tick per step, no intermediate waypoints, no reward;
    the ships are the scenario of record (assets/map arguments are accepted for signature parity and
    must describe that scenario; the configuration comes from `args` / `cfg`)."""

    def __init__(self, assets=None, map=None, ship_draw=False, collav=None, time_since_last_ship_drawing=30,
                 args=None, device=None, machinery="detailed", cfg=None):
        self.args = args if args is not None else default_args()
        self.collav = collav if collav is not None else getattr(self.args, "collav_mode", "sbmpc")
        if cfg is None:
            cfg = config_from_args(argparse.Namespace(**{**vars(self.args), "collav_mode": self.collav}), machinery)
        self._b = BatchedMultiShipRLEnv(self.args, 1, device=device, machinery=machinery, cfg=cfg)
        self.test, self.obs = ShipAssetView(self, 0), ShipAssetView(self, 1)
        self.assets = [self.test, self.obs]
        self.observation_space = self._b.observation_space
        self.action_space = Box(low=np.array([-np.pi / 6], np.float32), high=np.array([np.pi / 6], np.float32),
                                dtype=np.float32)
        self.obsv_dim, self.action_dim = 8, 1
        self.initial_states = self._b.initial_states
        self.states = self.initial_states
        self.next_states = self.initial_states
        self.map = map
        self.ship_draw = bool(ship_draw)
        self._snap = ShipSnapshots(self._b.cfg.time_step, float(time_since_last_ship_drawing))
        self._out = None
        self.record_trajectory = False

    @property
    def time_since_last_ship_drawing(self):
        return self._snap.timer

    def _record(self):
        raise RuntimeError("the legacy MultiShipEnv keeps no simulation_results on the device")

    def _ship_drawings(self, ship):
        return self._snap.drawings[ship]

    def _route(self, ship):
        return MultiShipRLEnv._route(self, ship)

    def reset(self):
        self._b.reset()
        self._snap.reset()
        return self.initial_states

    def step(self):
        self._out = self._b.legacy_step(1, out=self._out)
        states = [float(x) for x in self._out["states"][0].cpu().tolist()]
        bits = int(self._out["status"][0].item())
        done = bool(self._out["done"][0].item())
        if self.ship_draw:
            fire = self._snap.advance(1)
            if fire:
                empty = np.empty((0, abi.TRAJ_SHIP_COLS))
                self._snap.draw(fire, [empty, empty], [(states[0], states[1], self.test.ship_model.yaw_angle),
                                                       (states[3], states[4], states[5])])
        self.states = states
        cond = [bool(bits >> i & 1) for i in range(10)]
        return states, done, cond

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)

    def ensure_scalar(self, x):
        return float(x[0]) if isinstance(x, (np.ndarray, list)) else float(x)

    def close(self):
        self._b.close()
