"""The reference's non-IW two-ship environment (run_colav/env.py:37-677, MultiShipNonIWEnv) over the HIP simulator,
for the run_colav/run_simplified_model.py:245-249 loop (`init_step()`, then `_step()` while the test ship's clock is
below its simulation time).

* `BatchedMultiShipNonIWEnv` — N independent copies on one device (a KIND_NONIW handle, `noniw_tick_kernel`):
  `_step()` returns next_states (N, 6) float32, combined_done (N,) bool and env_info (event bits and flags) as
  torch tensors; `run()` is the whole loop.
* `MultiShipNonIWEnv` — the reference's one-env object API (numpy in / out) as a view of the batched env.

The ships are the reference scenario of record (SimpleShipModel + ThrustFromSpeedSetPoint, fixed routes, the
6-polygon map: `shipsim_abi.c1_config`); collav None / 'simple' / 'sbmpc' as the reference's `collav` argument.
Results are pinned to the reference's own run in tests/test_gpu_c1_noniw.py.
"""
import numpy as np
import torch

from .. import shipsim_abi as abi
from ..shipsim import ShipSim


class BatchedMultiShipNonIWEnv:
    def __init__(self, collav=None, n_envs=1, time_step=30, device=None):
        self.collav = "none" if collav is None else str(collav)
        self.cfg = abi.c1_config(self.collav, time_step=time_step)
        self.n_envs = int(n_envs)
        self.sim = ShipSim(self.cfg, self.n_envs, device=device)
        self.device = self.sim.device
        self.sim_time = float(self.cfg.simulation_time)
        self._events = torch.zeros(self.n_envs, dtype=torch.int32, device=self.device)

    def init_step(self):
        """reset + init_step (run_colav/env.py:223-323): every ship at its initial state, one control tick."""
        self.sim.reset()

    @property
    def time(self):
        """(N,) the test ship's clock (ship_model.int.time)."""
        return self.sim.get(abi.F_TIME).view(self.n_envs, 2)[:, 0]

    def stop_flags(self):
        """(N, 2) int32 ShipAssets.stop_flag of the test / obstacle ship."""
        return self.sim.get(abi.F_STOP).view(self.n_envs, 2)

    def _step(self):
        """MultiShipNonIWEnv._step (:613-676) for every env: (next_states (N, 6) float32, combined_done (N,) bool,
        env_info dict of (N,) tensors: events (bits, shipsim_abi.EV_*), terminal, test_ship_stop, obs_ship_stop)."""
        stopped = self.stop_flags().bool()  # a ship frozen before this step reports its yaw where e_ct would be
        self.sim.tick(1, self._events)
        n = self.sim.get(abi.F_NORTH).view(self.n_envs, 2)
        e = self.sim.get(abi.F_EAST).view(self.n_envs, 2)
        third = torch.where(stopped, self.sim.get(abi.F_YAW).view(self.n_envs, 2),
                            self.sim.get(abi.F_LOG_ECT).view(self.n_envs, 2))
        next_states = torch.stack([n[:, 0], e[:, 0], third[:, 0], n[:, 1], e[:, 1], third[:, 1]], -1).float()
        ev = self._events.clone()
        terminal = (ev & abi.EV_TERMINAL) != 0
        stops = self.stop_flags().bool()
        combined_done = terminal | (stops[:, 0] & stops[:, 1])
        info = dict(events=ev, terminal=terminal, test_ship_stop=(ev & abi.EV_TEST_STOP) != 0,
                    obs_ship_stop=(ev & abi.EV_OBS_STOP) != 0)
        return next_states, combined_done, info

    def run(self, max_steps=100000):
        """The run_simplified_model.py:245-249 loop: init_step, then _step while the test ship's time is below
        sim_time (every env advances on the same clock). Returns (events (T, N) int32, stops (T, N, 2) int32)."""
        self.init_step()
        events, stops = [], []
        for _ in range(max_steps):
            if not bool((self.time < self.sim_time).any()):
                break
            _, _, info = self._step()
            events.append(info["events"].clone())
            stops.append(self.stop_flags().clone())
        if not events:
            return (torch.zeros((0, self.n_envs), dtype=torch.int32, device=self.device),
                    torch.zeros((0, self.n_envs, 2), dtype=torch.int32, device=self.device))
        return torch.stack(events), torch.stack(stops)

    @staticmethod
    def events_strings(bits):
        return [abi.events_to_string(int(b)) for b in torch.as_tensor(bits).cpu().tolist()]


class MultiShipNonIWEnv:
    """One env of the batched environment with the reference's object API: init_step(), _step() ->
    (next_states np.float32 (6,), combined_done bool, env_info dict with 'events' as the reference's string and the
    'terminal' / 'test_ship_stop' / 'obs_ship_stop' booleans)."""

    def __init__(self, collav=None, time_step=30, device=None):
        self._b = BatchedMultiShipNonIWEnv(collav=collav, n_envs=1, time_step=time_step, device=device)
        self.collav = self._b.collav
        self.sim_time = self._b.sim_time

    def init_step(self):
        self._b.init_step()

    @property
    def time(self):
        return float(self._b.time[0])

    def _step(self):
        s, d, info = self._b._step()
        bits = int(info["events"][0])
        env_info = dict(events=abi.events_to_string(bits), terminal=bool(info["terminal"][0]),
                        test_ship_stop=bool(info["test_ship_stop"][0]), obs_ship_stop=bool(info["obs_ship_stop"][0]))
        return s[0].cpu().numpy(), bool(d[0]), env_info
