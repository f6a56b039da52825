"""BatchedPathCollector — MdpPathCollector + ast_sac_rollout for N device-resident envs.

Per env the semantics of ast_sac_rollout (rollout_functions.py:74-181) hold: an episode starts
with reset(), the policy picks an action from the current observation whenever the env waits for
a decision, the env runs that decision, the transition (o, a, r·reward_scale, o', terminal =
env_info['terminal']) is recorded, and the episode ends on done or after max_path_length
decisions. Unlike the reference, thousands of envs advance together: one sliced
`step_async(max_ticks)` call advances every env by ≤ max_ticks ticks, envs that complete a
decision emit their transition straight into a DeviceReplayBuffer, and finished envs are reset
in the same pass (masked reset).

Two ways to pick the actions:
* device_policy (the runner's, a FusedSACTrainer.device_policy): the trainer's current policy on the
  matrix cores (libsacfused sacf_policy_act) for every env, the result kept only where an env waits for
  a decision. A pass is then device work only — policy, env slice, replay append, path bookkeeping,
  masked reset — and is captured once in a HIP graph and replayed. `collect` checks the transition count
  on the host only every few passes (it plans the passes from the count per pass), and the episodes that
  ended go to a device ring that is copied to the host once per collect (record_paths).
  With `fused` (the default when the env library can run this policy itself: one obstacle ship, the
  TanhGaussianPolicy's obs dim 8 and hidden a multiple of 64 up to 512), the policy is evaluated INSIDE the env launch
  (shipsim_run_policy): an env that completes a decision gets its next action at once and keeps ticking,
  an ended episode is reset in place, so no env idles until the pass ends. The launch logs every decision
  (observation, action, reward, next observation, events); the pass turns the log into replay rows and
  path records. Same transitions as the sliced pass (test_gpu_run_policy.py pins the env side bitwise);
  only the noise stream differs.
* a torch policy module (any policy; the CPU tests): evaluated only on the envs that wait (their count is
  known on the host from the previous pass), one host sync per pass.
The epoch's paths (get_epoch_paths, as MdpPathCollector's, path_collector.py:77-78) feed
eval_util.get_generic_path_information (Rewards/Returns/Actions/Num Paths/Average Returns).

Shared envs (quirk Q10, run/ast-sac_runner.py:113-114): the reference's exploration and evaluation
wrappers share ONE env object, so evaluation episodes reset and advance the same env, and what reset()
leaves alone (the SBMPC memory P_ca_last / Chi_ca_last, quirk Q7) carries from evaluation episodes into
exploration ones. Two collectors over the same batched env reproduce that: a collector that finds the env
last driven by the other one resets every env first (the reference starts every path with env.reset(),
rollout_functions.py:100-106) and starts all its episodes afresh; the library's reset keeps the SBMPC
memory, as the reference's does.
"""
import math
import warnings
from collections import OrderedDict, deque

import numpy as np
import torch

from .... import shipsim_abi as abi
from ...core.eval_util import create_stats_ordered_dict


def _add_capacity(replay_buffer):
    """Rows one add_batch of the buffer can take (a ReplicatedReplayBuffer stages into a smaller ring)."""
    cap = getattr(replay_buffer, "add_capacity", None)
    return cap() if cap is not None else replay_buffer._max


def _staging_room(replay_buffer):
    """Rows the buffer can still stage before its next sync (host read), or None for a plain ring."""
    room = getattr(replay_buffer, "staging_room", None) if replay_buffer is not None else None
    return room() if room is not None else None


class BatchedPathCollector:
    SLICED_TICKS = 128   # sliced passes: an env idles after its decision until the pass ends
    FUSED_TICKS = 1024   # fused passes: envs chain decisions inside the launch; longer passes amortise its tail
    # fused passes: the launch's work-conserving tail. Off by default: where a launch ends then depends on timing,
    # and a stochastic policy's noise is drawn per pass, so runs would not repeat bit for bit; collection is ~1 % of
    # the C4 loop at the reference's update ratio. 512 gives +11.6 % env-ticks/s on collection alone.
    FUSED_TAIL = 0
    def __init__(self, env, policy, max_path_length=9, max_ticks=None, deterministic=False,
                 max_num_epoch_paths_saved=None, device_policy=None, use_graph=None, path_ring=None, fused=None,
                 stream_tail=None):
        self._env = env                       # BatchedNormalizedBoxEnv
        self._policy = policy
        self.max_path_length = int(max_path_length)
        self.max_ticks = int(max_ticks) if max_ticks is not None else None  # None: by pass kind, below
        self.deterministic = deterministic
        N = env.n_envs
        dev = env.device
        self.N, self.device = N, dev
        self._device_policy = device_policy
        if device_policy is not None:
            device_policy.reserve(N)
        self.use_graph = (device_policy is not None and dev.type == "cuda") if use_graph is None else bool(use_graph)
        if self.use_graph and device_policy is None:
            raise ValueError("graph-captured passes need a device_policy (the torch-policy path syncs per pass)")
        self._obs = env.reset().clone()                           # (N, 8) obs at the pending decision
        self._base_env().__dict__["_batched_collector_owner"] = id(self)
        self._act = torch.zeros((N, 1), dtype=torch.float32, device=dev)
        self._awaiting = torch.ones(N, dtype=torch.bool, device=dev)
        self._path_len = torch.zeros(N, dtype=torch.int32, device=dev)
        self._ret = torch.zeros(N, dtype=torch.float64, device=dev)
        f = lambda dt: torch.empty(N, dtype=dt, device=dev)
        self._out = dict(obs=torch.empty((N, 8), dtype=torch.float32, device=dev), reward=f(torch.float64),
                         done=f(torch.uint8), events=f(torch.int32), ticks=f(torch.int32), ready=f(torch.uint8))
        self._obs_reset = torch.empty((N, 8), dtype=torch.float32, device=dev)
        # device-side counters (read by get_diagnostics / collect's occasional checks)
        self._steps_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._paths_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._ticks_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._nonfinite_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._max_saved = max_num_epoch_paths_saved
        self._epoch_paths = deque(maxlen=max_num_epoch_paths_saved)
        self._n_awaiting = N                                      # host copy, None when unknown
        T = self.max_path_length
        # current episode, per decision: (N, T) views of flat buffers with one spare element (masked scatters)
        self._path_flat = [torch.zeros(N * T + 1, dtype=dt, device=dev) for dt in (torch.float64, torch.float32,
                                                                                  torch.int32)]
        self._path_rew, self._path_act, self._path_ev = [b[:N * T].view(N, T) for b in self._path_flat]
        self._rows = torch.arange(N, device=dev)
        self._trace_idx = None                                    # see trace()
        # ended episodes of the current collect (record_paths): a device ring, copied out once per collect
        self._ring_cap = int(path_ring) if path_ring else max(4096, 4 * N)
        self._ring_len = torch.zeros(self._ring_cap + 1, dtype=torch.int32, device=dev)   # + one spare row
        self._ring_rew = torch.zeros((self._ring_cap + 1, T), dtype=torch.float64, device=dev)
        self._ring_act = torch.zeros((self._ring_cap + 1, T), dtype=torch.float32, device=dev)
        self._ring_ev = torch.zeros((self._ring_cap + 1, T), dtype=torch.int32, device=dev)
        self._ring_top = torch.zeros((), dtype=torch.int64, device=dev)   # episodes written since the collect began
        self._graphs = {}
        self.fused = self._fused_supported() if fused is None else bool(fused)
        if self.fused and not self._fused_supported():
            raise ValueError("fused collection needs a device policy the env library can run (see _fused_supported)")
        if self.max_ticks is None:  # ticks per pass: the measured best of each kind (DESIGN.md §9, C4 shard)
            self.max_ticks = self.FUSED_TICKS if self.fused else self.SLICED_TICKS
        # fused passes: the env launch's work-conserving tail (ShipSim.set_stream_tail) — an env whose wave met
        # max_ticks ticks on, up to stream_tail more, while the launch's slowest wave has not (0: off; None:
        # FUSED_TAIL)
        self.stream_tail = self.FUSED_TAIL if stream_tail is None else max(0, int(stream_tail))
        self._mode = None                                         # "fused" / "sliced": the last pass's kind
        self._ep_idx = torch.zeros(N, dtype=torch.int32, device=dev)   # fused: episodes started per env
        self._dec_idx = torch.zeros(N, dtype=torch.int32, device=dev)  # fused: decisions of the current episode
        self._logs = {}                                           # fused: decision log per log capacity
        self._fused_out = dict(ticks=torch.zeros(N, dtype=torch.int32, device=dev),
                               decisions=torch.zeros(N, dtype=torch.int32, device=dev))

    def _fused_supported(self):
        """The env library can run this collector's policy inside the env launch (shipsim_run_policy): a
        device policy exposing its weights, one obstacle ship, obs dim 8, hidden a multiple of 64 up to 512, and the
        wrapper's action bounds equal to the env's (so the in-kernel NormalizedBoxEnv mapping is the
        wrapper's)."""
        dp = self._device_policy
        if dp is None or not hasattr(dp, "weights"):
            return False
        base = self._base_env()
        sim = getattr(base, "sim", None)
        if sim is None or sim.n_ships != 2 or not hasattr(sim, "run_policy"):
            return False
        _, _, o, h = dp.weights()
        if o != 8 or h % 64 or not 64 <= h <= 512:
            return False
        cfg = sim.cfg
        lb, ub = (-1.0, 1.0) if cfg.normalize_action else (cfg.action_low, cfg.action_high)
        w = self._env
        return bool(np.float32(getattr(w, "_lb", np.nan)) == np.float32(lb) and
                    np.float32(getattr(w, "_ub", np.nan)) == np.float32(ub))

    def _base_env(self):
        e = self._env
        while hasattr(type(e), "wrapped_env") or "_wrapped_env" in getattr(e, "__dict__", {}):
            e = e.wrapped_env
        return e

    def _take_over(self):
        """The env was last driven by another collector over the same env (Q10): its in-flight episodes
        are not ours. Reset every env and start all episodes afresh (SBMPC memory is not reset, Q7)."""
        base = self._base_env()
        if base.__dict__.get("_batched_collector_owner") == id(self):
            return
        base.__dict__["_batched_collector_owner"] = id(self)
        self._obs.copy_(self._env.reset())
        self._awaiting.fill_(True)
        self._path_len.zero_()
        self._ret.zero_()
        self._n_awaiting = self.N
        self._mode = None

    def _enter(self, mode):
        """A switch between pass kinds starts every episode afresh (as _take_over), in either direction:
        fused -> sliced because the sliced pass keeps the pending observations and awaiting flags on the
        host side, which fused passes do not maintain; sliced -> fused because a decision a sliced pass
        began is still in flight in the env, and only the policy stream's own decision prologue stores the
        action and observation its log record (and so its replay row) is built from."""
        if self._mode is not None and self._mode != mode:
            self._obs.copy_(self._env.reset())
            self._awaiting.fill_(True)
            self._path_len.zero_()
            self._ret.zero_()
            self._n_awaiting = self.N
        if mode == "fused" and self._mode != "fused":
            self._dec_idx.copy_(self._path_len)
        self._mode = mode

    def trace(self, env_indices):
        """Record every decision of the given envs (test / audit hook: one small host copy per pass, so
        passes are not graph-captured while tracing). trace_log()[j] lists env_indices[j]'s decisions in
        order as dicts: episode, decision, action (the policy's normalized action), obs (next observation),
        reward (the env's, unscaled), done, events, ticks (the decision's ticks summed over the slices it
        took)."""
        self._trace_idx = torch.as_tensor(env_indices, dtype=torch.long, device=self.device)
        self._trace_log = [[] for _ in range(len(env_indices))]
        self._trace_ticks = np.zeros(len(env_indices), dtype=np.int64)
        self._trace_ep = np.zeros(len(env_indices), dtype=np.int64)
        self._trace_dec = np.zeros(len(env_indices), dtype=np.int64)

    def trace_log(self):
        return self._trace_log

    def _trace_pass(self, out, end):
        i = self._trace_idx
        rows = torch.stack([out["ready"][i].double(), self._act[i, 0].double(), out["reward"][i].double(),
                            out["done"][i].double(), out["events"][i].double(), out["ticks"][i].double(),
                            end[i].double()], 1).cpu().numpy()
        obs = out["obs"][i].cpu().numpy()
        for j, (ready, a, r, d, ev, tk, e) in enumerate(rows):
            self._trace_ticks[j] += int(tk)
            if not ready:
                continue
            self._trace_log[j].append(dict(episode=int(self._trace_ep[j]), decision=int(self._trace_dec[j]),
                                           action=np.float32(a), obs=obs[j].copy(), reward=float(r), done=bool(d),
                                           events=int(ev) & 0xFFFFFFFF, ticks=int(self._trace_ticks[j])))
            self._trace_ticks[j] = 0
            self._trace_dec[j] += 1
            if e:
                self._trace_ep[j] += 1
                self._trace_dec[j] = 0

    @torch.no_grad()
    def _actions(self, obs):
        dist = self._policy(obs)
        if self.deterministic or not hasattr(dist, "rsample_with_pretanh"):
            return dist.mle_estimate() if hasattr(dist, "mle_estimate") else dist.sample()
        return dist.sample()

    def _choose_actions(self):
        if self._device_policy is not None:  # every row evaluated, kept where the env waits (in-kernel mask)
            self._device_policy.act(self._obs, self._awaiting, self._act)
            return
        k = self._n_awaiting
        if k is None:  # count unknown (step() called on its own): evaluate everywhere, keep the awaiting rows
            new_a = self._actions(self._obs)
            self._act = torch.where(self._awaiting.unsqueeze(1), new_a.to(torch.float32), self._act)
        elif k == self.N:
            self._act.copy_(self._actions(self._obs).to(torch.float32))
        elif k > 0:
            idx = torch.nonzero_static(self._awaiting, size=k).squeeze(1)
            self._act.index_copy_(0, idx, self._actions(self._obs.index_select(0, idx)).to(torch.float32))

    @staticmethod
    def log_cap_for(max_ticks, stream_tail):
        """Decision records per env per fused pass: a decision takes ~100 ticks (RoA + the turn), so a third
        of that leaves room; an env whose log fills just waits for the next pass (no record is lost)."""
        return max(4, -(-(max_ticks + stream_tail) // 32))

    def _log_cap(self):
        return self.log_cap_for(self.max_ticks, self.stream_tail)

    def _rows_per_pass(self):
        """The most replay rows one pass can add (fused: every log record; sliced: one per env)."""
        return self.N * self._log_cap() if self.fused and self._trace_idx is None else self.N

    @torch.no_grad()
    def _fused_pass(self, replay_buffer, record):
        """One pass with the policy inside the env launch: every env runs max_ticks ticks (less if its
        log fills), chaining decisions and resetting ended episodes in place; then the decision log ->
        replay rows (all at once) and, with record, the path buffers / ring (record by record). Device
        work only (graph-capturable). Returns the transitions of this pass as a device scalar."""
        N, T, cap = self.N, self.max_path_length, self._log_cap()
        lg = self._logs.get(cap)
        if lg is None:
            lg = self._logs[cap] = (torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device=self.device),
                                    torch.zeros(N, dtype=torch.int32, device=self.device))
        log, log_len = lg
        dp = self._device_policy
        log_len.zero_()
        sim = self._base_env().sim
        if getattr(sim, "stream_tail", 0) != self.stream_tail:  # (host state of the handle, read at launch)
            sim.set_stream_tail(self.stream_tail)
        sim.run_policy(dp.weights(), self.max_ticks, T, self._ep_idx, self._dec_idx, deterministic=dp.deterministic,
                       seed=dp.seed, counter=None if dp.deterministic else dp.counter, out=self._fused_out,
                       log=log, log_len=log_len)
        if not dp.deterministic:
            dp.counter.add_(1)
        valid = torch.arange(cap, device=self.device).unsqueeze(0) < log_len.unsqueeze(1)        # (N, cap)
        ev = log[:, :, abi.DL_EVENTS].to(torch.int64)
        rew = log[:, :, abi.DL_REWARD] * self._env._reward_scale
        nonfinite = (ev & abi.EV_NONFINITE) != 0
        good = valid & ~nonfinite
        dec = log[:, :, abi.DL_DECISION].to(torch.int64)
        end = valid & ((log[:, :, abi.DL_DONE] != 0) | nonfinite | (dec + 1 >= T))
        act = log[:, :, abi.DL_ACTION].to(torch.float32)
        if replay_buffer is not None:  # env-major, in env chunks no larger than one add can take
            step = max(1, _add_capacity(replay_buffer) // cap)
            for a in range(0, N, step):
                b = min(N, a + step)
                n = (b - a) * cap
                replay_buffer.add_batch(log[a:b, :, abi.DL_OBS0:abi.DL_OBS0 + 8].reshape(n, 8).to(torch.float32),
                                        act[a:b].reshape(n, 1), rew[a:b].reshape(n, 1).to(torch.float32),
                                        log[a:b, :, abi.DL_OBS:abi.DL_OBS + 8].reshape(n, 8).to(torch.float32),
                                        ((ev[a:b] & abi.EV_TERMINAL) != 0).reshape(n, 1).to(torch.float32),
                                        mask=good[a:b].reshape(-1))
        if record:  # record by record, in each env's order: the episode buffers, ended episodes -> the ring
            evi = ev.to(torch.int32)
            for j in range(cap):
                g, e = good[:, j], end[:, j]
                pos = dec[:, j].clamp(0, T - 1)
                for buf, v in ((self._path_rew, rew[:, j]), (self._path_act, act[:, j]), (self._path_ev, evi[:, j])):
                    buf[self._rows, pos] = torch.where(g, v.to(buf.dtype), buf[self._rows, pos])
                length = torch.where(e, dec[:, j] + g.to(torch.int64), torch.zeros_like(dec[:, j])).to(torch.int32)
                keep = e & (length > 0)
                k64 = keep.to(torch.int64)
                slot = (torch.cumsum(k64, 0) - k64 + self._ring_top) % self._ring_cap
                idx = torch.where(keep, slot, torch.full_like(slot, self._ring_cap))
                self._ring_len.index_copy_(0, idx, length)
                self._ring_rew.index_copy_(0, idx, self._path_rew)
                self._ring_act.index_copy_(0, idx, self._path_act)
                self._ring_ev.index_copy_(0, idx, self._path_ev)
                self._ring_top += k64.sum()
        else:  # the unfinished episode's decisions only (one write per element: graph-capturable scatter)
            cur = good & (log[:, :, abi.DL_EPISODE].to(torch.int32) == self._ep_idx.unsqueeze(1))
            flat = self._rows.unsqueeze(1) * T + dec.clamp(0, T - 1)
            idx = torch.where(cur, flat, torch.full_like(flat, N * T)).reshape(-1)
            for b, v in zip(self._path_flat, (rew, act, ev.to(torch.int32))):
                b.index_copy_(0, idx, v.reshape(-1).to(b.dtype))
        n_good = good.sum()
        self._steps_total += n_good
        self._paths_total += end.sum()
        self._ticks_total += self._fused_out["ticks"].sum()
        self._nonfinite_total += (valid & nonfinite).sum()
        self._path_len.copy_(self._dec_idx)  # the sliced pass's episode length, for a switch back (_enter)
        return n_good

    @torch.no_grad()
    def _pass(self, replay_buffer, record):
        """One sliced pass over all envs, device work only (graph-capturable with a device policy).
        Returns the transitions of this pass as a device scalar."""
        self._choose_actions()
        out = self._env.step_async(self._act, max_ticks=self.max_ticks, out=self._out)
        ready = out["ready"].bool()
        done = out["done"].bool()
        rew = out["reward"] * self._env._reward_scale
        terminal = (out["events"] & abi.EV_TERMINAL) != 0
        # a decision that ended on a NaN/Inf ship state (EV_NONFINITE; the env reports it done) is not a
        # transition: it never reaches the replay buffer or the epoch paths, the episode just ends
        nonfinite = (out["events"] & abi.EV_NONFINITE) != 0
        good = ready & ~nonfinite
        if replay_buffer is not None:
            replay_buffer.add_batch(self._obs, self._act, rew.to(torch.float32).unsqueeze(1), out["obs"],
                                    terminal.to(torch.float32).unsqueeze(1), mask=good)
        pos = self._path_len.clamp(max=self.max_path_length - 1).long()
        for buf, v in ((self._path_rew, rew), (self._path_act, self._act[:, 0]), (self._path_ev, out["events"])):
            buf[self._rows, pos] = torch.where(good, v.to(buf.dtype), buf[self._rows, pos])
        self._path_len += good.to(torch.int32)
        self._ret += torch.where(good, rew, torch.zeros_like(rew))
        self._nonfinite_total += (ready & nonfinite).sum()
        end = ready & (done | nonfinite | (self._path_len >= self.max_path_length))
        if record:  # ended episodes with at least one transition -> the ring (prefix-sum scatter, as add_batch)
            keep = end & (self._path_len > 0)
            k64 = keep.to(torch.int64)
            slot = (torch.cumsum(k64, 0) - k64 + self._ring_top) % self._ring_cap
            idx = torch.where(keep, slot, torch.full_like(slot, self._ring_cap))
            self._ring_len.index_copy_(0, idx, self._path_len)
            self._ring_rew.index_copy_(0, idx, self._path_rew)
            self._ring_act.index_copy_(0, idx, self._path_act)
            self._ring_ev.index_copy_(0, idx, self._path_ev)
            self._ring_top += k64.sum()
        self._obs.copy_(torch.where(ready.unsqueeze(1), out["obs"], self._obs))
        self._awaiting.copy_(ready)  # (non-finite decisions included: those envs were reset and wait too)
        self._n_ready = ready.sum()
        n_ready = good.sum()
        self._steps_total += n_ready
        self._paths_total += end.sum()
        self._ticks_total += out["ticks"].sum()
        self._last_end = end
        self._last_end_len = torch.where(end, self._path_len, torch.zeros_like(self._path_len))
        if self._trace_idx is not None:
            self._trace_pass(out, end)
        # masked auto-reset of finished episodes
        self._env.reset(mask=end.to(torch.uint8), obs_out=self._obs_reset)
        self._obs.copy_(torch.where(end.unsqueeze(1), self._obs_reset, self._obs))
        self._path_len.masked_fill_(end, 0)
        self._ret.masked_fill_(end, 0.0)
        return n_ready

    def step(self, replay_buffer=None):
        """One sliced pass over all envs (eager). Returns (ready mask, #transitions) as device tensors."""
        self._enter("sliced")
        n = self._pass(replay_buffer, False)
        self._n_awaiting = None
        return self._awaiting, n

    def _graph_pass(self, replay_buffer, record, fused=False):
        key = (id(replay_buffer) if replay_buffer is not None else None, bool(record), self.max_ticks, fused,
               self.stream_tail if fused else 0)
        g = self._graphs.get(key)
        pass_fn = self._fused_pass if fused else self._pass
        if g is None:
            # one eager pass on a side stream (allocations, library scratch), then the capture
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                pass_fn(replay_buffer, record)
            torch.cuda.current_stream(self.device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                pass_fn(replay_buffer, record)
            self._graphs[key] = g
            return  # the capture did not run the pass; the eager one did
        g.replay()

    def collect(self, num_steps, replay_buffer=None, record_paths=False):
        """Advance until ≥ num_steps transitions were produced. Device-policy collectors replay the
        graph-captured pass and read the transition count on the host only between batches of passes
        (planned from the count per pass so far); torch-policy collectors sync once per pass."""
        self._take_over()
        record = bool(record_paths)
        if record:
            self._ring_top.zero_()
        fused = self.fused and self._trace_idx is None
        self._enter("fused" if fused else "sliced")
        if self._device_policy is None or self._trace_idx is not None:
            got = 0
            while got < num_steps:
                n = self._pass(replay_buffer, record)
                got += int(n.item())                      # transitions (non-finite decisions left out)
                self._n_awaiting = int(self._n_ready.item())  # envs that wait for an action
        else:
            room0 = _staging_room(replay_buffer)
            if room0 is not None and room0 < num_steps + 2 * self._rows_per_pass():
                # checked once, before any pass: every rank of a replicated group has the same room (each sync
                # empties the stage), the same num_steps and the same pass size, so all of them fail here together
                # instead of one rank failing mid-collect while the others wait in the next sync's all-gather
                raise RuntimeError(
                    f"BatchedPathCollector: the replay buffer's staging ring has room for {room0} rows; a collect of "
                    f"{num_steps} decisions needs {num_steps + 2 * self._rows_per_pass()} (plus two passes of "
                    f"{self._rows_per_pass()} rows): sync() it after every collect or enlarge its stage_size "
                    f"(ast_sac_runner.replicated_stage_rows)")
            start = int(self._steps_total.item())
            got, passes, batch = 0, 0, 1
            while got < num_steps:
                room = _staging_room(replay_buffer)
                if room is not None:  # a staging ring (ReplicatedReplayBuffer) takes rows only until its next sync
                    fit = room // self._rows_per_pass()
                    if fit < 1:
                        raise RuntimeError(
                            f"BatchedPathCollector: the replay buffer's staging ring has room for {room} rows, less "
                            f"than one pass can add ({self._rows_per_pass()}); sync() it after every collect or "
                            f"enlarge its stage_size (ast_sac_runner.replicated_stage_rows)")
                    batch = min(batch, fit)
                for _ in range(batch):
                    if self.use_graph:
                        self._graph_pass(replay_buffer, record, fused)
                    elif fused:
                        self._fused_pass(replay_buffer, record)
                    else:
                        self._pass(replay_buffer, record)
                passes += batch
                got = int(self._steps_total.item()) - start
                per = max(got / passes, 1.0)
                batch = max(1, math.ceil((num_steps - got) / per))
            self._n_awaiting = None
        if record:
            self._drain_ring()
        self.check_nonfinite()
        return got

    def _drain_ring(self):
        """The episodes that ended during this collect -> reference path dicts (rollout_functions.py:161-181:
        rewards and actions (T, 1), terminals, env_infos with the reference's keys), one host copy."""
        top = int(self._ring_top.item())
        n = min(top, self._ring_cap)
        if n == 0:
            return
        if top > self._ring_cap:
            warnings.warn(f"BatchedPathCollector: {top} episodes ended during this collect but the path ring holds "
                          f"{self._ring_cap}; the epoch paths keep the newest {self._ring_cap} (construct the "
                          f"collector with a larger path_ring)", RuntimeWarning, stacklevel=2)
        order = [(top - n + j) % self._ring_cap for j in range(n)]  # oldest first
        sel = torch.as_tensor(order, dtype=torch.long, device=self.device)
        lens = self._ring_len[sel].cpu().numpy()
        rews = self._ring_rew[sel].cpu().numpy()
        acts = self._ring_act[sel].cpu().numpy()
        evs = self._ring_ev[sel].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        for L, r, a, ev in zip(lens, rews, acts, evs):
            L = int(L)
            ev = ev[:L]
            infos = [dict(terminal=bool(x & abi.EV_TERMINAL), test_ship_stop=bool(x & abi.EV_TEST_STOP),
                          obs_ship_stop=bool(x & abi.EV_OBS_STOP)) for x in ev]
            self._epoch_paths.append(dict(rewards=r[:L, None].copy(), actions=a[:L, None].copy(),
                                          terminals=np.array([[i["terminal"]] for i in infos]),
                                          env_infos=infos, agent_infos=[{} for _ in range(L)]))

    def check_nonfinite(self):
        """Warn (once per occurrence) when env decisions ended on a non-finite ship state since the last
        check: the env library's status (shipsim_synchronize), those rows were kept out of the buffer."""
        sim = getattr(self._env, "sim", None)
        if sim is None:
            return
        from ....shipsim import ShipSimNonFiniteError
        try:
            sim.synchronize()
        except ShipSimNonFiniteError as e:
            warnings.warn(f"BatchedPathCollector: {e} (transitions dropped from the replay buffer and paths)",
                          RuntimeWarning, stacklevel=2)

    # reference collector surface -------------------------------------------------------------
    def get_epoch_paths(self):
        return self._epoch_paths

    def end_epoch(self, epoch):
        self._epoch_paths = deque(maxlen=self._max_saved)

    def get_diagnostics(self):
        """MdpPathCollector.get_diagnostics (path_collector.py:83-92): the same keys, so progress.csv has
        the reference's columns (tests/golden/progress_header.json)."""
        st = OrderedDict([("num steps total", int(self._steps_total.item())),
                          ("num paths total", int(self._paths_total.item()))])
        st.update(create_stats_ordered_dict("path length", [len(p["actions"]) for p in self._epoch_paths],
                                            always_show_all_stats=True))
        return st

    def device_diagnostics(self):
        """What the batched collector counts beyond the reference's columns (logged as text, not to
        progress.csv): env ticks advanced and decisions dropped for a non-finite ship state."""
        return OrderedDict([("num env ticks total", int(self._ticks_total.item())),
                            ("num nonfinite decisions dropped", int(self._nonfinite_total.item()))])

    def get_snapshot(self):
        return dict(policy=self._policy)
