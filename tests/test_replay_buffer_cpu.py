"""a30: EnvReplayBuffer / SimpleReplayBuffer pinned against the reference's own buffer
(tests/golden/replay_buffer.npz, written by gen_golden.py gen_replay from
ast_sac/data_management/{env_replay_buffer.py:8-50, simple_replay_buffer.py:44-103,
replay_buffer.py:34-77}): add_paths over a wrapping 7-row ring, with and without env_info sizes —
stored arrays (values and dtypes, fp64 and uint8 terminals), top / size, and random_batch under the
same np.random seed, all identical; plus DeviceReplayBuffer's ring order and batch layout against
the same path rows."""
import numpy as np
import torch

from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer, EnvReplayBuffer
from ast_sac_amd.spaces import Box


def _paths(fx):
    paths = []
    for k in range(3):
        g = lambda key: fx[f"path{k}/{key}"]
        T = g("obs").shape[0]
        paths.append(dict(observations=g("obs"), actions=g("act"), rewards=g("rew"), next_observations=g("nobs"),
                          terminals=g("term"), agent_infos=[{} for _ in range(T)],
                          env_infos=[dict(x=g("info")[t], terminal=bool(g("term")[t, 0]), events="")
                                     for t in range(T)]))
    return paths


class _Env:
    observation_space = Box(-np.inf, np.inf, shape=(8,))
    action_space = Box(-1.0, 1.0, shape=(1,))


class _EnvInfo(_Env):
    info_sizes = {"x": 2}


def test_env_replay_buffer_matches_reference(golden):
    fx = golden("replay_buffer")
    for tag, env in (("plain", _Env()), ("info", _EnvInfo())):
        rb = EnvReplayBuffer(7, env)
        rb.add_paths(_paths(fx))
        np.random.seed(123)
        b = rb.random_batch(5)
        for key in ("_observations", "_actions", "_rewards", "_terminals", "_next_obs"):
            ref = fx[f"{tag}/{key}"]
            got = getattr(rb, key)
            assert got.dtype == ref.dtype and got.shape == ref.shape, (tag, key)
            np.testing.assert_array_equal(got, ref)
        assert [rb._top, rb._size] == fx[f"{tag}/top_size"].tolist()
        keys = sorted(k.split("/")[-1] for k in fx.files if k.startswith(f"{tag}/batch/"))
        assert sorted(b) == keys
        for key in keys:
            np.testing.assert_array_equal(b[key], fx[f"{tag}/batch/{key}"])
            assert b[key].dtype == fx[f"{tag}/batch/{key}"].dtype
        if tag == "info":
            np.testing.assert_array_equal(rb._env_infos["x"], fx["info/env_info_x"])
        assert rb.num_steps_can_sample() == 7


def test_device_replay_buffer_ring_matches_reference_rows(golden):
    """The device ring holds the same rows in the same slots (fp32), terminal as 0/1."""
    fx = golden("replay_buffer")
    rb = DeviceReplayBuffer(7, 8, 1, "cpu")
    for p in _paths(fx):
        f = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float32))
        rb.add_batch(f(p["observations"]), f(p["actions"]), f(p["rewards"]), f(p["next_observations"]),
                     f(p["terminals"]))
    for key, dev in (("_observations", rb._observations), ("_actions", rb._actions), ("_next_obs", rb._next_obs),
                     ("_rewards", rb._rewards), ("_terminals", rb._terminals)):
        np.testing.assert_array_equal(dev.cpu().numpy(), fx[f"plain/{key}"].astype(np.float32))
    assert rb.num_steps_can_sample() == 7
