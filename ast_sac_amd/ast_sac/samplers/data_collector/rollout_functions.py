"""ast_sac_rollout (ast_sac/samplers/data_collector/rollout_functions.py:74-181).

One episode of at most `max_path_length` decisions on a single (N=1 view) env; terminals are
env_info['terminal'], dones the env's combined done.
"""
import copy

import numpy as np


def ast_sac_rollout(env, agent, max_path_length=np.inf, render=False, render_kwargs=None,
                    preprocess_obs_for_policy_fn=None, get_action_kwargs=None, full_o_postprocess_func=None,
                    reset_callback=None):
    render_kwargs = render_kwargs or {}
    get_action_kwargs = get_action_kwargs or {}
    observations, actions, rewards, terminals, dones = [], [], [], [], []
    agent_infos, env_infos, next_observations = [], [], []
    path_length = 0
    agent.reset()
    o = env.reset()
    if reset_callback:
        reset_callback(env, agent, o)
    if render:
        env.render(**render_kwargs)
    while path_length < max_path_length:
        a, agent_info = agent.get_action(o, **get_action_kwargs)
        if full_o_postprocess_func:
            full_o_postprocess_func(env, agent, o)
        next_o, r, done, env_info = env.step(copy.deepcopy(a))
        if render:
            env.render(**render_kwargs)
        observations.append(o)
        rewards.append(r)
        terminals.append(env_info["terminal"])
        dones.append(done)
        actions.append(a)
        next_observations.append(next_o)
        agent_infos.append(agent_info)
        env_infos.append(env_info)
        path_length += 1
        if done:
            break
        o = next_o
    actions = np.array(actions)
    if len(actions.shape) == 1:
        actions = np.expand_dims(actions, 1)
    rewards = np.array(rewards)
    if len(rewards.shape) == 1:
        rewards = rewards.reshape(-1, 1)
    return dict(observations=np.array(observations), actions=actions, rewards=rewards,
                next_observations=np.array(next_observations), terminals=np.array(terminals).reshape(-1, 1),
                dones=np.array(dones).reshape(-1, 1), agent_infos=agent_infos, env_infos=env_infos)
