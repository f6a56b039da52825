"""The bench workload itself at full size (BASELINE.json configs[2]: 4096 two-ship AST envs, PTI
machinery, dt 4 s, the decision stream of shipsim_run_table in 128-tick launches, as bench.py runs
it, in 128-tick launches and in one 4096-tick launch, the bench default), checked two ways:
  - every env: size-independent invariants of the decision log (finite records, episode / decision
    counters in order, each episode ends on done or on the 9th decision, ticks per launch bounded);
  - every 4th env: decision by decision against the CPU oracle replaying the same episodes
    (reward, termination bits, done, obs, and the decision's tick count exactly), with the oracle's
    few-ulp initial-condition variants (gpu_harness.run_oracle_variants) as the acceptance
    envelope; at most 1 % of the checked envs may need a perturbed variant (every case so far: none).
Each case's statistics (fraction matched only by a perturbed oracle run, worst relative error) are printed and
appended as one JSON line to $SHIPSIM_PARITY_LOG (default gpurun_out/parity_fullsize.jsonl; committed copies under
profiles/).
Needs an MI355X."""
import copy
import json
import os
import time

import numpy as np
import pytest
import torch

import gpu_harness as H
from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim
from parity import rel_err

pytestmark = pytest.mark.gpu

N = 4096
N_EPS = 3


def _run(cfg, a_norm, SLICE, LAUNCHES, tail=0):
    sim = ShipSim(cfg, N)
    sim.reset()
    if tail:
        sim.set_stream_tail(tail)
    table = torch.from_numpy(abi.normalized_to_scoping(a_norm)).cuda()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    cap = 144 if not tail else 288  # (the tail case: up to 2 x 5120 ticks, decisions of >= ~76 ticks)
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    ticks = []
    for _ in range(LAUNCHES):
        o = sim.run_table(table, SLICE, ep, dec, log=log, log_len=log_len)
        ticks.append(o["ticks"].cpu().numpy())
    torch.cuda.synchronize()
    out = log.cpu().numpy(), log_len.cpu().numpy(), np.array(ticks), ep.cpu().numpy(), dec.cpu().numpy()
    sim.close()
    return out


def _episodes(rows):
    """decision-log rows of one env -> per episode [(obs, reward, done, bits, -1), ...] (harness tuples)"""
    eps = []
    for r in rows:
        e = int(r[abi.DL_EPISODE])
        while len(eps) <= e:
            eps.append([])
        eps[e].append((r[abi.DL_OBS:abi.DL_OBS + 8].astype(np.float32), r[abi.DL_REWARD], bool(r[abi.DL_DONE]),
                       int(r[abi.DL_EVENTS]), int(r[abi.DL_TICKS])))
    return eps


def _match(g_eps, o_rec, rtol=1e-5):
    """g_eps (possibly ending in an unfinished episode) against the oracle's episodes: bits, done and
    the decision's tick count exactly, obs and reward within rtol."""
    worst = 0.0
    for k, gd in enumerate(g_eps):
        od = o_rec[k][1]
        if len(gd) > len(od) or (k < len(g_eps) - 1 and len(gd) != len(od)):
            return np.inf
        for g, o in zip(gd, od):
            if (g[3] & 0x7FFFF) != (o[3] & 0x7FFFF) or g[2] != o[2] or g[4] != o[4]:
                return np.inf
            e = max(float(rel_err(g[0][None], o[0][None]).max()), float(abs(g[1] - o[1]) / (abs(o[1]) + 1e-6)))
            if e > rtol:
                return e
            worst = max(worst, e)
    return worst


# The last case is bench.py's headline launch exactly: sbmpc, detailed machinery, 4096 envs, 4096-tick launches with
# the 1024-tick work-conserving launch tail (shipsim_set_stream_tail), over bench.py's own 8-episode PCG64 table
# (seed 20251015, rank 0); two launches, so the second resumes every env where the tail left it.
@pytest.mark.parametrize("collav,SLICE,LAUNCHES,mach,tail,n_eps",
                         [("sbmpc", 128, 12, "detailed", 0, N_EPS), ("none", 128, 12, "detailed", 0, N_EPS),
                          ("sbmpc", 4096, 1, "detailed", 0, N_EPS), ("simple", 1024, 2, "detailed", 0, N_EPS),
                          ("sbmpc", 1024, 2, "simplified", 0, N_EPS), ("none", 1024, 2, "simplified", 0, N_EPS),
                          ("sbmpc", 4096, 2, "detailed", 1024, 8)])
def test_bench_workload_full_size(collav, SLICE, LAUNCHES, mach, tail, n_eps):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cfg = abi.ast_config(collav, machinery=abi.MACH_DETAILED if mach == "detailed" else abi.MACH_SIMPLIFIED)
    n_dec = cfg.max_sampling_frequency
    a_norm = np.random.Generator(np.random.PCG64(20251015)).uniform(-1, 1, (n_eps, n_dec, N)).astype(np.float32)
    log, log_len, ticks, ep, dec = _run(cfg, a_norm, SLICE, LAUNCHES, tail)

    # invariants, every env
    if tail:  # the tail extends a launch by whole chunks, up to `tail` more ticks per env
        assert ticks.max() <= SLICE + tail and (ticks >= SLICE).mean() > 0.99, (ticks.min(), ticks.max())
        print(f"\n[launch tail {tail}] ticks per env per launch: min {ticks.min()} mean {ticks.mean():.1f} "
              f"max {ticks.max()}")
    else:
        assert ticks.max() <= SLICE and (ticks == SLICE).mean() > 0.99  # the stream keeps every env busy
    assert (log_len >= 4).all() and log_len.max() <= log.shape[1]
    total_dec = 0
    for i in range(N):
        rows = log[i, :log_len[i]]
        assert np.isfinite(rows).all(), i
        e, d = rows[:, abi.DL_EPISODE].astype(int), rows[:, abi.DL_DECISION].astype(int)
        # counters advance by one decision, or start a new episode at decision 0
        nxt_same = (e[1:] == e[:-1]) & (d[1:] == d[:-1] + 1)
        nxt_new = (e[1:] == e[:-1] + 1) & (d[1:] == 0)
        assert (nxt_same | nxt_new).all(), i
        # an episode ends on done or on its n_dec-th decision, never otherwise
        ends = np.nonzero(nxt_new)[0]
        assert ((rows[ends, abi.DL_DONE] == 1) | (d[ends] == n_dec - 1)).all(), i
        assert (d < n_dec).all()
        total_dec += len(rows)
    assert total_dec == int(log_len.sum())

    # oracle, every 4th env
    idx = np.arange(0, N, 4)
    tables = [[a_norm[k % n_eps, :, i] for k in range(int(log[i, log_len[i] - 1, abi.DL_EPISODE]) + 1)] for i in idx]
    g_all = [_episodes(log[i, :log_len[i]]) for i in idx]
    orc = H.run_oracle(cfg, tables)
    worst, bad, perturbed = 0.0, [], 0
    for j, i in enumerate(idx):
        w = _match(g_all[j], orc[j][0])
        if not w <= 1e-5:
            perturbed += 1
            for eps in H.PERTURBATIONS[1:]:  # the oracle's own few-ulp envelope (gpu_harness)
                c = copy.deepcopy(cfg)
                c.ship[0].initial_north_position_m *= 1 + eps
                c.ship[1].initial_east_position_m *= 1 - eps
                w = min(w, _match(g_all[j], H.run_oracle(c, [tables[j]])[0][0]))
                if w <= 1e-5:
                    break
        if not w <= 1e-5:
            bad.append(int(i))
        else:
            worst = max(worst, w)
    frac = perturbed / len(idx)
    print(f"\n[{collav} {mach} slice {SLICE} tail {tail}] {len(idx)} envs vs oracle, {sum(len(e) for e in g_all)} decisions; "
          f"matched only by a perturbed oracle run: {perturbed} ({100 * frac:.2f} %); off the oracle: {len(bad)}; "
          f"worst rel err {worst:.2e}")
    _record(dict(collav=collav, machinery=mach, slice=SLICE, launches=LAUNCHES, tail=tail, episodes_in_table=n_eps,
                 envs_checked=len(idx), decisions_checked=int(sum(len(d) for e in g_all for d in e)),
                 perturbed=perturbed, perturbed_frac=frac, off_oracle=len(bad), worst_rel_err=worst,
                 ticks_per_env_launch=[int(ticks.min()), float(ticks.mean()), int(ticks.max())]))
    assert not bad, f"envs off the oracle: {bad[:20]}"
    assert frac <= 0.01, f"{perturbed} of {len(idx)} envs matched only by a perturbed oracle run"
    assert worst <= 1e-5


def _record(row):
    path = os.environ.get("SHIPSIM_PARITY_LOG") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity_fullsize.jsonl")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    row = dict(row, time=time.strftime("%Y-%m-%dT%H:%M:%S"),
               library=__import__("ast_sac_amd.shipsim", fromlist=["x"]).load_library().shipsim_build_info().decode())
    with open(path, "a") as f:
        f.write(json.dumps(row) + "\n")
