"""shipsim_sbmpc_eval_multi: SBMPC.get_optimal_ctrl_offset over a do_list of K obstacles (sbmpc.py:113-185) on the
device, through the C ABI — the optimiser the multi-obstacle env kernels (n_obs_ships = K > 1, configs[4]) run.

Pinned to the REFERENCE's own answers for K = 2, 3, 4 (tests/golden/sbmpc_multi.npz, made by
tests/golden/gen_golden.py gen_sbmpc_multi: one persistent controller per K, so the last-offset state carries from
call to call), and to the oracle on random batches. The batches cover both ways a wave serves requests: two
requests per pass (each lane taking its scenario's obstacles in turn) and a lone request whose obstacles the two
half-waves split."""
import numpy as np
import pytest

import oracle_ffi as O
from ast_sac_amd import shipsim_abi as abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _requests_from_fixture(g, K):
    ins, outs = g[f"k{K}_in"], g[f"k{K}_out"]
    reqs, refs = [], []
    p_last, chi_last = 1.0, 0.0
    for row, out in zip(ins, outs):
        slots = np.zeros(7 * abi.MAX_OBS)
        slots[:7 * K] = row[8:8 + 7 * K]
        reqs.append(np.concatenate([[p_last, chi_last], row[:8], slots]))
        refs.append(out[:3])
        p_last, chi_last = out[3], out[4]
    return np.array(reqs), np.array(refs)


@pytest.mark.parametrize("K", [2, 3, 4])
def test_sbmpc_eval_multi_matches_reference_known_answers(golden, torch_cuda, K):
    from ast_sac_amd.shipsim import sbmpc_eval_multi
    g = golden("sbmpc_multi")
    reqs, refs = _requests_from_fixture(g, K)
    assert reqs.shape[1] == abi.SBMPC_MULTI_IN
    got = sbmpc_eval_multi(reqs, K).cpu().numpy()  # every request in one launch (two per pass)
    np.testing.assert_array_equal(got, refs)
    for i in range(len(reqs)):  # each alone (one request per wave: the half-waves split its obstacles)
        if i % 7 == 0:
            np.testing.assert_array_equal(sbmpc_eval_multi(reqs[i:i + 1], K).cpu().numpy()[0], refs[i])


def _random_requests(rng, n, K):
    os_ = np.stack([rng.uniform(0, 20000, n), rng.uniform(0, 10000, n), rng.uniform(-np.pi, np.pi, n),
                    rng.uniform(0, 6, n), rng.uniform(-0.5, 0.5, n), rng.uniform(-0.01, 0.01, n)], 1)
    u_d, chi_d = rng.uniform(3, 5, n), rng.uniform(-4, 4, n)
    slots = np.zeros((n, 7 * abi.MAX_OBS))
    for k in range(K):
        ang, rad = rng.uniform(-np.pi, np.pi, n), rng.uniform(20, 4000, n)
        ob = np.stack([os_[:, 0] + rad * np.cos(ang), os_[:, 1] + rad * np.sin(ang), rng.uniform(-np.pi, np.pi, n),
                       rng.uniform(0, 6, n), rng.uniform(-0.5, 0.5, n)], 1)
        ahead = rng.uniform(size=n) < 0.5  # on a collision course: ahead of the nominal course, heading back
        r2, ax = rng.uniform(300, 1900, n), chi_d + rng.uniform(-0.6, 0.6, n)
        ob[ahead] = np.stack([os_[:, 0] - r2 * np.sin(ax), os_[:, 1] + r2 * np.cos(ax),
                              chi_d + np.pi + rng.uniform(-0.5, 0.5, n), rng.uniform(2, 6, n),
                              rng.uniform(-0.3, 0.3, n)], 1)[ahead]
        slots[:, 7 * k:7 * k + 5] = ob
        slots[:, 7 * k + 5] = np.where(rng.uniform(size=n) < 0.3, rng.uniform(40, 140, n), 80.0)
        slots[:, 7 * k + 6] = np.where(rng.uniform(size=n) < 0.3, rng.uniform(8, 30, n), 16.0)
    last = np.stack([rng.choice([0.4, 0.6, 0.8, 1.0], n), np.deg2rad(rng.choice(np.arange(-30, 31, 10), n))], 1)
    return np.concatenate([last, u_d[:, None], chi_d[:, None], os_, slots], 1)


def _oracle(reqs, K):
    return np.array([O.sbmpc_multi(r[0], r[1], r[2], r[3], r[4:10], r[10:10 + 7 * K].reshape(K, 7))[0] for r in reqs])


@pytest.mark.parametrize("K", [1, 2, 3, 4])
def test_sbmpc_eval_multi_matches_oracle(torch_cuda, K):
    """2048 random requests (half of the obstacles on a collision course, sizes varied) vs the oracle; then the same
    requests with only every 64th active (each wave serves one lone request: the split path) and every 32nd."""
    from ast_sac_amd.shipsim import sbmpc_eval_multi
    rng = np.random.Generator(np.random.PCG64(100 + K))
    n = 2048
    req = _random_requests(rng, n, K)
    ref = _oracle(req, K)
    got = sbmpc_eval_multi(req, K).cpu().numpy()
    assert got[:, 2].sum() > n // 2
    assert ((ref[:, 0] != 1) | (ref[:, 1] != 0)).sum() > n // 10  # the optimiser really chooses
    mism = np.nonzero((got != ref).any(axis=1))[0]
    assert len(mism) <= n // 1000, (len(mism), req[mism[:2]], got[mism[:2]], ref[mism[:2]])
    for stride in (64, 32):
        sparse = req.copy()
        far = np.ones(n, bool)
        far[::stride] = False
        for k in range(abi.MAX_OBS):  # every other request's obstacles out of D_INIT: inactive
            sparse[far, 10 + 7 * k] += 1e5
        got_s = sbmpc_eval_multi(sparse, K).cpu().numpy()
        assert got_s[far, 2].sum() == 0 and (got_s[far, :2] == [1.0, 0.0]).all()
        # the active requests' answers do not depend on how a wave served them (lone: split obstacles; paired)
        mism_s = np.nonzero((got_s[~far] != ref[~far]).any(axis=1))[0]
        assert len(mism_s) <= max(1, n // 1000), (stride, len(mism_s))


def test_sbmpc_eval_multi_k1_equals_single_obstacle_service(torch_cuda):
    """With one obstacle the multi-obstacle service is the reference's single-obstacle call: the same answers as
    shipsim_sbmpc_eval."""
    from ast_sac_amd.shipsim import sbmpc_eval, sbmpc_eval_multi
    rng = np.random.Generator(np.random.PCG64(9))
    req = _random_requests(rng, 1024, 1)
    single = np.concatenate([req[:, :10], req[:, 10:15], req[:, 15:17]], 1)
    np.testing.assert_array_equal(sbmpc_eval_multi(req, 1).cpu().numpy(), sbmpc_eval(single).cpu().numpy())


def test_sbmpc_eval_multi_rejects_bad_counts(torch_cuda):
    from ast_sac_amd.shipsim import ShipSimError, sbmpc_eval_multi
    req = np.zeros((4, abi.SBMPC_MULTI_IN))
    for k in (0, abi.MAX_OBS + 1):
        with pytest.raises(ShipSimError):
            sbmpc_eval_multi(req, k)
