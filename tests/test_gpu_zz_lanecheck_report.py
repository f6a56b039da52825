"""Read-out of a diagnostics build's lane / index checks (-DSHIPSIM_LANECHECK, scripts/build_abl.sh):
run last in a pytest invocation whose SHIPSIM_LIB is lib_lanecheck.so or lib_ilp_lanecheck.so, after the
env path's tests (scripts/gpu_r3_lanecheck.sh). Every cross-lane exchange of the step kernels read only
active lanes and every checked index was in range, over every launch of that invocation. Skipped on the
default build (the checks are compiled out). Needs an MI355X."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_no_lane_or_index_violations():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd.shipsim import diag_lane_faults
    d = diag_lane_faults()
    if d is None:
        pytest.skip("default build: lane checks compiled out")
    assert d["violations"] == 0, d
