"""Snapshot load (mt_load_snapshot) on a real MI355X vs the oracle: the checks of
tests/test_snapshot_load.py with the HIP engine (libmtgpu.so) in place of the
host emulation."""
import pytest

from test_gpu_parity import gpu_engine
from test_snapshot_load import (COLLAB_CASES, GOLDEN, LOADBODY_CASES, check_collab, check_golden,
                                check_golden_legacy, check_loadbody, check_quiescent)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", GOLDEN)
def test_gpu_loads_reference_snapshot(name):
    check_golden(name, gpu_engine)


@pytest.mark.parametrize("name", GOLDEN)
def test_gpu_legacy_snapshot_round_trip(name):
    check_golden_legacy(name, gpu_engine)


@pytest.mark.parametrize("case", COLLAB_CASES)
def test_gpu_collab_snapshot_load_and_continue(case):
    check_collab(case, gpu_engine)


def test_gpu_quiescent_long_snapshot_load_and_continue():
    check_quiescent(gpu_engine)


@pytest.mark.parametrize("name", list(LOADBODY_CASES))
def test_gpu_loadbody_reference_behaviour(name):
    check_loadbody(name, gpu_engine)
