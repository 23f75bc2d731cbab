"""Shared fixtures.  Markers: `gpu` = needs a real MI355X (run with -m gpu on the box)."""
import os
import sys
import warnings

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF_DATA = "/root/reference/pkg/recommender/recommender"
REF_PROM = "/root/reference/pkg/prom/test_data"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    warnings.filterwarnings("ignore", message=".*Early stopping criterion not reached.*")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def ref_data():
    """The reference's shipped training matrices (read in place, never copied); parity
    tests skip when the reference checkout is not mounted."""
    conf = os.path.join(REF_DATA, "configurations_train.ods")
    intf = os.path.join(REF_DATA, "interference_train.ods")
    if not (os.path.isfile(conf) and os.path.isfile(intf)):
        pytest.skip("reference data not mounted")
    return conf, intf


@pytest.fixture(scope="session")
def trained(ref_data):
    from k8s_gpu_scheduler_amd.recommender.tables import Table, TrainedTable
    conf, intf = ref_data
    return (TrainedTable.fit(Table.read_tsv(conf), "iterative", "c"),
            TrainedTable.fit(Table.read_tsv(intf), "iterative", "i"))
