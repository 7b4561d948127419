import os
import sys
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    # kernel choices the tests tune go to a throw-away user database: neither the shipped system
    # database (read-only anyway) nor the user's ~/.cache one sees per-test quick tunings
    os.environ.setdefault("DRN_TUNE_DB", os.path.join(tempfile.mkdtemp(prefix="drn-tune-"), "tune_db.json"))
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the in-tree HIP kernel library")
    config.addinivalue_line("markers", "slow: long-running integration test")


@pytest.fixture(scope="session")
def hip():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from distributed_resnet_tensorflow_amd.ops.backend import HipBackend
    return HipBackend("cuda")


@pytest.fixture(scope="session")
def ref():
    from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
    return RefBackend("cpu")
