import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built kernel library")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def fixtures_dir(tmp_path_factory):
    from flink_jpmml_amd.assets import write_fixtures

    d = tmp_path_factory.mktemp("pmml")
    return write_fixtures(str(d))


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
