import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def bonsai_tf(oracle):
    from cpp_volume_rendering_amd import datasets as D
    table = oracle.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    return oracle.tf_rgbt(table)


@pytest.fixture(scope="session")
def bonsai_tf_rgba(oracle):
    """GenerateTexture_1D_RGBA of the same TF (alpha = opacity, RGBA16F-rounded): the
    table the extinction volume of the occlusion renderer filters."""
    from cpp_volume_rendering_amd import datasets as D
    table = oracle.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    return oracle.tf_rgbt(table, extinction_input=True)
