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


# Run order of the GPU suites under `-x`: the headline parity first, the 1024^3 /
# 2048^2 full-size cases last, so one full-size failure (or OOM) never hides the
# faster parity rows. Files not listed keep their collection order in between.
_SUITE_ORDER = ("test_rc1pass_gpu.py", "test_filter8_gpu.py", "test_postpass_gpu.py", "test_split_gpu.py",
                "test_dos_gpu.py", "test_ebs_gpu.py", "test_iso_gpu.py",
                "test_selftest_gpu.py")
_SUITE_LAST = ("test_fullsize_gpu.py",)


def _suite_rank(item):
    name = os.path.basename(str(item.fspath))
    if name in _SUITE_ORDER:
        return _SUITE_ORDER.index(name)
    if name in _SUITE_LAST:
        return len(_SUITE_ORDER) + 1 + _SUITE_LAST.index(name)
    return len(_SUITE_ORDER)


def pytest_collection_modifyitems(session, config, items):
    # sorted() is stable: tests inside one file keep their own order.
    items[:] = sorted(items, key=_suite_rank)


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
