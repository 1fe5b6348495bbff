"""bench.py's roofline on the pipe that binds, on CPU: the vmem and
VALU fractions from a PMC record (scaled to the launch's frames), the fallback to the
kernel's own wave-load count, the choice of the busier pipe, and the TD split."""
import os

import pytest


@pytest.fixture(scope="module")
def bench():
    os.environ.setdefault("WORLD_SIZE", "1")
    import bench as B
    return B


def test_pipe_roofline_from_pmc(bench):
    pmc = {"frames_per_launch": 4, "sq_insts_vmem_rd": 4.586e6, "valu_wave_insts": 2.448e8,
           "td_busy_frac_per_cu": 0.771, "td_tc_stall_frac_per_cu": 0.418,
           "td_work_cycles_per_wave_load": 16.8, "tcp_accesses_per_wave_load": 18.9,
           "l1_miss_requests_per_wave_load": 2.1, "effective_clock_ghz_under_pmc": 2.17}
    r = bench.pipe_roofline(0.3202, 4, pmc, None)
    assert r["bound"] == "valu"
    # 2.448e8 wave-instructions in 0.3202 ms against 1024 SIMDs x 2.4 GHz / 2
    assert r["frac"] == pytest.approx(2.448e8 / 0.3202e-3 / (1024 * 2.4e9 / 2), rel=1e-3)
    assert r["pipes"]["vmem"]["frac"] == pytest.approx(
        4.586e6 * 1024 / 0.3202e-3 / (256 * 64 * 2.4e9), rel=1e-3)
    assert 0 < r["frac"] <= 1 and r["unit"] == "G wave-instr/s"
    assert r["vmem_detail"]["td_stalled_on_cache_per_cu"] == 0.418
    # a launch of 1 frame scales the record's 4-frame counts
    r1 = bench.pipe_roofline(0.3202 / 4, 1, pmc, None)
    assert r1["frac"] == pytest.approx(r["frac"], rel=1e-3)


def test_pipe_roofline_without_pmc(bench):
    r = bench.pipe_roofline(0.32, 4, {}, 4.5e6)
    assert r["bound"] == "vmem" and set(r["pipes"]) == {"vmem"}
    assert r["pipes"]["vmem"]["count"].startswith("kernel count")
    assert bench.pipe_roofline(0.32, 4, {}, None) == {}


def test_vmem_bound_when_busier(bench):
    pmc = {"frames_per_launch": 1, "sq_insts_vmem_rd": 2.166e9, "valu_wave_insts": 3.9e10}
    r = bench.pipe_roofline(72.57, 1, pmc, None)   # EBS-like: the TD path is the busier pipe
    assert r["bound"] == "vmem"
    assert r["frac"] == pytest.approx(2.166e9 * 1024 / 72.57e-3 / (256 * 64 * 2.4e9), rel=1e-3)
