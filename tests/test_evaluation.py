"""The evaluation sweep (cpp_volume_rendering_amd/evaluation.py) against the
reference's ParameterSpace semantics and its own sweep output: the isosurface
renderers' parameter space enumerates exactly the 200 rows of
data/4b skipping/skipping eval 4 blocks.csv (values as std::to_string prints
them, in the same order), and the PNG writer round-trips through PIL."""
import csv
import os

import numpy as np
import pytest

from cpp_volume_rendering_amd import evaluation as E
from cpp_volume_rendering_amd.renderer import (CustomRayCasting1PassIsoAdapt,
                                               RayCasting1Pass)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _sweep_rows(renderer):
    ps = E.ParameterSpace.from_renderer(renderer)
    ps.StartEvaluation()
    rows = []
    while True:
        rows.append([ps.GetDimensionValue(i) for i in range(ps.GetNumDimensions())])
        if not ps.IncrEvaluation():
            break
    ps.EndEvaluation()
    return ps, rows


def test_iso_parameter_space_matches_reference_sweep():
    r = CustomRayCasting1PassIsoAdapt()
    before = (r.m_u_step_size_small, r.m_u_step_size_large, r.m_u_step_size_range)
    ps, rows = _sweep_rows(r)
    assert [ps.GetDimensionName(i) for i in range(3)] == ["StepSizeSmall", "StepSizeLarge",
                                                          "StepSizeRange"]
    assert len(rows) == 200
    # NumSteps = 1 + ceil((end - start) / incr) overestimates when the range is not a
    # multiple of the step (6 x 8 x 6): the reference's UI estimate, kept as is
    assert ps.GetNumSamplePoints() == 288
    with open(os.path.join(GOLDEN, "iso_eval_4blocks_params.csv")) as f:
        ref = [row[:3] for row in csv.reader(f)][1:]
    assert rows == ref
    # EndEvaluation restores the renderer's values
    assert (r.m_u_step_size_small, r.m_u_step_size_large, r.m_u_step_size_range) == before


def test_rc1pass_parameter_space():
    ps, rows = _sweep_rows(RayCasting1Pass())
    # 0.2 += 0.1 in float reaches 2.0000002 > 2.0 after 1.9: 18 points (estimate 19)
    assert len(rows) == 18 and ps.GetNumSamplePoints() == 19
    assert rows[0] == ["0.200000"] and rows[-1] == ["1.900000"]


def test_parameter_range_counts_as_reference_test():
    """ParameterSpaceTest (parameterspace.cpp:120-149): [0, 1] by 0.1 -> 11 steps."""
    class T:
        v = 0.0
    t = T()
    p = E.ParameterRange("DTest", t, "v", 0, 1, 0.1, dtype=np.float64)
    n = 0
    p.Start()
    while not p.End():
        n += 1
        p.Incr()
    assert n == 11 == p.NumSteps()


def test_png_writer_round_trip(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    path = str(tmp_path / "x.png")
    E.write_png_rgb8(path, img)
    back = np.asarray(Image.open(path).convert("RGB"))
    assert np.array_equal(back, img[::-1])     # row 0 of the input is the bottom
