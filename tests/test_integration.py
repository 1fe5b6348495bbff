"""The reference-side adapters (integration/hip_*.cpp: BaseVolumeRenderer subclasses
that forward to include/cvr.h) type-check against the reference's own headers where
they lie (cppvolrend/volrenderbase.h:25-96, DataManager, StructuredGridVolume,
TransferFunction, Camera, RenderingParameters, RenderFrameToScreen, ParameterSpace).
Needs /root/reference (the build container); skipped elsewhere."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "cppvolrend")),
                    reason="reference tree not present")
def test_adapters_type_check_against_reference_headers():
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "integration"), "syntax"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "hip_renderers.cpp" in p.stdout and "hip_renderer_base.cpp" in p.stdout
