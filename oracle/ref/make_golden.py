"""Regenerate tests/golden/ref_vectors.json from the reference-built generator.

Runs here only (the reference tree is absent on the GPU box):
    make -C oracle/ref && python oracle/ref/make_golden.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_golden"),
                      os.path.join(REF, "data", "tf1dcp", "bonsai_01.tf1d"),
                      os.path.join(REF, "data", "#list_camera_states")],
                     check=True, capture_output=True, text=True).stdout
data = json.loads(out[out.index("{"):])
cones = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_cones")],
                       check=True, capture_output=True, text=True).stdout
data["cones"] = json.loads(cones[cones.index("{"):])
data["_generator"] = ("oracle/ref/ref_golden.cpp and ref_cones.cpp linked with the "
                      "reference's own sources")
with open(os.path.join(ROOT, "tests", "golden", "ref_vectors.json"), "w") as f:
    json.dump(data, f)
print("wrote tests/golden/ref_vectors.json:", sorted(data))
