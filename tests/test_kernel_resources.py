"""Per-kernel scratch of the built library, read from its gfx950 code objects (no GPU).

A device function the inliner leaves as a call takes its by-reference kernel
arguments from a copy in scratch: the DOS shader did so for filter_bits 8 (and after
small edits to its taps), ~1.9 KB per lane, and its frame ran ~7x slower (72 -> 11 ms,
DESIGN §6).  The guard: every kernel of libcvr.so keeps its private segment (register
spills included) at or below 128 B per lane.
"""
import os
import re
import subprocess

import pytest

from cpp_volume_rendering_amd import _native as N

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
MAX_PRIVATE = 128


def kernel_private_segments(lib, tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib,
                    os.path.join(tmp, "stripped")], check=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = {}
    for i, s in enumerate(starts):   # one offload bundle per translation unit
        piece = os.path.join(tmp, f"b{i}.bin")
        with open(piece, "wb") as f:
            f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(tmp, f"b{i}.o")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={piece}",
                        f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s*\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
            if m:
                out[name] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/clang-offload-bundler"), reason="no ROCm llvm tools")
def test_no_kernel_copies_its_arguments_to_scratch(tmp_path):
    lib = N.LIB_PATH
    if not os.path.exists(lib):
        pytest.skip("libcvr.so not built")
    seg = kernel_private_segments(lib, str(tmp_path))
    assert len(seg) > 100, "the library's kernels were not found"
    assert any("DosShaderTILi8" in k for k in seg), "the filter_bits 8 DOS kernels"
    big = {k: v for k, v in seg.items() if v > MAX_PRIVATE}
    assert not big, f"kernels with > {MAX_PRIVATE} B of scratch per lane: {big}"
