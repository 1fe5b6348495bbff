#!/usr/bin/env python3
"""VALU instructions of the headline ray-march loop by category, from the ISA
(DESIGN §5‴).

Compiles raymarch.hip for gfx950 with line tables (-gline-tables-only, the same
flags as the library otherwise), takes one rc1pass_tile_kernel instantiation
(default: the headline's K=4, EA, no macro skip, exact-range exp, buffer
addressing, exact weights, cell skip 3), finds its march loop (the innermost
region between the loop header label and the back-edge that spans the most
instructions) and attributes every instruction of the loop to the source line it
came from (.loc), then to a category by the function / line range of that source.
Prints JSON: per basic block, its instruction counts by category, and the totals.
Usage: python tools/isa_breakdown.py [--kernel SUBSTR] [--asm FILE] [--define X]"""
import argparse
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "cpp_volume_rendering_amd", "csrc")

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="rc1pass_tile_kernelILi4ELb0ELb0ELb0ELi1ELi2ELi0ELi3E")
ap.add_argument("--asm", default="")
ap.add_argument("--define", action="append", default=[])
a = ap.parse_args()

asm = a.asm
if not asm:
    asm = "/tmp/raymarch_isa.s"
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-ffp-contract=off", "--offload-arch=gfx950",
           "-gline-tables-only", "-x", "hip", os.path.join(CSRC, "raymarch.hip"), "--cuda-device-only",
           "-S", "-o", asm] + ["-D" + d for d in a.define]
    subprocess.run(cmd, check=True, cwd=CSRC, stderr=subprocess.DEVNULL)
lines = open(asm).read().split("\n")

files = {}
for ln in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
    if m:
        files[int(m.group(1))] = os.path.basename(m.group(3) or m.group(2))

# source function ranges: line -> enclosing function name
def func_ranges(fname):
    path = os.path.join(CSRC, fname)
    if not os.path.exists(path):
        return []
    out = []
    for i, l in enumerate(open(path).read().split("\n"), 1):
        m = re.match(r'^(?:template <[^>]*>\s*)?(?:__device__|__host__ __device__|__global__)[^(]*?\b(\w+)\s*\(', l)
        if m:
            out.append((i, m.group(1)))
    return out

franges = {f: func_ranges(f) for f in set(files.values())}

def func_at(fname, line):
    best = None
    for l0, n in franges.get(fname, []):
        if l0 <= line:
            best = n
    return best

# march_ray (raymarch.hip) line ranges -> categories, from markers in the source
_src = open(os.path.join(CSRC, "raymarch.hip")).read().split("\n")

def _find(pat, start=0):
    for i in range(start, len(_src)):
        if pat in _src[i]:
            return i + 1
    raise SystemExit(f"marker not found: {pat}")

L_MR = _find("void march_ray(")
L_LC = _find("auto load_cell", L_MR)
L_WH = _find("while (!done)", L_LC)
L_S1 = _find("// stage 1:", L_MR)
L_BOX = _find("if (wave_in_box) {", L_S1)
L_S2 = _find("// stage 2:", L_BOX)
L_VIS = _find("bool visible = false;", L_S2)
L_S3 = _find("// stage 3:", L_VIS)
L_RGB = _find("if (kAlphaFirst) {   // classify's rgb", L_S3)
L_X = _find("const float x = -(sc.w * hj[j]);", L_RGB)
L_OM = _find("const float om = 1.0f - dst.w;", L_X)
L_SS = _find("s = ss;", L_OM)
L_END = _find("// Value of `v` in lane L", L_SS)
MARCH_END = L_END

def march_cat(line):
    if L_S1 <= line < L_BOX:
        return "position: step recurrence (s, h, t)"
    if L_BOX <= line < L_S2:
        return "position: texel coordinates and cell address"
    if L_S2 <= line < L_VIS:
        return "classify: trilinear + TF alpha"
    if L_VIS <= line < L_S3:
        return "composite: exp of the batch (packed pairs)"
    if L_RGB <= line < L_X:
        return "composite: TF rgb (visible samples)"
    if L_X <= line < L_OM:
        return "composite: exp (per sample)"
    if L_OM <= line < L_SS:
        return "composite: blend + ERT"
    if L_S3 <= line < L_SS:
        return "composite: sample loop control"
    if L_SS <= line < L_END:
        return "loop control + distance skip"
    if L_LC <= line < L_WH:
        return "position: texel coordinates and cell address"
    if L_MR <= line < L_S1:
        return "loop head (skip probe, counters)"
    return "raymarch.hip other"

FUNC_CAT = {
    "sample_pos": "position: texel coordinates and cell address",
    "sample_pos_clamped": "position: texel coordinates and cell address",
    "mad_i24": "position: texel coordinates and cell address",
    "buffer_load_u4": "position: texel coordinates and cell address",
    "trilerp_cell": "classify: trilinear + TF alpha",
    "h2f": "classify: trilinear + TF alpha",
    "classify": "classify: trilinear + TF alpha",
    "filter_weight": "classify: trilinear + TF alpha",
    "lerpf": None,       # by its caller's line
    "cvt_flr": None,
    "cell_empty": "skip flags (cell_empty / cell_skip_q)",
    "cell_skip_q": "skip flags (cell_empty / cell_skip_q)",
}

k0 = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(a.kernel) + r"\S*:", l))
k1 = next(i for i in range(k0, len(lines)) if lines[i].strip().startswith("s_endpgm"))

# basic blocks with the compiler's loop annotations (".LBBx_y: ; in Loop: Header=BBx_z")
blocks = []
cur = (None, 0)
last_march = 0
for i in range(k0, k1 + 1):
    s_ = lines[i].strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s_)
    if m:
        f = files.get(int(m.group(1)), "?")
        cur = (f, int(m.group(2)))
        if f == "raymarch.hip" and L_MR <= cur[1] < MARCH_END:
            last_march = cur[1]
        continue
    m = re.match(r"^(\.LBB\w+):\s*(?:;(.*))?$", s_)
    if m:
        note = m.group(2) or ""
        hm = re.search(r"Header=BB(\w+)", note)
        pm = re.search(r"Parent Loop BB(\w+)", note)
        header = m.group(1) if "Loop Header" in note else None
        blocks.append({"name": m.group(1), "loop": ("BB" + hm.group(1)) if hm else None,
                       "parent": ("BB" + pm.group(1)) if pm else None, "header": header, "insts": []})
        continue
    if not blocks:
        blocks.append({"name": "entry", "loop": None, "parent": None, "header": None, "insts": []})
    if not s_ or s_.startswith((".", ";", "_Z")):
        continue
    blocks[-1]["insts"].append((s_, cur[0], cur[1], last_march))

def in_loop(b, hdr):
    return (b["name"].lstrip(".L") == hdr or b["loop"] == hdr or b["parent"] == hdr)

# the march loop: the outermost loop whose blocks hold the cell loads
hdrs = {b["name"].lstrip(".L") for b in blocks if b["header"]}
best = None
for h in hdrs:
    mem = [b for b in blocks if in_loop(b, h)]
    nl = sum("buffer_load_dwordx4" in x[0] for b in mem for x in b["insts"])
    if nl and (best is None or len(mem) > best[1]):
        best = (h, len(mem))
hdr = best[0]
loop_blocks = [b for b in blocks if in_loop(b, hdr)]

def category(f, line, lm):
    if f == "raymarch.hip":
        return march_cat(line)
    fn = func_at(f, line) if f else None
    c = FUNC_CAT.get(fn)
    if fn in FUNC_CAT and c is not None:
        return c
    if fn == "cvr_expf_neg2":
        return "composite: exp of the batch (packed pairs)"
    if fn and fn.startswith("cvr_expf"):
        return "composite: exp"
    return march_cat(lm) if lm else f"{f}:{fn}"

def kind(s_):
    op = s_.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"

out_blocks = []
tot = {}
bykind = {}
for b in loop_blocks:
    cats = {}
    for (s_, f, line, lm) in b["insts"]:
        k = kind(s_)
        bykind[k] = bykind.get(k, 0) + 1
        if k != "valu":
            continue
        c = category(f, line, lm)
        cats[c] = cats.get(c, 0) + 1
        tot[c] = tot.get(c, 0) + 1
    nv = sum(cats.values())
    if nv:
        out_blocks.append({"block": b["name"], "valu": nv,
                           "loads": sum("buffer_load_dwordx4" in x[0] for x in b["insts"]),
                           "by_category": dict(sorted(cats.items(), key=lambda kv: -kv[1]))})
res = {"kernel": a.kernel, "loop_header": hdr, "loop_blocks": len(loop_blocks), "by_kind": bykind,
       "valu_by_category_static": dict(sorted(tot.items(), key=lambda kv: -kv[1])),
       "blocks": out_blocks,
       "note": "static counts over the march loop's basic blocks (a batch of K samples; every "
               "branch side counted once, so the sum is not what a batch executes: per-block "
               "counts show which blocks each path runs)"}
print(json.dumps(res, indent=1))
