"""Copy three SSIM known-answer pairs out of the reference (data files only) into
tests/golden/ssim/: data/iso without skipping/img/N.png vs data/4b skipping/img/N.png
and the SSIM values eval.py stored for them in ssim_comparison_results.xlsx
(read as XML; the xlsx is a zip).  Run in the container that has /root/reference."""
import json
import os
import re
import shutil
import zipfile

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ssim")
PICK = [0, 7, 196]


def xlsx_values(path):
    sheet = zipfile.ZipFile(path).read("xl/worksheets/sheet1.xml").decode()
    vals = {}
    for row in re.finditer(r"<row r=\"\d+\">(.*?)</row>", sheet):
        cells = re.findall(r"<c r=\"[AB]\d+\"[^>]*>(?:<is><t>([^<]*)</t></is>|<v>([^<]*)</v>)</c>",
                           row.group(1))
        if len(cells) == 2 and cells[0][0].endswith(".png"):
            vals[cells[0][0]] = float(cells[1][1])
    return vals


def main():
    os.makedirs(OUT, exist_ok=True)
    vals = xlsx_values(os.path.join(REF, "ssim_comparison_results.xlsx"))
    pairs = []
    for i in PICK:
        name = f"{i:04d}.png"
        a = os.path.join(OUT, f"noskip_{name}")
        b = os.path.join(OUT, f"skip4b_{name}")
        shutil.copyfile(os.path.join(REF, "data", "iso without skipping", "img", name), a)
        shutil.copyfile(os.path.join(REF, "data", "4b skipping", "img", name), b)
        pairs.append({"a": os.path.basename(a), "b": os.path.basename(b), "ssim": vals[name]})
    with open(os.path.join(OUT, "pairs.json"), "w") as f:
        json.dump({"source": "ssim_comparison_results.xlsx (eval.py, magick compare -metric SSIM)",
                   "pairs": pairs}, f, indent=1)


if __name__ == "__main__":
    main()
