#!/usr/bin/env python3
"""Turn a tools/pmc_round.sh summary into profiles/pmc_rc1pass.json, the HBM
traffic bench.py reports as roofline.traffic.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE
and WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts 128-B
requests at 64 B, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
Both come from the L2's fabric-side requests, so Infinity-Cache hits are
included: the figure is an upper bound of the bytes HBM served.
Usage: python tools/pmc_traffic.py gpurun_out/pmc/summary.json <workload_key> <out.json>"""
import json
import sys

summ = json.load(open(sys.argv[1]))
key, out = sys.argv[2], sys.argv[3]
fetch = summ["FETCH_SIZE"] * 1024 * 2
write = summ["WRITE_SIZE"] * 1024
res = {
    "workload_key": key,
    "hbm_bytes_per_launch": int(round(fetch + write)),
    "read_bytes_per_launch": int(round(fetch)),
    "write_bytes_per_launch": int(round(write)),
    "raw": {"FETCH_SIZE_KiB": summ["FETCH_SIZE"], "WRITE_SIZE_KiB": summ["WRITE_SIZE"]},
    "kernel_ns_avg_under_pmc": summ.get("_kernel_ns_avg"),
    "dispatches": summ.get("_dispatches_per_counter", {}).get("FETCH_SIZE"),
    "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
              "FETCH x2 (gfx950), KiB -> bytes",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
