#!/usr/bin/env python3
"""One PMC record for bench.py's roofline (profiles/pmc_<renderer>.json) from a
tools/pmc_bench.sh summary and the bench line of the same workload.

  python tools/pmc_record.py gpurun_out/pmc_NAME/summary.json BENCH_LINE.json OUT.json

The record names the workload (workload_key), the dominant kernel and the library
build it was counted on (lib_sha16 = the first 16 hex digits of sha256(libcvr.so));
bench.py uses a record only when all three match the running bench, so counters of
an older kernel are never reported as the current one's.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE counts 128-B requests at 64 B,
so it is doubled.  Both are the L2's fabric-side requests (Infinity-Cache hits
included): an upper bound of the bytes HBM served.  busy = counter / 256 CUs /
(kernel ns x 2.4 GHz); VALU issue = SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / kernel
cycles (a wave64 VALU instruction issues over 2 cycles, the guide's constants table); VALU per sample = SQ_INSTS_VALU x 64 / samples; scratch estimate = write
bytes - the frame's algorithmic stores."""
import json
import sys

summ = json.load(open(sys.argv[1]))
bench = json.load(open(sys.argv[2]))
out = sys.argv[3]
roof = bench["roofline"]
ns = summ.get("_kernel_ns_avg")
cyc = ns * 2.4 if ns else None
fetch = summ["FETCH_SIZE"] * 1024 * 2 if "FETCH_SIZE" in summ else None
write = summ["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in summ else None
rec = {
    "workload_key": bench["config"]["workload_key"],
    "kernel": roof["kernel"],
    "lib_sha16": bench["config"]["lib_sha16"],
    "kernel_ns_avg_under_pmc": ns,
    "hbm_bytes_per_launch": int(round(fetch + write)) if fetch is not None and write is not None else None,
    "read_bytes_per_launch": int(round(fetch)) if fetch is not None else None,
    "write_bytes_per_launch": int(round(write)) if write is not None else None,
}
if "TCC_HIT_sum" in summ and "TCC_MISS_sum" in summ:
    rec["tcc_hit_rate"] = summ["TCC_HIT_sum"] / max(1.0, summ["TCC_HIT_sum"] + summ["TCC_MISS_sum"])
if cyc:
    for k, name in (("TA_TA_BUSY", "ta_busy_frac_per_cu"), ("TD_TD_BUSY", "td_busy_frac_per_cu")):
        if k in summ:
            rec[name] = summ[k] / 256.0 / cyc
    if "SQ_INSTS_VALU" in summ:
        rec["valu_wave_insts"] = summ["SQ_INSTS_VALU"]
        rec["valu_issue_frac_per_simd"] = summ["SQ_INSTS_VALU"] * 2.0 / 1024.0 / cyc
    if "SQ_WAIT_INST_ANY" in summ and "SQ_WAVE_CYCLES" in summ:
        rec["wait_any_over_wave_cycles"] = summ["SQ_WAIT_INST_ANY"] / max(1.0, summ["SQ_WAVE_CYCLES"])
samples = roof.get("samples_per_launch")
if "SQ_INSTS_VALU" in summ and samples and bench["metric"].startswith("Msamples/s (rays x steps), rc1pass"):
    rec["valu_per_sample"] = summ["SQ_INSTS_VALU"] * 64.0 / samples
for k in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES"):
    if k in summ:
        rec[k.lower()] = summ[k]
# the vector-memory pipe (DESIGN §5 "what a wave-load costs"): TD busy splits into
# cycles stalled on the cache (TD_TC_STALL: L1 misses in flight) and its own work;
# TCP accesses count (lane quad, 128-B line) pairs, 16 per coalesced dwordx4 wave-load
if cyc and "TD_TC_STALL" in summ:
    rec["td_tc_stall_frac_per_cu"] = summ["TD_TC_STALL"] / 256.0 / cyc
vm = summ.get("SQ_INSTS_VMEM_RD")
if vm:
    if "TD_TD_BUSY" in summ and "TD_TC_STALL" in summ:
        rec["td_work_cycles_per_wave_load"] = (summ["TD_TD_BUSY"] - summ["TD_TC_STALL"]) / vm
        rec["td_busy_cycles_per_wave_load"] = summ["TD_TD_BUSY"] / vm
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in summ:
        rec["tcp_accesses_per_wave_load"] = summ["TCP_TOTAL_CACHE_ACCESSES_sum"] / vm
    if "TCP_TCC_READ_REQ_sum" in summ:
        rec["l1_miss_requests_per_wave_load"] = summ["TCP_TCC_READ_REQ_sum"] / vm
if ns and "GRBM_GUI_ACTIVE" in summ:
    # the guide's effective clock: GRBM_GUI_ACTIVE summed over the 8 XCDs / kernel time
    rec["effective_clock_ghz_under_pmc"] = summ["GRBM_GUI_ACTIVE"] / 8.0 / ns
rec["frames_per_launch"] = bench["config"].get("frames_per_launch", 1)
rec["counters"] = {k: v for k, v in summ.items() if not k.startswith("_")}
rec["dispatches"] = summ.get("_dispatches_per_counter", {})
rec["method"] = ("rocprofv3 --kernel-trace --pmc, one pass per counter group (tools/pmc_bench.sh); "
                 "tools/pmc_summary.py averages the dominant kernel's dispatches; "
                 "tools/pmc_record.py (corrections in its docstring)")
rec["round"] = 5
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec, indent=1))
