# round 6, session s12: the paired exp -- bit-exact suites, A/B against the scalar-exp
# build (ablib/nopair, -DCVR_NO_PAIR_EXP), PMC VALU count
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s13; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_frames_gpu.py tests/test_tolerance_gpu.py "tests/test_fullsize_gpu.py::test_c2_raw_256_at_1024" "tests/test_fullsize_gpu.py::test_c3_phong_fd_512_at_1024" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  CVR_LIB_OVERRIDE=ablib/nopair/libcvr.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_nopair_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_pair2_$i.json 2>/dev/null || exit 1
done
export TMPDIR=/tmp
PMC_STEPS=8 timeout -k 10 300 bash tools/pmc_bench.sh pair2 rc1pass_tile_kernel "--streams 1 --no-cadence" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY;GRBM_GUI_ACTIVE GRBM_COUNT" > $O/pmc_pair2.log 2>&1 || exit 1
