# overlap probe: frames in flight vs quad share, per-GPU work of an N-way split
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 8 4 2 1; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 tools/overlap_probe.py --nranks $n --quads 0,10 --streams 3,4,5 --frames 48 2>/dev/null | grep nranks || exit 1
done
