# round 6, session s24: checkpoint of the current library: full GPU suite, smoke, bench, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh all
