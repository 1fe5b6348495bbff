# round 6, session s45: the final tree: full GPU suite, smoke, the driver's bench command, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh all
