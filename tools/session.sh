# round 6, session s39: final library (with the DOS tolerance variant): PMC records, full GPU suite, smoke, bench, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_session.sh rc1pass phong longray dos ebs || exit 1
bash tools/gpu_round.sh all
