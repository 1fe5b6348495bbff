# round 6, session s25: PMC records of the current library (all five workloads)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_session.sh rc1pass phong longray dos ebs
