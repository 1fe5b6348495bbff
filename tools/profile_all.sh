#!/bin/bash
# All round profiles in one GPU session (each step time-limited inside profile_round.sh).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/profile_round.sh rc1pass "--postpass" pmc && \
bash tools/profile_round.sh phong "--phong" && \
bash tools/profile_round.sh dos "--renderer dos" && \
bash tools/profile_round.sh ebs "--renderer ebs"
