#!/bin/bash
# round-3 session ad: the next sample's ratio computed at the end of the step (ahead, default)
# against the division at the top of each step (top); config 4 and config 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="top ahead" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="top ahead" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
AB="top ahead" AB_PP=0 AB_ARGS="--workload vcv --batch 8192" bash tools/ab.sh 2>&1 | sed 's/^/vcv /'
