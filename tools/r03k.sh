#!/bin/bash
# round-3 session k: A/B of scheduler options for the tree kernel (phase profile + 0.25 s bench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="base ilp minreg postra nocluster nosink" PP_SECONDS=0.05 AB_SECONDS=0.25 bash tools/ab.sh || exit 3
