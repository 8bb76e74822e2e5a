#!/bin/bash
# round-3 session l: A/B of scheduler options on top of iterative-ilp
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="base licm bias0 ilpnosink" PP_SECONDS=0.05 AB_SECONDS=0.25 bash tools/ab.sh || exit 3
