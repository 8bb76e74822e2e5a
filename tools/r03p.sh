#!/bin/bash
# round-3 session p: tree kernel without the SLP vectorizer / without any vectorizer
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="base noslp novec" PP_SECONDS=0.05 AB_SECONDS=0.25 bash tools/ab.sh || exit 3
