#!/bin/bash
# round-3 session w: A/B of the output filter's 16-entry window (filt) against the per-sample
# shift (base, -DAFS_OUTF_SHIFT) and the dense plan word loaded under a branch (br), hop records
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="${AB:-base filt br}" AB_PP=0 AB_SECONDS=${AB_SECONDS:-0.5} bash tools/ab.sh
