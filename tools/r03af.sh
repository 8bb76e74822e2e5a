#!/bin/bash
# round-3 session af: compiler options for the tree kernel on top of the build.py flags
# (rpu: -amdgpu-enable-rewrite-partial-reg-uses; nopre: -amdgpu-enable-pre-ra-optimizations=false;
# norp: -misched-regpressure=false), config 4, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="base rpu nopre norp" AB_PP=0 AB_SECONDS=0.5 bash tools/ab.sh || exit 3
