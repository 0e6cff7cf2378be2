#!/usr/bin/env bash
# LET tests (incl. the C4 8-rank digest) then the solo per-rank timing; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LET_PROF=0 bash tools/let_gpu.sh || exit $?
bash tools/solo_gpu.sh || exit $?
