#!/usr/bin/env bash
# End-of-round check: full GPU suite, smoke, driver bench, and the solo LET kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS="tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_check.sh || exit $?
LETS=1 bash tools/solo_prof.sh || exit $?
