#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, short bench.  Every GPU step has its own time
# limit; a crash/timeout (rc other than 0 or 1) stops the script before any further GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_bad() {  # $1 = rc, $2 = step name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (rc=$1)"; exit "$1"; fi
}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -x -q"}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_bad $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_if_bad $rc smoke
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
