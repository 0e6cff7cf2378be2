#!/usr/bin/env bash
# GPU box: parity tests on one candidate library build, then A/B timing (tools/ab.sh).
# TEST_LIB=<label> picks barnes-hut-n-body_amd/lib/lib<label>.so for the tests; LIBS, ROUNDS,
# AB_ARGS are passed to tools/ab.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=${TEST_LIB:-bh_engine}
BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/lib$L.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$L.log 2>&1
rc=$?; echo "pytest($L) rc=$rc"; tail -3 gpurun_out/pytest_$L.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab.sh
