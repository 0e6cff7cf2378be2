#!/usr/bin/env bash
# Round 3, GPU session 11: libMB (the merge mailbox header cleared on the overlapped stream while
# the second build runs, off the build -> traversal critical path) -- full GPU suite, C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
T=${TEST_LIB:-MB}
BH_ENGINE_LIB=$L/lib$T.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/s11_pytest.log 2>&1
rc=$?; echo "pytest($T) rc=$rc"; tail -3 gpurun_out/s11_pytest.log; [ $rc -eq 0 ] || exit $rc
cp $L/libbh_engine.so $L/libB.so
LIBS="B $T" ROUNDS=3 AB_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash tools/ab.sh || exit 1
