#!/usr/bin/env bash
# Round 3, GPU session 12: libSA (k_com_span loads span records three levels ahead instead of
# two) -- full GPU suite, then C3 and C4 A/B against the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
T=${TEST_LIB:-SA}
BH_ENGINE_LIB=$L/lib$T.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/s12_pytest.log 2>&1
rc=$?; echo "pytest($T) rc=$rc"; tail -3 gpurun_out/s12_pytest.log; [ $rc -eq 0 ] || exit $rc
cp $L/libbh_engine.so $L/libB.so
LIBS="B $T" ROUNDS=3 AB_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-verify" bash tools/ab.sh || exit 1
LIBS="B $T" ROUNDS=2 AB_ARGS="--config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-verify" bash tools/ab.sh || exit 1
