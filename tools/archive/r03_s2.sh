#!/usr/bin/env bash
# Round 3, GPU session 2: (1) parity suite on the spill-path build (libS: BH_RS_CAP=1), (2) the
# digest / theta = 0 tests on the default build (resume stack + scalar-streamed k_direct_s),
# (3) C3 A/B against libA (BH_TRAV_STACK=0), (4) C5 A/B against libD (LDS-tiled k_direct),
# (5) a C3 kernel timeline of the default build.  Any failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
if [ "${SKIP_S:-0}" != 1 ]; then
  BH_ENGINE_LIB=$L/libS.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_S.log 2>&1
  rc=$?; echo "pytest(S) rc=$rc"; tail -3 gpurun_out/s2_pytest_S.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "digest or theta0 or c5 or direct" \
  --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_def.log 2>&1
rc=$?; echo "pytest(default, digests/theta0) rc=$rc"; tail -3 gpurun_out/s2_pytest_def.log; [ $rc -eq 0 ] || exit $rc
cp $L/libbh_engine.so $L/libB.so
LIBS="A B" ROUNDS=${ROUNDS:-3} AB_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash tools/ab.sh || exit 1
LIBS="D B" ROUNDS=2 AB_ARGS="--config c5 --steps 2 --warmup 1 --no-cpu-baseline" bash tools/ab.sh || exit 1
if [ "${TRACE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl_c3 -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tl_c3.log 2>&1 || { echo "trace rc=$?"; exit 1; }
  f=$(find gpurun_out/tl_c3 -name '*kernel_trace.csv' | head -1); echo "trace: $f"
  python3 tools/timeline.py "$f" 2 gpurun_out/tl_c3_step.txt | tail -12
fi
