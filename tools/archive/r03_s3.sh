#!/usr/bin/env bash
# Round 3, GPU session 3: full parity suite on the default build (chain kernels at wave priority 3,
# mailbox header cleared before the second traversal), C3 A/B against libP0 (BH_CHAIN_PRIO=0),
# a C3 kernel timeline of the default build.  Any failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  BH_ENGINE_LIB=$L/lib${TEST_LIB:-bh_engine}.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/s3_pytest.log 2>&1
  rc=$?; echo "pytest(${TEST_LIB:-bh_engine}) rc=$rc"; tail -3 gpurun_out/s3_pytest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "digest or pipelined" \
    --timeout 300 --timeout-method thread > gpurun_out/s3_pytest_def.log 2>&1
  rc=$?; echo "pytest(default, digests/pipelined) rc=$rc"; tail -2 gpurun_out/s3_pytest_def.log; [ $rc -eq 0 ] || exit $rc
fi
cp $L/libbh_engine.so $L/libB.so
LIBS="${AB_LIBS:-P0 B Q6 QL4 QW7}" ROUNDS=${ROUNDS:-3} AB_ARGS="${AB_ARGS:---steps 20 --warmup 5 --no-cpu-baseline}" bash tools/ab.sh || exit 1
if [ "${TRACE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  BH_ENGINE_LIB=$L/lib${TRACE_LIB:-Q6}.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl3_c3 -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tl3_c3.log 2>&1 || { echo "trace rc=$?"; exit 1; }
  f=$(find gpurun_out/tl3_c3 -name '*kernel_trace.csv' | head -1); echo "trace: $f"
  python3 tools/timeline.py "$f" 3 gpurun_out/tl3_c3_step.txt | tail -5
fi
