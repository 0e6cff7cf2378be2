#!/usr/bin/env bash
# A/B of the pipelined step's stream priority: libA (no pipeline), libB (pipeline, default
# priority), libC (pipeline, highest priority = the default build) at C3, C2 and C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "pipelined or merge_rule or c3_1e6 or profiling" > gpurun_out/pipe2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pipe2_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 AB_ARGS="--steps 20 --warmup 3 --no-cpu-baseline" LIBS="A B C" bash tools/ab.sh || exit 1
ROUNDS=2 AB_ARGS="--config c4 --steps 6 --warmup 1 --no-cpu-baseline --no-counters" LIBS="A B C" bash tools/ab.sh || exit 1
ROUNDS=1 AB_ARGS="--config c2 --steps 50 --warmup 5 --no-cpu-baseline" LIBS="A B C" bash tools/ab.sh || exit 1
ROUNDS=2 AB_ARGS="--config c5 --steps 2 --warmup 1 --no-cpu-baseline" LIBS="C E" bash tools/ab.sh || exit 1
