#!/usr/bin/env bash
# Round 3, GPU session 5: full parity suite on the default build (the first traversal of the
# pipelined step writes the second build's Morton keys and bucket counts; k_direct with two
# bodies per lane), then C3 and C4 A/B against libK0 (BH_FUSE_KEYS=0) and a C3 kernel timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/s5_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s5_pytest.log; [ $rc -eq 0 ] || exit $rc
cp $L/libbh_engine.so $L/libB.so
LIBS="K0 B" ROUNDS=3 AB_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash tools/ab.sh || exit 1
LIBS="K0 B" ROUNDS=1 AB_ARGS="--config c4 --steps 6 --warmup 1 --no-cpu-baseline" bash tools/ab.sh || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl5_c3 -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tl5_c3.log 2>&1 || { echo "trace rc=$?"; exit 1; }
f=$(find gpurun_out/tl5_c3 -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$f" 3 gpurun_out/tl5_c3_step.txt | tail -4
