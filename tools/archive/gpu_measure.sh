#!/usr/bin/env bash
# One GPU session that refreshes the committed measurements: default bench (C3, with the CPU
# baseline), C4 and C5 bench lines, rocprofv3 kernel trace + HBM counter passes for C3 and C5,
# SQ counter passes for C3.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_c3.log 2>&1 || { echo "bench c3 rc=$?"; exit 1; }
echo "bench c3 ok"; tail -1 gpurun_out/bench_c3.log | cut -c1-300
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { echo "bench c4 rc=$?"; exit 1; }
echo "bench c4 ok"
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1 || { echo "bench c5 rc=$?"; exit 1; }
echo "bench c5 ok"
CONFIG=c3 bash tools/profile.sh || exit 1
CONFIG=c5 STEPS=2 bash tools/profile.sh || exit 1
bash tools/profile_sq.sh || exit 1
