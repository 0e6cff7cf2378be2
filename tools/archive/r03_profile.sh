#!/usr/bin/env bash
# Round-3 profile session: the GPU parity suite, then rocprofv3 kernel traces of the driver's C3
# bench command and of one rank's share of the 8-GPU C4 step (solo, LET builds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03p}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c3 -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > gpurun_out/${TAG}_c3.log 2>&1
rc=$?; echo "c3 prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/${TAG}_c3.log | tail -1 | cut -c1-300
BH_LET=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_solo -o run \
  --output-format csv -- python3 tools/solo_rank.py --world 8 --rank 0 --steps 10 --warmup 2 \
  > gpurun_out/${TAG}_solo.log 2>&1
rc=$?; echo "solo prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/${TAG}_solo.log | tail -1
