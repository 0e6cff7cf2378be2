#!/usr/bin/env bash
# LET (sharded multi-rank build) session: parity tests, then per-rank build cost LET vs
# replicated under rocprofv3 (C4 on 8 in-process ranks).  Each GPU step has its own limit; a
# failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${LET_TESTS:-1}" = "1" ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_digests.py -k "${LET_K:-let_ or multi_rank or rccl or eight_rank}" \
  > gpurun_out/let_tests.log 2>&1
rc=$?; echo "let tests rc=$rc"; tail -15 gpurun_out/let_tests.log
[ $rc -eq 0 ] || exit $rc
fi
[ "${LET_PROF:-1}" = "1" ] || exit 0
for mode in 1 0; do
  BH_LET=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/letprof$mode -o run --output-format csv \
    -- python3 tools/let_timing.py --world 8 --steps 5 > gpurun_out/let_timing$mode.log 2>&1
  rc=$?; echo "let timing BH_LET=$mode rc=$rc"; tail -2 gpurun_out/let_timing$mode.log
  [ $rc -eq 0 ] || exit $rc
  python3 tools/let_timing.py --summarize "$(ls gpurun_out/letprof$mode/*kernel_stats.csv | head -n 1)" \
    --world 8 --builds 12 > gpurun_out/let_summary$mode.json || exit 1
  head -8 gpurun_out/let_summary$mode.json
done
exit 0
