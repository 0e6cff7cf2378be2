#!/usr/bin/env bash
# rocprofv3 session on the GPU box: kernel trace + stats, then HBM counters in their own passes
# (FETCH_SIZE and WRITE_SIZE separately: TCC slots, MI355X_MICROARCH.md §rocprofv3 PMC slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${PROF_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok"; tail -1 $OUT/trace.log
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
  echo "fetch ok"
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
  echo "write ok"
fi
find $OUT -name "*.csv" | head -20
