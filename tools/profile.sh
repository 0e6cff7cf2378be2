#!/usr/bin/env bash
# rocprofv3 session on the GPU box: kernel trace + stats, then HBM counters in their own passes
# (FETCH_SIZE and WRITE_SIZE separately: TCC slots, MI355X_MICROARCH.md §rocprofv3 PMC slots).
# CONFIG=c3|c5|... selects the bench workload; output under gpurun_out/prof_<CONFIG>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c3}
OUT=gpurun_out/prof_$CONFIG
mkdir -p $OUT
STEPS=${STEPS:-10}
ARGS="--config $CONFIG --steps $STEPS --warmup 2 --no-cpu-baseline"
PMC_ARGS="--config $CONFIG --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok"; tail -1 $OUT/trace.log | cut -c1-400
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv \
    -- python3 bench.py $PMC_ARGS > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
  echo "fetch ok"
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv \
    -- python3 bench.py $PMC_ARGS > $OUT/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
  echo "write ok"
fi
