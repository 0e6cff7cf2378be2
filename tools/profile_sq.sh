#!/usr/bin/env bash
# SQ counter passes for the traversal kernel (VALU busy, waits) + the counter list.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_sq
mkdir -p $OUT
# CONFIG=c2 etc. for another workload; SQ_CACHE=1 adds a pass of scalar-cache and L2 hit counters
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
ARGS="--config ${CONFIG:-c3} --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES" \
           ${SQ_CACHE:+"SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ TCC_HIT TCC_MISS"} ; do
  i=$((i+1))
  timeout -s KILL 600 rocprofv3 --pmc $SET --kernel-trace -d $OUT/p$i -o run --output-format csv \
    -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
