#!/usr/bin/env bash
# Round-2 profile session on one GPU box: rocprofv3 kernel trace + stats of the driver's bench
# command (C3) and of C4; HBM counter passes (FETCH_SIZE, WRITE_SIZE separately) and SQ passes
# for C3.  Outputs under gpurun_out/prof_r02/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r02
mkdir -p $OUT
B="--no-cpu-baseline"
trace() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag/trace -o run --output-format csv \
    -- python3 bench.py "$@" > $OUT/$tag.log 2>&1 || { echo "$tag trace rc=$?"; tail -5 $OUT/$tag.log; exit 1; }
  echo "$tag trace ok"
}
trace c3 --steps 20 --warmup 5 $B
trace c4 --config c4 --steps 5 --warmup 1 $B
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/c3/$C -o run --output-format csv \
    -- python3 bench.py --steps 4 --warmup 1 $B > $OUT/c3_$C.log 2>&1 || { echo "$C rc=$?"; exit 1; }
  echo "$C ok"
done
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-trace -d $OUT/sq/p$i -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-counters $B > $OUT/sq_p$i.log 2>&1 || { echo "sq pass $i rc=$?"; exit 1; }
  echo "sq pass $i ok"
done
