#!/usr/bin/env bash
# One rank's share of the C4 step at world 2, 4, 8 (bh_create_solo), LET and replicated builds;
# then the 8-rank in-process kernel profile (tools/let_timing.py).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/solo_curve.jsonl
for w in 2 4 8; do
  for let in 1 0; do
    BH_LET=$let timeout -k 10 300 python3 tools/solo_rank.py --world $w --rank 0 --steps 10 \
      --warmup 2 --config c4 > gpurun_out/solo_w$w$let.log 2>&1
    rc=$?; echo "solo world=$w BH_LET=$let rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/solo_w$w$let.log; exit $rc; }
    grep '^{' gpurun_out/solo_w$w$let.log | tail -1 | tee -a gpurun_out/solo_curve.jsonl
  done
done
if [ "${PROFILE:-1}" = 1 ]; then LET_TESTS=0 bash tools/let_gpu.sh; fi
