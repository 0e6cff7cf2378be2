#!/usr/bin/env bash
# One GPU's share of the 8-GPU north-star step (C4), measured alone: LET vs replicated builds,
# ranks 0 and 5.  Each run has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/solo.jsonl
for let in 1 0; do
  for rank in 0 5; do
    BH_LET=$let timeout -k 10 300 python3 tools/solo_rank.py --world ${WORLD:-8} --rank $rank \
      --steps 10 --warmup 2 --config ${CONFIG:-c4} > gpurun_out/solo_$let$rank.log 2>&1
    rc=$?; echo "solo BH_LET=$let rank=$rank rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/solo_$let$rank.log; exit $rc; }
    grep '^{' gpurun_out/solo_$let$rank.log | tail -1 | tee -a gpurun_out/solo.jsonl
  done
done
