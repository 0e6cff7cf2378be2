#!/usr/bin/env bash
# LET parity tests, then one rank's share of the C4 step at world 8 (bh_create_solo) for several
# round-size weightings (BH_ROUND_FRACS).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LET_PROF=0 bash tools/let_gpu.sh || exit $?
: > gpurun_out/round_sweep.jsonl
for F in "1,1,1,1" "35,35,15,15" "40,40,10,10" "30,30,20,20" "45,45,5,5"; do
  BH_LET=1 BH_ROUND_FRACS=$F timeout -k 10 300 python3 tools/solo_rank.py --world 8 --rank 0 \
    --steps 10 --warmup 2 > gpurun_out/sweep.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/sweep.log; exit $rc; }
  echo "$F $(grep '^{' gpurun_out/sweep.log | tail -1)" | tee -a gpurun_out/round_sweep.jsonl | cut -c1-220
done
