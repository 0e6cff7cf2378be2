#!/usr/bin/env bash
# Kernel breakdown of one GPU's share of the 8-GPU C4 step (bh_create_solo), LET vs replicated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for let in ${LETS:-1 0}; do
  BH_LET=$let timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/soloprof$let -o run \
    --output-format csv -- python3 tools/solo_rank.py --world 8 --rank 0 --steps 10 --warmup 2 \
    > gpurun_out/soloprof$let.log 2>&1
  rc=$?; echo "solo prof BH_LET=$let rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/soloprof$let.log | tail -1
done
