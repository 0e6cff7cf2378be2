#!/usr/bin/env bash
# Round 3, GPU session 10: libSF (span super list filled by k_cells instead of a memset launch;
# solo: the peers' exchange tables zeroed once) -- the full GPU suite on it, then one rank's
# share of C4 / 8 (solo) A/B against the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
T=${TEST_LIB:-SF}
BH_ENGINE_LIB=$L/lib$T.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/s10_pytest.log 2>&1
rc=$?; echo "pytest($T) rc=$rc"; tail -3 gpurun_out/s10_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/s10.jsonl
for r in 1 2; do for lib in bh_engine $T; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/s10_$lib.log 2>&1
  rc=$?; echo "solo lib=$lib rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s10_$lib.log; exit $rc; }
  grep '^{' gpurun_out/s10_$lib.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", /" | tee -a gpurun_out/s10.jsonl | cut -c1-260
done; done
