#!/usr/bin/env bash
# kd wave groups (lib A) against Hilbert runs (lib B): multi-rank parity with A, then C3 and C4
# bench A/B, then one rank's share of the 8-GPU C4 step for both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "let_ or multi_rank or digest or massless" > gpurun_out/r03_kd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03_kd_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 AB_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash tools/ab.sh || exit 1
ROUNDS=2 AB_ARGS="--config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-verify" bash tools/ab.sh || exit 1
for L in A B; do
  BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/lib$L.so BH_LET=1 timeout -k 10 200 python3 \
    tools/solo_rank.py --world 8 --rank 0 --steps 10 --warmup 2 --config c4 \
    > gpurun_out/r03_kd_solo.log 2>&1 || { tail -3 gpurun_out/r03_kd_solo.log; exit 1; }
  echo "solo $L $(grep '^{' gpurun_out/r03_kd_solo.log | tail -1)"
done
