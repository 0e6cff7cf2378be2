#!/usr/bin/env bash
# Pipelined-step session: GPU parity suite with the default library, then an A/B of the
# library built with -DBH_PIPELINE=0 (libA) against the default (libB) at C3 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/valu_rate > gpurun_out/valu_rate.txt 2>&1; echo "valu_rate rc=$?"; cat gpurun_out/valu_rate.txt
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pipe_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pipe_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
ROUNDS=3 AB_ARGS="--steps 20 --warmup 3 --no-cpu-baseline" LIBS="A B D" bash tools/ab.sh || exit 1
ROUNDS=2 AB_ARGS="--config c2 --steps 50 --warmup 5 --no-cpu-baseline" LIBS="A B D" bash tools/ab.sh || exit 1
ROUNDS=1 AB_ARGS="--config c4 --steps 6 --warmup 1 --no-cpu-baseline" LIBS="A D" bash tools/ab.sh || exit 1
for r in 1 2; do
  for L in B D; do
    BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/lib$L.so BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py \
      --world 8 --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/pipe_solo_$L$r.log 2>&1 || { echo "solo $L failed"; tail -5 gpurun_out/pipe_solo_$L$r.log; exit 1; }
    echo "solo $L$r $(grep '^{' gpurun_out/pipe_solo_$L$r.log | tail -1 | head -c 400)"
  done
done
