#!/usr/bin/env bash
# Round 3, GPU session 9: longest-first wave dispatch (libLP: BH_TRAV_LPT=1) for the LET rounds
# of one rank's share of C4 / 8 (solo) and for C3, A/B against the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
T=${TEST_LIB:-LP}
: > gpurun_out/s9.jsonl
for r in 1 2; do for lib in bh_engine $T; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/s9_$lib.log 2>&1
  rc=$?; echo "solo lib=$lib rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s9_$lib.log; exit $rc; }
  grep '^{' gpurun_out/s9_$lib.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", /" | tee -a gpurun_out/s9.jsonl | cut -c1-260
done; done
cp $L/libbh_engine.so $L/libB.so
LIBS="B $T" ROUNDS=2 AB_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash tools/ab.sh || exit 1
