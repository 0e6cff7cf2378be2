#!/usr/bin/env bash
# Round 3, GPU session 7: the multi-rank parity tests on libLF (LET cell starts + table in one
# launch, top records + cell records in one launch, k_let_top_hi with 8 ranks' loads in flight),
# then one rank's share of C4 / 8 (solo) A/B against the default build.  Any failure stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
BH_ENGINE_LIB=$L/lib${TEST_LIB:-LF}.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  -k "let or multi_rank or group or dist or quads" --timeout 300 --timeout-method thread > gpurun_out/s7_pytest.log 2>&1
rc=$?; echo "pytest(${TEST_LIB:-LF}) rc=$rc"; tail -3 gpurun_out/s7_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/s7.jsonl
for r in 1 2; do for lib in bh_engine ${TEST_LIB:-LF}; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/s7_$lib.log 2>&1
  rc=$?; echo "solo lib=$lib rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s7_$lib.log; exit $rc; }
  grep '^{' gpurun_out/s7_$lib.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", /" | tee -a gpurun_out/s7.jsonl | cut -c1-300
done; done
