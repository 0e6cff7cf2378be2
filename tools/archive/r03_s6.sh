#!/usr/bin/env bash
# Round 3, GPU session 6: multi-rank engines end a call with a LET build (lastTree on demand from
# a position snapshot).  LET / group / RCCL / digest / quads tests on the default build, then solo
# C4 / 8 ranks 0 and 5 against libLZ0 (the call's last build full), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "let or rccl or group or rank or dist or digest or quads" \
  --timeout 300 --timeout-method thread > gpurun_out/s6_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s6_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/s6_solo.jsonl
for r in 1 2; do for rank in 0 5; do for lib in LZ0 bh_engine; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank $rank --steps 10 --warmup 2 --config c4 > gpurun_out/s6_$lib.log 2>&1
  rc=$?; echo "solo lib=$lib rank=$rank rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s6_$lib.log; exit $rc; }
  grep '^{' gpurun_out/s6_$lib.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", /" | tee -a gpurun_out/s6_solo.jsonl | cut -c1-230
done; done; done
