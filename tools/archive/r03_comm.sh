#!/usr/bin/env bash
# Round 3: all-gathers on a high-priority stream.  Multi-rank / RCCL / LET GPU tests on the default
# build, then solo C4 / 8 rank 0 with the emulated exchange (BH_SOLO_XCHG=1) against libC0
# (BH_COMM_PRIO=0), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "let or rccl or group or rank or dist" \
  --timeout 300 --timeout-method thread > gpurun_out/comm_pytest.log 2>&1
rc=$?; echo "pytest(let/rccl/group) rc=$rc"; tail -2 gpurun_out/comm_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/comm.jsonl
for r in 1 2; do for lib in C0 bh_engine; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 BH_SOLO_XCHG=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/comm_$lib.log 2>&1
  rc=$?; echo "solo lib=$lib rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/comm_$lib.log; exit $rc; }
  grep '^{' gpurun_out/comm_$lib.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", /" | tee -a gpurun_out/comm.jsonl | cut -c1-300
done; done
