#!/usr/bin/env bash
# Round 3, GPU session 4: the LET build with three launches folded into neighbours (default build):
# multi-rank / LET / RCCL tests and the digests, solo C4 / 8 rank 0 against libLF0 (before the
# folding), then C5 against libN2 (two bodies per lane in k_direct).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "let or rccl or group or rank or dist or digest" \
  --timeout 300 --timeout-method thread > gpurun_out/s4_pytest.log 2>&1
rc=$?; echo "pytest(let/rccl/group/digest) rc=$rc"; tail -2 gpurun_out/s4_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/s4_solo.jsonl
for r in 1 2; do for lib in LF0 bh_engine; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/s4_$lib.log 2>&1
  rc=$?; echo "solo lib=$lib rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s4_$lib.log; exit $rc; }
  grep '^{' gpurun_out/s4_$lib.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", /" | tee -a gpurun_out/s4_solo.jsonl | cut -c1-260
done; done
cp $L/libbh_engine.so $L/libB.so
LIBS="B N2" ROUNDS=2 AB_ARGS="--config c5 --steps 2 --warmup 1 --no-cpu-baseline" bash tools/ab.sh || exit 1
