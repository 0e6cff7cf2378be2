#!/usr/bin/env bash
# Round 3, GPU session 8: a LET evaluation's rounds in one traversal launch (libOL: TravPieces,
# per-piece wave counters, k_round_wait on the comm stream) -- multi-rank parity tests, then one
# rank's share of C4 / 8 (solo) A/B against the default build with and without the emulated
# exchange, then a kernel trace of the emulated run.  Any failure stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/barnes-hut-n-body_amd/lib
T=${TEST_LIB:-OL}
BH_ENGINE_LIB=$L/lib$T.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  -k "let or multi_rank or group or dist or quads or rccl" --timeout 300 --timeout-method thread > gpurun_out/s8_pytest.log 2>&1
rc=$?; echo "pytest($T) rc=$rc"; tail -3 gpurun_out/s8_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/s8.jsonl
for r in 1 2; do for lib in bh_engine $T; do for x in 0 1; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 BH_SOLO_XCHG=$x timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/s8_$lib$x.log 2>&1
  rc=$?; echo "solo lib=$lib xchg=$x rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/s8_$lib$x.log; exit $rc; }
  grep '^{' gpurun_out/s8_$lib$x.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", \"xchg\": $x, /" | tee -a gpurun_out/s8.jsonl | cut -c1-260
done; done; done
export TMPDIR=/tmp
BH_ENGINE_LIB=$L/lib$T.so BH_LET=1 BH_SOLO_XCHG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s8_tl -o run --output-format csv \
  -- python3 tools/solo_rank.py --world 8 --rank 0 --steps 4 --warmup 1 --config c4 > gpurun_out/s8_tl.log 2>&1 \
  || { echo "trace rc=$?"; exit 1; }
f=$(find gpurun_out/s8_tl -name '*kernel_trace.csv' | head -1); echo "trace: $f"
python3 tools/timeline.py "$f" 2 gpurun_out/s8_tl_step.txt k_let_flags | tail -6
