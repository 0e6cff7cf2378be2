#!/usr/bin/env bash
# Round 3: one rank's share of the C4 / 8 step alone (solo), with and without the emulated
# exchange (BH_SOLO_XCHG=1: each round's received bytes as device copies on the comm stream),
# then a kernel trace of the emulated run (when do the copies run against the rounds?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sx.jsonl
L=$PWD/barnes-hut-n-body_amd/lib
for r in 1 2; do for lib in bh_engine LQ; do for x in 0 1; do
  BH_ENGINE_LIB=$L/lib$lib.so BH_LET=1 BH_SOLO_XCHG=$x timeout -k 10 300 python3 tools/solo_rank.py --world 8 \
    --rank 0 --steps 10 --warmup 2 --config c4 > gpurun_out/sx_$lib$x.log 2>&1
  rc=$?; echo "solo lib=$lib xchg=$x rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sx_$lib$x.log; exit $rc; }
  grep '^{' gpurun_out/sx_$lib$x.log | tail -1 | sed "s/^{/{\"lib\": \"$lib\", \"xchg\": $x, /" | tee -a gpurun_out/sx.jsonl | cut -c1-300
done; done; done
if [ "${TRACE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  BH_ENGINE_LIB=$L/lib${TRACE_LIB:-bh_engine}.so BH_LET=1 BH_SOLO_XCHG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/sx_tl -o run --output-format csv \
    -- python3 tools/solo_rank.py --world 8 --rank 0 --steps 4 --warmup 1 --config c4 > gpurun_out/sx_tl.log 2>&1 \
    || { echo "trace rc=$?"; exit 1; }
  echo "trace ok"
fi
