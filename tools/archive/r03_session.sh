#!/usr/bin/env bash
# Round-3 GPU session: parity suite, smoke, the driver's bench command (C3, self-verified), one
# bench line per BASELINE configuration, and one rank's share of the 8-GPU C4 step (solo).
# Every GPU step has its own time limit; a crash / timeout (rc other than 0 or 1) stops the
# script before any further GPU step.  Output: gpurun_out/r03_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
stop_if_bad() {  # $1 = rc, $2 = step name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (rc=$1)"; exit "$1"; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; stop_if_bad $rc pytest
  [ $rc -eq 0 ] || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; stop_if_bad $rc smoke
fi
: > gpurun_out/${TAG}_bench_lines.jsonl
for spec in ${BENCH_SPECS:-"c3:20:5" "c1_baseline:100:5" "c1_code:50:5" "c2:50:5" "c4:10:2" "c5:3:1"}; do
  cfg=${spec%%:*}; rest=${spec#*:}; steps=${rest%%:*}; warm=${rest#*:}
  timeout -k 10 600 python -u bench.py --gpus 1 --config $cfg --steps $steps --warmup $warm \
    > gpurun_out/${TAG}_bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; stop_if_bad $rc "bench $cfg"
  grep '^{' gpurun_out/${TAG}_bench_$cfg.log | tail -1 >> gpurun_out/${TAG}_bench_lines.jsonl
  python - "$cfg" <<'EOF' || true
import json, sys
d = json.loads(open("gpurun_out/" + __import__("os").environ.get("TAG", "r03") + "_bench_lines.jsonl").read().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], d["value"], d["ms_per_step"], "kernel", r["kernel_ms"], "frac", r["frac"],
      "verify", (d.get("verify") or {}).get("digest_match"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
EOF
done
if [ "${SKIP_SOLO:-0}" != 1 ]; then
  : > gpurun_out/${TAG}_solo.jsonl
  for rank in ${SOLO_RANKS:-0 5}; do
    BH_LET=1 timeout -k 10 300 python3 tools/solo_rank.py --world 8 --rank $rank --steps 10 \
      --warmup 2 --config c4 > gpurun_out/${TAG}_solo_$rank.log 2>&1
    rc=$?; echo "solo rank=$rank rc=$rc"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_solo_$rank.log; exit $rc; }
    grep '^{' gpurun_out/${TAG}_solo_$rank.log | tail -1 | tee -a gpurun_out/${TAG}_solo.jsonl
  done
fi
