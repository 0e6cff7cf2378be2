#!/usr/bin/env bash
# Round 3: C3 ms per step against the steps per bh_step call (K) at warm-up 5 -- the per-call
# cost (the call's last step is not pipelined: lastTree; compaction; status read-back).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/calls.txt
for k in 1 2 5 10 20 40; do
  timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu-baseline --no-verify > gpurun_out/calls_$k.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "K=$k rc=$rc"; tail -3 gpurun_out/calls_$k.log; exit $rc; }
  python3 - $k gpurun_out/calls_$k.log <<'PY' | tee -a gpurun_out/calls.txt
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("K", sys.argv[1], "ms_per_step", d["ms_per_step"], "phase_ms", d["phase_ms"])
PY
done
