#!/usr/bin/env bash
# Traversal timing diagnosis on one GPU box: the driver's exact bench arguments, then the same
# with a longer warmup and a longer timed region, each printing per-launch kernel min/median/max
# and the GPU clock sampled during the timed region.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/diag_$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/diag_$tag.log; exit 1; }
  python - "$tag" gpurun_out/diag_$tag.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line); r = d["roofline"]
print(sys.argv[1], d["ms_per_step"], r["kernel_ms"], r.get("gpu_clock"), d["phase_ms"], r.get("achieved"), r.get("lane_efficiency"), r.get("contrib_per_body_eval"))
PY
}
run driver --gpus 1 --steps 20 --warmup 5 ${EXTRA:-}
run warm50 --gpus 1 --steps 20 --warmup 50 --no-cpu-baseline
run long --gpus 1 --steps 200 --warmup 5 --no-cpu-baseline
run driver2 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
