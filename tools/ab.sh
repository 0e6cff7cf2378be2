#!/usr/bin/env bash
# A/B timing on one GPU box: bench.py alternately against in-tree builds of the library
# (barnes-hut-n-body_amd/lib/lib<L>.so for L in $LIBS, default "A B", made by the caller),
# ROUNDS times each, so box-to-box clock differences cancel.  Prints one line per run:
# label ms_per_step kernel_ms phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3}
ARGS=${AB_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
for r in $(seq 1 $ROUNDS); do
  for L in ${LIBS:-A B}; do
    BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/lib$L.so timeout -k 10 300 python bench.py $ARGS \
      > gpurun_out/ab_$L$r.log 2>&1 || { echo "run $L$r failed"; tail -3 gpurun_out/ab_$L$r.log; exit 1; }
    python - "$L" gpurun_out/ab_$L$r.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]; di = d.get("drop_in") or {}
print(sys.argv[1], d["ms_per_step"], r.get("kernel_ms", {}).get("avg"), r.get("kernel_ms", {}).get("max"), d["phase_ms"],
      "drop_in", di.get("ms_per_step"), di.get("ms_per_step_with_get_bodies"), di.get("ms_per_step_with_mirror"),
      "verify", (d.get("verify") or {}).get("digest_match"))
PY
  done
done
