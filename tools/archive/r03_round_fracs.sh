#!/usr/bin/env bash
# Round 3: one rank's share of C4 / 8 (solo, rank 0) with the emulated exchange (BH_SOLO_XCHG=1)
# and without, for several round-size weights (BH_ROUND_FRACS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/fracs.txt
for r in 1 2; do for f in 1,1,1,1 3,3,2,2 4,4,3,1 2,2,2,1 1,1,1,2; do for x in 1 0; do
  BH_LET=1 BH_SOLO_XCHG=$x BH_ROUND_FRACS=$f timeout -k 10 300 python3 tools/solo_rank.py --world 8 --rank 0 \
    --steps 10 --warmup 2 --config c4 > gpurun_out/fr.log 2>&1 || { echo "fracs=$f rc=$?"; tail -3 gpurun_out/fr.log; exit 1; }
  python3 - "$f" "$x" gpurun_out/fr.log <<'PY' | tee -a gpurun_out/fracs.txt
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print("fracs", sys.argv[1], "xchg", sys.argv[2], "ms_per_step", d["ms_per_step"], d["phase_ms_per_step"])
PY
done; done; done
