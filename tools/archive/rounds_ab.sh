set -u
cd "${GRAFT_REPO_ROOT:-.}"
for rr in 1 2; do
  for L in bh_engine R3 R2 R1; do
    for X in 0 1; do
      BH_SOLO_XCHG=$X BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/lib$L.so timeout -k 10 300 python -u tools/solo_rank.py --config c4 --world 8 --rank 0 > gpurun_out/r04w_$L$X$rr.log 2>&1 || { echo "fail $L $X"; exit 1; }
      echo "$L xchg=$X $(grep '^{' gpurun_out/r04w_$L$X$rr.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["phase_ms_per_step"])')"
    done
  done
done
