#!/usr/bin/env bash
# Grid-size sweep of k_let_copy_blocks (libG<G>.so built by the caller with EXTRA=-DBH_LET_COPY_GRID=<G>):
# kernel traces of one rank of the 8-GPU C4 step alone (bh_create_solo, LET builds).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/gs
export TMPDIR=/tmp
for G in 2048 8192 32768; do
  BH_LET=1 BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/libG$G.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/gs/g$G -o run \
    --output-format csv -- python3 tools/solo_rank.py --world 8 --rank 0 --steps 10 --warmup 2 > gpurun_out/gs/g$G.log 2>&1 || { echo "G=$G rc=$?"; exit 1; }
  echo "G=$G ok"
done
