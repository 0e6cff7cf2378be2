#!/usr/bin/env bash
# The GPU session runner: every measurement and test step of a gpurun call, by name, in order.
#
#   TAG=r04b bash tools/session.sh STEP [STEP ...]
#
# Steps (outputs under gpurun_out/, prefixed with $TAG):
#   tests          python -m pytest tests -m gpu (PYTEST_K="expr" narrows it)  -> ${TAG}_pytest.log
#   smoke          __graft_entry__.smoke()                                     -> ${TAG}_smoke.log
#   bench          the driver's command: bench.py --steps 20 --warmup 5        -> ${TAG}_bench_lines.jsonl
#   configs        one bench line per BASELINE configuration (c1_baseline, c1_code, c2, c4, c5)
#   profile        rocprofv3 kernel trace + stats and FETCH_SIZE / WRITE_SIZE passes of C3
#                  (tools/profile.sh; CONFIG=c5 etc. for another workload) -> prof_<CONFIG>/
#   sq             SQ counters of the traversal (tools/profile_sq.sh; CONFIG=c2 etc., SQ_CACHE=1 adds
#                  scalar-cache and L2 hit counters)
#   timed          the C3 bench's timed call alone: kernel trace, FETCH / WRITE passes, summarised
#                  over that call only (tools/timed_window.py)               -> ${TAG}_c3_timed*
#   timeline       one C3 bench under a kernel trace, summarised per step (tools/timeline.py)
#   dropin         the front-end's one-step calls under a kernel + copy trace (tools/dropin_calls.py,
#                  summarised by tools/timeline.py)                             -> ${TAG}_dropin_*
#   solo           one rank's share of the 8-GPU C4 step, alone (tools/solo_rank.py, ranks 0, 5)
#   soloprof       the solo rank-0 step under rocprofv3 --kernel-trace --stats -> ${TAG}_soloprof/
#   soloab         the solo step of rank 0 (C4 / 8) alternately with lib/libA.so and the default
#                  build (SOLO_LIBS="A default" to change), 2 rounds          -> ${TAG}_soloab.jsonl
#   ab             A/B of in-tree library builds (tools/ab.sh; LIBS="A B", AB_ARGS=...)
#   kstats         C3 bench under rocprofv3 --kernel-trace --stats per library (KSTATS_LIBS)
#   rehearse       bench.py --gpus 2 --single-process --devices 0,0 (the watchdog parent + child)
#   envab          A/B of environment settings (ENVS="X=0 X=1", AB_ARGS, ROUNDS) -> ${TAG}_envab.jsonl
# Every GPU step runs under its own time limit; a failing step (any rc but 0) ends the session, so
# nothing else touches the GPU after a fault, an abort or a timeout.
# (Older one-off session scripts are kept in tools/archive/: committed profiles cite them; see tools/README.md.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-s}
O=gpurun_out/$TAG
run() {  # $1 = seconds, $2 = log, rest = command
  local t=$1 log=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$TAG] $* -> rc=$rc"
  tail -3 "$log" | cut -c1-600
  [ $rc -eq 0 ] || { echo "[$TAG] STOP (rc=$rc)"; exit $rc; }
}
bench_line() {  # bench.py args... -> one JSON line appended to ${O}_bench_lines.jsonl
  run 600 ${O}_bench.log python -u bench.py "$@"
  grep '^{' ${O}_bench.log | tail -1 >> ${O}_bench_lines.jsonl
}
for step in "$@"; do
  case $step in
    tests)
      run ${PYTEST_TIMEOUT:-1200} ${O}_pytest.log python -u -m pytest tests -m gpu -x -v \
        --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke) run 300 ${O}_smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) bench_line --steps 20 --warmup 5 ;;
    configs)
      for c in c1_baseline c1_code c2 c4; do bench_line --config $c --steps 10 --warmup 2; done
      bench_line --config c5 --steps 2 --warmup 1 ;;
    profile) run 1800 ${O}_profile.log bash tools/profile.sh ;;
    sq)
      run 900 ${O}_sq.log bash tools/profile_sq.sh
      run 120 ${O}_sq_sum.log python3 tools/summarize_sq.py gpurun_out/prof_sq ${O}_${CONFIG:-c3}
      rm -rf gpurun_out/prof_sq/p* ;;  # (raw counter files: gpurun_out travels back only under 64 MiB)
    timed)  # the driver's C3 call alone under rocprofv3 (no drop-in / counter / verify legs):
            # kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes, summarised over the timed
            # call's window only (tools/timed_window.py)                    -> ${TAG}_c3_timed*
      export TMPDIR=/tmp
      TA="--no-cpu-baseline --no-counters --no-drop-in --no-verify"
      run 600 ${O}_timed_trace.log rocprofv3 --kernel-trace --stats -d ${O}_timed_trace -o run \
        --output-format csv -- python3 bench.py --steps 20 --warmup 5 $TA
      grep '^{' ${O}_timed_trace.log | tail -1 >> ${O}_bench_lines.jsonl
      run 300 ${O}_timed_fetch.log timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace \
        -d ${O}_timed_fetch -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 $TA
      run 300 ${O}_timed_write.log timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace \
        -d ${O}_timed_write -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 $TA
      run 120 ${O}_timed_sum.log python3 tools/timed_window.py ${O}_timed_trace 40 ${O}_c3 \
        ${O}_timed_fetch ${O}_timed_write 8
      cp "$(find ${O}_timed_trace -name '*kernel_stats.csv' | head -1)" ${O}_c3_timed_kernel_stats.csv
      rm -rf ${O}_timed_trace ${O}_timed_fetch ${O}_timed_write ;;  # (raw traces: see sq)
    timeline)  # CONFIG=c2 etc. for another workload -> ${TAG}_${CONFIG}_timeline.txt
      export TMPDIR=/tmp
      C=${CONFIG:-c3}
      run 600 ${O}_timeline.log rocprofv3 --kernel-trace -d ${O}_tl_$C -o run --output-format csv \
        -- python3 bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --no-counters --no-drop-in --no-verify
      grep '^{' ${O}_timeline.log | tail -1 >> ${O}_bench_lines.jsonl
      kt=$(find ${O}_tl_$C -name '*kernel_trace.csv' | head -1)
      python3 tools/timeline.py "$kt" 2 ${O}_${C}_timeline.txt > /dev/null
      tail -3 ${O}_${C}_timeline.txt
      rm -rf ${O}_tl_$C ;;
    dropin)
      export TMPDIR=/tmp
      run 600 ${O}_dropin.log rocprofv3 --kernel-trace --memory-copy-trace -d ${O}_dropin_trace \
        -o run --output-format csv -- python3 tools/dropin_calls.py
      kt=$(find ${O}_dropin_trace -name '*kernel_trace.csv' | head -1)
      python3 tools/timeline.py "$kt" 2 ${O}_dropin_timeline.txt > /dev/null
      tail -4 ${O}_dropin_timeline.txt ;;
    solo)
      for r in 0 5; do
        run 600 ${O}_solo$r.log python -u tools/solo_rank.py --config c4 --world 8 --rank $r
        grep '^{' ${O}_solo$r.log | tail -1 >> ${O}_solo.jsonl
      done ;;
    soloprof)  # rocprofv3 kernel trace + stats of the solo C4 / 8 rank-0 step (LET builds)
      export TMPDIR=/tmp
      run 600 ${O}_soloprof.log rocprofv3 --kernel-trace --stats -d ${O}_soloprof -o run \
        --output-format csv -- python3 tools/solo_rank.py --config c4 --world 8 --rank 0 \
        --steps 10 --warmup 2
      grep '^{' ${O}_soloprof.log | tail -1 >> ${O}_solo.jsonl
      cp "$(find ${O}_soloprof -name '*kernel_stats.csv' | head -1)" ${O}_solo_kernel_stats.csv ;;
    soloab)  # SOLO_LIBS="A B ..." (lib/lib<X>.so; "default" = the in-tree build)
      for rr in 1 2; do
        for L in ${SOLO_LIBS:-A default}; do
          lib=$PWD/barnes-hut-n-body_amd/lib/libbh_engine.so
          [ $L = default ] || lib=$PWD/barnes-hut-n-body_amd/lib/lib$L.so
          export BH_ENGINE_LIB=$lib
          run 600 ${O}_soloab_$L$rr.log python -u tools/solo_rank.py --config c4 --world 8 --rank 0
          unset BH_ENGINE_LIB
          echo "{\"lib\": \"$L\", \"line\": $(grep '^{' ${O}_soloab_$L$rr.log | tail -1)}" >> ${O}_soloab.jsonl
        done
      done ;;
    rehearse)  # the N > 1 launch path on one GPU: bench.py's watchdog parent, the
               # --single-process child over a repeated device (device-to-device copies)
      bench_line --gpus 2 --single-process --devices 0,0 --config c2 --steps 3 --warmup 1 \
        --no-cpu-baseline --no-single-gpu --no-verify ;;
    ab) run 1800 ${O}_ab.log bash tools/ab.sh ;;
    envab)  # A/B of environment settings with the in-tree library: ENVS="A=1 A=2" (one
            # assignment per label, or 'none'), AB_ARGS, ROUNDS -> ${TAG}_envab.jsonl
      for rr in $(seq 1 ${ROUNDS:-2}); do
        for E in ${ENVS:-none}; do
          if [ "$E" = none ]; then
            run 600 ${O}_envab.log python -u bench.py ${AB_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}
          else
            run 600 ${O}_envab.log env "$E" python -u bench.py ${AB_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}
          fi
          echo "{\"env\": \"$E\", \"line\": $(grep '^{' ${O}_envab.log | tail -1)}" >> ${O}_envab.jsonl
        done
      done ;;
    kstats)  # kernel-trace stats of C3 per library (KSTATS_LIBS="default X ..."; lib/lib<X>.so)
      export TMPDIR=/tmp
      for L in ${KSTATS_LIBS:-default}; do
        lib=$PWD/barnes-hut-n-body_amd/lib/libbh_engine.so
        [ $L = default ] || lib=$PWD/barnes-hut-n-body_amd/lib/lib$L.so
        export BH_ENGINE_LIB=$lib
        run 600 ${O}_kstats_$L.log rocprofv3 --kernel-trace --stats -d ${O}_kstats_$L -o run \
          --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
          --no-counters --no-drop-in
        unset BH_ENGINE_LIB
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
