mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_native.py "tests/test_gpu_parity.py::test_carried_tree_error_is_reported_by_the_call_that_uses_it" > gpurun_out/r05a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05a_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
TAG=r05a bash tools/session.sh bench || exit 1
for L in SS S0; do
  BH_ENGINE_LIB=$PWD/barnes-hut-n-body_amd/lib/lib$L.so timeout -k 10 300 python -u tools/solo_rank.py --config c4 --world 8 --rank 0 > gpurun_out/r05a_solo_$L.log 2>&1 || exit 1
  tail -2 gpurun_out/r05a_solo_$L.log | cut -c1-1500
done
TAG=r05a bash tools/session.sh soloab
