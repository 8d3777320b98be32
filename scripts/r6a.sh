# round-6 session a: the new GPU tests, the level-0/1 tile micro at backward tile heights 16 / 32, quick bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_gpu.py tests/test_gpu_fp16_grads.py tests/test_gpu_c1dw_tile.py tests/test_gpu_wgrad_full.py -s > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for th in 16 32 16 32; do
  NBP_C1DW_BWD_TH=$th timeout -k 10 200 python scripts/c1dw_tile_micro.py 20 > $O/micro_th$th.txt 2>&1 || exit $?
  grep -E "bwd_new|C32|C64" $O/micro_th$th.txt
done
timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 > $O/bench.json 2> $O/bench_stderr.txt
rc=$?
tail -c 300 $O/bench.json
exit $rc
