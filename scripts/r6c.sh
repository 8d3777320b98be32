# round-6 session c: tile backward micro (balanced MFMA split on / off), the tile tests, then quick-bench A/Bs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
for bal in 0 1 0 1; do
  NBP_C1DW_BWD_BAL=$bal timeout -k 10 200 python scripts/c1dw_tile_micro.py 20 > $O/micro_bal$bal.txt 2>&1 || exit $?
  echo "bal=$bal"; grep -E "bwd_new" $O/micro_bal$bal.txt
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c1dw_tile.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/ab_env.sh r6c "-" "NBP_LATE_FLUSH=1" "NBP_C1DW_BWD_BAL=0"
