set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6v
mkdir -p $O
NBP_C1DW_BWD_TH=64,32 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c1dw_tile.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for th in 32,32 64,32; do
  NBP_C1DW_BWD_TH=$th timeout -k 10 300 python scripts/c1dw_tile_micro.py 20 > $O/micro_$th.txt 2>&1 || { tail $O/micro_$th.txt; exit 1; }
  echo "TH=$th"; grep -v amdgpu.ids $O/micro_$th.txt
done
bash scripts/ab_env.sh r6v "-" "NBP_C1DW_BWD_TH=64,32"
