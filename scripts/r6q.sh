set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6q
mkdir -p $O
NBP_FFN_PF=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ffn_rows.py > $O/pytest_pf.log 2>&1 || { tail -30 $O/pytest_pf.log; exit 1; }
tail -1 $O/pytest_pf.log
for pf in 0 1; do
  NBP_FFN_PF=$pf timeout -k 10 200 python scripts/ffn_cold_micro.py > $O/cold_pf$pf.txt 2>&1 || { tail $O/cold_pf$pf.txt; exit 1; }
  echo "PF=$pf"; grep ffn $O/cold_pf$pf.txt
done
bash scripts/ab_env.sh r6q "-" "NBP_FFN_PF=1"
