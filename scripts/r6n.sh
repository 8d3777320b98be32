set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ffn_rows.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
NBP_FFN_NT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ffn_rows.py > $O/pytest_nt.log 2>&1 || { tail -30 $O/pytest_nt.log; exit 1; }
tail -2 $O/pytest_nt.log
for nt in 0 1; do
  NBP_FFN_NT=$nt timeout -k 10 200 python scripts/ffn_cold_micro.py > $O/cold_nt$nt.txt 2>&1 || { tail $O/cold_nt$nt.txt; exit 1; }
  echo "NT=$nt"; grep ffn $O/cold_nt$nt.txt
done
bash scripts/ab_env.sh r6n "-" "NBP_FFN_NT=1"
