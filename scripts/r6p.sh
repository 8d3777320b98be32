set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ffn_rows.py > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert" $O/pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ffn_rows_micro.py 20 > $O/micro.txt 2>&1 || { tail $O/micro.txt; exit 1; }
cat $O/micro.txt
bash scripts/ab_env.sh r6p "-" "NBP_FFN_PRE=0"
