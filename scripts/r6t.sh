set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
NBP_WG_SIDE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ffn_rows.py tests/test_gpu_fp16_grads.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_env.sh r6t "-" "NBP_WG_SIDE=1"
