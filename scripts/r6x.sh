set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sca_fold.py tests/test_gpu_c1dw_tile.py > $O/pytest_fold.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" $O/pytest_fold.log | tail -30; exit 1; }
grep -c PASSED $O/pytest_fold.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp16_grads.py tests/test_gpu_configs.py > $O/pytest_net.log 2>&1 || { tail -30 $O/pytest_net.log; exit 1; }
tail -1 $O/pytest_net.log
bash scripts/ab_env.sh r6x "-" "NBP_SCA_FOLD=0"
