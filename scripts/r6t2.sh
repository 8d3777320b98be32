set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6t2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_reduce_bits.py tests/test_gpu_reduce_table.py tests/test_gpu_fp16_grads.py tests/test_dp_gpu.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ROUNDS=3 bash scripts/ab_env.sh r6t2 "-" "NBP_REDUCE_TABLE=0"
