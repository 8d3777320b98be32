set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
ALT=lowlight_image_enhancement_amd/_lib/ab/liblowlight_nbp.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ffn_rows.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python scripts/ffn_cold_micro.py > $O/cold_d8.txt 2>&1 || exit 1
NBP_LIB=$ALT timeout -k 10 200 python scripts/ffn_cold_micro.py > $O/cold_d4.txt 2>&1 || exit 1
echo D8; grep ffn $O/cold_d8.txt; echo D4; grep ffn $O/cold_d4.txt
ROUNDS=3 bash scripts/ab_env.sh r6d "-" "NBP_LIB=$ALT"
