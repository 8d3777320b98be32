set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sca_fold.py tests/test_gpu_c1dw_tile.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ROUNDS=3 bash scripts/ab_env.sh r6l "-" "NBP_LIB=lowlight_image_enhancement_amd/_lib/ab/liblowlight_nbp.so"
