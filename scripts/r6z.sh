set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sca_fold.py > $O/pytest_fold.log 2>&1 || { tail -30 $O/pytest_fold.log; exit 1; }
tail -1 $O/pytest_fold.log
ROUNDS=3 bash scripts/ab_env.sh r6z "-" "NBP_LIB=lowlight_image_enhancement_amd/_lib/ab/liblowlight_nbp.so"
