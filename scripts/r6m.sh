set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROUNDS=3 bash scripts/ab_env.sh r6m "-" "NBP_SCA_FOLD_L0=0"
