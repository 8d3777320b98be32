set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6s2
mkdir -p $O
NBP_FFN_SPLIT=1 timeout -k 10 200 python scripts/ffn_cold_micro.py > $O/cold_split.txt 2>&1 || { tail $O/cold_split.txt; exit 1; }
timeout -k 10 200 python scripts/ffn_cold_micro.py > $O/cold_row.txt 2>&1 || { tail $O/cold_row.txt; exit 1; }
echo split; grep ffn $O/cold_split.txt; echo row; grep ffn $O/cold_row.txt
bash scripts/ab_env.sh r6s2 "-" "NBP_FFN_SPLIT=1"
