#!/bin/bash
# SQ / TCC counter passes over the middle-level grouped weight gradient (scripts/wgroup_micro.py), one group per run.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/${OUT:-pmc_wg}
mkdir -p $O
timeout -k 10 120 python scripts/wgroup_micro.py > $O/time.txt 2>&1
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  REPS=5 timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --stats -d $O/p$i -o run --output-format csv \
      -- python scripts/wgroup_micro.py > $O/p$i.log 2>&1
done
python - "$O" <<'PY'
import csv, collections, sys
O = sys.argv[1]
for i in range(1, 7):
    acc = collections.defaultdict(list)
    try:
        rows = list(csv.DictReader(open(f"{O}/p{i}/run_counter_collection.csv")))
    except OSError as e:
        print(i, e)
        continue
    for r in rows:
        if "wgrad_bf16_wide_group" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
