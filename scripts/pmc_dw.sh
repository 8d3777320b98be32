#!/bin/bash
# SQ counter passes over the level-0 depthwise backward microbenchmark (scripts/dw_micro.py), one group per run.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
           "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --stats -d gpurun_out/pmc_dw$i -o run --output-format csv \
      -- python scripts/dw_micro.py > gpurun_out/pmc_dw$i.log 2>&1
done
python - <<'PY'
import csv, collections
for i in (1, 2, 3):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/pmc_dw{i}/run_counter_collection.csv")):
        if "dw_bwd_tiled" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
