#!/bin/bash
# PMC passes over the bench (eager launches so every dispatch is attributed), kernel trace + stats only, each counter
# group in its own run (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):
#   fetch: FETCH_SIZE   write: WRITE_SIZE   mfma: SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_{F16,BF16,F32}
# Output under gpurun_out/pmc_<pass>/; scripts/pmc_traffic.py turns them into profiles/<name>_pmc_traffic.json.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PREC=${PREC:-fp16}
WL=${WORKLOAD:-cfg2}
SUF=${SUFFIX:-}
BENCH="python bench.py --steps 3 --warmup 1 --quick --eager --precision $PREC --workload $WL"
pass() {
  local name=$1
  shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace --stats -d gpurun_out/pmc_$name$SUF -o run --output-format csv \
      -- $BENCH > gpurun_out/pmc_$name$SUF.log 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32
ls gpurun_out/pmc_fetch$SUF gpurun_out/pmc_mfma$SUF | head
