#!/bin/bash
# SQ counters of a micro program's kernels (default: the level-0/1 tile kernels, scripts/c1dw_tile_micro.py; PROG
# overrides, e.g. PROG="scripts/wgrad_ring_check.py /tmp/w.pt"), one rocprofv3 pass per counter group, kernel trace +
# stats only.  Output: gpurun_out/<tag>/pmc_<pass>/ and a per-kernel summary (scripts/pmc_sq_summary.py).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc_tile}
mkdir -p $O
run() {
  local name=$1
  shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --stats -d $O/pmc_$name -o run --output-format csv \
      -- python ${PROG:-scripts/c1dw_tile_micro.py 2} > $O/pmc_$name.log 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
run b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA
run c FETCH_SIZE
python scripts/pmc_sq_summary.py $O
