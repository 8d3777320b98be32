#!/bin/bash
# Two separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel trace + stats only,
# eager launches so every dispatch is attributed.  Output under gpurun_out/pmc_{fetch,write}/.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc_fetch -o run \
    --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmc_write -o run \
    --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/pmc_write.log 2>&1
ls -R gpurun_out/pmc_fetch | head -20
