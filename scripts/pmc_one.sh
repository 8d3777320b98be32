#!/bin/bash
# One PMC pass over the quick eager bench (kernel trace + stats only): bash scripts/pmc_one.sh <name> <counters...>
# Env is passed through (A/B knobs).  Output: gpurun_out/pmc1_<name>/
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
name=$1
shift
timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace --stats -d gpurun_out/pmc1_$name -o run --output-format csv \
    -- python bench.py --steps 2 --warmup 1 --quick --eager > gpurun_out/pmc1_$name.log 2>&1
