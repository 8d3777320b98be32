# full GPU suite + smoke (the driver's round-end commands), then the quick bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 > $O/bench.json 2> $O/bench_stderr.txt || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])"
