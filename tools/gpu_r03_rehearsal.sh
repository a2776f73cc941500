#!/bin/bash
# The driver's round-end order on the shipped tree: smoke, the GPU suite (-x -q), the default bench.
set -o pipefail
O=gpurun_out/r03rh
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().split('\n')[-1]); print('bench ms/update %.4f value %.4e frac %.4f traffic %s cpu %.3e' % (d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value']))"
