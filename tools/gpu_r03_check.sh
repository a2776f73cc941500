#!/bin/bash
# Checkpoint: smoke, the whole GPU suite, one default bench line (with the CPU baselines).
set -o pipefail
mkdir -p gpurun_out/r03chk
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03chk/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/r03chk/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/r03chk/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03chk/pytest.log | tail -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r03chk/bench.json 2> gpurun_out/r03chk/bench.err || { echo "bench rc=$?"; tail gpurun_out/r03chk/bench.err; exit 1; }
tail -c 400 gpurun_out/r03chk/bench.json
exit $rc
