#!/bin/bash
# Round 3: smoke + the whole GPU suite (one pytest process), then bench eager vs graph;
# logs under gpurun_out/r03t/.  Benches run only when pytest ended normally (rc 0 or 1).
set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03t/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/r03t/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r03t/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/r03t/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
[ -n "${SKIP_BENCH}" ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r03t/bench_eager.log 2>&1 || { echo "bench eager rc=$?"; tail -20 gpurun_out/r03t/bench_eager.log; exit 1; }
timeout -k 10 300 python -u bench.py --graph 1 > gpurun_out/r03t/bench_graph.log 2>&1 || { echo "bench graph rc=$?"; tail -20 gpurun_out/r03t/bench_graph.log; exit 1; }
tail -1 gpurun_out/r03t/bench_eager.log; tail -1 gpurun_out/r03t/bench_graph.log
exit $rc
