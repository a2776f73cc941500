# The driver's order (run via gpurun): smoke, the GPU suite, then three bench runs back to back.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/at
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/at/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/at/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/at/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
    MPPI_HOST_TRACE=1 timeout -k 10 300 python bench.py > gpurun_out/at/bench.$rep.json 2> gpurun_out/at/bench.$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/at/bench.$rep.json')); print('ms/update %.4f dyn %.4f cpu %.3g' % (d['ms_per_step'], d['kernel_ms']['rollout_dynamics'], d['cpu_baseline']['value']))"
    tail -1 gpurun_out/at/bench.$rep.err
done
