# GPU parity tests (objective in the launch), the cost-kernel path's tests, then A/B of MPPI_COSTS_IN_LAUNCH.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
MPPI_COSTS_IN_LAUNCH=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu0.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu0.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in 0 1; do
    MPPI_COSTS_IN_LAUNCH=$f timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/cil$f.$rep.json 2> gpurun_out/ab/cil$f.$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/cil$f.$rep.json')); k=d['kernel_ms']; print('in_launch=$f ms/update %.4f rollout %.4f cost %.4f frac %.4f' % (d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost'], d['roofline']['frac']))"
  done
done
