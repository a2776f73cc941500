# GPU parity tests, then bench A/B of an environment switch: ENV_AB="NAME" (values 0 / 1), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in 0 1; do
    env $ENV_AB=$f timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/env$f.$rep.json 2> gpurun_out/ab/env$f.$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/env$f.$rep.json')); k=d['kernel_ms']; b=k['breakdown_untimed']; print('$ENV_AB=$f ms/update %.4f rollout %.4f sample %.4f reduce %.4f' % (d['ms_per_step'], k['rollout_dynamics'], b['sample'], b['reduce']))"
  done
done
