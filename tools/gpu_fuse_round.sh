# GPU parity tests, prologue traces (gpurun_variants/wtrace), then fused-sampling A/B (run via gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pro_trace.sh || exit 1
for rep in 1 2; do
  for f in 0 1; do
    MPPI_FUSE_SAMPLE=$f timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/fuse$f.$rep.json 2> gpurun_out/ab/fuse$f.$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/fuse$f.$rep.json')); k=d['kernel_ms']; print('fuse=$f ms/update %.4f dyn %.4f cost %.4f' % (d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost']))"
  done
done
