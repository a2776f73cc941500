# GPU parity tests, then a kernel trace of the bench on the in-tree library (run via gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/tp/bench.json 2> gpurun_out/tp/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/tp/bench.json')); k=d['kernel_ms']; print('ms/update %.4f dyn %.4f cost %.4f' % (d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/tp/traced.json 2> gpurun_out/tp/trace.err || exit 1
python3 tools/trace_gaps.py gpurun_out/tp/trace/run_kernel_trace.csv tp
