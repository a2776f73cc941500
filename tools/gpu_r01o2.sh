# GPU parity tests, the bench line and its kernel-trace profile (run via gpurun from the repo root).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t2 gpurun_out/o2
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t2/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/t2/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/o2/smoke.log 2>&1 && tail -1 gpurun_out/o2/smoke.log || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/o2/bench.json 2> gpurun_out/o2/bench.err && cat gpurun_out/o2/bench.json || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/o2/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/o2/bench_prof.json 2> gpurun_out/o2/prof.err && echo prof ok
