# GPU parity tests + a short bench line (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/t/pytest_gpu.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/t/bench.json 2> gpurun_out/t/bench.err && cat gpurun_out/t/bench.json
