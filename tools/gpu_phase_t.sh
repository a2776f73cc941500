# GPU parity tests, then phase traces + A/B (tools/gpu_phase.sh); run via gpurun
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/t/pytest_gpu.log; [ $rc -eq 0 ] && bash tools/gpu_phase.sh
