# GPU parity tests, then A/B bench lines and kernel traces of gpurun_variants/* (run via gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_run.sh || exit 1
bash tools/ab_prof.sh
