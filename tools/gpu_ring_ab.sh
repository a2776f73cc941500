set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t2
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "event_ring or config3 or draws_ahead" --timeout 120 --timeout-method thread > gpurun_out/t2/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/t2/pytest.log; [ $rc -eq 0 ] && bash tools/gpu_ab_gaps.sh
