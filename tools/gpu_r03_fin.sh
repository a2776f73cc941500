set -o pipefail
mkdir -p gpurun_out/t1
timeout -k 10 600 python -u -m pytest tests/test_gpu_launch_paths.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t1/pytest.log 2>&1 || { tail -40 gpurun_out/t1/pytest.log; exit 1; }
tail -3 gpurun_out/t1/pytest.log
bash tools/gpu_ab3.sh
