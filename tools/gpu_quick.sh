# parity tests + bench (no CPU leg) + one SQ counter pass (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/q/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/q/pytest_gpu.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err && cat gpurun_out/q/bench.json && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/q -o sq --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/q/sq.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/q/sq_counter_collection.csv
