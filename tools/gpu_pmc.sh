# microbenchmark + PMC passes for the rollout kernel (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value tools/ubench.hip -o /tmp/ubench && \
timeout -k 10 120 /tmp/ubench > gpurun_out/ubench.txt 2>&1 && cat gpurun_out/ubench.txt && \
B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline" && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/pmc -o sq --output-format csv -- $B > gpurun_out/pmc/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc -o fetch --output-format csv -- $B > gpurun_out/pmc/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc -o write --output-format csv -- $B > gpurun_out/pmc/write.log 2>&1 && echo "pmc ok"
