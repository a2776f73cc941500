#!/bin/bash
# Wave traces of the rollout launch (COOP_TRACE + COST_TRACE build) with and without take_over.
set -o pipefail
mkdir -p gpurun_out/r03wt
for ho in 1 0; do
  rm -f gpurun_out/r03wt/t$ho.bin
  MPPI_HANDOVER=$ho MPPI_WAVE_TRACE=$PWD/gpurun_out/r03wt/t$ho.bin MPPI_AMD_LIB=$PWD/gpurun_variants/wtrace/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03wt/b$ho.json 2> gpurun_out/r03wt/b$ho.err || { echo "rc=$?"; tail gpurun_out/r03wt/b$ho.err; exit 1; }
  echo "== handover=$ho"; python3 tools/wave_trace_r03.py gpurun_out/r03wt/t$ho.bin 1026 relay || exit 1
done
