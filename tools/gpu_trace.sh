# per-block timing of the rollout kernel (COOP_TRACE variant; run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace
for s in ${SWEEP:-2046 4094}; do
  rm -f gpurun_out/trace/s$s.bin
  MPPI_WAVE_TRACE=$PWD/gpurun_out/trace/s$s.bin MPPI_AMD_LIB=$PWD/gpurun_variants/trace/libmppi_amd.so \
    timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --samples-per-gpu $s > gpurun_out/trace/s$s.json 2>&1 || exit 1
  echo "== samples $s"
  python3 tools/wave_trace.py gpurun_out/trace/s$s.bin $(( (s + 2) / 4 + 2 ))
done
