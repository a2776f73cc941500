set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wt
rm -f gpurun_out/wt/t.bin
MPPI_WAVE_TRACE=$PWD/gpurun_out/wt/t.bin MPPI_AMD_LIB=$PWD/gpurun_variants/wtrace/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/wt/b.json 2> gpurun_out/wt/b.err || exit 1
python3 tools/wave_trace.py gpurun_out/wt/t.bin 1026
