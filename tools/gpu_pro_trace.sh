# Per-wave kernel entry / loop start / end of the update launch (COOP_TRACE + PRO_TRACE build), fused and not.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wt
for f in 0 1; do
rm -f gpurun_out/wt/t$f.bin
MPPI_FUSE_SAMPLE=$f MPPI_WAVE_TRACE=$PWD/gpurun_out/wt/t$f.bin MPPI_AMD_LIB=$PWD/gpurun_variants/wtrace/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/wt/b$f.json 2> gpurun_out/wt/b$f.err || exit 1
echo "fuse=$f"; python3 tools/prologue_trace.py gpurun_out/wt/t$f.bin 1026
done
