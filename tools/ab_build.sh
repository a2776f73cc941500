# Build kernel variants for A/B timing: tools/ab_build.sh name "-DFLAG ..." [name "-D..."]...
# Each lands in gpurun_variants/<name>/libmppi_amd.so (travels to the GPU box; run with MPPI_AMD_LIB).
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
    d=gpurun_variants/$1
    mkdir -p $d/obj
    make -s -C assistedmanipulation_amd/csrc OUT=../../$d OBJ=../../$d/obj EXTRA="$2" ARCH=gfx950
    shift 2
done
