#!/bin/bash
# A/B: weights_gradient_kernel with its control components split over blockIdx.z (GRAD_CSPLIT
# 2 / 3 / 4 builds in gpurun_variants/cs*) against the default, interleaved, default bench.
set -o pipefail
O=gpurun_out/r03cs
mkdir -p $O
b() {   # name lib
    local n=$1 lib=$2
    timeout -k 10 300 env MPPI_AMD_LIB=$lib python -u bench.py --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -5 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().split('\n')[-1]); k=d['kernel_ms']; print('%-10s ms/update %.4f launch %.4f reduce %.4f' % ('$n', d['ms_per_step'], k['rollout_launch'], k['breakdown_untimed']['reduce']))"
}
for i in 1 2 3; do
  b base_$i assistedmanipulation_amd/lib/libmppi_amd.so || exit 1
  b cs2_$i gpurun_variants/cs2/libmppi_amd.so || exit 1
  b cs3_$i gpurun_variants/cs3/libmppi_amd.so || exit 1
  b cs4_$i gpurun_variants/cs4/libmppi_amd.so || exit 1
done
