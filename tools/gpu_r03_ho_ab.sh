#!/bin/bash
# Same-box A/B of take_over's tuning (gpurun_variants/*: HO_BIAS / HO_SELF builds) against the tree's build.
set -o pipefail
mkdir -p gpurun_out/r03hoab
for i in 1 2 3; do
  for v in tree b2s0 b4s0 b4s3 b6s0; do
    if [ $v = tree ]; then L=assistedmanipulation_amd/lib/libmppi_amd.so; else L=gpurun_variants/$v/libmppi_amd.so; fi
    f=gpurun_out/r03hoab/${v}_$i.log
    MPPI_AMD_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-cpu-baseline > $f 2>&1 || { echo "bench $v rc=$?"; tail -5 $f; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('%-5s %.4f %.4f %s %s' % (sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'], d['engine']['handover'], d['engine']['wait_timeouts']))" $f $v
  done
done
