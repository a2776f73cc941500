#!/bin/bash
# Bisect builds: tools/diag_lib.py per library (bounded device waits in all of them).
set -o pipefail
mkdir -p gpurun_out/r03diag
for v in new v_gjserial; do
  if [ $v = new ]; then L=assistedmanipulation_amd/lib/libmppi_amd.so; else L=gpurun_variants/$v/libmppi_amd.so; fi
  echo "== $v"
  MPPI_AMD_LIB=$PWD/$L PYTHONPATH=$PWD timeout -k 10 150 python -u tools/diag_lib.py 2>&1 | tee gpurun_out/r03diag/$v.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; exit $rc; fi
done
