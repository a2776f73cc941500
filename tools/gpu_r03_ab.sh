#!/bin/bash
# Round 3: the whole GPU suite, interleaved bench runs over builds x handover, the microbenchmark
# and the phase traces.  old3 = gpurun_variants/v_old3 (serial pivots, select masks, dummy body 0),
# new = the tree's build.  Logs under gpurun_out/r03ab/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03ab
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r03ab/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|handover steps" gpurun_out/r03ab/pytest.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
  for lib in old3 new; do
    for ho in 0 1; do
      if [ $lib = old3 ]; then L=gpurun_variants/v_old3/libmppi_amd.so; else L=assistedmanipulation_amd/lib/libmppi_amd.so; fi
      f=gpurun_out/r03ab/bench_${lib}_ho${ho}_$i.log
      MPPI_AMD_LIB=$PWD/$L MPPI_HANDOVER=$ho timeout -k 10 200 python -u bench.py --no-cpu-baseline > $f 2>&1 || { echo "bench $lib ho=$ho rc=$?"; tail -20 $f; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'])" $f "$lib ho=$ho"
    done
  done
done
timeout -k 10 120 tools/bin/ubench > gpurun_out/r03ab/ubench.txt 2>&1 || { echo "ubench rc=$?"; exit 1; }
grep -E "blocks=    1 " gpurun_out/r03ab/ubench.txt
for n in phase phasefk; do
  for ho in 0 1; do
    rm -f gpurun_out/r03ab/$n$ho.bin
    MPPI_HANDOVER=$ho MPPI_WAVE_TRACE=$PWD/gpurun_out/r03ab/$n$ho.bin MPPI_AMD_LIB=$PWD/gpurun_variants/$n/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03ab/$n$ho.json 2> gpurun_out/r03ab/$n$ho.err || { echo "$n rc=$?"; exit 1; }
    echo "== $n handover=$ho"; case $n in *fk*) m=fk;; *) m=;; esac; python3 tools/phase_trace.py gpurun_out/r03ab/$n$ho.bin 1026 $m || exit 1
  done
done
exit $rc
