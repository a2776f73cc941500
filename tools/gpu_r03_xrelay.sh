#!/bin/bash
# Round 3: the relay across workgroups with sleeping hosts against the chunked build of the
# previous commit (gpurun_variants/v_chunk): equality tests, the whole GPU suite, interleaved
# bench runs over MPPI_RELAY_CUS, wave traces.  Logs under gpurun_out/r03xr/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03xr
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "handover or draws_ahead" -v -s --timeout 120 --timeout-method thread > $O/pytest_relay.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|handover steps" $O/pytest_relay.log | tail -30
if [ $rc -ne 0 ]; then tail -80 $O/pytest_relay.log; exit $rc; fi
if [ -n "$FULL" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for i in 1 2; do
  for v in chunk r1 r2 r3 r4; do
    case $v in
      chunk) L=gpurun_variants/v_chunk/libmppi_amd.so; n=4;;
      r*) L=assistedmanipulation_amd/lib/libmppi_amd.so; n=${v#r};;
    esac
    f=$O/bench_${v}_$i.log
    MPPI_RELAY_CUS=$n MPPI_AMD_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-cpu-baseline > $f 2>&1 || { echo "bench $v rc=$?"; tail -20 $f; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'])" $f "$v"
  done
done
for n in 2 3; do
  MPPI_RELAY_CUS=$n MPPI_WAVE_TRACE=$PWD/$O/t$n.bin MPPI_AMD_LIB=$PWD/gpurun_variants/wtrace/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/wt$n.json 2> $O/wt$n.err || { echo "trace rc=$?"; tail $O/wt$n.err; exit 1; }
  echo "== relay CUs $n"; python3 tools/wave_trace_r03.py $O/t$n.bin 1030 relay || exit 1
done
exit 0
