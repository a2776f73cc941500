#!/bin/bash
# Round 3: the objective in chunks beside the loops (cost_work) against the relay build (v_relay).
# The relay's equality tests, the whole GPU suite, interleaved bench runs, then wave traces
# (COOP_TRACE + COST_TRACE build in gpurun_variants/wtrace).  Logs under gpurun_out/r03chunk/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03chunk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "handover or draws_ahead" -v -s --timeout 120 --timeout-method thread > $O/pytest_relay.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|handover steps" $O/pytest_relay.log | tail -30
if [ $rc -ne 0 ]; then tail -60 $O/pytest_relay.log; exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in relay chunks chunks0; do
    case $v in
      relay) L=gpurun_variants/v_relay/libmppi_amd.so; ho=1;;
      chunks) L=assistedmanipulation_amd/lib/libmppi_amd.so; ho=1;;
      chunks0) L=assistedmanipulation_amd/lib/libmppi_amd.so; ho=0;;
    esac
    f=$O/bench_${v}_$i.log
    MPPI_AMD_LIB=$PWD/$L MPPI_HANDOVER=$ho timeout -k 10 200 python -u bench.py --no-cpu-baseline > $f 2>&1 || { echo "bench $v rc=$?"; tail -20 $f; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'])" $f "$v"
  done
done
for ho in 1 0; do
  MPPI_HANDOVER=$ho MPPI_WAVE_TRACE=$PWD/$O/t$ho.bin MPPI_AMD_LIB=$PWD/gpurun_variants/wtrace/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/wt$ho.json 2> $O/wt$ho.err || { echo "trace rc=$?"; tail $O/wt$ho.err; exit 1; }
  echo "== handover=$ho"; python3 tools/wave_trace_r03.py $O/t$ho.bin 1026 relay || exit 1
done
exit 0
