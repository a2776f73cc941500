#!/bin/bash
# Round 3: the relay (fr_coop.hip relay_stage) against take_over (gpurun_variants/v_take, the
# previous tree's build): the relay's equality tests, the whole GPU suite, then interleaved bench
# runs.  Logs under gpurun_out/r03relay/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03relay
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
  for v in take relay relay0; do
    case $v in
      take) L=gpurun_variants/v_take/libmppi_amd.so; ho=1;;
      relay) L=assistedmanipulation_amd/lib/libmppi_amd.so; ho=1;;
      relay0) L=assistedmanipulation_amd/lib/libmppi_amd.so; ho=0;;
    esac
    f=$O/bench_${v}_$i.log
    MPPI_AMD_LIB=$PWD/$L MPPI_HANDOVER=$ho timeout -k 10 200 python -u bench.py --no-cpu-baseline > $f 2>&1 || { echo "bench $v rc=$?"; tail -20 $f; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'])" $f "$v"
  done
done
exit 0
