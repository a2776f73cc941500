# gj_rows on the GPU: the standalone probe, then the parity subset through the in-tree library
mkdir -p gpurun_out/gjv
timeout -k 5 60 ./tools/probe/gj_probe > gpurun_out/gjv/probe.txt 2>&1 || exit $?
head -1 gpurun_out/gjv/probe.txt; sed -n 15p gpurun_out/gjv/probe.txt
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "config1 or config3 or default_stack" > gpurun_out/gjv/tree.log 2>&1
rc=$?; echo "tree rc=$rc $(tail -1 gpurun_out/gjv/tree.log)"; exit $rc
