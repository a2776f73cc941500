# Host turnaround probe (tools/host_loop_probe.py) on the GPU box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp
MPPI_HOST_TRACE=1 timeout -k 10 180 python tools/host_loop_probe.py wrapper raw bench raw wrapper > gpurun_out/hp/probe.log 2>&1; rc=$?; cat gpurun_out/hp/probe.log; exit $rc
