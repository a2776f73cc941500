#!/bin/bash
# Round 3 profile set (run via gpurun): default bench line, rocprofv3 --kernel-trace --stats of the
# same command, PMC passes for the rollout kernel's traffic and issue counters, then the other
# BASELINE workloads (point mass configs[1], 32768 x 64, 8192 x 128 SG, 65536 x 128 SG).
# Output: gpurun_out/r03prof/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03prof
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
echo "bench ok"; tail -c 600 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err || { echo "trace rc=$?"; exit 1; }
echo "trace ok"
B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline"
D=$O/pmc
mkdir -p $D
run() {   # name counters...
    local n=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $D -o $n --output-format csv -- $B > $D/$n.log 2>&1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY && echo "pmc sq ok" && \
run lat SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && echo "pmc lat ok" && \
run flops SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL && echo "pmc flops ok" && \
run fetch FETCH_SIZE GRBM_GUI_ACTIVE && echo "pmc fetch ok" && \
run write WRITE_SIZE && echo "pmc write ok" || exit 1
for n in sq lat flops fetch write; do python3 tools/pmc_summary.py $D/${n}_counter_collection.csv > $D/${n}_summary.txt; done
python3 tools/pmc_traffic.py $D $O/pmc_rollout.json && cat $O/pmc_rollout.json
size() {   # name args...
    local n=$1; shift
    timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/size_$n.json 2> $O/size_$n.err || { echo "size $n rc=$?"; tail -5 $O/size_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/size_$n.json').read().strip().split('\n')[-1]); print('%-14s ms/update %.4f value %.3e launch %s' % ('$n', d['ms_per_step'], d['value'], d['kernel_ms'].get('rollout_launch')))"
}
size pm --workload point_mass --steps 200 --warmup 10
size s32k --steps 20 --warmup 3 --samples-per-gpu 32768
size s8k_h128_sg --steps 40 --warmup 3 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10
size s64k_h128_sg --steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10
