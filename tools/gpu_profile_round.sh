# One round's profile set (run via gpurun): tools/gpu_profile_round.sh <tag>
#   bench line, rocprofv3 --kernel-trace --stats of the same command, PMC passes (SQ, LDS/latency,
#   fp64 work, FETCH_SIZE, WRITE_SIZE) and the rollout kernel's per-launch traffic JSON.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo "bench ok"; cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err || exit 1
echo "trace ok"
B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline"
D=$O/pmc
mkdir -p $D
run() {   # name counters...
    local n=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $D -o $n --output-format csv -- $B > $D/$n.log 2>&1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY && \
run lat SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
run flops SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL && \
run fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
run write WRITE_SIZE || exit 1
for n in sq lat flops fetch write; do python3 tools/pmc_summary.py $D/${n}_counter_collection.csv > $D/${n}_summary.txt; done
python3 tools/pmc_traffic.py $D $O/pmc_rollout.json
