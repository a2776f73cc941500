#!/bin/bash
# The one GPU-box launcher (run through gpurun from the repo root): every step under its own time
# limit, steps chained so that the first failure ends the call.  Replaces rounds 1-3's one-off
# tools/gpu_*.sh scripts (in git history before round 4).
#
#   TAG=r04a bash tools/gpu_run.sh STEP [STEP ...]
#
# STEP is one of
#   smoke              __graft_entry__.smoke()
#   tests[:EXPR]       the whole -m gpu suite in one pytest process (or -k EXPR)
#   softtests[:EXPR]   the same, but test failures (not crashes or timeouts) let the later steps run
#   bench              the default bench line (N = 1, with the CPU baseline)
#   trace[:NAME]       rocprofv3 --kernel-trace --stats of the bench (no CPU baseline; BENCH_ARGS apply;
#                      NAME names the output, default "trace")
#   tracepm            trace of the point-mass workload (configs[1]), 200 updates
#   pmc                rocprofv3 PMC passes (one counter set per run) -> pmc summaries + traffic JSON
#   pmcpm              the fetch / write / fp64 passes over the fused point-mass launch (configs[1])
#   pmcsize:NAME:KERN  the PMC passes over BENCH_ARGS's workload, kernel names containing KERN
#   sizes              the other BASELINE workloads on one GPU (point mass, 32768x64, 8192x128 SG,
#                      65536x128 SG)
#   absizes:V1,V2:N    N interleaved rounds of the 4096x64, 32768x64, 8192x128 SG and 65536x128 SG benches
#                      over library variants (as ab)
#   graphab[:ROUNDS]   configs[4]'s shapes as the hipGraph against eager launches, unsharded and through a
#                      one-rank RCCL communicator (bench.py --graph / --comm1)
#   ab:V1,V2,..:N      N interleaved rounds of bench over kernel variants (gpurun_variants/<V>/,
#                      built by tools/ab_build.sh; "tree" = the in-tree library); BENCH_ARGS and
#                      AB_ENV_<V> (extra env for variant V, e.g. AB_ENV_tree0="MPPI_HANDOVER=0") apply
#   pmstamps[:VARIANT] the fused point-mass kernel's phase stamps (MPPI_PM_STAMPS=1), in-tree or a variant
#   wtrace:VARIANT     per-wave trace of VARIANT's COOP_TRACE build (tools/wave_trace_r03.py)
#   kpmc:V1,V2,..      PMC of the kernels outside the rollout launch (weights / finish / rank), per library
# Output: gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-run}
O=gpurun_out/$TAG
mkdir -p $O
BENCH_ARGS=${BENCH_ARGS:-}

summary() {   # file label
    python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split('\n')[-1])
k = d.get("kernel_ms", {})
r = d.get("roofline", {})
print("%-16s ms/update %.4f value %.4e launch %s frac %s" % (sys.argv[2], d["ms_per_step"], d["value"],
      k.get("rollout_launch"), r.get("frac")))
PY
}

step_smoke() {
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { echo "smoke rc=$?"; tail -30 $O/smoke.log; return 1; }
    echo "smoke ok"
}

step_tests() {   # [expr] [soft]: soft = test failures (pytest rc 1) do not stop the run; anything
                 # else (a timeout, an abort, a crash) does
    local k=()
    [ -n "$1" ] && k=(-k "$1")
    timeout -k 10 1000 python -u -m pytest tests -m gpu "${k[@]}" -v -s --timeout 240 --timeout-method thread \
        > $O/pytest.log 2>&1
    local rc=$?
    grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
    if [ "$2" = soft ] && [ $rc -eq 1 ]; then echo "tests: failures (continuing)"; return 0; fi
    return $rc
}

step_bench() {
    timeout -k 10 300 python -u bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err \
        || { echo "bench rc=$?"; tail -20 $O/bench.err; return 1; }
    summary $O/bench.json bench
}

step_trace() {   # [name] [extra bench args...]
    local n=${1:-trace}; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline $BENCH_ARGS "$@" > $O/${n}_bench.json 2> $O/$n.err \
        || { echo "trace rc=$?"; tail -20 $O/$n.err; return 1; }
    summary $O/${n}_bench.json $n
    local st
    st=$(find $O/$n -name "run_kernel_stats.csv" | head -n 1)
    [ -n "$st" ] && cp "$st" $O/${n}_kernel_stats.csv && head -8 $O/${n}_kernel_stats.csv
    local tr
    tr=$(find $O/$n -name "run_kernel_trace.csv" | head -n 1)
    [ -n "$tr" ] && python3 tools/trace_seq.py "$tr" > $O/${n}_seq.txt 2>&1
    return 0
}

step_pmc() {   # [pm | NAME PREFIX]: NAME: a size's passes (BENCH_ARGS) into $O/pmc_NAME, the kernel matched by PREFIX
    local B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline $BENCH_ARGS" D=$O/pmc out=$O/pmc_rollout.json prefix=
    if [ -n "$2" ]; then
        D=$O/pmc_$1 out=$O/pmc_$1.json prefix=$2
    fi
    if [ "$1" = pm ]; then
        B="python3 bench.py --workload point_mass --steps 50 --warmup 5 --no-cpu-baseline"
        D=$O/pmcpm out=$O/pmc_pm.json prefix=pm_update_kernel
    fi
    mkdir -p $D
    run() {   # name counters...
        local n=$1; shift
        timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $D -o $n --output-format csv -- $B > $D/$n.log 2>&1
    }
    local names="sq lat flops fetch write"
    if [ "$1" = pm ]; then
        names="flops fetch write"
    else
        run sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY && echo "pmc sq ok" && \
        run lat SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && echo "pmc lat ok" || return 1
    fi
    run flops SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL && echo "pmc flops ok" && \
    run fetch FETCH_SIZE GRBM_GUI_ACTIVE && echo "pmc fetch ok" && \
    run write WRITE_SIZE && echo "pmc write ok" || return 1
    for n in $names; do python3 tools/pmc_summary.py $D/${n}_counter_collection.csv > $D/${n}_summary.txt; done
    python3 tools/pmc_traffic.py $D $out $prefix && cat $out
}

step_kpmc() {   # V1,V2,..: counters of the kernels outside the rollout launch, per library ("tree" = in-tree)
    local vs
    IFS=, read -ra vs <<< "$1"
    for v in "${vs[@]}"; do
        local lib=$PWD/gpurun_variants/$v/libmppi_amd.so D=$O/kpmc_$v
        [ "$v" = tree ] && lib=$PWD/assistedmanipulation_amd/lib/libmppi_amd.so
        mkdir -p $D
        local B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
        krun() {   # name counters...
            local n=$1; shift
            MPPI_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "weights|finish|rank_draw" \
                -d $D -o $n --output-format csv -- $B > $D/$n.log 2>&1
        }
        krun sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE && \
        krun ta TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum && \
        krun fetch FETCH_SIZE && echo "kpmc $v ok" || return 1
        for n in sq ta fetch; do python3 tools/pmc_summary.py $D/${n}_counter_collection.csv > $D/${n}_summary.txt; cat $D/${n}_summary.txt; done
    done
}

step_sizes() {
    size() {   # name args...
        local n=$1; shift
        timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/size_$n.json 2> $O/size_$n.err \
            || { echo "size $n rc=$?"; tail -5 $O/size_$n.err; return 1; }
        summary $O/size_$n.json $n
    }
    size pm --workload point_mass --steps 200 --warmup 10 && \
    size s32k --steps 20 --warmup 3 --samples-per-gpu 32768 && \
    size s8k_h128_sg --steps 40 --warmup 3 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 && \
    size s64k_h128_sg --steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10
}

step_graphab() {   # [rounds]: configs[4]'s shapes, the hipGraph against eager launches, unsharded and through a
                  # one-rank RCCL communicator (--comm1), interleaved on one box
    local rounds=${1:-2} i
    gsize() {   # name args...
        local n=$1; shift
        timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/size_$n.json 2> $O/size_$n.err \
            || { echo "size $n rc=$?"; tail -5 $O/size_$n.err; return 1; }
        summary $O/size_$n.json $n
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print('   graph_updates_timed', d['engine']['graph_updates_timed'], 'of', d['steps'])" $O/size_$n.json
    }
    for i in $(seq 1 $rounds); do
        for c in 0 1; do
            for g in 0 1; do
                gsize s8k_sg_c${c}_g${g}_$i --steps 60 --warmup 5 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 \
                    --graph $g --comm1 $c || return 1
            done
        done
    done
    for g in 0 1; do
        gsize s64k_sg_g${g} --steps 12 --warmup 3 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10 --graph $g || return 1
    done
}

step_absizes() {   # V1,V2,..  rounds: interleaved A/B of the library variants over BASELINE's workloads
    local vs rounds=${2:-2} i v w
    IFS=, read -ra vs <<< "$1"
    local shapes=("s4k:--steps 200 --warmup 10" "s32k:--steps 20 --warmup 3 --samples-per-gpu 32768"
                  "s8k_sg:--steps 40 --warmup 3 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10"
                  "s64k_sg:--steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10")
    for i in $(seq 1 $rounds); do
        for w in "${shapes[@]}"; do
            for v in "${vs[@]}"; do
                local lib=$PWD/assistedmanipulation_amd/lib/libmppi_amd.so n=${w%%:*} f
                case $v in tree*) ;; *) lib=$PWD/gpurun_variants/$v/libmppi_amd.so;; esac
                f=$O/abs_${n}_${v}_$i.json
                MPPI_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline ${w#*:} > $f 2> ${f%.json}.err \
                    || { echo "absizes $n $v rc=$?"; tail -20 ${f%.json}.err; return 1; }
                summary $f "$n/$v/$i"
            done
        done
    done
}

step_ab() {   # V1,V2,..  rounds
    local vs rounds=${2:-3}
    IFS=, read -ra vs <<< "$1"
    for i in $(seq 1 $rounds); do
        for v in "${vs[@]}"; do
            local lib=$PWD/assistedmanipulation_amd/lib/libmppi_amd.so
            case $v in tree*) ;; *) lib=$PWD/gpurun_variants/$v/libmppi_amd.so;; esac
            local envv="AB_ENV_$v" f=$O/ab_${v}_$i.json
            env MPPI_AMD_LIB=$lib ${!envv} timeout -k 10 200 python -u bench.py --no-cpu-baseline $BENCH_ARGS \
                > $f 2> $O/ab_${v}_$i.err || { echo "ab $v rc=$?"; tail -20 $O/ab_${v}_$i.err; return 1; }
            summary $f "$v/$i"
        done
    done
}

step_pmstamps() {   # [variant]: the fused point-mass kernel's phase stamps (MPPI_PM_STAMPS=1, printed at destroy)
    local lib=$PWD/assistedmanipulation_amd/lib/libmppi_amd.so n=pmstamps${1:+_$1}
    [ -n "$1" ] && lib=$PWD/gpurun_variants/$1/libmppi_amd.so
    MPPI_AMD_LIB=$lib MPPI_PM_STAMPS=1 timeout -k 10 200 python -u bench.py --workload point_mass --steps 100 --warmup 10 \
        --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$n rc=$?"; tail -20 $O/$n.err; return 1; }
    grep "pm_update_kernel phases" $O/$n.err
    summary $O/$n.json $n
}


step_wtrace() {   # variant
    local lib=$PWD/gpurun_variants/$1/libmppi_amd.so
    MPPI_WAVE_TRACE=$PWD/$O/wt.bin MPPI_AMD_LIB=$lib timeout -k 10 120 python bench.py --steps 40 --warmup 10 \
        --no-cpu-baseline $BENCH_ARGS > $O/wt.json 2> $O/wt.err || { echo "wtrace rc=$?"; tail $O/wt.err; return 1; }
    python3 tools/wave_trace_r06.py $O/wt.bin 1064 | tee $O/wave_trace.txt
}

for s in "$@"; do
    name=${s%%:*}
    arg=${s#*:}
    [ "$arg" = "$s" ] && arg=""
    case $name in
        smoke) step_smoke ;;
        tests) step_tests "$arg" ;;
        softtests) step_tests "$arg" soft ;;
        bench) step_bench ;;
        trace) step_trace "$arg" ;;
        tracepm) step_trace tracepm --workload point_mass --steps 200 ;;
        pmc) step_pmc ;;
        pmcsize) step_pmc "${arg%%:*}" "${arg#*:}" ;;
        pmcpm) step_pmc pm ;;
        sizes) step_sizes ;;
        kpmc) step_kpmc "$arg" ;;
        graphab) step_graphab "$arg" ;;
        absizes) step_absizes "${arg%%:*}" "$( [ "${arg#*:}" != "$arg" ] && echo ${arg#*:} )" ;;
        ab) step_ab "${arg%%:*}" "$( [ "${arg#*:}" != "$arg" ] && echo ${arg#*:} )" ;;
        wtrace) step_wtrace "$arg" ;;
        pmstamps) step_pmstamps "$arg" ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac || { echo "step $s failed"; exit 1; }
done
exit 0
