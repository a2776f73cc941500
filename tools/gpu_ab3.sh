#!/bin/bash
# Same-box interleaved A/B (run via gpurun): ROUNDS rounds over the libraries in gpurun_variants/*/
# (a variant's optional env file holds VAR=value lines), the default bench line (200 updates) per
# run; one summary line per run: ms/update, the rollout launch, the untimed reduce phase.
# Output: gpurun_out/ab3/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab3
mkdir -p $O
for i in $(seq 1 ${ROUNDS:-3}); do
    for d in gpurun_variants/*/; do
        n=$(basename $d)
        envs=""
        [ -f $d/env ] && envs=$(cat $d/env)
        env $envs MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "$n rc=$?"; tail -5 $O/${n}_$i.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/${n}_$i.json').read().strip().split('\n')[-1]); k=d['kernel_ms']; print('%-10s %d ms/update %.4f launch %.4f reduce %.4f' % ('$n', $i, d['ms_per_step'], k['rollout_launch'], k['breakdown_untimed']['reduce']))"
    done
done
