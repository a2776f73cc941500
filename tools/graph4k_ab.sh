mkdir -p gpurun_out/g4k
for i in 1 2 3; do for g in 0 1; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --graph $g > gpurun_out/g4k/g${g}_$i.json 2> gpurun_out/g4k/g${g}_$i.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], d['ms_per_step'], d['engine']['graph_updates_timed'], d['steps'])" gpurun_out/g4k/g${g}_$i.json g${g}_$i
done; done
