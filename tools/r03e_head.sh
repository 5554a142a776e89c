#!/bin/bash
# HEAD record: GPU tests, the driver's bench command, its rocprofv3 kernel stats, other workloads
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps({k:v for k,v in d['kernel_ms_per_step'].items() if v})); print(json.dumps(d['e2e'])[:600])"
bash tools/driver_prof.sh $1/driver || exit 1
for w in c1 c4 c5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > $O/bench_$w.json 2> $O/bench_$w.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], json.dumps({k:v for k,v in d['kernel_ms_per_step'].items() if v}))"
done
for c in natural noise-patches; do
  timeout -k 10 200 python bench.py --content $c --no-cpu-baseline --no-e2e > $O/bench_c2_$c.json 2> $O/bench_c2_$c.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_c2_$c.json')); print('$c', d['value'], d['ms_per_step'], json.dumps({k:v for k,v in d['kernel_ms_per_step'].items() if v}))"
done
echo done
