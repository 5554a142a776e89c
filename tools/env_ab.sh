#!/bin/bash
# GPU-box job: bench.py lines under several environment settings, interleaved (round-robin, R
# rounds), for A/Bs of runtime switches (MJG_MERGE, MJG_MERGE_HOLD, ...).
# Usage: bash tools/env_ab.sh TAG "NAME=ENV ...;NAME=ENV ..." [bench args...]   (R=2 rounds by default)
set -o pipefail
TAG=$1; SETS=$2; shift 2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
IFS=';' read -ra S <<< "$SETS"
for r in $(seq 1 ${R:-2}); do
  for s in "${S[@]}"; do
    name=${s%%=*}; envs=${s#*=}
    env $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e "$@" > $O/${name}_$r.json 2> $O/${name}_$r.err || { tail -5 $O/${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${name}_$r.json')); print('%-14s %s %10.1f %.4f' % ('$name', '$r', d['value'], d['ms_per_step']))" | tee -a $O/ab.txt
  done
done
echo done
