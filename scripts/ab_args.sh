#!/bin/bash
# A/B of bench.py argument sets on one library: bash scripts/ab_args.sh TAG REPS "name1:args1" "name2:args2" ...
# (each line: config name, Mpx/s, ms per frame, the dominant kernel's live launch time)
set -o pipefail
TAG=$1; REPS=$2; shift 2
mkdir -p gpurun_out
: > gpurun_out/${TAG}_ab.txt
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 300 python bench.py $args > gpurun_out/${TAG}_ab_one.json 2> gpurun_out/${TAG}_ab_one.err \
      || { tail -5 gpurun_out/${TAG}_ab_one.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline',{})
print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame', 'dom', r.get('launch_ms_live'))" gpurun_out/${TAG}_ab_one.json "$name rep$rep" | tee -a gpurun_out/${TAG}_ab.txt || exit 1
  done
done
