#!/bin/bash
# round3_ak: records per launch (CESS_BLS_LAUNCH_RECORDS: light kernels of part
# i+1 on the second stream beside the Miller loop / final exponentiation of
# part i) on the current build, config[1] bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 1048576 524288 262144 1048576 524288 262144; do
  CESS_BLS_LAUNCH_RECORDS=$q timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/round3_ak_$q.json 2> gpurun_out/round3_ak_$q.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/round3_ak_$q.json')); print($q, round(d['value']), d['verdicts_ok'], round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['stage_ms_per_step'].items()})"
done
