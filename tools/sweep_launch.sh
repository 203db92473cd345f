#!/bin/bash
# Sweep of the pipeline part size (records per kernel launch) on the bench workload.
# Usage (GPU box, repo root): TAG=r02c bash tools/sweep_launch.sh 1048576 262144 ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in "$@"; do
  CESS_BLS_LAUNCH_RECORDS=$q timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG}_launch_$q.json 2> gpurun_out/${TAG}_launch_$q.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_launch_$q.json')); print($q, round(d['value']), d['verdicts_ok'], {k: round(v,1) for k,v in d['stage_ms_per_step'].items()})"
done
