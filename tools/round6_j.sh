#!/bin/bash
# Round 6: pipelined parts with the lane-pair kernels: CESS_BLS_LAUNCH_RECORDS
# = 1 M (one part, default) / 512 K / 256 K (light kernels of part i+1 on
# stream2 beside the Miller + final kernels of part i), same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6j}
for q in 1048576 524288 262144 1048576 524288; do
  CESS_BLS_LAUNCH_RECORDS=$q timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_q$q.json 2> gpurun_out/${T}_q$q.err || { tail -5 gpurun_out/${T}_q$q.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_q$q.json')); print('q$q', round(d['value']), d['verdicts_ok'], round(d['ms_per_step'],1), {k: round(x,2) for k,x in d['stage_ms_per_step'].items()})"
done
