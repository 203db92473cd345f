#!/bin/bash
# Round 6: stability of the final library's config[1] rate -- one long run
# (40 timed steps, ~14 s of sustained load) and three default runs back to
# back on the same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6x}
timeout -k 10 300 python bench.py --steps 40 --warmup 2 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_long.json 2> gpurun_out/${T}_long.err || { tail -5 gpurun_out/${T}_long.err; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_rep$r.json 2> gpurun_out/${T}_rep$r.err || { tail -5 gpurun_out/${T}_rep$r.err; exit 2; }
done
for f in gpurun_out/${T}_long.json gpurun_out/${T}_rep*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['steps'], round(d['value']), round(d['ms_per_step'],2), {k: round(v,1) for k,v in d['stage_ms_per_step'].items()})"; done
