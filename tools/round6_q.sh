#!/bin/bash
# Round 6: scale checks on one GPU -- the whole of config[2] (16 M signatures)
# through the multi-part pipeline, config[4]'s adversarial mix at 8 M, and the
# audit-round RLC shape at 4 M records; every run checks its verdicts.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6q}
timeout -k 10 400 python bench.py --n 16777216 --steps 2 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_bench_16m.json 2> gpurun_out/${T}_bench_16m.err || { tail -5 gpurun_out/${T}_bench_16m.err; exit 1; }
timeout -k 10 400 python bench.py --mode adversarial --n 8388608 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/${T}_bench_adv8m.json 2> gpurun_out/${T}_bench_adv8m.err || { tail -5 gpurun_out/${T}_bench_adv8m.err; exit 2; }
timeout -k 10 400 python bench.py --mode rlc --n 4194304 --forged-count 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/${T}_bench_rlc4m.json 2> gpurun_out/${T}_bench_rlc4m.err || { tail -5 gpurun_out/${T}_bench_rlc4m.err; exit 3; }
for f in gpurun_out/${T}_bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['config'].get('n_per_gpu', d['config']), round(d['value']), d.get('verdicts_ok'), round(d['ms_per_step'],1))"; done
