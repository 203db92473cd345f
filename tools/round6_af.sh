#!/bin/bash
# Round 6: the N>1 path rehearsed with 4 ranks on one GPU over the shared-memory
# transport (bench.py --transport shm --one-device; the rate is NOT a 4-GPU
# figure): per-signature (config[2] shape), adversarial (config[4] shape) and
# RLC with the Gt-partial all-gather (config[3] shape), verdicts checked.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6af}
run() {  # name, port, extra args
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $2 \
    bench.py --gpus 4 --transport shm --one-device --steps 2 --warmup 1 --cpu-sample 0 ${@:3} > gpurun_out/${T}_$1.json 2> gpurun_out/${T}_$1.err
}
run persig 29511 --host-steps 0 || { tail -20 gpurun_out/${T}_persig.err; exit 1; }
run adv 29512 --mode adversarial || { tail -20 gpurun_out/${T}_adv.err; exit 2; }
run rlc 29513 --mode rlc --forged-count 2 || { tail -20 gpurun_out/${T}_rlc.err; exit 3; }
for f in persig adv rlc; do python3 -c "import json; d=json.loads(open('gpurun_out/${T}_$f.json').read().strip().splitlines()[-1]); print('$f', d['n_gpus'], round(d['value']), d.get('verdicts_ok'), d['config'].get('parallelism'), d['config'].get('transport'), d.get('bitmap_popcount'))"; done
