# round5_ab: the per-GPU shape of config[2] (2 M signatures per GPU) and the
# whole 16 M batch of config[2] through one GPU (chunked by the context)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --n 2097152 --steps 2 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/r5ab_2m.json 2> gpurun_out/r5ab_2m.err || { tail -20 gpurun_out/r5ab_2m.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5ab_2m.json')); print('2M', round(d['value']), d['verdicts_ok'], d['ms_per_step'])"
timeout -k 10 600 python bench.py --n 16777216 --steps 1 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/r5ab_16m.json 2> gpurun_out/r5ab_16m.err || { tail -20 gpurun_out/r5ab_16m.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5ab_16m.json')); print('16M', round(d['value']), d['verdicts_ok'], d['ms_per_step'])"
