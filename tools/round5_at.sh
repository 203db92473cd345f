# round5_at: distinct-key RLC, 2-rank shm rehearsal on one GPU (four records
# per Miller lane), one forgery per rank
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --transport shm --one-device --mode rlcd --n 262144 --forged-count 2 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r5at_rlcd_n2.json 2> gpurun_out/r5at_rlcd_n2.err || { tail -30 gpurun_out/r5at_rlcd_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5at_rlcd_n2.json')); print(round(d['value']), d['n_gpus'], d['verdicts_ok'], d['rlc_stats'])"
