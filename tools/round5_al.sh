# round5_al: re-measure the part pipeline (light kernels of part i+1 beside
# k_miller of part i) with the round-5 kernels: CESS_BLS_LAUNCH_RECORDS sweep
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 1048576 524288 262144 1048576 524288; do
  CESS_BLS_LAUNCH_RECORDS=$q timeout -k 10 200 python bench.py --steps 5 --cpu-sample 0 > gpurun_out/r5al_$q.json 2> gpurun_out/r5al_$q.err || { tail -20 gpurun_out/r5al_$q.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5al_$q.json')); print($q, round(d['value']), round(d['ms_per_step'],1), d['verdicts_ok'], {k: round(v,1) for k,v in d['stage_ms_per_step'].items()})"
done
