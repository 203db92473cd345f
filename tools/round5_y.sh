# round5_y: the final round-5 library on this box: three default bench runs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/r5y_bench_$r.json 2> gpurun_out/r5y_bench_$r.err || { tail -20 gpurun_out/r5y_bench_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5y_bench_$r.json')); print($r, round(d['value']), {k: round(v,2) for k,v in d['stage_ms_per_step'].items()}, d['runtime']['lib_sha256'][:12] if 'runtime' in d and 'lib_sha256' in d['runtime'] else '')"
done
rocm-smi --showclocks --showpower 2>/dev/null | head -20 || true
