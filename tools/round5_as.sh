# round5_as: distinct-key RLC with shared N-pair Miller loop (staged.hpp) and g1_mul_glv32 in curve.hpp: RLC
# tests, the rlcd benches, kernel times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rlc_distinct.py tests/test_gpu_rlc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5as_pytest.txt 2>&1 || { tail -30 gpurun_out/r5as_pytest.txt; exit 1; }
tail -2 gpurun_out/r5as_pytest.txt
timeout -k 10 300 python bench.py --mode rlcd --steps 3 --cpu-sample 0 > gpurun_out/r5as_bench_rlcd.json 2> gpurun_out/r5as_bench_rlcd.err || { tail -20 gpurun_out/r5as_bench_rlcd.err; exit 1; }
timeout -k 10 300 python bench.py --mode rlcd --forged-count 4 --steps 3 --cpu-sample 0 > gpurun_out/r5as_bench_rlcd_f4.json 2> gpurun_out/r5as_bench_rlcd_f4.err || { tail -20 gpurun_out/r5as_bench_rlcd_f4.err; exit 1; }
for f in gpurun_out/r5as_bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), d['verdicts_ok'], d.get('rlc_stats'))"; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5as_prof -o run -- python3 bench.py --mode rlcd --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r5as_prof.log 2>&1 || { tail -20 gpurun_out/r5as_prof.log; exit 1; }
f=$(find gpurun_out/r5as_prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print(r['Name'].split('(')[0][:40].ljust(40), r['Calls'].rjust(6), '%10.2f ms total' % (float(r['TotalDurationNs'])/1e6), '%10.3f ms avg' % (float(r['AverageNs'])/1e6))
PY
