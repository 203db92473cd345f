# round5_ai: GPU suite + the RLC benches after the lane-group final exponentiation
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ai_pytest.txt 2>&1 || { tail -30 gpurun_out/r5ai_pytest.txt; exit 1; }
tail -2 gpurun_out/r5ai_pytest.txt
for m in rlc; do
  timeout -k 10 300 python bench.py --mode $m --steps 3 --cpu-sample 0 > gpurun_out/r5ai_bench_$m.json 2> gpurun_out/r5ai_bench_$m.err || { tail -20 gpurun_out/r5ai_bench_$m.err; exit 1; }
  timeout -k 10 300 python bench.py --mode $m --forged-count 4 --steps 3 --cpu-sample 0 > gpurun_out/r5ai_bench_${m}_f4.json 2> gpurun_out/r5ai_bench_${m}_f4.err || { tail -20 gpurun_out/r5ai_bench_${m}_f4.err; exit 1; }
done
for f in gpurun_out/r5ai_bench_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), d['verdicts_ok'], d.get('rlc_stats'))"; done
