# round5_q: replay probe; GPU suite and benches after the SSWU park became the default
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/replay_probe > gpurun_out/r5q_replay.txt 2>&1 || { cat gpurun_out/r5q_replay.txt; exit 1; }
cat gpurun_out/r5q_replay.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5q_pytest.txt 2>&1 || { tail -30 gpurun_out/r5q_pytest.txt; exit 1; }
tail -2 gpurun_out/r5q_pytest.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/r5q_bench.json 2> gpurun_out/r5q_bench.err || { tail -20 gpurun_out/r5q_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5q_bench.json')); print(round(d['value']), {k: round(v,2) for k,v in d['stage_ms_per_step'].items()})"
timeout -k 10 300 python bench.py --mode sign --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/r5q_bench_sign.json 2> gpurun_out/r5q_bench_sign.err || { tail -20 gpurun_out/r5q_bench_sign.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5q_bench_sign.json')); print('sign', round(d['value']))"
