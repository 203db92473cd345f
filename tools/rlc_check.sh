#!/bin/bash
# RLC bucket-path check on the GPU box: RLC tests, bench --mode rlc (clean and 4 forgeries), rocprof kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-rlc_b}
timeout -k 10 400 python -u -m pytest tests/test_gpu_rlc.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.txt
timeout -k 10 200 python3 bench.py --mode rlc --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 2; }
cat gpurun_out/${TAG}_bench.json | cut -c1-200
timeout -k 10 200 python3 bench.py --mode rlc --steps 3 --warmup 1 --cpu-sample 0 --forged-count 4 > gpurun_out/${TAG}_bench_f4.json 2> gpurun_out/${TAG}_bench_f4.err || { tail -20 gpurun_out/${TAG}_bench_f4.err; exit 3; }
cat gpurun_out/${TAG}_bench_f4.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --mode rlc --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG}_prof.log 2>&1 || exit 4
echo done
