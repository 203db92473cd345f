#!/bin/bash
# Round 6: first GPU run of k_miller2 (lane pair per signature): the GPU parity
# file with CESS_BLS_MILLER=pair, then a same-box A/B of the bench (lane / pair
# twice each) and a rocprofv3 kernel-stats pass of the pair build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6a}
CESS_BLS_MILLER=pair timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_pair.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_pair.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_pair.txt
for v in lane pair lane pair; do
  CESS_BLS_MILLER=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_bench_$v.json 2> gpurun_out/${T}_bench_$v.err || { tail -5 gpurun_out/${T}_bench_$v.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench_$v.json')); print('$v', round(d['value']), d['verdicts_ok'], {k: round(x,2) for k,x in d['stage_ms_per_step'].items()})"
done
CESS_BLS_MILLER=pair timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 3; }
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${T}_pair_kernel_stats.csv
head -8 gpurun_out/${T}_pair_kernel_stats.csv
