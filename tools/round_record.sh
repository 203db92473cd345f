#!/bin/bash
# End-of-session record on one GPU box (repo root): -m gpu tests, smoke, the
# default bench (with cpu_baseline), the mode benches, rocprofv3 kernel stats +
# PMC traffic (tools/profile.sh) and the stall counters of the two Fp12
# kernels (tools/pmc_stall.sh).  Every GPU step has its own time limit and the
# script stops at the first failure.  Usage: TAG=round3_r bash tools/round_record.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-round3_r}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -20 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit 3
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_n1.json 2> gpurun_out/${T}_bench_n1.err || exit 4
for m in adversarial keyed rsa sign; do
  timeout -k 10 300 python bench.py --mode $m --steps 3 --cpu-sample 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.err || exit 5
done
timeout -k 10 300 python bench.py --mode rlc --steps 3 --cpu-sample 0 > gpurun_out/${T}_bench_rlc.json 2> gpurun_out/${T}_bench_rlc.err || exit 6
timeout -k 10 300 python bench.py --mode rlc --forged-count 4 --steps 3 --cpu-sample 0 > gpurun_out/${T}_bench_rlc_forged4.json 2> gpurun_out/${T}_bench_rlc_forged4.err || exit 7
timeout -k 10 300 python bench.py --mode rlcd --steps 3 --cpu-sample 0 > gpurun_out/${T}_bench_rlcd.json 2> gpurun_out/${T}_bench_rlcd.err || exit 6
timeout -k 10 300 python bench.py --mode rlcd --forged-count 4 --steps 3 --cpu-sample 0 > gpurun_out/${T}_bench_rlcd_forged4.json 2> gpurun_out/${T}_bench_rlcd_forged4.err || exit 7
for f in gpurun_out/${T}_bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']), d.get('verdicts_ok'))"; done
[ -n "$NOPROF" ] && exit 0
timeout -k 10 560 bash tools/profile.sh $T 1048576 > gpurun_out/${T}_profile.log 2>&1 || { tail -5 gpurun_out/${T}_profile.log; exit 8; }
tail -1 gpurun_out/${T}_profile.log
timeout -k 10 400 bash tools/pmc_stall.sh $T 262144 "k_final|k_miller" > gpurun_out/${T}_stall.log 2>&1 || { tail -5 gpurun_out/${T}_stall.log; exit 9; }
tail -3 gpurun_out/${T}_stall.log
timeout -k 10 600 bash tools/profile_rlcd.sh $T > gpurun_out/${T}_profile_rlcd.log 2>&1 || { tail -5 gpurun_out/${T}_profile_rlcd.log; exit 10; }
tail -1 gpurun_out/${T}_profile_rlcd.log
