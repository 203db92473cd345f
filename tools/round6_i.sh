#!/bin/bash
# Round 6: lane-pair block size A/B (CESS_PAIR_THREADS 256 / 128 / 64 for
# k_miller2 and k_final2), same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6i}
CESS_BLS_LIB=$PWD/cess_amd/lib_variants/t64/libcess_bls.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_t64.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_t64.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_t64.txt
TAG=$T bash tools/sweep_ab.sh t128 t64 t64
# distinct-key RLC with the lane-pair record kernel (k_miller_rr2, default) and
# the one-lane k_miller_rr (CESS_BLS_MILLER=lane)
timeout -k 10 400 python -u -m pytest tests/test_gpu_rlc_distinct.py tests/test_gpu_rlc_gt_oracle.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_rlcd.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_rlcd.txt; exit 4; }
tail -1 gpurun_out/${T}_pytest_rlcd.txt
for v in lane pair lane pair; do
  CESS_BLS_MILLER=$v timeout -k 10 300 python bench.py --mode rlcd --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${T}_rlcd_$v.json 2> gpurun_out/${T}_rlcd_$v.err || { tail -5 gpurun_out/${T}_rlcd_$v.err; exit 5; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_rlcd_$v.json')); print('rlcd $v', round(d['value']), d['verdicts_ok'], {k: round(x,2) for k,x in d['stage_ms_per_step'].items()})"
done
