#!/bin/bash
# Round 6: k_final2 (lane-pair final exponentiation, accumulator in LDS):
# GPU parity file + RLC files with CESS_BLS_FINAL=pair, bench A/B (k_final /
# k_final2, k_miller2 in both), PMC traffic + stall counters of k_final2.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6e}
CESS_BLS_FINAL=pair timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_pair.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_pair.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_pair.txt
for v in lane pair lane pair; do
  CESS_BLS_FINAL=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_bench_$v.json 2> gpurun_out/${T}_bench_$v.err || { tail -5 gpurun_out/${T}_bench_$v.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench_$v.json')); print('$v', round(d['value']), d['verdicts_ok'], {k: round(x,2) for k,x in d['stage_ms_per_step'].items()})"
done
for v in lane pair; do
  OUT=gpurun_out/stall_${T}_$v; mkdir -p $OUT; i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_IFETCH GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    CESS_BLS_FINAL=$v timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_final" --output-format csv -d $OUT/p$i -o run -- python3 bench.py --n 262144 --steps 1 --warmup 0 --cpu-sample 0 --host-steps 0 > $OUT/p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit 3; fi
  done
done
