#!/bin/bash
# Round 6: k_miller (lane) vs k_miller2 (pair) on one box: bench A/B and the
# stall counters of the Miller kernel (two PMC passes per variant, 256 K sigs).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6b}
for v in lane pair lane pair; do
  CESS_BLS_MILLER=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_bench_$v.json 2> gpurun_out/${T}_bench_$v.err || { tail -5 gpurun_out/${T}_bench_$v.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench_$v.json')); print('$v', round(d['value']), d['verdicts_ok'], {k: round(x,2) for k,x in d['stage_ms_per_step'].items()})"
done
for v in lane pair; do
  OUT=gpurun_out/stall_${T}_$v; mkdir -p $OUT; i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_IFETCH GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    CESS_BLS_MILLER=$v timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_miller" --output-format csv -d $OUT/p$i -o run -- python3 bench.py --n 262144 --steps 1 --warmup 0 --cpu-sample 0 --host-steps 0 > $OUT/p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit 3; fi
  done
done
CESS_BLS_MILLER=pair timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 4; }
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -3
