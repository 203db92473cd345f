#!/bin/bash
# Round-5 diagnostics on one GPU box (repo root): the in-kernel issue probe and
# the instruction-cache counters of the six verify kernels.  Usage: TAG=r5a bash tools/round5_probe.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r5a}
timeout -k 10 120 ./tools/issue_probe > gpurun_out/${T}_issue_probe.txt 2>&1 || { cat gpurun_out/${T}_issue_probe.txt; exit 1; }
cat gpurun_out/${T}_issue_probe.txt
RX="k_final|k_miller|k_prepare|k_decode_pk|k_hash|k_decode_sig"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_pmc$i -o run -- python3 bench.py --n 262144 --steps 1 --warmup 0 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_pmc$i.log; exit $rc; }
done
