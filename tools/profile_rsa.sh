#!/bin/bash
# rocprofv3 passes for the RSA-2048 bench (bench.py --mode rsa) on the GPU box,
# from the repo root: kernel trace + stats, then PMC passes (traffic: FETCH_SIZE
# and WRITE_SIZE apart; issue/stall counters), then the bench line itself with
# its CPU baseline.  Usage: tools/profile_rsa.sh <tag> [n]
set -o pipefail
TAG=${1:-round3_rsa}
N=${2:-4194304}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
sha256sum cess_amd/lib/libcess_bls.so > $OUT/lib_sha256.txt
export TMPDIR=/tmp
RX="k_rsa_verify_2048|k_rsa_classify|k_rsa_count|k_rsa_scatter"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --mode rsa --n $N --steps 3 --warmup 1 --cpu-sample 0 > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
echo "trace ok"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_p$i -o run -- python3 bench.py --mode rsa --n $N --steps 1 --warmup 0 --cpu-sample 0 > $OUT/pmc_p$i.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_p$i.log; exit $rc; fi
done
timeout -k 10 300 python3 bench.py --mode rsa --n $N --steps 5 --warmup 1 --cpu-sample 20000 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; exit $rc
