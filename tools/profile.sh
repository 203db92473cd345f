#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats.  Passes 2-4: PMC counters, one group per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Usage: tools/profile.sh <tag> [n]
set -o pipefail
TAG=${1:-r01}
N=${2:-1048576}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
sha256sum cess_amd/lib/libcess_bls.so > $OUT/lib_sha256.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BENCH="python3 bench.py --n $N --steps 2 --warmup 1 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
echo "trace ok"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_final|k_miller|k_prepare|k_hash|k_decode_sig|k_decode_pk" --output-format csv -d $OUT/pmc_$name -o run -- python3 bench.py --n $N --steps 1 --warmup 0 --cpu-sample 0 > $OUT/pmc_$name.log 2>&1 || { echo "pmc pass $grp failed"; tail -5 $OUT/pmc_$name.log; }
done
find $OUT -name "*.csv" | head -50
