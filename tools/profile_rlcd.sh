#!/bin/bash
# rocprofv3 passes for the distinct-key RLC bench (bench.py --mode rlcd, run on
# the GPU box from the repo root): kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE (separate passes) of k_miller_rr, k_hash and k_decode_sig.
# Usage: tools/profile_rlcd.sh <tag>   -> gpurun_out/prof_<tag>_rlcd
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/prof_${TAG}_rlcd
mkdir -p $OUT
sha256sum cess_amd/lib/libcess_bls.so > $OUT/lib_sha256.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BENCH="python3 bench.py --mode rlcd --steps 1 --warmup 0 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
echo "trace ok"
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_miller_rr|k_hash|k_decode_sig" --output-format csv -d $OUT/pmc_$grp -o run -- $BENCH > $OUT/pmc_$grp.log 2>&1 || { echo "pmc pass $grp failed"; tail -5 $OUT/pmc_$grp.log; exit 2; }
done
echo "pmc ok"
