#!/bin/bash
# Round 6: instruction-cache counters of the verify kernels with the lane-pair
# Fp12 kernels (one PMC pass, as tools/round5_probe.sh's first pass).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6aa}
RX="k_final|k_miller|k_prepare|k_decode_pk|k_hash|k_decode_sig"
timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_pmc1 -o run -- python3 bench.py --n 262144 --steps 1 --warmup 0 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_pmc1.log 2>&1
rc=$?
echo "pass 1 rc=$rc"
[ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_pmc1.log; exit $rc; }
find gpurun_out/${T}_pmc1 -name "*counter_collection.csv" | head -3
