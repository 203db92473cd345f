#!/bin/bash
# round3_z: k_miller with the G1 points held in registers (main) against the
# build before (head): stage times on the bench workload and k_miller's
# FETCH_SIZE / WRITE_SIZE (one PMC pass each).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=round3_z bash tools/sweep_variants.sh head main head main || exit 1
for v in head main; do
  if [ $v = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    CESS_BLS_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex k_miller --output-format csv -d gpurun_out/round3_z_${v}_$c -o run -- python3 bench.py --n 262144 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/round3_z_${v}_$c.log 2>&1 || exit 2
  done
done
echo pmc ok
