#!/bin/bash
# round3_al: non-temporal loads of the per-signature coefficient rows in
# k_miller (mnt) against the build (main): stage times (two passes), k_miller
# FETCH_SIZE + WRITE_SIZE, then the -m gpu tests with mnt.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=round3_al bash tools/sweep_variants.sh main mnt main mnt || exit 1
for v in main mnt; do
  if [ $v = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    CESS_BLS_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex "k_miller" --output-format csv -d gpurun_out/round3_al_${v}_$c -o run -- python3 bench.py --n 262144 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/round3_al_${v}_$c.log 2>&1 || exit 2
  done
done
CESS_BLS_LIB=$PWD/cess_amd/lib_variants/mnt/libcess_bls.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/round3_al_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/round3_al_pytest.txt; exit $rc
