#!/bin/bash
# round3_ah: systolic 8-row Montgomery product of the loop-form RSA class
# (main) against the one-row form (prev): big-key rates at 65,536 and
# 1,048,576 records, then the RSA GPU tests with main.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${VARIANTS:-prev main}; do
  if [ $v = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  for n in 65536 1048576; do
    echo "== $v $n"
    CESS_BLS_LIB=$lib timeout -k 10 240 python tools/rsa_big_rate.py $n || exit 1
  done
done
[ -n "$NOTEST" ] && exit 0
timeout -k 10 300 python -u -m pytest tests/test_rsa.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/round3_ah_pytest_rsa.txt 2>&1; rc=$?; tail -3 gpurun_out/round3_ah_pytest_rsa.txt; exit $rc
