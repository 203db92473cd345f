#!/bin/bash
# Round 6: FE_MUL as a three-iteration loop over one Fp6 product body
# (pair_fe.hpp CESS_PAIR_FE_LOOP, variant feloop) against the default;
# parity with the feloop library first.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6ac}
CESS_BLS_LIB=$PWD/cess_amd/lib_variants/feloop/libcess_bls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_rlc_gt_oracle.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
TAG=$T bash tools/sweep_ab.sh feloop || exit 1
