#!/bin/bash
# Round 6: smaller Miller step bodies for the instruction cache
# (pair.hpp CESS_PAIR_LOOP): psqr12's two Fp6 products as a loop (loop1),
# plus the normalised 014 product's two halves (loop5), against the default;
# parity with the loop5 library first.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6ab}
CESS_BLS_LIB=$PWD/cess_amd/lib_variants/loop5/libcess_bls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
TAG=$T bash tools/sweep_ab.sh loop1 loop5 || exit 1
