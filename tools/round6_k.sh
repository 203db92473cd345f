#!/bin/bash
# Round 6: schoolbook dot3 Fp6 products in the pair kernels (main, CESS_PAIR_SB=1)
# against Karatsuba (variant kar): parity files, then a same-box bench A/B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6k}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_rlc_gt_oracle.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
TAG=$T bash tools/sweep_ab.sh kar kar
