#!/bin/bash
# Round 6: scheduler strategy of the lane-pair kernels (Makefile PAIR_SCHED /
# FINAL2_SCHED): max-ilp (mil), max-memory-clause (mmc), iterative-maxocc
# (imo) against the default, same box, config[1] bench; the variants' stage
# times give k_miller2 and k_final2 separately.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
TAG=$T bash tools/sweep_ab.sh mil mmc imo
