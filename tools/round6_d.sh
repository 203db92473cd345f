#!/bin/bash
# Round 6: the whole GPU suite with k_miller2 as the default Miller kernel
# (and the new RLC Gt-vs-oracle file), then smoke().
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -5 gpurun_out/${T}_smoke.txt; exit 3; }
tail -1 gpurun_out/${T}_smoke.txt
