#!/bin/bash
# Round 6: the whole GPU suite + smoke with the pair kernels as defaults and
# the product-split compressed squarings (CESS_PAIR_KCYC_PS=1), then a
# same-box A/B against the component-split squarings (variant kcyc_cs).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -5 gpurun_out/${T}_smoke.txt; exit 3; }
tail -1 gpurun_out/${T}_smoke.txt
TAG=$T bash tools/sweep_ab.sh kcyc_cs noprep
