#!/bin/bash
# Round 6: fixed-exponent powering with a uniform switch for the window table (field.hpp pow_fixed) against
# the previous build (variant head): the whole GPU suite, then same-box
# bench A/Bs on the per-signature and distinct-key RLC workloads.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6an}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
TAG=$T bash tools/sweep_ab.sh head || exit 1
for v in main head main; do
  if [ "$v" = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  CESS_BLS_LIB=$lib timeout -k 10 300 python bench.py --mode rlcd --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_rlcd_$v.json 2> gpurun_out/${T}_rlcd_$v.err || { tail -5 gpurun_out/${T}_rlcd_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_rlcd_$v.json')); print('rlcd $v', round(d['value']), {k: round(v,2) for k,v in d['stage_ms_per_step'].items()})"
done
