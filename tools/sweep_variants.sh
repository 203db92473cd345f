#!/bin/bash
# Stage times of library variants (tools/build_variant.sh) on the bench workload.
# Usage (GPU box, repo root): TAG=r02g bash tools/sweep_variants.sh main w1norm ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  CESS_BLS_LIB=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG}_var_$v.json 2> gpurun_out/${TAG}_var_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_var_$v.json')); print('$v', round(d['value']), d['verdicts_ok'], {k: round(v,1) for k,v in d['stage_ms_per_step'].items()})"
done
