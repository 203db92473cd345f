#!/bin/bash
# Same-box A/B sweep of library variants (tools/build_variant.sh) on the bench
# workload (config[1], 1 M signatures, 3 timed steps each), the product
# library ("main") run first and last so drift on the box shows.  Prints the
# rate and per-kernel HIP-event stage times of each run.
# Usage (GPU box, repo root): TAG=round5_d bash tools/sweep_ab.sh v1 v2 ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in main "$@" main; do
  if [ "$v" = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  CESS_BLS_LIB=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${TAG}_var_$v.json 2> gpurun_out/${TAG}_var_$v.err || { tail -5 gpurun_out/${TAG}_var_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_var_$v.json')); print('$v', round(d['value']), d['verdicts_ok'], {k: round(v,2) for k,v in d['stage_ms_per_step'].items()})"
done
