#!/bin/bash
# Round 6: the general 014 product as a loop too (CESS_PAIR_LOOP = 7, bb formed
# inside the first iteration: no spill) against the default 5;
# parity with the loop7 library first (incl. the distinct-key RLC lane kernel).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r6ae}
CESS_BLS_LIB=$PWD/cess_amd/lib_variants/loop7/libcess_bls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_rlc_distinct.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
TAG=$T bash tools/sweep_ab.sh loop7 || exit 1
for v in main loop7 main; do if [ "$v" = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi; CESS_BLS_LIB=$lib timeout -k 10 300 python bench.py --mode rlcd --steps 3 --warmup 1 --cpu-sample 0 --host-steps 0 > gpurun_out/${T}_rlcd_$v.json 2> gpurun_out/${T}_rlcd_$v.err || exit 2; python3 -c "import json; d=json.load(open('gpurun_out/${T}_rlcd_$v.json')); print('rlcd $v', round(d['value']), round(d['stage_ms_per_step']['k_miller'],2))"; done
