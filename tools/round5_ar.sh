# round5_ar: distinct-key RLC records per Miller lane, 4 (default) vs 8 (variant)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/cess_amd/lib_variants/per8/libcess_bls.so
timeout -k 10 300 env CESS_BLS_LIB=$V python -u -m pytest tests/test_gpu_rlc_distinct.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ar_pytest8.txt 2>&1 || { tail -30 gpurun_out/r5ar_pytest8.txt; exit 1; }
tail -1 gpurun_out/r5ar_pytest8.txt
for rep in 1 2; do
for v in default per8; do
  if [ $v = per8 ]; then L=$V; else L=$PWD/cess_amd/lib/libcess_bls.so; fi
  CESS_BLS_LIB=$L timeout -k 10 300 python bench.py --mode rlcd --steps 5 --cpu-sample 0 > gpurun_out/r5ar_${v}_$rep.json 2> gpurun_out/r5ar_${v}_$rep.err || { tail -20 gpurun_out/r5ar_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5ar_${v}_$rep.json')); print('$v', $rep, round(d['value']), d['verdicts_ok'], d['runtime']['lib_sha256'][:8])"
done
done
