# round5_av: k_miller_rr with looped (half-size) sparse-product / squaring
# bodies (CESS_MUL014_LOOP, CESS_SQR12_LOOP, its translation unit only) against
# the default, distinct-key RLC bench, two rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in rrloop rrloop2; do
  CESS_BLS_LIB=$PWD/cess_amd/lib_variants/$v/libcess_bls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rlc_distinct.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5av_pytest_$v.txt 2>&1 || { tail -30 gpurun_out/r5av_pytest_$v.txt; exit 1; }
  tail -1 gpurun_out/r5av_pytest_$v.txt
done
for rep in 1 2; do
for v in default rrloop rrloop2; do
  if [ $v = default ]; then L=$PWD/cess_amd/lib/libcess_bls.so; else L=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  CESS_BLS_LIB=$L timeout -k 10 300 python bench.py --mode rlcd --steps 5 --cpu-sample 0 > gpurun_out/r5av_${v}_$rep.json 2> gpurun_out/r5av_${v}_$rep.err || { tail -20 gpurun_out/r5av_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5av_${v}_$rep.json')); print('$v', $rep, round(d['value']), d['verdicts_ok'])"
done
done
