TAG=round3_t bash tools/sweep_variants.sh head main noload noloadpt || exit 1
for v in head main; do
  if [ $v = main ]; then lib=$PWD/cess_amd/lib/libcess_bls.so; else lib=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  CESS_BLS_LIB=$lib timeout -k 10 300 python bench.py --mode adversarial --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/round3_t_adv_$v.json 2> gpurun_out/round3_t_adv_$v.err || exit 2
  python3 -c "import json; d=json.load(open('gpurun_out/round3_t_adv_$v.json')); print('adv $v', round(d['value']), d['verdicts_ok'], {k: round(v,1) for k,v in d['stage_ms_per_step'].items()})"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/round3_t_pytest.txt 2>&1; tail -3 gpurun_out/round3_t_pytest.txt
