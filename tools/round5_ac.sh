# round5_ac: distinct-key RLC (CESS_BLS_F_RLC_DISTINCT): GPU tests, then the
# config[1]-shaped bench through it (all valid, and with 4 forgeries)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rlc_distinct.py tests/test_gpu_rlc.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5ac_pytest.txt 2>&1 || { tail -40 gpurun_out/r5ac_pytest.txt; exit 1; }
tail -3 gpurun_out/r5ac_pytest.txt
timeout -k 10 300 python bench.py --mode rlcd --steps 3 --warmup 1 > gpurun_out/r5ac_rlcd.json 2> gpurun_out/r5ac_rlcd.err || { tail -20 gpurun_out/r5ac_rlcd.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5ac_rlcd.json')); print('rlcd', round(d['value']), d['verdicts_ok'], d['ms_per_step'], d['rlc_stats'])"
timeout -k 10 300 python bench.py --mode rlcd --forged-count 4 --steps 3 --warmup 1 > gpurun_out/r5ac_rlcd_f4.json 2> gpurun_out/r5ac_rlcd_f4.err || { tail -20 gpurun_out/r5ac_rlcd_f4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5ac_rlcd_f4.json')); print('rlcd forged4', round(d['value']), d['verdicts_ok'], d['ms_per_step'], d['rlc_stats'])"
