cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/round3_l_pytest.txt 2>&1 || { tail -30 gpurun_out/round3_l_pytest.txt; exit 1; }
tail -1 gpurun_out/round3_l_pytest.txt
timeout -k 10 300 python -u bench.py --mode sign > gpurun_out/round3_l_bench_sign.json 2> gpurun_out/round3_l_bench_sign.err || { tail gpurun_out/round3_l_bench_sign.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/round3_l_bench_sign.json')); print('sign', d['value'], d['verdicts_ok'], d['roofline']['frac'])"
timeout -k 10 560 bash tools/profile.sh round3_j 1048576 > gpurun_out/round3_j_profile.log 2>&1 || { tail -5 gpurun_out/round3_j_profile.log; exit 1; }
tail -2 gpurun_out/round3_j_profile.log
timeout -k 10 560 bash tools/profile_rsa.sh round3_rsa_c 4194304 > gpurun_out/round3_rsa_c_profile.log 2>&1 || { tail -5 gpurun_out/round3_rsa_c_profile.log; exit 1; }
tail -2 gpurun_out/round3_rsa_c_profile.log
