cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/icache_probe > gpurun_out/r5c_icache_probe.txt 2>&1 || { cat gpurun_out/r5c_icache_probe.txt; exit 1; }
cat gpurun_out/r5c_icache_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_rlc.py tests/test_service.py tests/test_c_abi.py tests/test_cabi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5c_pytest.txt 2>&1; rc=$?; tail -15 gpurun_out/r5c_pytest.txt; exit $rc
