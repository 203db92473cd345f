cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CESS_BLS_LIB=$PWD/cess_amd/lib_variants/diag/libcess_bls.so timeout -k 10 300 python tools/diag_run.py > gpurun_out/r5b_diag.json 2> gpurun_out/r5b_diag.err || { tail -20 gpurun_out/r5b_diag.err; exit 1; }
cat gpurun_out/r5b_diag.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_rlc.py tests/test_service.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5b_pytest.txt 2>&1; rc=$?; tail -15 gpurun_out/r5b_pytest.txt; exit $rc
