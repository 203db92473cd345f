cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r02a}_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/${TAG:-r02a}_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r02a}_smoke.txt 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG:-r02a}_bench.json 2> gpurun_out/${TAG:-r02a}_bench.err
rc=$?; cat gpurun_out/${TAG:-r02a}_bench.json; exit $rc
