# round5_o: latency probe, the GPU suite, smoke and one default bench run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/lat_probe > gpurun_out/r5o_lat_probe.txt 2>&1 || { cat gpurun_out/r5o_lat_probe.txt; exit 1; }
cat gpurun_out/r5o_lat_probe.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5o_pytest.txt 2>&1 || { tail -30 gpurun_out/r5o_pytest.txt; exit 1; }
tail -3 gpurun_out/r5o_pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5o_smoke.txt 2>&1 || { tail -20 gpurun_out/r5o_smoke.txt; exit 1; }
tail -1 gpurun_out/r5o_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r5o_bench.json 2> gpurun_out/r5o_bench.err || { tail -20 gpurun_out/r5o_bench.err; exit 1; }
cat gpurun_out/r5o_bench.json
