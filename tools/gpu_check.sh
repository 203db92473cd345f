# Round check on one MI355X box: -m gpu tests, smoke, the N=1 bench, and a
# rehearsal of the N=2 sharded path (two ranks on GPU 0 over the shared-memory
# transport; its throughput is not an N-GPU figure).  Usage: TAG=round3_x bash tools/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${TAG:-round3}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/${T}_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; cat gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
if [ -n "$REHEARSE" ]; then
  timeout -k 10 300 python bench.py --gpus 2 --transport shm --one-device --n 262144 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${T}_bench_n2_shm.json 2> gpurun_out/${T}_bench_n2_shm.err
  rc=$?; cat gpurun_out/${T}_bench_n2_shm.json; exit $rc
fi
