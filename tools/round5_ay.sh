# round5_ay: k_final with the two-pass compressed-squaring loop (CESS_KCYC_LOOP,
# half the loop body's code) against the default: kernel times, two rounds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/cess_amd/lib_variants/kcyc/libcess_bls.so
CESS_BLS_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ay_pytest.txt 2>&1 || { tail -30 gpurun_out/r5ay_pytest.txt; exit 1; }
tail -1 gpurun_out/r5ay_pytest.txt
for rep in 1 2; do
for v in default kcyc; do
  if [ $v = default ]; then L=$PWD/cess_amd/lib/libcess_bls.so; else L=$V; fi
  CESS_BLS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ay_${v}_$rep -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r5ay_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r5ay_${v}_$rep.log; exit 1; }
  f=$(find gpurun_out/r5ay_${v}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if r['Name'].startswith('k_final'): print('$v', $rep, 'k_final calls', r['Calls'], 'avg %.3f ms' % (float(r['AverageNs'])/1e6))"
done
done
