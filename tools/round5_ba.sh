# round5_ba: k_rlcd_scale at one wave per SIMD (512 registers, no scratch)
# against two waves (256 registers, 184 B/lane of scratch): kernel times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/cess_amd/lib_variants/w1/libcess_bls.so
CESS_BLS_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_rlc_distinct.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ba_pytest.txt 2>&1 || { tail -30 gpurun_out/r5ba_pytest.txt; exit 1; }
tail -1 gpurun_out/r5ba_pytest.txt
for rep in 1 2; do
for v in default w1; do
  if [ $v = default ]; then L=$PWD/cess_amd/lib/libcess_bls.so; else L=$V; fi
  CESS_BLS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ba_${v}_$rep -o run -- python3 bench.py --mode rlcd --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r5ba_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r5ba_${v}_$rep.log; exit 1; }
  f=$(find gpurun_out/r5ba_${v}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if r['Name'].startswith('k_rlcd_scale'): print('$v', $rep, 'k_rlcd_scale calls', r['Calls'], 'avg %.3f ms' % (float(r['AverageNs'])/1e6))"
done
done
