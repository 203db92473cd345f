# round5_aw: k_miller_rr kernel time, default vs CESS_MUL014_LOOP (rocprofv3 stats, two rounds)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in default rrloop rrloop2; do
  if [ $v = default ]; then L=$PWD/cess_amd/lib/libcess_bls.so; else L=$PWD/cess_amd/lib_variants/$v/libcess_bls.so; fi
  CESS_BLS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5aw_${v}_$rep -o run -- python3 bench.py --mode rlcd --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r5aw_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r5aw_${v}_$rep.log; exit 1; }
  f=$(find gpurun_out/r5aw_${v}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if r['Name'].startswith('k_miller_rr'): print('$v', $rep, 'k_miller_rr avg %.3f ms' % (float(r['AverageNs'])/1e6))"
done
done
