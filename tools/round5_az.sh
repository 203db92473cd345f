# round5_az: kernel times of the distinct-key RLC bench with 4 forgeries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5az_prof -o run -- python3 bench.py --mode rlcd --forged-count 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r5az.log 2>&1 || { tail -20 gpurun_out/r5az.log; exit 1; }
f=$(find gpurun_out/r5az_prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:26]:
    print(r['Name'].split('(')[0][:40].ljust(40), r['Calls'].rjust(6), '%10.2f ms total' % (float(r['TotalDurationNs'])/1e6), '%10.3f ms avg' % (float(r['AverageNs'])/1e6))
PY
