# round5_ad: kernel times of the distinct-key RLC bench (rocprofv3 stats)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ad_prof -o run -- python3 bench.py --mode rlcd --steps 2 --warmup 1 > gpurun_out/r5ad.log 2>&1 || { tail -20 gpurun_out/r5ad.log; exit 1; }
f=$(find gpurun_out/r5ad_prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print(r['Name'].split('(')[0][:40].ljust(40), r['Calls'].rjust(6), '%10.2f ms total' % (float(r['TotalDurationNs'])/1e6), '%10.3f ms avg' % (float(r['AverageNs'])/1e6))
PY
