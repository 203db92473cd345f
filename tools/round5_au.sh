# round5_au: stall counters of k_miller_rr (distinct-key RLC) beside k_miller's
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/stall_r5au
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY --kernel-include-regex "k_miller" --output-format csv -d $OUT/p1 -o run -- python3 bench.py --mode rlcd --n 1048576 --steps 1 --warmup 0 --cpu-sample 0 > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
f=$(find $OUT/p1 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    key = (k, r["Dispatch_Id"])
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
for (k, d), c in sorted(agg.items()):
    if c["SQ_WAVES"] < 1000: continue
    wc = c["SQ_WAVE_CYCLES"]
    print(k, d, "waves", int(c["SQ_WAVES"]), "WAIT_ANY %.3f" % (c["SQ_WAIT_ANY"] / wc), "WAIT_INST %.3f" % (c["SQ_WAIT_INST_ANY"] / wc),
          "VALU %.3f" % (c["SQ_ACTIVE_INST_VALU"] / wc), "VALU/wave %.3g" % (c["SQ_INSTS_VALU"] / c["SQ_WAVES"]),
          "VMEM_RD/wave %.3g" % (c["SQ_INSTS_VMEM_RD"] / c["SQ_WAVES"]), "cyc/VALU %.2f" % (wc / c["SQ_INSTS_VALU"]))
PY
