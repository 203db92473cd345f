# round5_s: stall counters of the latency and replay probes (what SQ_WAIT_ANY
# counts when no memory instruction runs)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/r5s_lat -o run -- ./tools/lat_probe > gpurun_out/r5s_lat.log 2>&1 || { tail -5 gpurun_out/r5s_lat.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/r5s_rp -o run -- ./tools/replay_probe > gpurun_out/r5s_rp.log 2>&1 || { tail -5 gpurun_out/r5s_rp.log; exit 1; }
echo done
