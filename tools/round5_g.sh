cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/fp_probe > gpurun_out/r5g_fp_probe.txt 2>&1; rc=$?; cat gpurun_out/r5g_fp_probe.txt; [ $rc -eq 0 ] || exit $rc
TAG=round5_g bash tools/sweep_ab.sh mul2
