# round5_v: k_final in-kernel region stamps with the slots in HBM (diag) and
# L2-resident (diagl2, CESS_FE_L2PROBE: wrong verdicts, timing only)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in diag diagl2; do
  CESS_BLS_LIB=$PWD/cess_amd/lib_variants/$v/libcess_bls.so timeout -k 10 300 python tools/diag_run.py > gpurun_out/r5v_$v.json 2> gpurun_out/r5v_$v.err || { tail -20 gpurun_out/r5v_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5v_$v.json')); k=d['kernels']['k_final']
print('$v', round(d['stage_ms_per_step']['k_final'],1), 'clk', round(k['in_kernel_clock_ghz'],3), {a: round(b) for a,b in k['region_cycles_per_wave'].items()})"
done
