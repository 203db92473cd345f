# round5_m: in-kernel region stamps, k_miller with and without CESS_MONT_SEP
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in diag diagsep diag; do
  CESS_BLS_LIB=$PWD/cess_amd/lib_variants/$v/libcess_bls.so timeout -k 10 300 python tools/diag_run.py > gpurun_out/r5m_$v.json 2> gpurun_out/r5m_$v.err || { tail -20 gpurun_out/r5m_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5m_$v.json')); k=d['kernels']['k_miller']
print('$v', round(d['sigs_per_s']), {a: round(b,1) for a,b in d['stage_ms_per_step'].items()}, 'clk', round(k['in_kernel_clock_ghz'],3), {a: round(b) for a,b in k['region_cycles_per_wave'].items()})"
done
