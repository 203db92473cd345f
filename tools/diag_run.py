"""Run the bench workload once on a DIAGNOSTIC build (tools/build_variant.sh
diag "-DCESS_DIAG" k_pairing k_final) and print the in-kernel cycle stamps of
k_miller and k_final (bls/diag.hpp): cycles per region summed over waves, each
region's share, and the in-kernel clock d(s_memtime) / d(s_memrealtime) x
100 MHz (MI355X_MICROARCH.md, DVFS item 6).

Usage (GPU box, repo root):
  CESS_BLS_LIB=cess_amd/lib_variants/diag/libcess_bls.so python tools/diag_run.py [--n N] [--reps R]
The first launches warm the chip (>= 2 s of back-to-back work) and are not
recorded; the last `reps` steps are."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REGIONS = {
    "k_miller": ["pair1 loads", "pair1 mul014", "pair0 loads", "pair0 mul014_one", "sqr12", "prologue/epilogue"],
    "k_final": ["other opcodes", "FE_MUL", "FE_INV", "compressed squarings", "decompression", "verdict"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    from cess_amd import bls
    lib = bls.load_library()
    import numpy as np
    import bench
    ctx = bls.Context(device=0, max_batch=min(args.n, 1 << 20), profile=True)
    S, P, M, forged = bench.make_dataset(ctx, args.n, seed=(0x00C0FFEE, 0), forged_frac=0.0)
    d_sig, d_pk, d_msg = ctx.to_device(S), ctx.to_device(P), ctx.to_device(M)
    d_off = ctx.to_device(np.arange(args.n + 1, dtype=np.uint64) * 32)
    wpr = (args.n + 63) // 64
    d_codes, d_bitmap = ctx.device_alloc(wpr * 64), ctx.device_alloc(wpr * 8)
    readers = {}
    for k in REGIONS:
        f = getattr(lib, f"cess_diag_read_{k}")
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        readers[k] = f
    buf = (ctypes.c_ulonglong * 16)()
    for _ in range(args.warmup):
        ctx.verify_device(args.n, d_sig, d_pk, d_msg, d_off, d_codes, d_bitmap)
    ctx.synchronize()
    for f in readers.values():
        assert f(buf, 1) == 16
    ctx.stage_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ctx.verify_device(args.n, d_sig, d_pk, d_msg, d_off, d_codes, d_bitmap)
    ctx.synchronize()
    el = time.perf_counter() - t0
    stages = {k: v[0] for k, v in ctx.stage_stats(reset=True).items() if v[1] > 0}
    codes = np.frombuffer(ctx.from_device(d_codes, wpr * 64), dtype=np.uint8)[: args.n]
    out = {"n": args.n, "reps": args.reps, "sigs_per_s": args.n * args.reps / el, "codes_ok": bool((codes == 0).all()),
           "stage_ms_per_step": {k: v / args.reps for k, v in stages.items()}, "kernels": {}}
    for k, names in REGIONS.items():
        assert readers[k](buf, 0) == 16
        v = list(buf)
        waves, cyc, rt = v[12], v[13], v[14]
        reg = {names[r]: v[r] for r in range(len(names))}
        tot = sum(reg.values())
        out["kernels"][k] = {
            "waves": waves,
            "in_kernel_clock_ghz": cyc / rt * 0.1 if rt else None,
            "cycles_per_wave": cyc / waves if waves else None,
            "region_share": {r: c / tot for r, c in reg.items()} if tot else None,
            "region_cycles_per_wave": {r: c / waves for r, c in reg.items()} if waves else None,
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
