"""Benchmark: verified BLS12-381 signatures/s on MI355X (BASELINE.json metric).

Workloads (one process per GPU):
  N = 1 : BASELINE config[1] -- 1,048,576 independent signatures with distinct
          random keys over 32-byte messages, per-signature two-pairing verify.
  N > 1 : BASELINE config[2] shape -- 2,097,152 signatures per GPU (16 M at
          N = 8) sharded by index; each rank verifies its shard and the verdict
          bitmap words (and code bytes) are all-gathered over RCCL (xGMI) INSIDE
          the library (cess_bls_verify_batch_sharded_device), so every rank
          holds the whole batch's verdicts.  Weak scaling: fixed work per GPU.

A "step" = one verify_batch over the shard (inputs resident in HBM) + the
all-gather.  Keys/signatures are generated on the GPU with the library's own
keygen/sign kernels (untimed); their parity with the CPU oracle is pinned by the
tests.

Launch: `python bench.py --gpus N` with no WORLD_SIZE in the environment starts
N ranks itself (torch.distributed.run, 127.0.0.1) from this parent, which never
touches the GPU; under torchrun (the driver's form) each rank runs directly.

Runtime provenance: libcess_bls.so is loaded BEFORE anything else can pull in a
HIP runtime, and the data path never calls torch, so the kernels and RCCL are
the /opt/rocm builds the tests use; the JSON line records the mapped
libamdhip64 / librccl paths and the library's SHA-256, and `roofline.traffic`
is taken only from a PMC profile of that same library build.

Prints ONE JSON line on rank 0 (contract in the task brief), including
`roofline` (dominant kernel vs the v_mad_u64_u32 peak) and `cpu_baseline`
(CPU ports on a bounded sample: the 64-bit-limb restatement
tests/hostemu/cpu64_verify.cpp as the main value, the kernels' 32-bit-limb
algorithms for the host, tests/hostemu/cpu_verify.cpp, as "alt").
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# v_mad_u64_u32 peak (integer-multiply roofline): 256 CUs x 64 lanes/clk (half
# rate; measured 53 lane-ops/CU/clk at the nominal clock by tools/mad_peak.hip,
# profiles/r01_mad_peak.txt) x 2.4 GHz.
PEAK_MADS = 256 * 64 * 2.4e9
ALG_MADS_PER_FP_MUL = 288   # 12^2 (a*b) + 12^2 (m*p) 32x32-bit limb products
N1_DEFAULT = 1 << 20        # config[1]
NPER_MULTI = 1 << 21        # config[2]: 16 M over 8 GPUs


def parse():
    """Command-line flags; ranks started by launch() receive the parent's flags
    through CESS_BENCH_ARGV (torch.distributed.run would otherwise try to
    prefix-match flags such as --n against its own options)."""
    argv = json.loads(os.environ["CESS_BENCH_ARGV"]) if "CESS_BENCH_ARGV" in os.environ else None
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=None,
                    help="signatures per GPU (default: 1,048,576 at N=1 = config[1]; 2,097,152 at N>1 = config[2])")
    ap.add_argument("--forged-frac", type=float, default=0.0)
    ap.add_argument("--cpu-sample", type=int, default=40960, help="records for the CPU baseline (0: skip)")
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                    help="host threads for the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--mode", choices=["persig", "rlc", "rlcd", "adversarial", "keyed", "rsa", "sign"], default="persig",
                    help="persig: BASELINE config[1]/[2] (default); rlc: config[3] shape (few keys, RLC batch "
                         "mode + Gt-partial all-gather); adversarial: config[4] shape (1%% invalid mix, exact codes); "
                         "keyed: config[3] shape with per-signature verdicts; rsa: SURVEY §8(f) rank 4, RSA-2048 "
                         "PKCS#1 v1.5 raw verify (cp_enclave_verify::verify_rsa) over 32-byte messages; sign: SURVEY §8(f) "
                         "rank 3, batch PrivateKey::sign")
    ap.add_argument("--host-steps", type=int, default=2,
                    help="N=1 persig: extra steps from host buffers (cess_bls_verify_batch incl. PCIe), reported as "
                         "host_buffers_sigs_per_s beside the device-resident value (0: skip)")
    ap.add_argument("--keys", type=int, default=16, help="distinct keys (rlc / keyed modes)")
    ap.add_argument("--forged-count", type=int, default=0, help="forgeries per rank (rlc mode)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rendezvous/sharding only, no GPU (CPU test of the N>1 path)")
    ap.add_argument("--transport", choices=["rccl", "shm"], default="rccl",
                    help="communicator of the sharded entry points: rccl (xGMI, one GPU per rank; default) or "
                         "shm (host shared memory: ranks may share a GPU -- a rehearsal of the N>1 path on one box)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on GPU 0 (with --transport shm: N>1 rehearsal on a one-GPU box; the "
                         "throughput is then NOT an N-GPU figure)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher + rendezvous (no GPU in this process)
# ---------------------------------------------------------------------------
def node_gpu_count():
    """GPUs this job may use, counted WITHOUT a HIP call (the launcher parent
    must not initialise the GPU): KFD topology nodes that have SIMDs, narrowed
    by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.
    CESS_BENCH_DEVICE_COUNT overrides it (the CPU test of the fail-fast path).
    None when it cannot be told (no KFD topology: a CPU container)."""
    o = os.environ.get("CESS_BENCH_DEVICE_COUNT")
    if o is not None:
        return int(o)
    topo = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for d in os.listdir(topo):
            with open(os.path.join(topo, d, "properties")) as f:
                props = dict(line.split() for line in f if len(line.split()) == 2)
            n += int(props.get("simd_count", "0")) > 0
    except OSError:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def fail(kind: str, code: int, **info):
    """One JSON error line on stderr and a non-zero exit, before any rank has
    a communicator (nothing to hang on, nothing to abort)."""
    print(json.dumps(dict({"error": kind}, **info)), file=sys.stderr, flush=True)
    sys.exit(code)


def launch(args) -> int:
    """Start args.gpus ranks with torch.distributed.run and return its exit code.
    This parent process makes no HIP call (it only imports the launcher).  A
    node with fewer visible GPUs than ranks fails here, before any rank starts
    (each rank checks again under an external torchrun)."""
    ndev = node_gpu_count()
    if ndev is not None and ndev < args.gpus and not args.one_device and (
            not args.dry_run or "CESS_BENCH_DEVICE_COUNT" in os.environ):
        fail("devices", 4, need=args.gpus, visible=ndev, where="launcher")
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               CESS_BENCH_ARGV=json.dumps(sys.argv[1:]))
    return subprocess.call(cmd, env=env)


def rdv_dir() -> str:
    """Per-job rendezvous directory: all ranks of one torchrun job share the
    agent (parent) pid and the master port."""
    key = f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"
    d = os.path.join(tempfile.gettempdir(), f"cess_bls_rdv_{key}")
    os.makedirs(d, exist_ok=True)
    return d


def rdv_put(name: str, data: bytes):
    d = rdv_dir()
    tmp = os.path.join(d, f".{name}.{os.getpid()}")
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, os.path.join(d, name))


def rdv_get(name: str, timeout: float = None) -> bytes:
    """Wait for rank 0's file; bounded by the same deadline as the
    communicator (CESS_BLS_COMM_TIMEOUT_MS, 120 s by default for N > 1)."""
    if timeout is None:
        timeout = float(os.environ.get("CESS_BLS_COMM_TIMEOUT_MS", "120000")) / 1000.0
    p = os.path.join(rdv_dir(), name)
    t0 = time.time()
    while not os.path.exists(p):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"rendezvous: {p} never appeared")
        time.sleep(0.05)
    with open(p, "rb") as f:
        return f.read()


def rdv_cleanup(rank: int, world: int):
    if rank == 0:
        import shutil
        shutil.rmtree(rdv_dir(), ignore_errors=True)


def comm_setup(ctx, rank: int, world: int, transport: str = "rccl", one_device: bool = False) -> dict:
    """ncclUniqueId (or the shared-memory job name) from rank 0 to every rank
    (file rendezvous), then the communicator inside the library.  Returns what
    the communicator itself reports (cess_bls_comm_info: a collective, every
    rank asks); under RCCL with one GPU per rank the job must span WORLD_SIZE
    distinct devices, else every rank exits non-zero here, before any data."""
    from cess_amd import bls
    if transport == "shm":
        if rank == 0:
            rdv_put("comm_name", bls.comm_shm_name().encode())
        ctx.comm_init_shm(world, rank, rdv_get("comm_name").decode())
        ctx.comm_barrier()
        rdv_cleanup(rank, world)
    else:
        if rank == 0:
            rdv_put("comm_id", bls.comm_id())
        cid = rdv_get("comm_id")
        try:
            ctx.comm_init(world, rank, cid)
            ctx.comm_barrier()
        except bls.BlsInfraError as ex:
            # a peer never arrived (CESS_BLS_COMM_TIMEOUT_MS) or RCCL failed: exit
            # non-zero at once.  _exit, because a rank whose RCCL bootstrap never
            # completed keeps a helper thread blocked inside RCCL (include/cess_bls.h)
            print(json.dumps({"error": "communicator", "status": ex.status, "rank": rank, "message": str(ex)}),
                  file=sys.stderr, flush=True)
            os._exit(3)
        rdv_cleanup(rank, world)
    ci = ctx.comm_info()
    info = {"kind": ctx.comm_kind, "nranks": ci["nranks"], "rank": ci["rank"], "bus_ids": ci["bus_ids"],
            "distinct_devices": len(set(ci["bus_ids"]))}
    if info["nranks"] != world or info["rank"] != rank:
        print(json.dumps(dict(info, error="communicator shape", world=world)), file=sys.stderr, flush=True)
        os._exit(5)
    if transport == "rccl" and not one_device and info["distinct_devices"] != world:
        # every rank saw the same gathered bus ids, so every rank exits here
        print(json.dumps(dict(info, error="ranks share a device", world=world)), file=sys.stderr, flush=True)
        os._exit(5)
    return info


def runtime_provenance() -> dict:
    maps = {}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.strip() else ""
                for key in ("libamdhip64", "librccl", "libcess_bls"):
                    if key in p and "/" in p:
                        maps.setdefault(key, p)
    except OSError:
        pass
    return maps


def lib_sha256() -> str:
    p = os.path.join(ROOT, "cess_amd", "lib", "libcess_bls.so")
    with open(p, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


# resident waves per SIMD of the two Fp12 kernels, fixed by their LDS images:
# the Miller stage runs k_miller2 (a lane pair per signature, 72 KiB per
# 128-signature block, two blocks per CU) unless CESS_BLS_MILLER=lane selects
# the one-lane k_miller (144 KiB per block, one wave per SIMD); k_final 72 KiB
# 
WAVES_PER_SIMD = {"k_miller": 1 if os.environ.get("CESS_BLS_MILLER") == "lane" else 2, "k_final": 2}
# the kernel that runs a stage (its name in the rocprofv3 PMC summaries): the
# lane-pair kernels by default, the one-lane ones with CESS_BLS_MILLER / _FINAL = lane
KERNEL_OF_STAGE = {"k_miller": "k_miller" if os.environ.get("CESS_BLS_MILLER") == "lane" else "k_miller2",
                   "k_final": "k_final" if os.environ.get("CESS_BLS_FINAL") == "lane" else "k_final2"}


def load_opcount():
    with open(os.path.join(ROOT, "profiles", "opcount.json")) as f:
        return json.load(f)


def load_pmc_traffic(sha: str, kernel=None, n=None):
    """HBM bytes per launch from a committed rocprofv3 PMC summary
    (profiles/*_pmc_traffic.json) measured on THIS library build (same
    SHA-256), for `kernel` at launch size `n` when given; None when no profile
    of this build exists."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json"))):
        with open(p) as f:
            d = json.load(f)
        if d.get("lib_sha256") != sha:
            continue
        if kernel is not None and kernel not in d.get("all", {}):
            continue
        if n is not None and d.get("n") != n:
            continue
        d["_file"] = os.path.relpath(p, ROOT)
        return d
    return None


# ---------------------------------------------------------------------------
# synthetic datasets (generated on the GPU by the library's keygen/sign kernels)
# ---------------------------------------------------------------------------
def make_dataset(ctx, n, seed, forged_frac):
    import numpy as np
    rng = np.random.default_rng(seed)
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x3F          # < 2^254 < r
    sk[:, 31] |= 1            # nonzero
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    P = ctx.public_keys_raw(sk.tobytes())
    sign_msgs = msgs.copy()
    forged = np.zeros(n, dtype=bool)
    if forged_frac > 0:
        idx = rng.choice(n, size=max(1, int(n * forged_frac)), replace=False)
        forged[idx] = True
        sign_msgs[idx, 0] ^= 0xFF      # valid signature over a different message
    offs = np.arange(n + 1, dtype=np.uint64) * 32
    S = ctx.sign_raw(sk.tobytes(), sign_msgs.tobytes(), offs)
    return S, P, msgs.tobytes(), forged


def make_keyed_dataset(ctx, n, k, seed, forged_frac):
    """Few-keys workload (BASELINE config[3]'s shape, per-signature verdicts):
    k distinct keys, signature i by key i % k over its own 32-byte message."""
    import numpy as np
    rng = np.random.default_rng(seed)
    sk = rng.integers(0, 256, size=(k, 32), dtype=np.uint8)
    sk[:, 0] &= 0x3F
    sk[:, 31] |= 1
    kp = ctx.public_keys_raw(sk.tobytes())
    pks = [kp[96 * j:96 * j + 96] for j in range(k)]
    who = (np.arange(n) % k).astype(np.uint32)
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sign_msgs = msgs.copy()
    forged = np.zeros(n, dtype=bool)
    if forged_frac > 0:
        idx = rng.choice(n, size=max(1, int(n * forged_frac)), replace=False)
        forged[idx] = True
        sign_msgs[idx, 0] ^= 0xFF
    offs = np.arange(n + 1, dtype=np.uint64) * 32
    S = ctx.sign_raw(sk[who].tobytes(), sign_msgs.tobytes(), offs)
    return S, pks, who, msgs.tobytes(), forged


def inject_adversarial(S, P, M, n, seed, frac=0.01):
    """BASELINE config[4] mix: `frac` of the records invalid -- half forged
    (valid signature over another message, code 5), half replaced by the
    fixed-length adversarial golden records (non-subgroup and off-curve points,
    x >= p, bad flag combinations, identity pairs; tests/golden/vectors.json,
    generated by the oracle).  Returns the new buffers and expected codes."""
    import numpy as np
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        cases = [c for c in json.load(f)["cases"]
                 if len(c["sig"]) == 96 and len(c["pk"]) == 192 and len(c["msg"]) == 64]
    rng = np.random.default_rng(seed)
    S, P, M = bytearray(S), bytearray(P), bytearray(M)
    expect = np.zeros(n, dtype=np.uint8)
    idx = rng.choice(n, size=max(2, int(n * frac)), replace=False)
    half = len(idx) // 2
    for i in idx[:half]:
        M[32 * i] ^= 0xFF
        expect[i] = 5
    for j, i in enumerate(idx[half:]):
        c = cases[j % len(cases)]
        S[48 * i:48 * i + 48] = bytes.fromhex(c["sig"])
        P[96 * i:96 * i + 96] = bytes.fromhex(c["pk"])
        M[32 * i:32 * i + 32] = bytes.fromhex(c["msg"])
        expect[i] = c["code"]
    return bytes(S), bytes(P), bytes(M), expect, len(cases)


CPU_LIB = os.path.join(ROOT, "tests", "hostemu", "libcpu_verify.so")
CPU64_LIB = os.path.join(ROOT, "tests", "hostemu", "libcpu64_verify.so")


def _time_cpu_lib(path, fn, sigs, msgs, pks, n, threads):
    import ctypes
    lib = ctypes.CDLL(path)
    codes = (ctypes.c_uint8 * n)()
    t = time.perf_counter()
    if fn == "cpu64_verify_batch":
        offs = (ctypes.c_uint64 * (n + 1))(*[32 * i for i in range(n + 1)])
        lib.cpu64_verify_batch(ctypes.c_uint64(n), sigs, pks, msgs, offs, codes, ctypes.c_int(threads))
    else:
        lib.cpu_verify_batch(ctypes.c_uint64(n), sigs, msgs, ctypes.c_uint32(32), pks, codes, ctypes.c_int(threads))
    return time.perf_counter() - t, sum(1 for c in codes if c == 0)


def cpu_baseline(S, M, P, idx, threads):
    """CPU baselines (reported, not a target) on a bounded sample of the same
    records, std::thread x `threads`.  The reference crate (Rust bls12_381
    0.7.1) cannot be built in this image, so both are kind
    "port":
      * main: tests/hostemu/cpu64_verify.cpp -- the crate's representation,
        6 x u64 Montgomery limbs with unsigned __int128;
      * "alt": tests/hostemu/cpu_verify.cpp -- the kernels' own 32-bit-limb
        algorithms compiled for the host (-DCESS_HOSTEMU)."""
    if not idx:
        return None
    n = len(idx)
    sigs = b"".join(S[48 * i:48 * i + 48] for i in idx)
    msgs = b"".join(M[32 * i:32 * i + 32] for i in idx)
    pks = b"".join(P[96 * i:96 * i + 96] for i in idx)
    out = {}
    for key, path, fn, what in (
            ("main", CPU64_LIB, "cpu64_verify_batch",
             "tests/hostemu/cpu64_verify.cpp: 6 x u64 Montgomery (the crate's limb layout), g++ -O3"),
            ("alt", CPU_LIB, "cpu_verify_batch",
             "tests/hostemu/cpu_verify.cpp: the kernels' 32-bit-limb algorithms for the host, g++ -O3")):
        if not os.path.exists(path):
            out[key] = {"value": None, "unit": "sigs/s", "cores": 0, "kind": "port",
                        "sample": f"skipped: {os.path.relpath(path, ROOT)} not built (run __graft_entry__.build())"}
            continue
        dt, ok = _time_cpu_lib(path, fn, sigs, msgs, pks, n, threads)
        out[key] = {"value": n / dt, "unit": "sigs/s", "cores": threads, "kind": "port",
                    "sample": f"{n} records of the same workload (distinct keys, 32-byte msgs), {what}, "
                              f"{threads} std::threads, {dt:.1f}s wall; not the reference crate",
                    "codes_ok": ok}
    rec = dict(out["main"])
    rec["alt"] = out["alt"]
    return rec


# RSA-2048 PKCS#1 v1.5 raw verify (e = 65537), algorithmic work per signature
# in 32x32-bit limb products: to-Montgomery product (2 * 64^2), 16 squarings
# (64 * 65 / 2 + 64^2 each), the final product (2 * 64^2) and the reduction out
# of Montgomery form (64^2)
RSA2048_ALG_MADS = 2 * 64 * 64 + 16 * (64 * 65 // 2 + 64 * 64) + 2 * 64 * 64 + 64 * 64


def cpu_baseline_rsa(pool, n, e, sample):
    """CPU baseline for the RSA mode (reported, not a target): the oracle's
    restatement (oracle/rsa_oracle.py verify_code: CPython big-int pow + the
    EMSA check), one thread, on a bounded sample of the same records."""
    from oracle import rsa_oracle as o
    t = time.perf_counter()
    ok = sum(1 for i in range(sample) if o.verify_code(n, e, pool[i % len(pool)][0], pool[i % len(pool)][1]) == 0)
    dt = time.perf_counter() - t
    return {"value": sample / dt, "unit": "sigs/s", "cores": 1, "kind": "port",
            "sample": f"{sample} records of the same workload through oracle/rsa_oracle.py (CPython pow), 1 thread, "
                      f"{dt:.1f}s; not the rsa crate", "codes_ok": ok}


def run_rsa(args, ctx, rank, world):
    """batch RSA-2048 PKCS#1 v1.5 raw verification
    (cp_enclave_verify::verify_rsa) with inputs resident in HBM: n records
    over the committed pool of valid signatures (tests/golden/rsa_vectors.json,
    key 0), 1 % corrupted; codes checked against the construction."""
    import numpy as np
    n = args.n or (1 << 22)
    with open(os.path.join(ROOT, "tests", "golden", "rsa_vectors.json")) as f:
        rv = json.load(f)
    key = bytes.fromhex(rv["keys"][0]["spki"])
    assert ctx.rsa_keys_load([key]) == [0]
    pool = [(bytes.fromhex(p["msg"]), bytes.fromhex(p["sig"])) for p in rv["bench_pool_key0"]]
    rng = np.random.default_rng((0x525341, rank))
    pick = rng.integers(0, len(pool), size=n)
    M = np.frombuffer(b"".join(p[0] for p in pool), dtype=np.uint8).reshape(len(pool), 32)[pick].copy()
    S = np.frombuffer(b"".join(p[1] for p in pool), dtype=np.uint8).reshape(len(pool), 256)[pick].copy()
    bad = rng.choice(n, size=max(1, n // 100), replace=False)
    M[bad, 0] ^= 0xFF                                   # message no longer matches: code 4
    expect = np.zeros(n, dtype=np.uint8)
    expect[bad] = 4
    d_idx = ctx.to_device(np.zeros(n, dtype=np.uint32))
    d_sig = ctx.to_device(S)
    d_soff = ctx.to_device(np.arange(n + 1, dtype=np.uint64) * 256)
    d_msg = ctx.to_device(M)
    d_moff = ctx.to_device(np.arange(n + 1, dtype=np.uint64) * 32)
    d_codes = ctx.device_alloc(n)

    def step():
        ctx.rsa_verify_batch_device(n, d_idx, d_sig, d_soff, d_msg, d_moff, d_codes)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    ctx.stage_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    elapsed = time.perf_counter() - t0
    # HIP events around each launch on its stream (CESS_BLS_F_PROFILE)
    st = {k: v for k, v in ctx.stage_stats(reset=True).items() if v[1] > 0}
    codes = np.frombuffer(ctx.from_device(d_codes, n), dtype=np.uint8)
    ok = bool((codes == expect).all())
    if world > 1:
        elapsed = ctx.comm_max(elapsed)
        ok = ctx.comm_max(0.0 if ok else 1.0) == 0.0
    if rank == 0:
        value = n * world * args.steps / elapsed
        ver_ms, ver_launches = st["k_rsa_verify"]
        assert ver_launches == args.steps, st
        verify_ms = ver_ms / ver_launches                  # average launch duration, HIP events
        achieved = n * RSA2048_ALG_MADS / (verify_ms * 1e-3)
        sha = lib_sha256()
        # one key, many records: the key-uniform kernel (host_rsa.cpp policy)
        pmc = load_pmc_traffic(sha, "k_rsa_verify_2048u", n)
        kd = (pmc or {}).get("all", {}).get("k_rsa_verify_2048u", {})
        cpu = None
        if world == 1 and args.cpu_sample > 0:
            kn, ke = bls_rsa_key(key)
            cpu = cpu_baseline_rsa([(bytes(M[i]), bytes(S[i])) for i in range(256)], kn, ke, min(args.cpu_sample, 20000))
        print(json.dumps({
            "metric": "verified RSA-2048 PKCS#1 v1.5 (raw) sigs/sec", "value": value, "unit": "sigs/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32 (2048-bit Montgomery, 74x28-bit limb products via v_mad_u64_u32)",
            "data": "synthetic: 256 distinct valid raw signatures under one 2048-bit key (e = 65537, committed "
                    "fixture pool) replicated, 1% corrupted messages",
            "config": {"workload": f"SURVEY §8(f) rank 4, cp_enclave_verify::verify_rsa: {n} sigs per GPU, inputs in HBM",
                       "parallelism": f"shard-by-index x{world}"},
            "verdicts_ok": ok,
            "stage_ms_per_step": {k: v[0] / args.steps for k, v in st.items()},
            "roofline": {"bound": "valu-int", "kernel": "k_rsa_verify_2048u",
                         "achieved": achieved / 1e12, "peak": PEAK_MADS / 1e12,
                         "unit": "T mad/s (32x32-bit limb products, v_mad_u64_u32)", "frac": achieved / PEAK_MADS,
                         "traffic": kd.get("hbm_bytes_per_launch"), "traffic_source": pmc["_file"] if pmc else None,
                         "pmc_valu_active_per_wave": (kd["SQ_ACTIVE_INST_VALU"] / kd["SQ_WAVE_CYCLES"]
                                                      if kd.get("SQ_WAVE_CYCLES") else None),
                         "alg_mads_per_sig": RSA2048_ALG_MADS,
                         "whole_step_frac": value / world * RSA2048_ALG_MADS / PEAK_MADS,
                         "note": "achieved = algorithmic mads of one launch / its HIP-event duration; 28-bit limbs "
                                 "issue 74^2-based products (1.34x the 32-bit count)"},
            "cpu_baseline": cpu,
            "runtime": dict(runtime_provenance(), lib_sha256=sha),
        }), flush=True)
    for p in (d_idx, d_sig, d_soff, d_msg, d_moff, d_codes):
        ctx.device_free(p)


def bls_rsa_key(der):
    from cess_amd import bls
    mod, e = bls.rsa_parse_key(der)
    return int.from_bytes(mod, "big"), e


# ---------------------------------------------------------------------------
# rank body
# ---------------------------------------------------------------------------
def run_sign(args, ctx, rank, world):
    """the TEE side's batch signer, PrivateKey::sign
    (src/lib.rs:233-236) = compress([sk] H(m)), n records resident in HBM
    (cess_bls_sign_batch_device, one k_sign launch per step).  Untimed check:
    every signature verifies against its key (cess_bls_verify_batch_device)."""
    import numpy as np
    n = args.n or N1_DEFAULT
    rng = np.random.default_rng((0x5167, rank))
    sk = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sk[:, 0] &= 0x3F                                   # < 2^254 < r
    M = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    d_sk = ctx.to_device(sk)
    d_msg = ctx.to_device(M)
    d_off = ctx.to_device(np.arange(n + 1, dtype=np.uint64) * 32)
    d_sig = ctx.device_alloc(48 * n)

    def step():
        ctx.sign_device(n, d_sk, d_msg, d_off, d_sig)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    if world > 1:
        ctx.comm_barrier()
    ctx.stage_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    if world > 1:
        ctx.comm_barrier()
    elapsed = time.perf_counter() - t0
    st = {k: v for k, v in ctx.stage_stats(reset=True).items() if v[1] > 0}
    # untimed: the signatures verify against keys from the keygen kernel
    pks = ctx.public_keys_raw(sk.tobytes())
    d_pk = ctx.to_device(np.frombuffer(pks, dtype=np.uint8))
    d_codes = ctx.device_alloc(n)
    d_bm = ctx.device_alloc(8 * ((n + 63) // 64))
    ctx.verify_device(n, d_sig, d_pk, d_msg, d_off, d_codes, d_bm)
    ctx.synchronize()
    ok = bool((np.frombuffer(ctx.from_device(d_codes, n), dtype=np.uint8) == 0).all())
    if world > 1:
        elapsed = ctx.comm_max(elapsed)
        ok = ctx.comm_max(0.0 if ok else 1.0) == 0.0
    if rank == 0:
        value = n * world * args.steps / elapsed
        sign_ms, launches = st["k_sign"]
        assert launches == args.steps, st
        with open(os.path.join(ROOT, "profiles", "opcount.json")) as f:
            g = json.load(f)["generator"]["k_sign"]
        alg = (g["mul"] + g["sqr"]) * ALG_MADS_PER_FP_MUL
        achieved = n * alg / (sign_ms / launches * 1e-3)
        print(json.dumps({
            "metric": "BLS12-381 signatures produced/sec (PrivateKey::sign)", "value": value, "unit": "sigs/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32 (381-bit Montgomery, 14x28-bit limb products via v_mad_u64_u32)",
            "data": "synthetic: random secret keys < 2^254 and 32-byte messages, inputs in HBM",
            "config": {"workload": f"SURVEY §8(f) rank 3, batch PrivateKey::sign: {n} records per GPU",
                       "parallelism": f"shard-by-index x{world}"},
            "verdicts_ok": ok,
            "stage_ms_per_step": {k: v[0] / args.steps for k, v in st.items()},
            "roofline": {"bound": "valu-int", "kernel": "k_sign", "achieved": achieved / 1e12,
                         "peak": PEAK_MADS / 1e12, "unit": "T mad/s (32x32-bit limb products, v_mad_u64_u32)",
                         "frac": achieved / PEAK_MADS, "traffic": None,
                         "alg_mads_per_sig": alg,
                         "note": "achieved = algorithmic mads of one launch (profiles/opcount.json generator.k_sign "
                                 "x 288) / its HIP-event duration"},
            "cpu_baseline": None,
            "runtime": dict(runtime_provenance(), lib_sha256=lib_sha256()),
        }), flush=True)
    for d in (d_sk, d_msg, d_off, d_sig, d_pk, d_codes, d_bm):
        ctx.device_free(d)


def run_dry(args, rank, world):
    """CPU rehearsal of the N>1 path: rendezvous of a 128-byte id through the
    launcher's job directory, then the shard ranges of the config[2] batch from
    the library's own cess_bls_shard_range (pure function, no device)."""
    from cess_amd import bls
    n_per = args.n or NPER_MULTI
    n_total = n_per * world
    if rank == 0:
        rdv_put("comm_id", hashlib.sha256(b"dry" + os.urandom(16)).digest() * 4)
    cid = rdv_get("comm_id")
    b, e, w = bls.shard_range(n_total, world, rank)
    rdv_put(f"shard_{rank}", json.dumps({"rank": rank, "begin": b, "end": e, "wpr": w,
                                         "id": hashlib.sha256(cid).hexdigest()}).encode())
    if rank == 0:
        shards = [json.loads(rdv_get(f"shard_{r}")) for r in range(world)]
        covered = sorted((s["begin"], s["end"]) for s in shards)
        ok = covered[0][0] == 0 and covered[-1][1] == n_total and all(
            covered[i][1] == covered[i + 1][0] for i in range(world - 1))
        same_id = len({s["id"] for s in shards}) == 1
        print(json.dumps({"dry_run": True, "n_gpus": world, "n_total": n_total, "sigs_per_gpu": n_per,
                          "shards": shards, "cover_ok": ok, "same_comm_id": same_id}), flush=True)
        rdv_put("done", b"1")
    else:
        rdv_get("done")
    if rank == 0:
        time.sleep(0.2)
        rdv_cleanup(rank, world)


def rlc_roofline(ctx, stages, n, distinct):
    """Roofline of an RLC line's dominant chunk kernel: its algorithmic mads per
    launch (profiles/opcount.json: k_miller_rr per record in the distinct-key
    mode, the per-signature kernels' counts otherwise) / its average HIP-event
    launch time; HBM traffic from a committed PMC profile of this library
    build (same SHA-256) when one exists."""
    if not stages:
        return None
    oc = load_opcount()
    dom = max(stages, key=lambda k: stages[k][0])
    ms, launches = stages[dom]
    chunk = min(n, ctx.launch_records)
    if distinct and dom == "k_miller":
        kernel, per = "k_miller_rr", oc.get("rlcd", {}).get("k_miller_rr")
    else:
        kernel, per = dom, oc["per_stage"].get(dom)
    if not per or not launches:
        return None
    alg = (per["mul"] + per["sqr"]) * ALG_MADS_PER_FP_MUL * chunk
    achieved = alg / (ms / launches * 1e-3)
    sha = lib_sha256()
    pmc = load_pmc_traffic(sha, kernel)
    kd = (pmc or {}).get("all", {}).get(kernel) or {}
    return {"bound": "valu-int", "kernel": kernel, "stage": dom, "achieved": achieved / 1e12,
            "peak": PEAK_MADS / 1e12, "unit": "T mad/s (32x32-bit limb products, v_mad_u64_u32)",
            "frac": achieved / PEAK_MADS, "launch_ms": ms / launches, "records_per_launch": chunk,
            "alg_mads_per_record": (per["mul"] + per["sqr"]) * ALG_MADS_PER_FP_MUL,
            "traffic": kd.get("hbm_bytes_per_launch"), "traffic_source": pmc["_file"] if pmc else None}


def run_rlc(args, ctx, rank, world):
    """RLC batch mode (BASELINE config[3] shape): each rank holds n records
    signed by `keys` distinct TEE keys; one combination per rank, the Gt
    partials all-gathered over RCCL and multiplied on the device inside the
    library (cess_bls_verify_batch_rlc_sharded), bisection iff a rank's own
    check fails.  Timed through the host-buffer API (key dedup + PCIe)."""
    import numpy as np
    distinct = args.mode == "rlcd"
    n = args.n or ((1 << 20) if distinct else (4 << 20))
    nkeys = n if distinct else args.keys
    rng = np.random.default_rng((0x0A0D17, rank))
    ksk = rng.integers(0, 256, size=(nkeys, 32), dtype=np.uint8)
    ksk[:, 0] &= 0x3F
    ksk[:, 31] |= 1
    kp = ctx.public_keys_raw(ksk.tobytes())
    owner = np.arange(n) if distinct else rng.integers(0, nkeys, size=n)
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sign_msgs = msgs.copy()
    forged = rng.choice(n, size=args.forged_count, replace=False) if args.forged_count else np.array([], dtype=int)
    sign_msgs[forged, 0] ^= 0xFF
    offs = np.arange(n + 1, dtype=np.uint64) * 32
    S = ctx.sign_raw(ksk[owner].tobytes(), sign_msgs.tobytes(), offs)
    kpa = np.frombuffer(kp, dtype=np.uint8).reshape(nkeys, 96)
    P, M = kpa[owner].tobytes(), msgs.tobytes()
    offl = offs

    def step():
        if world > 1:
            return ctx.verify_rlc_sharded(S, P, M, offl)          # seed: library CSPRNG
        return ctx.verify_rlc(S, P, M, offl)

    for _ in range(args.warmup):
        step()
    if world > 1:
        ctx.comm_barrier()
    ctx.synchronize()
    ctx.stage_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        codes, words, st = step()
    ctx.synchronize()
    if world > 1:
        ctx.comm_barrier()
    elapsed = time.perf_counter() - t0
    # HIP-event times of the chunk kernels inside the timed steps (the library
    # records them with CESS_BLS_F_PROFILE; host_rlc.cpp RLAUNCH)
    stages = {k: v for k, v in ctx.stage_stats(reset=True).items() if v[1] > 0}
    expect = np.zeros(n, dtype=np.uint8)
    expect[forged] = 5
    ok = bool((np.frombuffer(codes, dtype=np.uint8) == expect).all())
    if world > 1:
        elapsed = ctx.comm_max(elapsed)
        ok = ctx.comm_max(0.0 if ok else 1.0) == 0.0
    if rank == 0:
        total = n * world * args.steps
        if distinct:
            what = (f"BASELINE config[1] shape through the distinct-key RLC mode (CESS_BLS_F_RLC_DISTINCT): {n} sigs per "
                    f"GPU, {n} distinct keys, {args.forged_count} forged per GPU, one pairing per record, four records per "
                    f"Miller lane, one final exponentiation per check, bisection over the stored lane values")
        else:
            what = (f"BASELINE config[3] shape: {n} sigs per GPU, {args.keys} distinct keys, "
                    f"{args.forged_count} forged per GPU, RLC + Gt-partial RCCL all-gather + bisection")
        roofline = rlc_roofline(ctx, stages, n, distinct)
        print(json.dumps({
            "metric": "verified BLS12-381 sigs/sec (node), RLC batch mode", "value": total / elapsed,
            "unit": "sigs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: random keys (distinct)" if distinct else "synthetic: few random keys, 32-byte msgs",
            "config": {"workload": what,
                       "timing": "host-buffer API incl. PCIe" + ("" if distinct else " and key dedup"),
                       "parallelism": f"shard-by-index x{world}"},
            "verdicts_ok": ok,
            "rlc_stats": {k: (int(v) if not isinstance(v, bool) else v) for k, v in st.items()},
            "stage_ms_per_step": {k: v[0] / args.steps for k, v in stages.items()},
            "roofline": roofline,
            "runtime": runtime_provenance(),
        }), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1 and not args.one_device and "CESS_BENCH_DEVICE_COUNT" in os.environ:
            ndev = int(os.environ["CESS_BENCH_DEVICE_COUNT"])
            if ndev < world or local >= ndev:
                fail("devices", 4, need=world, visible=ndev, rank=rank, where="rank")
        run_dry(args, rank, world)
        return
    if world > 1:
        # the communicator's init (and every wait on it) gives up after this
        # deadline with CESS_BLS_E_COMM: a job with a missing peer ends in two
        # minutes, well inside any driver time limit, instead of 300 s
        os.environ.setdefault("CESS_BLS_COMM_TIMEOUT_MS", "120000")

    # the library (and with it /opt/rocm's HIP runtime and RCCL) first
    from cess_amd import bls
    lib = bls.load_library()
    import numpy as np
    if world > 1 and not args.one_device:
        # one GPU per rank: fewer visible devices than ranks (or a local rank
        # past them) fails every rank at once, before any context or
        # communicator exists
        # (the env override first: the library is asked only without it, and a
        # library without the symbol -- an older build in an A/B sweep -- falls
        # back to the KFD topology count the launcher parent uses)
        env_n = os.environ.get("CESS_BENCH_DEVICE_COUNT")
        if env_n is not None:
            ndev = int(env_n)
        elif hasattr(lib, "cess_bls_device_count"):
            ndev = int(lib.cess_bls_device_count())
        else:
            ndev = node_gpu_count()
        if ndev < world or local >= ndev:
            fail("devices", 4, need=world, visible=ndev, rank=rank, local_rank=local, where="rank")

    n = args.n or (N1_DEFAULT if world == 1 else NPER_MULTI)
    if args.mode == "rsa":
        ctx = bls.Context(device=local, max_batch=1 << 16, profile=True)
        if world > 1:
            comm_setup(ctx, rank, world, args.transport, args.one_device)
        run_rsa(args, ctx, rank, world)
        ctx.close()
        return
    if args.mode == "sign":
        ctx = bls.Context(device=local, max_batch=min(n, 1 << 20), profile=True)
        if world > 1:
            comm_setup(ctx, rank, world, args.transport, args.one_device)
        run_sign(args, ctx, rank, world)
        ctx.close()
        return
    if args.mode in ("rlc", "rlcd"):
        ctx = bls.Context(device=local, max_batch=min(args.n or (4 << 20), 1 << 20), rlc_distinct=args.mode == "rlcd",
                          profile=True)
        if world > 1:
            comm_setup(ctx, rank, world, args.transport, args.one_device)
        run_rlc(args, ctx, rank, world)
        ctx.close()
        return

    ctx = bls.Context(device=local, max_batch=min(n, 1 << 20), profile=True)
    comm = None
    if world > 1:
        comm = comm_setup(ctx, rank, world, args.transport, args.one_device)
    n_total = n * world
    keyed = args.mode == "keyed"
    if keyed:
        S, key_list, who, M, forged = make_keyed_dataset(ctx, n, args.keys, seed=(0x00C0FFEE, rank),
                                                         forged_frac=args.forged_frac)
        P = b"".join(key_list[w] for w in who)     # expanded records, for the CPU baseline only
        assert ctx.load_keys(key_list) == bytes(len(key_list))
        d_idx = ctx.to_device(who.astype(np.uint32))
    else:
        S, P, M, forged = make_dataset(ctx, n, seed=(0x00C0FFEE, rank), forged_frac=args.forged_frac)
    expect = np.where(forged, 5, 0).astype(np.uint8)
    n_adv_kinds = 0
    if args.mode == "adversarial":
        S, P, M, expect, n_adv_kinds = inject_adversarial(S, P, M, n, seed=(0xADD, rank))
    if world > 1:
        b, e, wpr = bls.shard_range(n_total, world, rank)
        assert (b, e) == (rank * n, rank * n + n), (b, e)
    else:
        wpr = (n + 63) // 64
    d_sig = ctx.to_device(S)
    d_pk = None if keyed else ctx.to_device(P)
    d_msg = ctx.to_device(M)
    d_off = ctx.to_device(np.arange(n + 1, dtype=np.uint64) * 32)
    d_codes = ctx.device_alloc(world * wpr * 64)
    d_bitmap = ctx.device_alloc(world * wpr * 8)

    def step():
        if keyed:
            ctx.verify_keyed_device(n, d_sig, d_idx, d_msg, d_off, d_codes, d_bitmap)
        elif world > 1:
            ctx.verify_sharded_device(n_total, d_sig, d_pk, d_msg, d_off, d_codes, d_bitmap)
        else:
            ctx.verify_device(n, d_sig, d_pk, d_msg, d_off, d_codes, d_bitmap)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    ctx.stage_stats(reset=True)
    if world > 1:
        ctx.comm_barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    if world > 1:
        ctx.comm_barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = None
    if world > 1:   # every rank's own step time (min / max over ranks)
        rank_ms = {"min": -ctx.comm_max(-elapsed) / args.steps * 1e3, "max": ctx.comm_max(elapsed) / args.steps * 1e3}
    # per-launch HIP events on each kernel's own stream, timed region only
    stats = {k: v for k, v in ctx.stage_stats(reset=True).items() if v[1] > 0}
    if keyed:   # the keyed pipeline runs k_merge_pk in k_decode_pk's slot and has no per-signature prepare
        stats["k_merge_pk"] = stats.pop("k_decode_pk")
        stats.pop("k_prepare", None)
    stages = {k: v[0] for k, v in stats.items()}
    launches_of = {k: v[1] for k, v in stats.items()}
    if world > 1:
        elapsed = ctx.comm_max(elapsed)

    # correctness of the last step: this rank's codes + the gathered bitmap
    codes_all = np.frombuffer(ctx.from_device(d_codes, world * wpr * 64), dtype=np.uint8)
    my = codes_all[rank * wpr * 64: rank * wpr * 64 + n] if world > 1 else codes_all[:n]
    local_ok = bool((my == expect).all())                 # bit-exact per-record codes
    words = np.frombuffer(ctx.from_device(d_bitmap, world * wpr * 8), dtype=np.uint64)
    popcount = int(np.unpackbits(words.view(np.uint8)).sum())
    ok = local_ok if world == 1 else ctx.comm_max(0.0 if local_ok else 1.0) == 0.0
    # `comm`: what the communicator itself reported at setup (comm_setup)

    # the same records from HOST buffers (cess_bls_verify_batch: H2D copies,
    # the pipeline, D2H of codes + bitmap), as node callers pass them; reported
    # beside the device-resident `value`, never as it
    host_rate = None
    if world == 1 and args.mode == "persig" and args.host_steps > 0:
        o_host = np.arange(n + 1, dtype=np.uint64) * 32
        ctx.synchronize()
        th = time.perf_counter()
        for _ in range(args.host_steps):
            hc, _hw = ctx.verify_fixed(S, P, M, o_host)
        th = time.perf_counter() - th
        host_rate = {"sigs_per_s": n * args.host_steps / th, "steps": args.host_steps,
                     "ms_per_step": th / args.host_steps * 1e3,
                     "codes_ok": bool((np.frombuffer(hc, dtype=np.uint8) == expect).all())}
        ctx.stage_stats(reset=True)

    if rank == 0:
        total = n_total * args.steps
        value = total / elapsed
        oc = load_opcount()
        per = oc["per_stage"]
        whole_mads = oc["algorithmic_mads_per_sig"]
        if keyed:   # per-key decode + prepare are done once per key, outside the per-signature work
            whole_mads -= sum((per[k]["mul"] + per[k]["sqr"]) * ALG_MADS_PER_FP_MUL for k in ("k_decode_pk", "k_prepare"))
        chunk = min(n, ctx.launch_records)                # records per kernel launch (pipeline part)
        dom = max(stages, key=lambda k: stages[k])
        launches = launches_of[dom]
        assert launches == args.steps * ((n + chunk - 1) // chunk), (launches, chunk)
        dom_ms = stages[dom] / launches                   # average launch duration (chunk records each)
        alg = (per[dom]["mul"] + per[dom]["sqr"]) * ALG_MADS_PER_FP_MUL * chunk
        achieved = alg / (dom_ms * 1e-3)
        sha = lib_sha256()
        dom_kernel = KERNEL_OF_STAGE.get(dom, dom)
        pmc = load_pmc_traffic(sha, dom_kernel, chunk)
        traffic = valu_active = None
        if pmc and pmc.get("n") == chunk:
            kd = pmc.get("all", {}).get(dom_kernel) or {}
            traffic = kd.get("hbm_bytes_per_launch")
            # the issue bound the kernels sit on: share of each wave's cycles
            # with a VALU instruction issued (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
            # of the same build; x waves per SIMD = SIMD VALU busy share)
            if kd.get("SQ_WAVE_CYCLES"):
                valu_active = kd.get("SQ_ACTIVE_INST_VALU", 0.0) / kd["SQ_WAVE_CYCLES"]
        cpu = None
        if world == 1 and args.cpu_sample > 0:
            import random
            rr = random.Random(5)
            idx = rr.sample(range(n), min(n, args.cpu_sample))
            cpu = cpu_baseline(S, M, P, idx, args.cpu_threads)
        if args.mode == "persig":
            wl = (f"BASELINE config[1]: {n} independent sigs, distinct keys, per-sig 2-pairing verify" if world == 1
                  else f"BASELINE config[2] shape: {n_total} sigs ({n} per GPU) sharded by index across {world} GPUs, "
                       f"distinct keys, per-sig 2-pairing verify, "
                       f"{'RCCL' if ctx.comm_kind == 'rccl' else 'shared-memory'} all-gather of verdict bitmap + codes"
                       + (" (REHEARSAL: all ranks share GPU 0)" if args.one_device else ""))
        elif keyed:
            wl = (f"BASELINE config[3] shape, per-signature verdicts: {n} sigs per GPU over {args.keys} keys, key "
                  f"decode + G2Prepared once per key (keyed batch)")
        else:
            wl = (f"BASELINE config[4] shape: {n} sigs per GPU, 1% invalid (half forged, half {n_adv_kinds} kinds of "
                  f"malformed/non-subgroup/identity records), exact codes")
        rec = {
            "metric": "verified BLS12-381 sigs/sec (node)",
            "value": value,
            "unit": "sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (381-bit Montgomery, 14x28-bit limb products via v_mad_u64_u32)",
            "data": "synthetic: random distinct keys + 32-byte messages, keys/sigs generated on GPU",
            "config": {"workload": wl, "sigs_per_gpu": n, "sigs_total": n_total, "msg_bytes": 32,
                       "forged_frac": args.forged_frac, "parallelism": f"shard-by-index x{world}",
                       "transport": ctx.comm_kind if world > 1 else None,
                       "ranks_share_gpu0": bool(args.one_device and world > 1),
                       "launch_chunk": chunk},
            "verdicts_ok": ok,
            "host_buffers_sigs_per_s": host_rate["sigs_per_s"] if host_rate else None,
            "host_buffers": host_rate,
            "comm": comm,
            "rank_ms_per_step": rank_ms,
            "bitmap_popcount": popcount,
            "stage_ms_per_step": {k: v / args.steps for k, v in stages.items()},
            "stage_launches_per_step": {k: v / args.steps for k, v in launches_of.items()},
            "roofline": {"bound": "valu-int", "kernel": dom_kernel, "stage": dom, "achieved": achieved / 1e12,
                         "peak": PEAK_MADS / 1e12,
                         "unit": "T mad/s (32x32-bit limb products, v_mad_u64_u32)",
                         "frac": achieved / PEAK_MADS, "traffic": traffic,
                         "traffic_source": pmc["_file"] if pmc else None,
                         "pmc_valu_active_per_wave": valu_active,
                         "waves_per_simd": WAVES_PER_SIMD.get(dom),
                         "alg_mads_per_sig": (per[dom]["mul"] + per[dom]["sqr"]) * ALG_MADS_PER_FP_MUL,
                         "whole_path_frac": whole_mads * value / world / PEAK_MADS},
            "cpu_baseline": cpu,
            "runtime": dict(runtime_provenance(), lib_sha256=sha),
        }
        print(json.dumps(rec), flush=True)
    for d in (d_sig, d_pk, d_msg, d_off, d_codes, d_bitmap) + ((d_idx,) if keyed else ()):
        if d:
            ctx.device_free(d)
    ctx.close()


if __name__ == "__main__":
    main()
