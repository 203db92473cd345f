"""Diagnostic: one process inits rank 0 of a 2-rank RCCL communicator alone
(the peer never arrives) and reports the status and the time it took.
Usage (GPU box): CESS_BLS_COMM_TIMEOUT_MS=4000 CESS_BLS_COMM_TRACE=1 python tools/rccl_lone_rank.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cess_amd import bls  # noqa: E402

bls.load_library()
c = bls.Context(max_batch=256)
t0 = time.time()
try:
    c.comm_init(2, 0, bls.comm_id())
    print("STATUS 0", time.time() - t0, flush=True)
except bls.BlsInfraError as ex:
    print("STATUS", ex.status, time.time() - t0, flush=True)
c.close()
print("CLOSED", time.time() - t0, flush=True)
os._exit(0)
