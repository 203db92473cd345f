// Transport seam of the sharded entry points (host_multi.cpp; SURVEY §8(e),
// §4 "a fake-RCCL single-process shim ... to test shard and merge logic").
//
// The shard/merge code of cess_bls_verify_batch_sharded[_device] and
// cess_bls_verify_batch_rlc_sharded is written against this interface only:
//
//  * RcclTransport (host_multi.cpp): production -- one process per GPU,
//    ncclAllGather / ncclAllReduce over xGMI.  RCCL refuses two ranks on one
//    device, so it cannot run N > 1 on a one-GPU box.
//  * ShmTransport (comm_shm.cpp): the same collectives over a POSIX
//    shared-memory segment between processes of one host.  The ranks may
//    share a GPU (the -m gpu two-rank tests) or have none at all (the CPU
//    world-2 tests of the merge code through cess_bls_comm_open_shm).
//
// Collective contract (both transports): every rank of the communicator
// issues the same collectives in the same order.  The sharded entry points
// keep it by agreeing on a status (agree(): the worst status of any rank)
// after their local, possibly failing, work and before any data collective,
// so a rank that fails returns that failure on every rank instead of leaving
// the others blocked in an all-gather (host_multi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/cess_bls.h"

namespace cess_host {

struct Transport {
  int nranks = 1, rank = 0;
  virtual ~Transport() {}
  virtual const char* kind() const = 0;
  // Host memory, in place: rank r's block of `bytes` is buf + r * bytes; on
  // return every block holds its rank's data.
  virtual int allgather_host(void* buf, size_t bytes) = 0;
  // Device memory of device `dev`, in place, ordered on stream s.  The default
  // stages through host memory with allgather_host (synchronises s).
  virtual int allgather_dev(int dev, void* dbuf, size_t bytes, hipStream_t s);
  // Element-wise maximum over ranks of n host values, in place.
  virtual int max_i64(int64_t* v, int n) = 0;
  virtual int max_f64(double* v) = 0;
  // What the communicator itself reports (RCCL: ncclCommCount /
  // ncclCommUserRank; shm: the segment's rank count and this rank).
  virtual int comm_count(int* count, int* my_rank) {
    *count = nranks;
    *my_rank = rank;
    return CESS_BLS_OK;
  }
};

// POSIX shared-memory transport (comm_shm.cpp).  `name` (from
// cess_bls_comm_shm_name, distributed out of band) identifies the job; rank 0
// creates the segment, the others attach; returns after all nranks attached.
int make_shm_transport(const char* name, int nranks, int rank, Transport** out);

// The worst (most negative) status over all ranks; every rank gets the same
// value.  A transport failure is returned as itself.
int agree(Transport& t, int status);

// Merge of per-rank verdicts: shard_codes holds this rank's shard of an
// n-record batch (cess_bls_shard_range order, shard_n bytes); every rank
// receives the codes (n bytes, may be NULL) and the LSB-first bitmap
// (ceil(n/64) words, may be NULL) of the whole batch.  Collective; n must
// be equal on every rank (checked: CESS_BLS_E_INVALID_ARG on all ranks).
int gather_verdicts(Transport& t, uint64_t n, const uint8_t* shard_codes, uint8_t* codes_out, uint64_t* bitmap_out);

// every rank passed the same value (one collective step)
int same_on_all_ranks(Transport& t, uint64_t v, bool* same);

// Bounded waits of both transports: CLOCK_MONOTONIC in ms, and the deadline
// of one wait, env CESS_BLS_COMM_TIMEOUT_MS (default 300 s)
double comm_now_ms();
double comm_timeout_ms();

// shard of a batch for rank r of R (whole bitmap words, equal word count per rank; host.cpp)
void shard_of(uint64_t n, int nranks, int rank, uint64_t* begin, uint64_t* end, uint64_t* words_per_rank);

}  // namespace cess_host
