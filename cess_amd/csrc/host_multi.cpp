// Multi-GPU paths of include/cess_bls.h.
//
// Signatures are independent (reference src/lib.rs:243 is per signature), so a
// batch shards by index with no exchange during compute.  Two deployments:
//
//  * one process per GPU (cess_bls_comm_init / _init_shm): the context owns a
//    communicator behind the transport seam of comm.hpp -- RCCL over xGMI in
//    production, host shared memory for ranks that share a GPU (tests on a
//    one-GPU box).  The sharded entry points verify the rank's shard, agree on
//    a status, and all-gather the verdict-bitmap words and code bytes (in RLC
//    mode the 576-byte Gt partials).  Shards are whole bitmap words with an
//    equal word count per rank, so the all-gather is in place and needs no
//    re-packing.
//  * one process driving several GPUs (cess_bls_config.n_devices > 1): the
//    context holds one sub-context per device and the host-buffer batches are
//    split the same way across them, one host thread per device, each writing
//    its verdicts straight into the caller's buffers (no collective needed in
//    one address space).
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <atomic>
#include <memory>
#include <thread>

#include "host.hpp"

using namespace cess_host;

#define NCCLCHK(x)                                 \
  do {                                             \
    if ((x) != ncclSuccess) return CESS_BLS_E_RCCL; \
  } while (0)

#define ENTRY(c)                          \
  if (!(c)) return CESS_BLS_E_INVALID_ARG; \
  CtxLock lock_(c);                        \
  if (!lock_.ok()) return CESS_BLS_E_BUSY

// single-device workers (host.cpp)
int cess_keys_load_one(cess_bls_ctx* c, size_t k, const uint8_t* pks, uint8_t* key_codes_out);
int cess_keyed_one(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint32_t* key_idx, const uint8_t* msgs,
                   const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out);
int cess_gen_one(cess_bls_ctx* c, int kind, size_t n, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs,
                 uint8_t* out);

// ---------------------------------------------------------------------------
// RCCL transport (comm.hpp): production, one process per GPU, xGMI
// ---------------------------------------------------------------------------
namespace {
// Every RCCL call is bounded: the communicator is created NON-BLOCKING
// (ncclCommInitRankConfig, blocking = 0) and each wait -- init, a collective's
// enqueue, the control stream draining -- polls ncclCommGetAsyncError against
// a deadline (CESS_BLS_COMM_TIMEOUT_MS, default 300 s, the shm transport's).
// A dead or stuck peer therefore ends in ncclCommAbort and CESS_BLS_E_COMM on
// this rank instead of a hang; an RCCL-reported error ends in ncclCommAbort
// and CESS_BLS_E_RCCL.  After either, the transport is broken and every later
// call returns CESS_BLS_E_COMM at once.
// env CESS_BLS_COMM_TRACE=1: timestamped trace of the transport's RCCL calls on stderr
static bool comm_trace() {
  static const bool on = getenv("CESS_BLS_COMM_TRACE") != nullptr;
  return on;
}
#define CTRACE(...)                                                                   \
  do {                                                                                \
    if (comm_trace()) {                                                               \
      fprintf(stderr, "[cess comm %.3f] ", comm_now_ms() * 1e-3);                      \
      fprintf(stderr, __VA_ARGS__);                                                   \
      fprintf(stderr, "\n");                                                          \
      fflush(stderr);                                                                 \
    }                                                                                 \
  } while (0)

class RcclTransport final : public Transport {
 public:
  ~RcclTransport() override {
    if (ctl_) (void)hipSetDevice(dev_);
    if (comm_) {
      // drain our own control work, then a bounded finalize; abort if the
      // peers never complete it
      int r = ctl_ ? wait_stream(ctl_) : CESS_BLS_OK;
      if (!r && comm_) r = issue(ncclCommFinalize(comm_));
      if (!r && comm_) (void)ncclCommDestroy(comm_);
      comm_ = nullptr;   // (a failed wait aborted it already)
    }
    if (ctl_) (void)hipStreamDestroy(ctl_);
  }
  const char* kind() const override { return "rccl"; }

  int init(cess_bls_ctx* c, int nranks, int rank, const ncclUniqueId& id) {
    dev_ = c->device;
    ctx_ = c;
    this->nranks = nranks;
    this->rank = rank;
    HIPCHK(hipSetDevice(dev_));
    HIPCHK(hipStreamCreateWithFlags(&ctl_, hipStreamNonBlocking));
    // RCCL's bootstrap blocks the calling thread until every rank has
    // connected, even for a non-blocking communicator (measured on MI355X:
    // ncclCommInitRankConfig never returned for a lone rank), so the whole
    // init -- the call and, for the non-blocking communicator, polling its
    // state to ncclSuccess -- runs on a helper thread (which also owns the
    // config RCCL may read asynchronously), and this thread waits for it
    // against the deadline.  A helper that finishes after the caller gave up
    // aborts its communicator itself; one that never returns stays blocked in
    // the bootstrap (detached: it holds only the shared job state).
    struct InitJob {
      std::atomic<int> state{0};   // 0 running, 1 done, 2 abandoned by the caller
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      ncclComm_t comm = nullptr;
      ncclResult_t res = ncclInternalError;
    };
    auto job = std::make_shared<InitJob>();
    job->cfg.blocking = 0;
    CTRACE("init rank %d of %d: ncclCommInitRankConfig (non-blocking) on a helper thread", rank, nranks);
    std::thread([job, dev = dev_, nranks, rank, id]() {
      (void)hipSetDevice(dev);
      ncclComm_t comm = nullptr;
      ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, id, rank, &job->cfg);
      while (r == ncclInProgress && comm && job->state.load() == 0) {
        ncclResult_t st = ncclInProgress;
        if (ncclCommGetAsyncError(comm, &st) != ncclSuccess) st = ncclInternalError;
        r = st;
        if (r == ncclInProgress) usleep(200);
      }
      job->comm = comm;
      job->res = r;
      int running = 0;
      if (!job->state.compare_exchange_strong(running, 1) && comm) (void)ncclCommAbort(comm);
    }).detach();
    const double t_end = comm_now_ms() + comm_timeout_ms();
    for (int spins = 0; job->state.load() == 0; spins++) {
      if (comm_now_ms() > t_end) {
        int running = 0;
        if (job->state.compare_exchange_strong(running, 2)) {
          CTRACE("init: deadline passed with the bootstrap still waiting for peers");
          return CESS_BLS_E_COMM;
        }
        break;   // it finished just now
      }
      if (spins > 256) usleep(spins > 4096 ? 1000 : 50);
    }
    comm_ = job->comm;
    CTRACE("init finished: %d", (int)job->res);
    if (job->res != ncclSuccess) {
      if (comm_) (void)ncclCommAbort(comm_);
      comm_ = nullptr;
      return CESS_BLS_E_RCCL;
    }
    return CESS_BLS_OK;
  }

  int allgather_dev(int dev, void* dbuf, size_t bytes, hipStream_t s) override {
    (void)dev;
    if (!comm_) return CESS_BLS_E_COMM;
    char* b = static_cast<char*>(dbuf);
    return issue(ncclAllGather(b + (size_t)rank * bytes, b, bytes, ncclUint8, comm_, s));
  }

  // Host-side collectives run on the control stream after the context's
  // previous work (order_begin): RCCL then executes this communicator's
  // collectives in the order every rank issued them.
  int allgather_host(void* buf, size_t bytes) override {
    if (!comm_) return CESS_BLS_E_COMM;
    HIPCHK(hipSetDevice(dev_));
    int r = order_begin(ctx_, ctl_);
    if (r) return r;
    if (buf_.ensure(std::max<size_t>(1, (size_t)nranks * bytes))) return CESS_BLS_E_OOM;
    char* d = buf_.as<char>();
    char* h = static_cast<char*>(buf);
    if (bytes) HIPCHK(hipMemcpyAsync(d + (size_t)rank * bytes, h + (size_t)rank * bytes, bytes, hipMemcpyHostToDevice, ctl_));
    r = issue(ncclAllGather(d + (size_t)rank * bytes, d, bytes, ncclUint8, comm_, ctl_));
    if (r) return r;
    if (bytes) HIPCHK(hipMemcpyAsync(h, d, (size_t)nranks * bytes, hipMemcpyDeviceToHost, ctl_));
    r = wait_stream(ctl_);
    if (r) return r;
    return order_end(ctx_, ctl_);
  }

  int max_i64(int64_t* v, int n) override { return allreduce_max(v, n, ncclInt64); }
  int max_f64(double* v) override { return allreduce_max(v, 1, ncclFloat64); }

  int comm_count(int* count, int* my_rank) override {
    if (!comm_) return CESS_BLS_E_COMM;
    if (ncclCommCount(comm_, count) != ncclSuccess || ncclCommUserRank(comm_, my_rank) != ncclSuccess)
      return CESS_BLS_E_RCCL;
    return CESS_BLS_OK;
  }

 private:
  template <class T>
  int allreduce_max(T* v, int n, ncclDataType_t t) {
    if (!comm_) return CESS_BLS_E_COMM;
    HIPCHK(hipSetDevice(dev_));
    int r = order_begin(ctx_, ctl_);
    if (r) return r;
    if (buf_.ensure(std::max<size_t>(64, n * sizeof(T)))) return CESS_BLS_E_OOM;
    T* d = buf_.as<T>();
    HIPCHK(hipMemcpyAsync(d, v, n * sizeof(T), hipMemcpyHostToDevice, ctl_));
    r = issue(ncclAllReduce(d, d, n, t, ncclMax, comm_, ctl_));
    if (r) return r;
    HIPCHK(hipMemcpyAsync(v, d, n * sizeof(T), hipMemcpyDeviceToHost, ctl_));
    r = wait_stream(ctl_);
    if (r) return r;
    return order_end(ctx_, ctl_);
  }

  // abort the communicator (releases kernels waiting on peers) and mark the
  // transport broken (comm_ null: every later call returns CESS_BLS_E_COMM)
  int fail(int status) {
    CTRACE("fail(%d): ncclCommAbort", status);
    if (comm_) (void)ncclCommAbort(comm_);
    CTRACE("abort returned");
    comm_ = nullptr;
    return status;
  }
  // result of an RCCL call on the non-blocking communicator
  int issue(ncclResult_t r) {
    if (r == ncclSuccess) return CESS_BLS_OK;
    if (r == ncclInProgress) return wait_ready();
    return fail(CESS_BLS_E_RCCL);
  }
  // Poll `done` (true: finished, or a status < 0 to fail with) and the
  // communicator's asynchronous error until the deadline.
  template <class Done>
  int poll(Done&& done) {
    const double t_end = comm_now_ms() + comm_timeout_ms();
    for (int spins = 0;; spins++) {
      ncclResult_t st = ncclInProgress;
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) return fail(CESS_BLS_E_RCCL);
      if (st != ncclSuccess && st != ncclInProgress) return fail(CESS_BLS_E_RCCL);
      const int d = done(st);
      if (d > 0) return CESS_BLS_OK;
      if (d < 0) return fail(d);
      if (comm_now_ms() > t_end) {
        CTRACE("deadline passed (state %d)", (int)st);
        return fail(CESS_BLS_E_COMM);
      }
      if (spins > 256) usleep(spins > 4096 ? 200 : 20);
    }
  }
  // the communicator's state leaves ncclInProgress (init, an enqueue, finalize)
  int wait_ready() {
    if (!comm_) return CESS_BLS_E_COMM;
    return poll([](ncclResult_t st) { return st == ncclSuccess ? 1 : 0; });
  }
  // stream s drained while the communicator stays healthy
  int wait_stream(hipStream_t s) {
    if (!comm_) return CESS_BLS_E_COMM;
    return poll([s](ncclResult_t) {
      const hipError_t q = hipStreamQuery(s);
      return q == hipSuccess ? 1 : q == hipErrorNotReady ? 0 : CESS_BLS_E_HIP;
    });
  }

  int dev_ = 0;
  cess_bls_ctx* ctx_ = nullptr;
  ncclComm_t comm_ = nullptr;
  hipStream_t ctl_ = nullptr;
  DevBuf buf_;
};
}  // namespace

// ---------------------------------------------------------------------------
// communicator setup
// ---------------------------------------------------------------------------
extern "C" int cess_bls_shard_range(uint64_t n, int nranks, int rank, uint64_t* begin, uint64_t* end,
                                    uint64_t* words_per_rank) {
  if (nranks <= 0 || rank < 0 || rank >= nranks) return CESS_BLS_E_INVALID_ARG;
  shard_of(n, nranks, rank, begin, end, words_per_rank);
  return CESS_BLS_OK;
}

extern "C" int cess_bls_comm_id(uint8_t id_out[CESS_BLS_COMM_ID_BYTES]) {
  if (!id_out) return CESS_BLS_E_INVALID_ARG;
  static_assert(sizeof(ncclUniqueId) == CESS_BLS_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return CESS_BLS_OK;
}

extern "C" int cess_bls_comm_init(cess_bls_ctx* c, int nranks, int rank, const uint8_t id_in[CESS_BLS_COMM_ID_BYTES]) {
  ENTRY(c);
  if (!c->subs.empty() || !id_in || nranks <= 0 || rank < 0 || rank >= nranks || c->xport) return CESS_BLS_E_INVALID_ARG;
  ncclUniqueId id;
  memcpy(&id, id_in, sizeof(id));
  RcclTransport* t = new RcclTransport();
  const int r = t->init(c, nranks, rank, id);
  if (r) {
    delete t;
    return r;
  }
  c->xport = t;
  c->nranks = nranks;
  c->rank = rank;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_comm_init_shm(cess_bls_ctx* c, int nranks, int rank, const char* name) {
  ENTRY(c);
  if (!c->subs.empty() || c->xport) return CESS_BLS_E_INVALID_ARG;
  Transport* t = nullptr;
  const int r = make_shm_transport(name, nranks, rank, &t);
  if (r) return r;
  c->xport = t;
  c->nranks = nranks;
  c->rank = rank;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_comm_info(cess_bls_ctx* c, int* nranks_out, int* rank_out, char* bus_ids_out) {
  ENTRY(c);
  if (!c->xport) return CESS_BLS_E_NO_COMM;
  int nr = 0, rk = 0;
  int st = c->xport->comm_count(&nr, &rk);
  if (!st) {
    if (nranks_out) *nranks_out = nr;
    if (rank_out) *rank_out = rk;
  }
  if (!bus_ids_out) return st;
  // collective: every rank's PCI bus id, gathered in rank order; a local
  // failure (count or bus id) still joins the agreement, so no peer is left
  // waiting in it
  std::vector<char> ids((size_t)c->nranks * CESS_BLS_BUS_ID_BYTES, 0);
  char* mine = &ids[(size_t)c->rank * CESS_BLS_BUS_ID_BYTES];
  if (!st && hipDeviceGetPCIBusId(mine, CESS_BLS_BUS_ID_BYTES - 1, c->device) != hipSuccess) st = CESS_BLS_E_HIP;
  int r = agree(*c->xport, st);
  if (r) return r;
  r = c->xport->allgather_host(ids.data(), CESS_BLS_BUS_ID_BYTES);
  if (r) return r;
  memcpy(bus_ids_out, ids.data(), ids.size());
  return CESS_BLS_OK;
}

extern "C" const char* cess_bls_comm_kind(cess_bls_ctx* c) {
  return (c && c->xport) ? c->xport->kind() : "none";
}

// ---------------------------------------------------------------------------
// sharded entry points
// ---------------------------------------------------------------------------
// Every rank runs the same collective sequence whatever happens locally:
// (1) the batch size must agree, (2) local work, (3) agree() on the worst
// status -- a failure anywhere returns that failure on every rank, before any
// data moves -- (4) the data all-gathers.
extern "C" int cess_bls_verify_batch_sharded(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                             const uint8_t* msgs, const uint64_t* offs, uint8_t* codes_out,
                                             uint64_t* bitmap_out) {
  ENTRY(c);
  if (!c->xport) return CESS_BLS_E_NO_COMM;
  Transport& t = *c->xport;
  uint64_t b, e, wpr;
  shard_of(n, c->nranks, c->rank, &b, &e, &wpr);
  const uint64_t m = e - b;
  // the whole batch is validated on every rank (the same inputs give the same
  // answer everywhere; agree() covers ranks given different ones)
  int st = CESS_BLS_OK;
  if (n && (!sigs || !pks || !offs)) st = CESS_BLS_E_INVALID_ARG;
  for (uint64_t i = 0; st == CESS_BLS_OK && i < n; i++)
    if (offs[i + 1] < offs[i]) st = CESS_BLS_E_INVALID_ARG;
  if (st == CESS_BLS_OK && n && !msgs && offs[n] != offs[0]) st = CESS_BLS_E_INVALID_ARG;
  std::vector<uint8_t> codes(std::max<uint64_t>(m, 1), 0xff);
  if (st == CESS_BLS_OK && m)
    st = verify_host(c, m, sigs + 48 * b, pks + 96 * b, msgs, offs + b, nullptr, codes.data(), nullptr, nullptr);
  int r = agree(t, st);
  if (r) return r;
  return gather_verdicts(t, n, codes.data(), codes_out, bitmap_out);
}

extern "C" int cess_bls_verify_batch_var_sharded(cess_bls_ctx* c, size_t n, const uint8_t* sig_data,
                                                 const uint64_t* sig_offsets, const uint8_t* pk_data,
                                                 const uint64_t* pk_offsets, const uint8_t* msgs,
                                                 const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out) {
  ENTRY(c);
  if (!c->xport) return CESS_BLS_E_NO_COMM;
  Transport& t = *c->xport;
  uint64_t b, e, wpr;
  shard_of(n, c->nranks, c->rank, &b, &e, &wpr);
  const uint64_t m = e - b;
  // the whole batch's offsets are validated on every rank (as the fixed form)
  int st = CESS_BLS_OK;
  if (!sig_offsets || !pk_offsets || !msg_offsets) st = CESS_BLS_E_INVALID_ARG;
  for (uint64_t i = 0; st == CESS_BLS_OK && i < n; i++)
    if (sig_offsets[i + 1] < sig_offsets[i] || pk_offsets[i + 1] < pk_offsets[i] || msg_offsets[i + 1] < msg_offsets[i])
      st = CESS_BLS_E_INVALID_ARG;
  std::vector<uint8_t> codes(std::max<uint64_t>(m, 1), CESS_BLS_CODE_UNAVAILABLE);
  if (st == CESS_BLS_OK && m)
    st = verify_var_host(c, m, sig_data, sig_offsets + b, pk_data, pk_offsets + b, msgs, msg_offsets + b, codes.data(),
                         nullptr);
  int r = agree(t, st);
  if (r) return r;
  return gather_verdicts(t, n, codes.data(), codes_out, bitmap_out);
}

extern "C" int cess_bls_verify_batch_sharded_device(cess_bls_ctx* c, size_t n_total, const uint8_t* d_sigs,
                                                    const uint8_t* d_pks, const uint8_t* d_msgs,
                                                    const uint64_t* d_offs, uint8_t* d_codes_all,
                                                    uint64_t* d_bitmap_all, void* stream) {
  ENTRY(c);
  if (!c->xport) return CESS_BLS_E_NO_COMM;
  Transport& t = *c->xport;
  uint64_t b, e, wpr;
  shard_of(n_total, c->nranks, c->rank, &b, &e, &wpr);
  const uint64_t m = e - b;
  // (1) + local checks and allocations, then (3): nothing is enqueued before
  // every rank knows it can run
  // n_total and whether codes are gathered fix the collective sequence
  bool same = false;
  int r = same_on_all_ranks(t, ((uint64_t)n_total << 1) | (d_codes_all ? 1u : 0u), &same);
  if (r) return r;
  int st = same ? CESS_BLS_OK : CESS_BLS_E_INVALID_ARG;
  if (!d_bitmap_all || (m && (!d_sigs || !d_pks || !d_offs))) st = CESS_BLS_E_INVALID_ARG;
  if (st == CESS_BLS_OK && hipSetDevice(c->device) != hipSuccess) st = CESS_BLS_E_HIP;
  if (st == CESS_BLS_OK && !d_codes_all && c->comm_codes.ensure(std::max<uint64_t>(m, 1))) st = CESS_BLS_E_OOM;
  r = agree(t, st);
  if (r) return r;
  if (wpr == 0) return CESS_BLS_OK;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  r = order_begin(c, s);
  uint64_t* my_words = d_bitmap_all + c->rank * wpr;
  uint8_t* codes = d_codes_all ? d_codes_all + c->rank * wpr * 64 : c->comm_codes.as<uint8_t>();
  // (2) the shard's pipeline; words of the rank's run past its last record (a
  // short or empty last shard) are zero
  const uint64_t used = (m + 63) / 64;
  if (!r && used < wpr && hipMemsetAsync(my_words + used, 0, (wpr - used) * 8, s) != hipSuccess) r = CESS_BLS_E_HIP;
  for (uint64_t off = 0; !r && off < m; off += c->cap) {
    const uint64_t q = std::min<uint64_t>(c->cap, m - off);
    r = run_chunk(c, s, q, d_sigs + 48 * off, d_pks + 96 * off, d_msgs, d_offs + off, nullptr, codes + off,
                  my_words + off / 64, nullptr);
    if (!r && (c->flags & CESS_BLS_F_PROFILE)) r = collect_profile(c, s);
  }
  if (r) {
    // past the agreement the peers are committed to the all-gathers: take part
    // with a block that holds no verdict -- no bitmap bit, and every code of
    // the shard CESS_BLS_CODE_UNAVAILABLE, so records this rank never verified
    // cannot read as OK (0) from whatever the caller's buffer held
    (void)hipMemsetAsync(my_words, 0, wpr * 8, s);
    if (d_codes_all) (void)hipMemsetAsync(codes, CESS_BLS_CODE_UNAVAILABLE, wpr * 64, s);
  }
  // (4)
  int g = t.allgather_dev(c->device, d_bitmap_all, wpr * 8, s);
  if (d_codes_all) {
    const int g2 = t.allgather_dev(c->device, d_codes_all, wpr * 64, s);
    if (!g) g = g2;
  }
  const int oe = order_end(c, s);
  // (5) a second status agreement, ordered after the all-gathers (the
  // transport's host collectives wait for the context's last stream): a
  // failure on any rank after (3) is returned on every rank
  return agree(t, r ? r : g ? g : oe);
}

extern "C" int cess_bls_verify_batch_rlc_sharded(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks,
                                                 const uint8_t* msgs, const uint64_t* offs, const uint8_t* seed32,
                                                 uint8_t* codes_out, uint64_t* bitmap_out, uint64_t* stats4,
                                                 int* global_ok_out) {
  ENTRY(c);
  if (!c->xport) return CESS_BLS_E_NO_COMM;
  Transport& t = *c->xport;
  // (2) this rank's combination (its shard; scalars distinct across ranks)
  std::vector<uint8_t> gts((size_t)c->nranks * 576, 0);
  int st = rlc_begin(c, n, sigs, pks, msgs, offs, seed32, &gts[(size_t)c->rank * 576]);
  // (3), then the Gt partials: one 576-byte block per rank, multiplied on the
  // device (RCCL has no Fp12 reduction operator)
  int r = agree(t, st);
  if (r) return r;
  r = t.allgather_host(gts.data(), 576);
  if (r) return r;
  int one = 0;
  r = gt_product_is_one(c, c->nranks, gts.data(), false, &one);
  if (r) return r;
  if (global_ok_out) *global_ok_out = one;
  // bisection is shard-local: a rank bisects iff its own check failed
  return rlc_finish(c, codes_out, bitmap_out, stats4);
}

extern "C" int cess_bls_comm_barrier(cess_bls_ctx* c) {
  double v = 0;
  return cess_bls_comm_max_f64(c, &v);
}

extern "C" int cess_bls_comm_max_f64(cess_bls_ctx* c, double* value) {
  ENTRY(c);
  if (!c->xport) return CESS_BLS_E_NO_COMM;
  // a NULL value still takes part (the collective must not depend on it)
  double v = value ? *value : 0.0;
  const int r = c->xport->max_f64(&v);
  if (r) return r;
  if (!value) return CESS_BLS_E_INVALID_ARG;
  *value = v;
  return CESS_BLS_OK;
}

// ---------------------------------------------------------------------------
// one process, several GPUs (cess_bls_config.n_devices > 1)
// ---------------------------------------------------------------------------
int cess_multi_create(const cess_bls_config* cfg, int ndev, cess_bls_ctx* c) {
  const int nd = cfg->n_devices;
  c->device = -1;
  c->flags = cfg->flags;
  c->mode = cfg->mode;
  for (int k = 0; k < nd; k++) {
    const int dev = cfg->devices ? cfg->devices[k] : k;
    if (dev < 0 || dev >= ndev) return CESS_BLS_E_INVALID_ARG;
    cess_bls_config sc = *cfg;
    sc.device = dev;
    sc.n_devices = 1;
    sc.devices = nullptr;
    cess_bls_ctx* s = nullptr;
    int r = cess_bls_ctx_create(&sc, &s);
    if (r) return r;
    c->subs.push_back(s);
  }
  c->cap = c->subs[0]->cap;
  return CESS_BLS_OK;
}

// Run f(sub, begin, end) for every sub-context's shard of n records on its own
// host thread; shards are whole bitmap words (shard_of).  First failure wins.
template <class F>
static int for_each_shard(cess_bls_ctx* c, uint64_t n, F&& f) {
  const int nd = (int)c->subs.size();
  std::vector<int> st(nd, CESS_BLS_OK);
  std::vector<std::thread> th;
  for (int k = 0; k < nd; k++) {
    uint64_t b, e;
    shard_of(n, nd, k, &b, &e, nullptr);
    if (e <= b) continue;
    th.emplace_back([&, k, b, e] { st[k] = f(c->subs[k], b, e); });
  }
  for (auto& t : th) t.join();
  for (int v : st)
    if (v) return v;
  return CESS_BLS_OK;
}

int cess_multi_verify(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                      const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out, bool rlc, const uint8_t* seed32,
                      uint64_t* stats4) {
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !pks || !offs) return CESS_BLS_E_INVALID_ARG;
  if (!rlc)
    return for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
      return verify_host(s, e - b, sigs + 48 * b, pks + 96 * b, msgs, offs + b, nullptr,
                         codes_out ? codes_out + b : nullptr, bitmap_out ? bitmap_out + b / 64 : nullptr, nullptr);
    });
  // RLC: every device checks its shard (distinct scalar index ranges), the Gt
  // partials are multiplied on device 0 (the batch-level verdict, unused for
  // the codes), and each device bisects iff its own check failed
  const int nd = (int)c->subs.size();
  std::vector<uint8_t> gts((size_t)nd * 576, 0);
  std::vector<std::vector<uint64_t>> st(nd, std::vector<uint64_t>(4, 0));
  uint8_t seed[32];
  if (seed32) memcpy(seed, seed32, 32);
  else if (os_random(seed, 32)) return CESS_BLS_E_INVALID_ARG;
  for (int k = 0; k < nd; k++) gts[(size_t)k * 576 + 47] = 1;   // an empty shard's partial is one
  // the device index goes into the scalar index (k << 40), as the rank does
  // across processes, so no r_i is shared between shards under one seed
  int r = for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    int k = 0;
    while (c->subs[k] != s) k++;
    return rlc_begin_at(s, e - b, sigs + 48 * b, pks + 96 * b, msgs, offs + b, seed, (uint64_t)k << 40,
                        &gts[(size_t)k * 576]);
  });
  if (r) return r;
  int one = 0;
  r = gt_product_is_one(c->subs[0], nd, gts.data(), false, &one);
  if (r) return r;
  r = for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    int k = 0;
    while (c->subs[k] != s) k++;
    return rlc_finish(s, codes_out ? codes_out + b : nullptr, bitmap_out ? bitmap_out + b / 64 : nullptr,
                      st[k].data());
  });
  if (r) return r;
  if (stats4) {
    for (int q = 0; q < 3; q++) {
      stats4[q] = 0;
      for (int k = 0; k < nd; k++) stats4[q] += st[k][q];
    }
    stats4[3] = 0;
    for (int k = 0; k < nd; k++) stats4[3] = std::max(stats4[3], st[k][3]);
  }
  return CESS_BLS_OK;
}

int cess_multi_verify_var(cess_bls_ctx* c, size_t n, const uint8_t* sig_data, const uint64_t* sig_offsets,
                          const uint8_t* pk_data, const uint64_t* pk_offsets, const uint8_t* msgs,
                          const uint64_t* msg_offsets, uint8_t* codes_out, uint64_t* bitmap_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!sig_offsets || !pk_offsets || !msg_offsets) return CESS_BLS_E_INVALID_ARG;
  return for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    return verify_var_host(s, e - b, sig_data, sig_offsets + b, pk_data, pk_offsets + b, msgs, msg_offsets + b,
                           codes_out ? codes_out + b : nullptr, bitmap_out ? bitmap_out + b / 64 : nullptr);
  });
}

int cess_multi_keys_load(cess_bls_ctx* c, size_t k, const uint8_t* pks, uint8_t* key_codes_out) {
  // the table is replicated on every device; codes from device 0
  const int nd = (int)c->subs.size();
  std::vector<int> st(nd, CESS_BLS_OK);
  std::vector<std::thread> th;
  for (int d = 0; d < nd; d++)
    th.emplace_back([&, d] { st[d] = cess_keys_load_one(c->subs[d], k, pks, d == 0 ? key_codes_out : nullptr); });
  for (auto& t : th) t.join();
  for (int v : st)
    if (v) return v;
  return CESS_BLS_OK;
}

int cess_multi_keyed(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint32_t* key_idx, const uint8_t* msgs,
                     const uint64_t* offs, uint8_t* codes_out, uint64_t* bitmap_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !key_idx || !offs) return CESS_BLS_E_INVALID_ARG;
  return for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    return cess_keyed_one(s, e - b, sigs + 48 * b, key_idx + b, msgs, offs + b, codes_out ? codes_out + b : nullptr,
                          bitmap_out ? bitmap_out + b / 64 : nullptr);
  });
}

int cess_multi_gen(cess_bls_ctx* c, int kind, size_t n, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs,
                   uint8_t* out) {
  if (n == 0) return CESS_BLS_OK;
  const size_t ob = kind == 0 ? 96 : 48;
  return for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    return cess_gen_one(s, kind, e - b, sks ? sks + 32 * b : nullptr, msgs, offs ? offs + b : nullptr, out + ob * b);
  });
}

int cess_multi_gt(cess_bls_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                  const uint64_t* offs, uint8_t* codes_out, uint8_t* gt_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!sigs || !pks || !offs) return CESS_BLS_E_INVALID_ARG;
  return for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    return verify_host(s, e - b, sigs + 48 * b, pks + 96 * b, msgs, offs + b, nullptr,
                       codes_out ? codes_out + b : nullptr, nullptr, gt_out + 576 * b);
  });
}

int cess_rsa_one(cess_bls_ctx* s, size_t n, const uint32_t* key_idx, const uint8_t* sigs, const uint64_t* soffs,
                 const uint8_t* msgs, const uint64_t* moffs, uint8_t* codes_out, uint64_t* bitmap_out);

int cess_multi_rsa(cess_bls_ctx* c, size_t n, const uint32_t* key_idx, const uint8_t* sigs, const uint64_t* soffs,
                   const uint8_t* msgs, const uint64_t* moffs, uint8_t* codes_out, uint64_t* bitmap_out) {
  if (n == 0) return CESS_BLS_OK;
  if (!key_idx || !soffs || !moffs) return CESS_BLS_E_INVALID_ARG;
  return for_each_shard(c, n, [&](cess_bls_ctx* s, uint64_t b, uint64_t e) {
    return cess_rsa_one(s, e - b, key_idx + b, sigs, soffs + b, msgs, moffs + b, codes_out ? codes_out + b : nullptr,
                        bitmap_out ? bitmap_out + b / 64 : nullptr);
  });
}
