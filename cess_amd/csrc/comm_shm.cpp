// Host shared-memory transport of the sharded entry points (comm.hpp), the
// transport-independent merge (gather_verdicts, agree) and the context-free
// communicator of include/cess_bls.h (cess_bls_comm_open_shm & co).
//
// Segment layout: one 4 KiB header page (magic, rank count, slot size, a
// generation barrier, attach and abort flags), then one slot of kSlotBytes per
// rank.  An all-gather moves its blocks through the slots in chunks of at
// most kSlotBytes: every rank writes its chunk into its own slot, a barrier,
// every rank reads the others' slots, a barrier.  Waits are bounded
// (CESS_BLS_COMM_TIMEOUT_MS, default 300 s): a rank that times out marks the
// segment aborted, so its peers fail fast with CESS_BLS_E_COMM instead of
// hanging.
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/random.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "comm.hpp"

namespace cess_host {

double comm_now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

double comm_timeout_ms() {
  if (const char* e = getenv("CESS_BLS_COMM_TIMEOUT_MS")) {
    const double v = strtod(e, nullptr);
    if (v > 0) return v;
  }
  return 300e3;
}

namespace {

constexpr uint64_t kMagic = 0x434553535f534d31ull;   // "CESS_SM1"
constexpr size_t kHeaderBytes = 4096;
constexpr size_t kSlotBytes = 8u << 20;

struct ShmHeader {
  std::atomic<uint64_t> magic;
  uint32_t nranks;
  uint32_t pad;
  uint64_t slot_bytes;
  std::atomic<uint32_t> arrived;
  std::atomic<uint32_t> gen;
  std::atomic<uint32_t> attached;
  std::atomic<uint32_t> aborted;
};
static_assert(sizeof(ShmHeader) <= kHeaderBytes, "header page");
static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<uint64_t>::is_always_lock_free,
              "process-shared atomics must be lock-free");

double now_ms() { return comm_now_ms(); }
double timeout_ms() { return comm_timeout_ms(); }

// spin briefly, then yield, then sleep: ranks may wait seconds for a peer's
// verification to finish
void backoff(int& spins) {
  if (++spins < 256) return;
  if (spins < 4096) {
    sched_yield();
    return;
  }
  usleep(100);
}

class ShmTransport final : public Transport {
 public:
  ~ShmTransport() override {
    if (base_) munmap(base_, bytes_);
  }
  const char* kind() const override { return "shm"; }

  int open(const char* name, int nranks, int rank) {
    if (!name || !name[0] || nranks <= 0 || rank < 0 || rank >= nranks) return CESS_BLS_E_INVALID_ARG;
    this->nranks = nranks;
    this->rank = rank;
    tmo_ = timeout_ms();
    bytes_ = kHeaderBytes + (size_t)nranks * kSlotBytes;
    const double t0 = now_ms();
    int fd = -1;
    if (rank == 0) {
      fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) return CESS_BLS_E_COMM;   // the name must be fresh (cess_bls_comm_shm_name)
      if (ftruncate(fd, (off_t)bytes_) != 0) {
        close(fd);
        shm_unlink(name);
        return CESS_BLS_E_COMM;
      }
    } else {
      int spins = 0;
      while ((fd = shm_open(name, O_RDWR, 0600)) < 0) {
        if (errno != ENOENT || now_ms() - t0 > tmo_) return CESS_BLS_E_COMM;
        backoff(spins);
      }
      // wait until rank 0 has sized the segment
      spins = 0;
      for (;;) {
        struct stat st;
        if (fstat(fd, &st) != 0) {
          close(fd);
          return CESS_BLS_E_COMM;
        }
        if ((size_t)st.st_size >= bytes_) break;
        if (now_ms() - t0 > tmo_) {
          close(fd);
          return CESS_BLS_E_COMM;
        }
        backoff(spins);
      }
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      if (rank == 0) shm_unlink(name);
      return CESS_BLS_E_COMM;
    }
    base_ = static_cast<char*>(p);
    h_ = reinterpret_cast<ShmHeader*>(base_);
    if (rank == 0) {
      h_->nranks = (uint32_t)nranks;
      h_->slot_bytes = kSlotBytes;
      h_->arrived.store(0, std::memory_order_relaxed);
      h_->gen.store(0, std::memory_order_relaxed);
      h_->attached.store(0, std::memory_order_relaxed);
      h_->aborted.store(0, std::memory_order_relaxed);
      h_->magic.store(kMagic, std::memory_order_release);
    } else {
      int spins = 0;
      while (h_->magic.load(std::memory_order_acquire) != kMagic) {
        if (now_ms() - t0 > tmo_) return CESS_BLS_E_COMM;
        backoff(spins);
      }
      if (h_->nranks != (uint32_t)nranks || h_->slot_bytes != kSlotBytes) return CESS_BLS_E_INVALID_ARG;
    }
    h_->attached.fetch_add(1, std::memory_order_acq_rel);
    const int r = barrier();
    // every rank has the segment mapped: the name can go (no /dev/shm leak)
    if (rank == 0) shm_unlink(name);
    return r;
  }

  int barrier() {
    if (h_->aborted.load(std::memory_order_acquire)) return CESS_BLS_E_COMM;
    const uint32_t g = h_->gen.load(std::memory_order_acquire);
    if (h_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)nranks) {
      h_->arrived.store(0, std::memory_order_relaxed);
      h_->gen.fetch_add(1, std::memory_order_release);
      return CESS_BLS_OK;
    }
    const double t0 = now_ms();
    int spins = 0;
    while (h_->gen.load(std::memory_order_acquire) == g) {
      if (h_->aborted.load(std::memory_order_acquire)) return CESS_BLS_E_COMM;
      if (now_ms() - t0 > tmo_) {
        h_->aborted.store(1, std::memory_order_release);
        return CESS_BLS_E_COMM;
      }
      backoff(spins);
    }
    return CESS_BLS_OK;
  }

  char* slot(int r) const { return base_ + kHeaderBytes + (size_t)r * kSlotBytes; }

  int allgather_host(void* buf, size_t bytes) override {
    char* b = static_cast<char*>(buf);
    if (bytes == 0) return barrier();
    for (size_t off = 0; off < bytes; off += kSlotBytes) {
      const size_t len = std::min(kSlotBytes, bytes - off);
      memcpy(slot(rank), b + (size_t)rank * bytes + off, len);
      int r = barrier();
      if (r) return r;
      for (int q = 0; q < nranks; q++)
        if (q != rank) memcpy(b + (size_t)q * bytes + off, slot(q), len);
      r = barrier();   // slots are rewritten by the next chunk
      if (r) return r;
    }
    return CESS_BLS_OK;
  }

  int max_i64(int64_t* v, int n) override {
    std::vector<int64_t> all((size_t)nranks * n);
    memcpy(&all[(size_t)rank * n], v, n * sizeof(int64_t));
    int r = allgather_host(all.data(), n * sizeof(int64_t));
    if (r) return r;
    for (int q = 0; q < nranks; q++)
      for (int j = 0; j < n; j++) v[j] = std::max(v[j], all[(size_t)q * n + j]);
    return CESS_BLS_OK;
  }

  int max_f64(double* v) override {
    std::vector<double> all(nranks);
    all[rank] = *v;
    int r = allgather_host(all.data(), sizeof(double));
    if (r) return r;
    for (double x : all) *v = std::max(*v, x);
    return CESS_BLS_OK;
  }

 private:
  char* base_ = nullptr;
  size_t bytes_ = 0;
  ShmHeader* h_ = nullptr;
  double tmo_ = 300e3;
};

}  // namespace

int make_shm_transport(const char* name, int nranks, int rank, Transport** out) {
  *out = nullptr;
  ShmTransport* t = new ShmTransport();
  const int r = t->open(name, nranks, rank);
  if (r) {
    delete t;
    return r;
  }
  *out = t;
  return CESS_BLS_OK;
}

int Transport::allgather_dev(int dev, void* dbuf, size_t bytes, hipStream_t s) {
  if (bytes == 0) return allgather_host(nullptr, 0);
  if (hipSetDevice(dev) != hipSuccess) return CESS_BLS_E_HIP;
  std::vector<char> h((size_t)nranks * bytes);
  char* d = static_cast<char*>(dbuf);
  const size_t mine = (size_t)rank * bytes;
  // a failed copy still takes part in the all-gather (the peers are in it);
  // the failure is returned afterwards
  int st = CESS_BLS_OK;
  if (hipMemcpyAsync(h.data() + mine, d + mine, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    st = CESS_BLS_E_HIP;
  int r = allgather_host(h.data(), bytes);
  if (r) return r;
  if (st) return st;
  for (int q = 0; q < nranks; q++) {
    if (q == rank) continue;
    if (hipMemcpyAsync(d + (size_t)q * bytes, h.data() + (size_t)q * bytes, bytes, hipMemcpyHostToDevice, s) !=
        hipSuccess)
      return CESS_BLS_E_HIP;
  }
  // h is a host temporary: the copies must finish before it goes
  if (hipStreamSynchronize(s) != hipSuccess) return CESS_BLS_E_HIP;
  return CESS_BLS_OK;
}

int agree(Transport& t, int status) {
  int64_t v = status < 0 ? -(int64_t)status : 0;   // statuses are 0 or negative
  const int r = t.max_i64(&v, 1);
  if (r) return r;
  return (int)-v;
}

int same_on_all_ranks(Transport& t, uint64_t v, bool* same) {
  // max over ranks of (v, -v) is (v, -v) on every rank iff all v are equal
  // (values below 2^63; larger ones never pass)
  int64_t m[2] = {(int64_t)(v & 0x7fffffffffffffffull), -(int64_t)(v & 0x7fffffffffffffffull)};
  const int64_t want0 = m[0], want1 = m[1];
  const int r = t.max_i64(m, 2);
  if (r) return r;
  *same = m[0] == want0 && m[1] == want1 && v < (1ull << 63);
  return CESS_BLS_OK;
}

int gather_verdicts(Transport& t, uint64_t n, const uint8_t* shard_codes, uint8_t* codes_out, uint64_t* bitmap_out) {
  uint64_t b, e, wpr;
  shard_of(n, t.nranks, t.rank, &b, &e, &wpr);
  const uint64_t m = e - b;
  // the block sizes of the all-gathers follow from n: a rank with another n
  // would desynchronise the chunked transfers, so n is checked first, and a
  // missing shard buffer is agreed on before any data moves
  bool same = false;
  int r = same_on_all_ranks(t, n, &same);
  if (r) return r;
  if (!same) return CESS_BLS_E_INVALID_ARG;
  r = agree(t, (m && !shard_codes) ? CESS_BLS_E_INVALID_ARG : CESS_BLS_OK);
  if (r) return r;
  if (wpr == 0) return CESS_BLS_OK;   // empty batch
  // per-rank blocks of wpr words / wpr * 64 code bytes; 0xff marks the code
  // bytes past a short last shard (never a verdict)
  std::vector<uint64_t> words((size_t)t.nranks * wpr, 0);
  // (both all-gathers run on every rank whatever its output pointers: the
  // collective sequence must not depend on per-rank arguments)
  std::vector<uint8_t> codes((size_t)t.nranks * wpr * 64, 0xff);
  uint64_t* mw = &words[(size_t)t.rank * wpr];
  for (uint64_t i = 0; i < m; i++)
    if (shard_codes[i] == 0) mw[i >> 6] |= 1ull << (i & 63);
  r = t.allgather_host(words.data(), wpr * 8);
  if (r) return r;
  if (m) memcpy(&codes[(size_t)t.rank * wpr * 64], shard_codes, m);
  r = t.allgather_host(codes.data(), wpr * 64);
  if (r) return r;
  if (codes_out) memcpy(codes_out, codes.data(), n);
  if (bitmap_out) memcpy(bitmap_out, words.data(), ((n + 63) / 64) * 8);
  return CESS_BLS_OK;
}

}  // namespace cess_host

// ---------------------------------------------------------------------------
// context-free communicator (include/cess_bls.h)
// ---------------------------------------------------------------------------
struct cess_bls_comm {
  cess_host::Transport* t = nullptr;
};

extern "C" int cess_bls_comm_shm_name(char name_out[CESS_BLS_COMM_NAME_BYTES]) {
  if (!name_out) return CESS_BLS_E_INVALID_ARG;
  uint8_t rnd[8];
  size_t got = 0;
  while (got < sizeof(rnd)) {
    const ssize_t r = getrandom(rnd + got, sizeof(rnd) - got, 0);
    if (r <= 0) return CESS_BLS_E_COMM;
    got += (size_t)r;
  }
  uint64_t x;
  memcpy(&x, rnd, 8);
  snprintf(name_out, CESS_BLS_COMM_NAME_BYTES, "/cess_bls_%d_%016llx", (int)getpid(), (unsigned long long)x);
  return CESS_BLS_OK;
}

extern "C" int cess_bls_comm_open_shm(const char* name, int nranks, int rank, cess_bls_comm** out) {
  if (!out) return CESS_BLS_E_INVALID_ARG;
  *out = nullptr;
  cess_host::Transport* t = nullptr;
  const int r = cess_host::make_shm_transport(name, nranks, rank, &t);
  if (r) return r;
  *out = new cess_bls_comm{t};
  return CESS_BLS_OK;
}

extern "C" void cess_bls_comm_close(cess_bls_comm* comm) {
  if (!comm) return;
  delete comm->t;
  delete comm;
}

extern "C" int cess_bls_comm_agree(cess_bls_comm* comm, int status, int* agreed_out) {
  if (!comm || !agreed_out) return CESS_BLS_E_INVALID_ARG;
  int64_t v = status < 0 ? -(int64_t)status : 0;
  const int r = comm->t->max_i64(&v, 1);
  if (r) return r;
  *agreed_out = (int)-v;
  return CESS_BLS_OK;
}

extern "C" int cess_bls_comm_gather_verdicts(cess_bls_comm* comm, uint64_t n_total, const uint8_t* shard_codes,
                                             uint8_t* codes_out, uint64_t* bitmap_out) {
  if (!comm) return CESS_BLS_E_INVALID_ARG;
  return cess_host::gather_verdicts(*comm->t, n_total, shard_codes, codes_out, bitmap_out);
}
