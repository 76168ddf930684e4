// RCCL communicators of the row-sharded step (N > 1), enqueued on the CALLER's stream.
//
// The row exchange (route ids -> owner gather -> rows back; per-entry gradient rows -> owner)
// and the dense-gradient all-reduce are collectives between kernels of the same step.  Issued
// through torch.distributed they run on the process group's internal stream, and every one of
// them costs two cross-queue event edges (compute -> collective -> compute): ~10-20 us each on
// MI355X, ~55 us of idle GPU per step at one rank (profiles/r04_shard_gaps.txt).  Here the
// collectives are RCCL calls on the stream the step's kernels run on -- no edges at all.
//
// RCCL is the one torch already loaded (its librccl.so, passed to fbn_comm_load by path and
// bound with dlopen/dlsym): one RCCL runtime per process, whatever rccl the system also has.
// The unique id travels over torch.distributed (exchange.py NativeComm); only the data path is
// here.  All-to-all with per-peer counts = grouped ncclSend/ncclRecv (the counts are host ints,
// read at call time); equal-split all-to-all = ncclAllToAll; sum all-reduce in place.
//
// Watchdog (fbn_comm_watch / fbn_comm_heartbeat): torch.distributed aborts a process group whose
// collective does not complete in time; these communicators bypass that, so a rank whose peer
// never posts would wait forever.  The step calls fbn_comm_heartbeat at its end (a recordable entry
// point: every step-program replay posts it too), which notes the host time and records an event on
// the step's stream.  A monitor thread aborts EVERY live communicator (ncclCommAbort: RCCL's kernels
// poll the abort flag and exit, so the blocked stream -- and the host waiting on it -- drain) once
// the last heartbeat is older than the timeout while its event has not completed.  An idle process
// (the event complete) is never aborted.  Every call on an aborted communicator then fails with the
// watchdog's message.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <set>
#include <thread>

void fbn_set_error(const char* msg);

namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllToAll) all_to_all = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;   // optional (the watchdog)
};

Rccl g_rccl;

struct Comm {
  ncclComm_t comm;
  int world;
  int rank;
  std::atomic<int> aborted{0};
};

// the watchdog's state (one per process: a hang anywhere in the step aborts every communicator)
struct Watch {
  std::mutex mu;
  std::set<Comm*> live;
  std::thread th;
  std::atomic<bool> running{false};
  std::atomic<long long> timeout_ms{0};
  std::atomic<long long> beat_ms{0};        // host time of the last heartbeat (0 = none yet)
  std::atomic<int> fired{0};
  hipEvent_t ev = nullptr;                  // recorded by each heartbeat on the step's stream
  int device = -1;
  bool ev_recorded = false;
};
Watch g_watch;

long long now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void abort_all() {
  std::lock_guard<std::mutex> g(g_watch.mu);
  for (Comm* c : g_watch.live) {
    if (c->aborted.exchange(1)) continue;
    if (g_rccl.comm_abort && c->comm) (void)g_rccl.comm_abort(c->comm);
  }
}

void monitor() {
  if (g_watch.device >= 0) (void)hipSetDevice(g_watch.device);
  while (g_watch.running.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const long long beat = g_watch.beat_ms.load(), tmo = g_watch.timeout_ms.load();
    if (beat == 0 || tmo <= 0 || g_watch.fired.load()) continue;
    if (now_ms() - beat <= tmo) continue;
    bool pending = true;   // a heartbeat without an event (host-only callers, tests) counts as pending
    {
      std::lock_guard<std::mutex> g(g_watch.mu);
      if (g_watch.ev && g_watch.ev_recorded) pending = hipEventQuery(g_watch.ev) == hipErrorNotReady;
    }
    if (!pending) continue;   // idle: the last step finished long ago
    fprintf(stderr, "[fbn_comm] watchdog: no step completed for %lld ms -- aborting every RCCL communicator\n",
            now_ms() - beat);
    g_watch.fired.store(1);
    abort_all();
  }
}

bool aborted(const Comm* c, const char* where) {
  if (!c->aborted.load()) return false;
  char msg[224];
  snprintf(msg, sizeof(msg), "%s: the communicator was aborted by the watchdog (no step completed within %lld ms)",
           where, g_watch.timeout_ms.load());
  fbn_set_error(msg);
  return true;
}

int fail(const char* where, ncclResult_t r) {
  char msg[256];
  snprintf(msg, sizeof(msg), "%s: %s%s", where, g_rccl.error_string ? g_rccl.error_string(r) : "rccl error",
           g_watch.fired.load() ? " (the watchdog aborted the communicators: no step completed in time)" : "");
  fbn_set_error(msg);
  return 3;
}

int need_loaded(const char* where) {
  if (g_rccl.handle) return 0;
  char msg[160];
  snprintf(msg, sizeof(msg), "%s: RCCL not loaded (fbn_comm_load first)", where);
  fbn_set_error(msg);
  return 1;
}

template <typename F>
bool bind(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  return *out != nullptr;
}

}  // namespace

// Bind the RCCL library at `path` (torch's own librccl.so: already mapped, so no second copy).
extern "C" int fbn_comm_load(const char* path) {
  if (g_rccl.handle) return 0;
  if (!path) {
    fbn_set_error("fbn_comm_load: null path");
    return 1;
  }
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    char msg[512];
    snprintf(msg, sizeof(msg), "fbn_comm_load: dlopen(%s) failed: %s", path, dlerror());
    fbn_set_error(msg);
    return 1;
  }
  Rccl r;
  r.handle = h;
  bool ok = bind(h, "ncclGetUniqueId", &r.get_unique_id) && bind(h, "ncclCommInitRank", &r.comm_init_rank) &&
            bind(h, "ncclCommDestroy", &r.comm_destroy) && bind(h, "ncclSend", &r.send) &&
            bind(h, "ncclRecv", &r.recv) && bind(h, "ncclGroupStart", &r.group_start) &&
            bind(h, "ncclGroupEnd", &r.group_end) && bind(h, "ncclAllReduce", &r.all_reduce) &&
            bind(h, "ncclAllToAll", &r.all_to_all) && bind(h, "ncclAllGather", &r.all_gather) &&
            bind(h, "ncclGetErrorString", &r.error_string);
  if (!ok) {
    fbn_set_error("fbn_comm_load: the library lacks an RCCL entry point");
    dlclose(h);
    return 1;
  }
  bind(h, "ncclCommAbort", &r.comm_abort);
  g_rccl = r;
  return 0;
}

extern "C" int fbn_comm_id_bytes() { return (int)sizeof(ncclUniqueId); }

// rank 0: a fresh unique id (NCCL_UNIQUE_ID_BYTES bytes into `out`) for every rank's fbn_comm_init
extern "C" int fbn_comm_unique_id(void* out) {
  if (int rc = need_loaded("fbn_comm_unique_id")) return rc;
  if (!out) {
    fbn_set_error("fbn_comm_unique_id: null out");
    return 1;
  }
  ncclUniqueId id;
  ncclResult_t r = g_rccl.get_unique_id(&id);
  if (r != ncclSuccess) return fail("fbn_comm_unique_id", r);
  memcpy(out, &id, sizeof(id));
  return 0;
}

// collective over the `world` ranks: every rank calls it with the same id, on its own device
extern "C" int fbn_comm_init(void** out, const void* id, int world, int rank) {
  if (int rc = need_loaded("fbn_comm_init")) return rc;
  if (!out || !id || world < 1 || rank < 0 || rank >= world) {
    fbn_set_error("fbn_comm_init: bad arguments");
    return 1;
  }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  Comm* c = new Comm{nullptr, world, rank};
  ncclResult_t r = g_rccl.comm_init_rank(&c->comm, world, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail("fbn_comm_init", r);
  }
  *out = c;
  std::lock_guard<std::mutex> g(g_watch.mu);
  g_watch.live.insert(c);
  return 0;
}

extern "C" int fbn_comm_destroy(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return 0;
  {
    std::lock_guard<std::mutex> g(g_watch.mu);
    g_watch.live.erase(c);
  }
  // (an aborted communicator was already torn down by ncclCommAbort)
  if (g_rccl.handle && c->comm && !c->aborted.load()) (void)g_rccl.comm_destroy(c->comm);
  delete c;
  return 0;
}

// Abort one communicator now (its pending and future operations fail; RCCL's kernels exit).
extern "C" int fbn_comm_abort(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return 0;
  std::lock_guard<std::mutex> g(g_watch.mu);
  if (!c->aborted.exchange(1) && g_rccl.comm_abort && c->comm) (void)g_rccl.comm_abort(c->comm);
  return 0;
}

// Start (or retune) the watchdog: timeout_ms <= 0 disarms it.  The calling thread's current device is
// the one whose step events the monitor queries.
extern "C" int fbn_comm_watch(long long timeout_ms) {
  g_watch.timeout_ms.store(timeout_ms);
  if (g_watch.running.load() || timeout_ms <= 0) return 0;
  (void)hipGetDevice(&g_watch.device);
  g_watch.running.store(true);
  g_watch.th = std::thread(monitor);
  g_watch.th.detach();   // lives as long as the process (joined by nobody: it only sleeps and polls)
  return 0;
}

// The end of a step: the host time now, and an event on `stream` (NULL stream + host-only callers: no
// event, the beat alone) -- the monitor aborts when the beat is older than the timeout and the event
// has not completed.
extern "C" int fbn_comm_heartbeat(void* stream) {
  if (stream) {
    std::lock_guard<std::mutex> g(g_watch.mu);
    if (!g_watch.ev && hipEventCreateWithFlags(&g_watch.ev, hipEventDisableTiming) != hipSuccess) {
      g_watch.ev = nullptr;
      fbn_set_error("fbn_comm_heartbeat: hipEventCreateWithFlags failed");
      return 2;
    }
    if (hipEventRecord(g_watch.ev, static_cast<hipStream_t>(stream)) != hipSuccess) {
      fbn_set_error("fbn_comm_heartbeat: hipEventRecord failed");
      return 2;
    }
    g_watch.ev_recorded = true;
  }
  g_watch.beat_ms.store(now_ms());
  return 0;
}

// 1 once the watchdog has aborted the communicators (0 otherwise); a communicator's own state with
// a handle: 1 if it was aborted (by the watchdog or fbn_comm_abort).
extern "C" int fbn_comm_watchdog_fired(void* comm) {
  if (comm) return static_cast<Comm*>(comm)->aborted.load();
  return g_watch.fired.load();
}

// All-to-all with per-peer counts (rows of `row_bytes` bytes; send_counts / recv_counts: host
// int arrays of `world` entries, read now).  Blocks are packed in rank order on both sides.
extern "C" int fbn_comm_alltoallv(void* comm, const void* send, const int* send_counts, void* recv,
                                  const int* recv_counts, long long row_bytes, void* stream) {
  if (int rc = need_loaded("fbn_comm_alltoallv")) return rc;
  Comm* c = static_cast<Comm*>(comm);
  if (!c || !send_counts || !recv_counts || row_bytes <= 0) {
    fbn_set_error("fbn_comm_alltoallv: bad arguments");
    return 1;
  }
  if (aborted(c, "fbn_comm_alltoallv")) return 3;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const char* sp = static_cast<const char*>(send);
  char* rp = static_cast<char*>(recv);
  for (int p = 0; p < c->world; ++p) {
    if (send_counts[p] < 0 || recv_counts[p] < 0) {
      fbn_set_error("fbn_comm_alltoallv: negative count");
      return 1;
    }
  }
  ncclResult_t r = g_rccl.group_start();
  if (r != ncclSuccess) return fail("fbn_comm_alltoallv", r);
  size_t so = 0, ro = 0;
  for (int p = 0; p < c->world && r == ncclSuccess; ++p) {
    size_t sb = (size_t)send_counts[p] * (size_t)row_bytes, rb = (size_t)recv_counts[p] * (size_t)row_bytes;
    if (sb) r = g_rccl.send(sp + so, sb, ncclUint8, p, c->comm, s);
    if (r == ncclSuccess && rb) r = g_rccl.recv(rp + ro, rb, ncclUint8, p, c->comm, s);
    so += sb;
    ro += rb;
  }
  ncclResult_t e = g_rccl.group_end();
  if (r != ncclSuccess) return fail("fbn_comm_alltoallv", r);
  if (e != ncclSuccess) return fail("fbn_comm_alltoallv", e);
  return 0;
}

// Equal-split all-to-all: `bytes_per_peer` bytes to and from every rank.
extern "C" int fbn_comm_alltoall(void* comm, const void* send, void* recv, long long bytes_per_peer, void* stream) {
  if (int rc = need_loaded("fbn_comm_alltoall")) return rc;
  Comm* c = static_cast<Comm*>(comm);
  if (!c || bytes_per_peer < 0) {
    fbn_set_error("fbn_comm_alltoall: bad arguments");
    return 1;
  }
  if (aborted(c, "fbn_comm_alltoall")) return 3;
  if (bytes_per_peer == 0) return 0;
  ncclResult_t r = g_rccl.all_to_all(send, recv, (size_t)bytes_per_peer, ncclUint8, c->comm,
                                     static_cast<hipStream_t>(stream));
  return r == ncclSuccess ? 0 : fail("fbn_comm_alltoall", r);
}

// Equal-split all-to-all WITHOUT the caller's own block (grouped ncclSend / ncclRecv to every
// peer): the fixed-capacity exchange keeps a rank's requests to itself in place -- the owner side
// reads / writes the requester's buffers for that block directly -- so no self copy crosses RCCL.
// A one-rank communicator does nothing here.
extern "C" int fbn_comm_alltoall_peers(void* comm, const void* send, void* recv, long long bytes_per_peer,
                                       void* stream) {
  if (int rc = need_loaded("fbn_comm_alltoall_peers")) return rc;
  Comm* c = static_cast<Comm*>(comm);
  if (!c || bytes_per_peer < 0) {
    fbn_set_error("fbn_comm_alltoall_peers: bad arguments");
    return 1;
  }
  if (aborted(c, "fbn_comm_alltoall_peers")) return 3;
  if (bytes_per_peer == 0 || c->world <= 1) return 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  ncclResult_t r = g_rccl.group_start();
  if (r != ncclSuccess) return fail("fbn_comm_alltoall_peers", r);
  for (int p = 0; p < c->world && r == ncclSuccess; ++p) {
    if (p == c->rank) continue;
    r = g_rccl.send(static_cast<const char*>(send) + (size_t)p * bytes_per_peer, (size_t)bytes_per_peer, ncclUint8,
                    p, c->comm, st);
    if (r == ncclSuccess)
      r = g_rccl.recv(static_cast<char*>(recv) + (size_t)p * bytes_per_peer, (size_t)bytes_per_peer, ncclUint8, p,
                      c->comm, st);
  }
  ncclResult_t e = g_rccl.group_end();
  if (r != ncclSuccess) return fail("fbn_comm_alltoall_peers", r);
  if (e != ncclSuccess) return fail("fbn_comm_alltoall_peers", e);
  return 0;
}

// In-place sum all-reduce of n elements: dtype 0 = f32, 1 = f64, 2 = i32.
extern "C" int fbn_comm_allreduce(void* comm, void* buf, long long n, int dtype, void* stream) {
  if (int rc = need_loaded("fbn_comm_allreduce")) return rc;
  Comm* c = static_cast<Comm*>(comm);
  if (!c || n < 0 || dtype < 0 || dtype > 2) {
    fbn_set_error("fbn_comm_allreduce: bad arguments");
    return 1;
  }
  if (aborted(c, "fbn_comm_allreduce")) return 3;
  if (n == 0) return 0;
  ncclDataType_t t = dtype == 0 ? ncclFloat32 : (dtype == 1 ? ncclFloat64 : ncclInt32);
  ncclResult_t r = g_rccl.all_reduce(buf, buf, (size_t)n, t, ncclSum, c->comm, static_cast<hipStream_t>(stream));
  return r == ncclSuccess ? 0 : fail("fbn_comm_allreduce", r);
}

// All-gather of `bytes_per_rank` bytes from every rank into recv (rank order) -- with fbn_sum_slices,
// deterministic mode's all-reduce: the ranks' contributions summed in rank order, the same bits on
// every rank and whatever reduction algorithm RCCL would have picked.
extern "C" int fbn_comm_allgather(void* comm, const void* send, void* recv, long long bytes_per_rank, void* stream) {
  if (int rc = need_loaded("fbn_comm_allgather")) return rc;
  Comm* c = static_cast<Comm*>(comm);
  if (!c || bytes_per_rank < 0 || (bytes_per_rank > 0 && (!send || !recv))) {
    fbn_set_error("fbn_comm_allgather: bad arguments");
    return 1;
  }
  if (aborted(c, "fbn_comm_allgather")) return 3;
  if (bytes_per_rank == 0) return 0;
  ncclResult_t r = g_rccl.all_gather(send, recv, (size_t)bytes_per_rank, ncclUint8, c->comm,
                                     static_cast<hipStream_t>(stream));
  return r == ncclSuccess ? 0 : fail("fbn_comm_allgather", r);
}
