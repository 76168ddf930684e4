// A host-memory stand-in for the RCCL entry points csrc/comm.cpp binds (TEST INFRASTRUCTURE:
// tests/test_comm_mock.py builds it with g++ and hands its path to fbn_comm_load).  The ranks of a
// "world" are threads of one process; a unique id names the world.  ncclSend copies its bytes into
// the peer's mailbox at once (never blocks); ncclRecv, inside a group, is completed at
// ncclGroupEnd by waiting for the matching message (same (src, dst) pair, in posting order, as
// NCCL's send/recv matching).  Buffers are host pointers, streams are ignored.  The point is the
// world > 1 bookkeeping of fbn_comm_alltoallv / fbn_comm_alltoall / fbn_comm_allreduce (per-peer
// offsets, zero and uneven counts, row sizes), which RCCL itself cannot run on a one-GPU box.
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

extern "C" {
typedef enum { ncclSuccess = 0, ncclInvalidArgument = 4, ncclInternalError = 3 } ncclResult_t;
typedef enum { ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclFloat32 = 7, ncclFloat64 = 8 } ncclDataType_t;
typedef enum { ncclSum = 0 } ncclRedOp_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef struct MockComm* ncclComm_t;
typedef void* hipStream_t;
}

namespace {

struct World {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::deque<std::vector<char>>> box;   // (src, dst) -> messages
  // all-reduce rendezvous
  int arrived = 0, generation = 0;
  std::vector<double> acc, result;   // result: the last completed generation's sums
  bool aborted = false;              // ncclCommAbort on any rank: every wait returns an error
};

std::mutex g_mu;
std::map<uint64_t, std::shared_ptr<World>> g_worlds;
uint64_t g_next = 1;

struct PendingRecv {
  void* buf;
  size_t bytes;
  int peer;
};
thread_local int t_depth = 0;
thread_local std::vector<PendingRecv> t_recvs;
thread_local struct MockComm* t_comm = nullptr;

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclFloat32: return 4;
    case ncclFloat64: return 8;
  }
  return 0;
}

}  // namespace

struct MockComm {
  std::shared_ptr<World> w;
  int rank;
};

static ncclResult_t complete_recvs(MockComm* c) {
  World& w = *c->w;
  std::unique_lock<std::mutex> lk(w.mu);
  for (const PendingRecv& r : t_recvs) {
    auto key = std::make_pair(r.peer, c->rank);
    if (!w.cv.wait_for(lk, std::chrono::seconds(20), [&] { return w.aborted || !w.box[key].empty(); }) || w.aborted)
      return ncclInternalError;
    std::vector<char> msg = std::move(w.box[key].front());
    w.box[key].pop_front();
    if (msg.size() != r.bytes) return ncclInvalidArgument;   // a send / recv size mismatch
    memcpy(r.buf, msg.data(), r.bytes);
  }
  t_recvs.clear();
  return ncclSuccess;
}

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::lock_guard<std::mutex> g(g_mu);
  memset(id, 0, sizeof(*id));
  const uint64_t k = g_next++;
  memcpy(id->internal, &k, sizeof(k));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  uint64_t k;
  memcpy(&k, id.internal, sizeof(k));
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto& slot = g_worlds[k];
    if (!slot) {
      slot = std::make_shared<World>();
      slot->n = nranks;
    }
    w = slot;
  }
  if (w->n != nranks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  *comm = new MockComm{w, rank};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}

// the world's waits end with an error (a real abort also frees the communicator)
ncclResult_t ncclCommAbort(ncclComm_t comm) {
  {
    std::lock_guard<std::mutex> lk(comm->w->mu);
    comm->w->aborted = true;
  }
  comm->w->cv.notify_all();
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidArgument;
  if (--t_depth == 0 && t_comm) {
    ncclResult_t r = complete_recvs(t_comm);
    t_comm = nullptr;
    return r;
  }
  return ncclSuccess;
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t) {
  World& w = *comm->w;
  if (peer < 0 || peer >= w.n) return ncclInvalidArgument;
  const size_t bytes = count * type_size(dt);
  {
    std::lock_guard<std::mutex> lk(w.mu);
    w.box[std::make_pair(comm->rank, peer)].emplace_back((const char*)buf, (const char*)buf + bytes);
  }
  w.cv.notify_all();
  return ncclSuccess;
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t) {
  if (peer < 0 || peer >= comm->w->n) return ncclInvalidArgument;
  t_recvs.push_back({buf, count * type_size(dt), peer});
  t_comm = comm;
  if (t_depth == 0) return complete_recvs(comm);
  return ncclSuccess;
}

ncclResult_t ncclAllToAll(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclComm_t comm,
                          hipStream_t s) {
  const size_t bytes = count * type_size(dt);
  ncclGroupStart();
  for (int p = 0; p < comm->w->n; ++p) {
    ncclSend((const char*)send + p * bytes, count, dt, p, comm, s);
    ncclRecv((char*)recv + p * bytes, count, dt, p, comm, s);
  }
  return ncclGroupEnd();
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t s) {
  const size_t bytes = count * type_size(dt);
  ncclGroupStart();
  for (int p = 0; p < comm->w->n; ++p) {
    ncclSend(send, count, dt, p, comm, s);
    ncclRecv((char*)recv + p * bytes, count, dt, p, comm, s);
  }
  return ncclGroupEnd();
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t,
                           ncclComm_t comm, hipStream_t) {
  World& w = *comm->w;
  std::unique_lock<std::mutex> lk(w.mu);
  const int gen = w.generation;
  if (w.arrived == 0) w.acc.assign(count, 0.0);
  for (size_t i = 0; i < count; ++i) {
    double x = 0.0;
    if (dt == ncclFloat32) x = ((const float*)send)[i];
    else if (dt == ncclFloat64) x = ((const double*)send)[i];
    else if (dt == ncclInt32) x = ((const int32_t*)send)[i];
    w.acc[i] += x;
  }
  if (++w.arrived == w.n) {
    w.arrived = 0;
    w.result = w.acc;   // a rank of the next generation cannot complete it before every rank left this one
    ++w.generation;
    w.cv.notify_all();
  } else if (!w.cv.wait_for(lk, std::chrono::seconds(20), [&] { return w.aborted || w.generation != gen; }) ||
             w.generation == gen) {
    return ncclInternalError;
  }
  for (size_t i = 0; i < count; ++i) {
    if (dt == ncclFloat32) ((float*)recv)[i] = (float)w.result[i];
    else if (dt == ncclFloat64) ((double*)recv)[i] = w.result[i];
    else if (dt == ncclInt32) ((int32_t*)recv)[i] = (int32_t)w.result[i];
  }
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "mock rccl error"; }

}  // extern "C"
