// Step programs: the native step driver of the training loop (src/train_fibinet.py:113-123).
//
// One training step is ~25 launches of this library's C-ABI entry points on two streams with a
// few cross-stream edges.  Issued from Python (ctypes conversion + the trainer's sequencing) that
// costs ~0.4 ms of host time per step at C3 -- as much as the GPU work.  hipGraph replay avoids
// the host cost but adds its own per-edge cost for multi-stream graphs.  A step program is the
// third way: the host records the step's calls ONCE (entry point, its arguments, the stream
// edges) while running it, and replays them natively: the same launches on the same streams in
// the same order, so a replay is bit-identical to the eager step it was recorded from.
//
// Replay calls each recorded entry point through a packed-argument thunk generated from
// include/fibinet.h (csrc/plan_thunks.inc, ctr_recommendation_amd/gen_thunks.py): the thunk
// takes the recorded arguments as two arrays -- integer-class values (pointers, int, long long,
// size_t) as 64-bit words, float / double values as doubles (a float in the low 32 bits of its
// double) -- and makes an ordinary, well-typed call of the entry point's declared prototype.
// A recording names the entry point; its argument counts are checked against the thunk's.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "fibinet.h"

void fbn_set_error(const char* msg);

namespace {

constexpr int kMaxInt = 48;
constexpr int kMaxFlt = 8;

typedef uint64_t U;
typedef int (*ThunkFn)(const U* i, const double* f);

struct PlanThunk {
  const char* name;
  ThunkFn fn;
  int ni, nf;
};

// a float argument: the low 32 bits of its double slot (the recorder's encoding)
inline float plan_f32(double d) {
  uint64_t b;
  memcpy(&b, &d, sizeof(b));
  const uint32_t lo = (uint32_t)b;
  float x;
  memcpy(&x, &lo, sizeof(x));
  return x;
}

#include "plan_thunks.inc"

const PlanThunk* find_thunk(const char* name) {
  size_t lo = 0, hi = sizeof(kPlanThunks) / sizeof(kPlanThunks[0]);
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    const int c = strcmp(kPlanThunks[mid].name, name);
    if (c == 0) return &kPlanThunks[mid];
    if (c < 0) lo = mid + 1;
    else hi = mid;
  }
  return nullptr;
}

enum OpKind { kCall = 0, kRecord = 1, kWait = 2 };

struct Op {
  int kind;
  int slot;                // kRecord / kWait: event slot
  ThunkFn fn;              // kCall
  hipStream_t stream;      // kRecord / kWait
  U i[kMaxInt];
  double f[kMaxFlt];
};

struct Plan {
  int device;
  std::vector<Op> ops;
  std::vector<hipEvent_t> events;
};

int call_op(const Op& o) { return o.fn(o.i, o.f); }

// The program's events only order work between streams of one device, so their release need not be
// system scope (the default: an L2 writeback + invalidate at every record, ~6 us of idle on the
// recording stream before its next kernel).  FBN_PLAN_EVENT_SCOPE (A/B knob, read at event creation):
// "device" (default) -- hipEventDisableSystemFence; "release_device" -- hipEventReleaseToDevice;
// "system" -- the runtime's default fence.
unsigned event_flags() {
  const char* e = getenv("FBN_PLAN_EVENT_SCOPE");
  if (e && !strcmp(e, "system")) return hipEventDisableTiming;
  if (e && !strcmp(e, "release_device")) return hipEventDisableTiming | hipEventReleaseToDevice;
  return hipEventDisableTiming | hipEventDisableSystemFence;
}

int ensure_event(Plan* p, int slot) {
  while ((int)p->events.size() <= slot) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, event_flags()) != hipSuccess) {
      fbn_set_error("fbn_plan: hipEventCreateWithFlags failed");
      return 2;
    }
    p->events.push_back(e);
  }
  return 0;
}

}  // namespace

extern "C" int fbn_plan_create(void** out) {
  if (!out) {
    fbn_set_error("fbn_plan_create: null out");
    return 1;
  }
  Plan* p = new Plan();
  if (hipGetDevice(&p->device) != hipSuccess) p->device = 0;
  *out = p;
  return 0;
}

extern "C" int fbn_plan_destroy(void* plan) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p) return 0;
  for (hipEvent_t e : p->events) (void)hipEventDestroy(e);
  delete p;
  return 0;
}

extern "C" int fbn_plan_size(void* plan) { return plan ? (int)static_cast<Plan*>(plan)->ops.size() : 0; }

extern "C" int fbn_plan_add_call(void* plan, const char* name, const unsigned long long* iargs, int ni,
                                 const double* fargs, int nf) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p || !name || ni < 0 || nf < 0 || ni > kMaxInt || nf > kMaxFlt || (ni && !iargs) || (nf && !fargs)) {
    fbn_set_error("fbn_plan_add_call: bad arguments");
    return 1;
  }
  const PlanThunk* t = find_thunk(name);
  if (!t) {
    fbn_set_error("fbn_plan_add_call: not a recordable entry point of fibinet.h");
    return 1;
  }
  if (t->ni != ni || t->nf != nf) {
    fbn_set_error("fbn_plan_add_call: argument counts differ from the entry point's prototype");
    return 1;
  }
  Op o;
  memset(&o, 0, sizeof(o));
  o.kind = kCall;
  o.fn = t->fn;
  for (int k = 0; k < ni; ++k) o.i[k] = iargs[k];
  for (int k = 0; k < nf; ++k) o.f[k] = fargs[k];
  p->ops.push_back(o);
  return 0;
}

// stream edge, first half: record event `slot` on `stream` (hipEventRecord)
extern "C" int fbn_plan_add_record(void* plan, int slot, void* stream) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p || slot < 0) {
    fbn_set_error("fbn_plan_add_record: bad arguments");
    return 1;
  }
  if (int rc = ensure_event(p, slot)) return rc;
  Op o;
  memset(&o, 0, sizeof(o));
  o.kind = kRecord;
  o.slot = slot;
  o.stream = static_cast<hipStream_t>(stream);
  p->ops.push_back(o);
  return 0;
}

// stream edge, second half: `stream` waits for event `slot` (hipStreamWaitEvent)
extern "C" int fbn_plan_add_wait(void* plan, void* stream, int slot) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p || slot < 0) {
    fbn_set_error("fbn_plan_add_wait: bad arguments");
    return 1;
  }
  if (int rc = ensure_event(p, slot)) return rc;
  Op o;
  memset(&o, 0, sizeof(o));
  o.kind = kWait;
  o.slot = slot;
  o.stream = static_cast<hipStream_t>(stream);
  p->ops.push_back(o);
  return 0;
}

// Host wait for the program's event `slot` as its last replay (or the recording run) left it -- the
// sharded step's host check of the routed-ahead overflow flag waits for the routing this way.
extern "C" int fbn_plan_event_sync(void* plan, int slot) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p || slot < 0 || slot >= (int)p->events.size()) {
    fbn_set_error("fbn_plan_event_sync: bad arguments");
    return 1;
  }
  if (hipEventSynchronize(p->events[slot]) != hipSuccess) {
    fbn_set_error("fbn_plan_event_sync: hipEventSynchronize failed");
    return 2;
  }
  return 0;
}

// Replay every recorded op in order.  Returns 0, or the failing entry point's code (its
// message stays in fbn_last_error) with *failed = the op index.
extern "C" int fbn_plan_run(void* plan, int* failed) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p) {
    fbn_set_error("fbn_plan_run: null plan");
    return 1;
  }
  int n = (int)p->ops.size();
  for (int k = 0; k < n; ++k) {
    const Op& o = p->ops[k];
    int rc = 0;
    if (o.kind == kCall) {
      rc = call_op(o);
    } else if (o.kind == kRecord) {
      if (hipEventRecord(p->events[o.slot], o.stream) != hipSuccess) {
        fbn_set_error("fbn_plan_run: hipEventRecord failed");
        rc = 2;
      }
    } else {
      if (hipStreamWaitEvent(o.stream, p->events[o.slot], 0) != hipSuccess) {
        fbn_set_error("fbn_plan_run: hipStreamWaitEvent failed");
        rc = 2;
      }
    }
    if (rc) {
      if (failed) *failed = k;
      return rc;
    }
  }
  return 0;
}
