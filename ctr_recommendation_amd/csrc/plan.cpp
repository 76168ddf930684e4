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
// Replay calls each recorded entry point through one generic signature.  Every fbn_* entry
// point takes only INTEGER-class arguments (pointers, int, long long, size_t, unsigned) and
// SSE-class scalars (float, double), and returns int.  Under the x86-64 System V calling
// convention integer-class arguments occupy rdi, rsi, rdx, rcx, r8, r9 and then 8-byte stack
// slots in order, and SSE-class arguments occupy xmm0..xmm7 in order, independently of each
// other.  So a call through `int (*)(u64 x 48, double x 8)` with the integer arguments in
// order (int32 values sign-extended) and the float arguments as doubles whose low 32 bits
// hold the float's bits (a float argument is read from the low 32 bits of its xmm register)
// passes exactly what the real prototype expects; the callee ignores the unused tail, and the
// caller pops the stack.  Entry points with more than 48 integer or 8 float arguments are
// refused at record time.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#if !defined(__x86_64__) || !defined(__linux__)
#error "step programs rely on the x86-64 System V calling convention"
#endif

void fbn_set_error(const char* msg);

namespace {

constexpr int kMaxInt = 48;
constexpr int kMaxFlt = 8;

typedef uint64_t U;
typedef int (*GenericFn)(U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U,
                         U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, U, double, double, double,
                         double, double, double, double, double);

enum OpKind { kCall = 0, kRecord = 1, kWait = 2 };

struct Op {
  int kind;
  int slot;                // kRecord / kWait: event slot
  void* fn;                // kCall
  hipStream_t stream;      // kRecord / kWait
  U i[kMaxInt];
  double f[kMaxFlt];
};

struct Plan {
  int device;
  std::vector<Op> ops;
  std::vector<hipEvent_t> events;
};

int call_op(const Op& o) {
  GenericFn fn = reinterpret_cast<GenericFn>(o.fn);
  const U* a = o.i;
  const double* f = o.f;
  return fn(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13], a[14], a[15],
            a[16], a[17], a[18], a[19], a[20], a[21], a[22], a[23], a[24], a[25], a[26], a[27], a[28], a[29], a[30],
            a[31], a[32], a[33], a[34], a[35], a[36], a[37], a[38], a[39], a[40], a[41], a[42], a[43], a[44], a[45],
            a[46], a[47], f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]);
}

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

extern "C" int fbn_plan_add_call(void* plan, void* fn, const unsigned long long* iargs, int ni, const double* fargs,
                                 int nf) {
  Plan* p = static_cast<Plan*>(plan);
  if (!p || !fn || ni < 0 || nf < 0 || ni > kMaxInt || nf > kMaxFlt || (ni && !iargs) || (nf && !fargs)) {
    fbn_set_error("fbn_plan_add_call: bad arguments (at most 48 integer and 8 float arguments)");
    return 1;
  }
  Op o;
  memset(&o, 0, sizeof(o));
  o.kind = kCall;
  o.fn = fn;
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
