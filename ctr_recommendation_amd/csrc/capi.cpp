// C-ABI housekeeping for libfibinet_hip.so: error reporting and version/arch queries.
// Every compute entry point lives next to its kernels (gemm.hip, fields.hip, mlp.hip,
// optim.hip, exchange.hip) and is declared in include/fibinet.h.
#include <hip/hip_runtime.h>
#include <string.h>

static thread_local char g_err[512] = {0};

void fbn_set_error(const char* msg) {
  strncpy(g_err, msg ? msg : "", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

extern "C" const char* fbn_last_error(void) { return g_err; }

extern "C" int fbn_version(void) { return 1; }

// ---- bench probes: slot k is an event pair.  fbn_probe_arm(k) .. fbn_probe_disarm() brackets one
// entry-point call: the first kernel the library launches in between records the start event at its
// own start, every one records the stop event at its end (fbn_launch -> hipExtLaunchKernelGGL), so the
// pair spans exactly the call's kernels -- no marker packets or dispatch latency around them.  The
// events carry no system-scope fence (timing only), so probes inside timed steps (recorded into step
// programs) cost no cache writeback.
#include <vector>
namespace {
std::vector<hipEvent_t> g_probe_ev;      // [2k] start, [2k + 1] stop
std::vector<char> g_probe_taken;         // [k]: a launch recorded slot k since its last arm
int g_probe_armed = -1;
}  // namespace

bool fbn_probe_take(hipEvent_t* start, hipEvent_t* stop) {
  if (g_probe_armed < 0) return false;
  const bool first = !g_probe_taken[g_probe_armed];
  *start = first ? g_probe_ev[2 * g_probe_armed] : nullptr;
  *stop = g_probe_ev[2 * g_probe_armed + 1];
  g_probe_taken[g_probe_armed] = 1;
  return true;
}

extern "C" int fbn_probe_arm(int slot) {
  if (slot < 0) {
    fbn_set_error("fbn_probe_arm: slot >= 0");
    return 1;
  }
  while ((int)g_probe_ev.size() < 2 * (slot + 1)) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
      fbn_set_error("fbn_probe_arm: hipEventCreateWithFlags failed");
      return 2;
    }
    g_probe_ev.push_back(e);
  }
  if ((int)g_probe_taken.size() <= slot) g_probe_taken.resize(slot + 1, 0);
  g_probe_armed = slot;
  g_probe_taken[slot] = 0;
  return 0;
}

extern "C" int fbn_probe_disarm(void) {
  g_probe_armed = -1;
  return 0;
}

// span of slot k's kernels in ms (after they completed), or -1 when no launch took the slot
extern "C" float fbn_probe_elapsed(int slot) {
  if (slot < 0 || slot >= (int)g_probe_taken.size() || !g_probe_taken[slot]) return -1.f;
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, g_probe_ev[2 * slot], g_probe_ev[2 * slot + 1]) != hipSuccess) return -1.f;
  return ms;
}

// 1 if the current device is gfx950 (the only target this library is built for)
extern "C" int fbn_device_ok(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}
