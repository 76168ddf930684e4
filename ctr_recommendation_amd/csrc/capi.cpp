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
// pair spans exactly the call's kernels -- no marker packets or dispatch latency around them.
#include <vector>
namespace {
std::vector<hipEvent_t> g_probe_ev;      // [2k] start, [2k + 1] stop
int g_probe_armed = -1;
bool g_probe_first = false;
}  // namespace

bool fbn_probe_take(hipEvent_t* start, hipEvent_t* stop) {
  if (g_probe_armed < 0) return false;
  *start = g_probe_first ? g_probe_ev[2 * g_probe_armed] : nullptr;
  *stop = g_probe_ev[2 * g_probe_armed + 1];
  g_probe_first = false;
  return true;
}

extern "C" int fbn_probe_arm(int slot) {
  if (slot < 0) {
    fbn_set_error("fbn_probe_arm: slot >= 0");
    return 1;
  }
  while ((int)g_probe_ev.size() < 2 * (slot + 1)) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) {
      fbn_set_error("fbn_probe_arm: hipEventCreate failed");
      return 2;
    }
    g_probe_ev.push_back(e);
  }
  g_probe_armed = slot;
  g_probe_first = true;
  return 0;
}

// 1 if a kernel launch took the armed slot (0: the call launched nothing); disarms it
extern "C" int fbn_probe_disarm(void) {
  const int taken = (g_probe_armed >= 0 && !g_probe_first) ? 1 : 0;
  g_probe_armed = -1;
  return taken;
}

// span of slot k's kernels in ms (after they completed), or -1
extern "C" float fbn_probe_elapsed(int slot) {
  if (slot < 0 || 2 * slot + 1 >= (int)g_probe_ev.size()) return -1.f;
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
