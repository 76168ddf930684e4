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

// 1 if the current device is gfx950 (the only target this library is built for)
extern "C" int fbn_device_ok(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}
