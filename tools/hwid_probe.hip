// Probe: which (XCC, SE, SH, CU) ids do workgroups report on this GPU (HW_REG_HW_ID / XCC_ID)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <set>
#include <tuple>
__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}
int main() {
  const int nb = 8192;
  unsigned* d; hipMalloc(&d, nb * 8);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 0, 0, d);
  unsigned h[2 * nb]; hipMemcpy(h, d, nb * 8, hipMemcpyDeviceToHost);
  std::set<std::tuple<int, int, int, int>> cus;
  std::map<int, int> cu_hist, se_hist, xcc_hist, sh_hist;
  for (int i = 0; i < nb; ++i) {
    unsigned hw = h[2 * i], x = h[2 * i + 1] & 0xf;
    int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    cus.insert({(int)x, se, sh, cu});
    cu_hist[cu]++; se_hist[se]++; xcc_hist[x]++; sh_hist[sh]++;
  }
  printf("distinct (xcc,se,sh,cu): %zu\n", cus.size());
  printf("cu ids:"); for (auto& kv : cu_hist) printf(" %d:%d", kv.first, kv.second); printf("\n");
  printf("se ids:"); for (auto& kv : se_hist) printf(" %d:%d", kv.first, kv.second); printf("\n");
  printf("sh ids:"); for (auto& kv : sh_hist) printf(" %d:%d", kv.first, kv.second); printf("\n");
  printf("xcc ids:"); for (auto& kv : xcc_hist) printf(" %d:%d", kv.first, kv.second); printf("\n");
  printf("first 16 blocks:"); for (int i = 0; i < 16; ++i) printf(" %08x/%u", h[2 * i], h[2 * i + 1]); printf("\n");
  return 0;
}
