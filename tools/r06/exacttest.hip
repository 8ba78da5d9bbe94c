// Debug harness (r06): k_sig_exact on one SignatureShare encoding: status, leaf count, inf.
#include "hbtc_sig.hip"
#include <cstdio>
#include <cstring>
using namespace hbtc;
int main(int argc, char** argv) {
  uint8_t b[96];
  for (int i = 0; i < 96; ++i) sscanf(argv[1] + 2 * i, "%2hhx", &b[i]);
  const uint32_t n = argc > 2 ? atoi(argv[2]) : 1;
  std::vector<uint8_t> sigs(96 * n);
  for (uint32_t i = 0; i < n; ++i) memcpy(sigs.data() + 96 * i, b, 96);
  Tile tile{0, 0, n, 0};
  std::vector<uint32_t> idx(n, 0);
  int32_t pks = HBTC_ACCEPT;
  Tile* dt; uint32_t *didx, *dcnt, *dleaves, *dinf; uint8_t* dsig; int32_t *dpks, *dst; G2A* ddec; Fq2* dtab;
  (void)hipMalloc(&dt, sizeof(Tile)); (void)hipMalloc(&didx, 4 * n); (void)hipMalloc(&dcnt, 8);
  (void)hipMalloc(&dleaves, 8 * n); (void)hipMalloc(&dinf, 4 * n); (void)hipMalloc(&dsig, 96 * n);
  (void)hipMalloc(&dpks, 4); (void)hipMalloc(&dst, 4 * n); (void)hipMalloc(&ddec, sizeof(G2A) * n);
  (void)hipMalloc(&dtab, sizeof(Fq2) * PLINES_FQ2 * n);
  (void)hipMemcpy(dt, &tile, sizeof(Tile), hipMemcpyHostToDevice);
  (void)hipMemcpy(didx, idx.data(), 4 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsig, sigs.data(), 96 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dpks, &pks, 4, hipMemcpyHostToDevice);
  (void)hipMemset(dcnt, 0, 8);
  (void)hipMemset(dst, 0x55, 4 * n);
  hipError_t e = launch_sig_exact(0, n, didx, dsig, dpks, 1, dt, 1, dcnt, dleaves, ddec, dtab, dinf, dst);
  (void)hipDeviceSynchronize();
  std::vector<int32_t> st(n);
  uint32_t cnt;
  (void)hipMemcpy(st.data(), dst, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&cnt, dcnt, 4, hipMemcpyDeviceToHost);
  printf("launch %d, leaf_count %u, status", (int)e, cnt);
  for (uint32_t i = 0; i < n; ++i) printf(" %d", st[i]);
  printf("\n");
  return 0;
}
