// Operand layout of v_mfma_i32_32x32x32_i8 on this GPU, checked against the
// layout the matrix-core CRC tables assume (crc32.cpp, crc_device.hpp
// mfma_*): A lane l byte e -> row l % 32, K block l / 32 (B the same with
// columns), accumulator j of lane l -> C[8 (j / 4) + 4 (l / 32) + j % 4][l % 32].
// Random small A and B, one wave; the host recomputes C under two K orders
// within a block (contiguous, or two 8-byte halves 16 apart) and says which
// one matches.  Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_probe.hip.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void probe(const v4i* a, const v4i* b, v16i* c) {
  const int l = threadIdx.x;
  c[l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], v16i{}, 0, 0, 0);
}
// v_mfma_i32_16x16x64_i8 (the A/B 16x16x64 CRC form): A lane l -> row l % 16,
// K block l / 16; accumulator j -> C[4 (l / 16) + j][l % 16].
__global__ void probe16(const v4i* a, const v4i* b, v4i* c) {
  const int l = threadIdx.x;
  c[l] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], v4i{}, 0, 0, 0);
}

static int k_of(int order, int l, int e) {
  return order == 0 ? 16 * (l / 32) + e : 8 * (l / 32) + (e % 8) + 16 * (e / 8);
}

int main() {
  int8_t ha[64][16], hb[64][16];
  int32_t hc[64][16];
  srand(7);
  for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 16; ++e) {
      ha[l][e] = static_cast<int8_t>(rand() % 7 - 3);
      hb[l][e] = static_cast<int8_t>(rand() % 7 - 3);
    }
  void *da, *db, *dc;
  if (hipMalloc(&da, sizeof ha) || hipMalloc(&db, sizeof hb) || hipMalloc(&dc, sizeof hc)) return 2;
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(static_cast<const v4i*>(da), static_cast<const v4i*>(db), static_cast<v16i*>(dc));
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
  int matched = -1;
  for (int order = 0; order < 2; ++order) {
    int A[32][32] = {}, B[32][32] = {};
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 16; ++e) {
        A[l % 32][k_of(order, l, e)] = ha[l][e];
        B[k_of(order, l, e)][l % 32] = hb[l][e];
      }
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 16; ++j) {
        const int r = 8 * (j / 4) + 4 * (l / 32) + j % 4, n = l % 32;
        int want = 0;
        for (int k = 0; k < 32; ++k) want += A[r][k] * B[k][n];
        bad += want != hc[l][j];
      }
    printf("K order %s: %d of 1024 accumulators differ\n", order == 0 ? "contiguous" : "halves", bad);
    if (bad == 0 && matched < 0) matched = order;
  }
  printf(matched == 0 ? "layout as the CRC tables assume\n" : matched == 1 ? "C layout ok, K in halves (same for A and B: the CRC tables hold)\n" : "C LAYOUT DIFFERS\n");
  // 16x16x64: K block of 16 per lane group of 16 (order within a block is
  // the same for A and B either way, as above)
  int32_t hc16[64][4];
  void* dc16;
  if (hipMalloc(&dc16, sizeof hc16)) return 2;
  probe16<<<1, 64>>>(static_cast<const v4i*>(da), static_cast<const v4i*>(db), static_cast<v4i*>(dc16));
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipMemcpy(hc16, dc16, sizeof hc16, hipMemcpyDeviceToHost);
  int bad16 = 0;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * (l / 16) + j, n = l % 16;
      int want = 0;
      for (int g = 0; g < 4; ++g)
        for (int e = 0; e < 16; ++e) want += ha[r + 16 * g][e] * hb[n + 16 * g][e];
      bad16 += want != hc16[l][j];
    }
  printf("16x16x64: %d of 256 accumulators differ from the assumed layout\n", bad16);
  return (matched < 0 || bad16) ? 1 : 0;
}
