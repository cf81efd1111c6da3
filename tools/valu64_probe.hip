// valu64_probe.hip -- issue rate of 64-bit VALU shifts on gfx950
// (v_lshrrev_b64 / v_lshlrev_b64) against 32-bit shifts and bitop3, to decide
// whether the bit-slice transposition's SWAPMOVE layers can shift two dwords
// per instruction (rs_bitslice_core.h).
// Every variant: 16 independent dword chains per lane, ITER rounds; full
// occupancy (8 waves per SIMD). Reported: dword-ops per second, i.e. a 64-bit
// shift counts 2 dwords. Then v_bitop3_b32 at 1, 2, 4 and 8 waves per SIMD
// with 16 independent chains and with one dependent chain per lane: the
// issue rate a kernel gets at its own occupancy.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 valu64_probe.hip -o _build/valu64_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr int ITER = 4096;

__global__ __launch_bounds__(256) void k_b32(uint32_t *out) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = threadIdx.x * 16 + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(v[i]));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_b64(uint32_t *out) {
  uint64_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = (uint64_t)(threadIdx.x * 16 + i) * 0x100000001ull;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(v[i]));
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}

__global__ __launch_bounds__(256) void k_bitop3(uint32_t *out) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = threadIdx.x * 16 + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < 16; i++)
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(v[(i + 1) & 15]), "v"(v[(i + 2) & 15]));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void k_chain(uint32_t *out) {
  uint32_t v[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) v[i] = threadIdx.x * 16 + i;
  for (int it = 0; it < ITER * 16 / CH; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++)
      asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(v[(i + 1) % CH]), "v"(v[(i + 2) % CH]));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < CH; i++) s ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 8;  // 8 x 256 lanes per CU = 8 waves per SIMD
  uint32_t *out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V { const char *name; void (*f)(uint32_t *); double dwords_per_inst; int insts; };
  V vs[] = {{"v_lshrrev_b32", k_b32, 1, 16}, {"v_lshrrev_b64", k_b64, 2, 8},
            {"v_bitop3_b32", k_bitop3, 1, 16}};
  for (int round = 0; round < 3; round++)
    for (auto &v : vs) {
      hipLaunchKernelGGL(v.f, dim3(blocks), dim3(256), 0, 0, out);
      CK(hipEventRecord(a));
      for (int r = 0; r < 4; r++) hipLaunchKernelGGL(v.f, dim3(blocks), dim3(256), 0, 0, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double lanes = (double)blocks * 256 * 4;
      const double inst = lanes * ITER * v.insts;
      std::printf("%-16s %8.3f ms  %7.2f T lane-inst/s  %7.2f T dword-ops/s\n", v.name, ms,
                  inst / (ms * 1e-3) / 1e12, inst * v.dwords_per_inst / (ms * 1e-3) / 1e12);
    }
  // occupancy sweep: w workgroups of 4 waves per CU = w waves per SIMD
  for (int w : {1, 2, 4, 8})
    for (int ch : {16, 1}) {
      auto f = ch == 16 ? k_chain<16> : k_chain<1>;
      hipLaunchKernelGGL(f, dim3(cus * w), dim3(256), 0, 0, out);
      CK(hipEventRecord(a));
      for (int r = 0; r < 4; r++) hipLaunchKernelGGL(f, dim3(cus * w), dim3(256), 0, 0, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double inst = (double)cus * w * 256 * 4 * ITER * 16;
      std::printf("v_bitop3_b32 %d wave(s)/SIMD, %2d chain(s): %7.2f T lane-inst/s  %.3f wave-inst/cycle/SIMD at 2.4 GHz\n",
                  w, ch, inst / (ms * 1e-3) / 1e12, inst / 64 / (ms * 1e-3) / (cus * 4.0) / 2.4e9);
    }
  return 0;
}
