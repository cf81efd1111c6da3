// valu_rate.hip -- issue rate of the VOP3 integer ops the kernels lean on
// (v_perm_b32, v_bitop3_b32, v_alignbit_b32, v_add3_u32, v_xor_b32) on
// gfx950: 8 independent chains per lane, 4096 dependent steps each, every
// CU fully occupied; reports wave-instructions per cycle per SIMD
// (0.5 = one wave64 instruction every 2 cycles = full rate).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed, int iters) {
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = seed * (threadIdx.x + i + 1);
  const uint32_t c1 = seed ^ 0x5a5a5a5a, c2 = seed + 0x12345;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if constexpr (OP == 0) v[i] = v[i] ^ c1;
      if constexpr (OP == 1) v[i] = __builtin_amdgcn_perm(c1, v[i], c2);
      if constexpr (OP == 2) v[i] = __builtin_amdgcn_bitop3_b32(v[i], c1, c2, 0x96);
      if constexpr (OP == 3) v[i] = __builtin_amdgcn_alignbit(v[i], v[i], 7);
      if constexpr (OP == 4) v[i] = v[i] + c1 + c2;
      if constexpr (OP == 5) v[i] = __builtin_amdgcn_perm(c1, c2, v[i]);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  const int blocks = 256 * 8, iters = 4096;
  uint32_t *out;
  hipMalloc(&out, blocks * 256 * 4);
  const char *names[] = {"v_xor_b32", "v_perm_b32 (data as src1)", "v_bitop3_b32",
                         "v_alignbit_b32", "v_add3_u32", "v_perm_b32 (data as selector)"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  for (int rep = 0; rep < 2; rep++)
    for (int op = 0; op < 6; op++) {
      auto launch = [&] {
        switch (op) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); break;
          case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); break;
          case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, 3u, iters); break;
        }
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double winst = (double)blocks * 4 * iters * 8;  // wave-instructions
      const double per_simd_per_ns = winst / 1024.0 / (ms * 1e6);
      if (rep)
        std::printf("%-30s %.3f ms  %.3f wave-inst/ns/SIMD  (= %.2f per cycle at %.2f GHz)\n",
                    names[op], ms, per_simd_per_ns, per_simd_per_ns / (clk_khz / 1e6),
                    clk_khz / 1e6);
    }
  return 0;
}
