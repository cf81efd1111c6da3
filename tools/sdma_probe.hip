// sdma_probe.hip -- do H2D and D2H copies overlap, and in which stream
// arrangements? (torch's two-stream pinned copies run
// 97 GB/s both ways at once, the batch encode's SDMA pipeline ~55 GB/s.)
// Page-locked host buffers, 64 MiB in / 32 MiB out per batch (RS(4,2)'s 1.5
// bytes per user byte), 16 batches per sample:
//   A  H2D on stream 0 and D2H on stream 1, no kernels (torch's test);
//   B  the product pipeline: batch i on stream i % 2 as H2D -> kernel -> D2H;
//   C  three streams: H2D on an in-stream, kernel on a compute stream after
//      an event, D2H on an out-stream after an event (copy engines per
//      direction never wait on the other direction's stream);
//   D  as B with four streams.
// The kernel is a trivial device copy of 32 MiB (in -> out), standing in for
// the encode. Prints GB/s of PCIe traffic per arrangement.
//
// build: make -C tools sdma_probe   run: tools/_build/sdma_probe [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,                 \
                   hipGetErrorString(e));                                            \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void half_copy(const uint4 *in, uint4 *out, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    out[i] = in[i];
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  constexpr size_t IN = 64u << 20, OUT = 32u << 20;
  constexpr int NB = 16, NS = 4;
  uint8_t *hin, *hout, *din[NS], *dout[NS];
  CK(hipHostMalloc(reinterpret_cast<void **>(&hin), IN * NB, hipHostMallocDefault));
  CK(hipHostMalloc(reinterpret_cast<void **>(&hout), OUT * NB, hipHostMallocDefault));
  for (int i = 0; i < NS; i++) {
    CK(hipMalloc(&din[i], IN));
    CK(hipMalloc(&dout[i], OUT));
  }
  std::memset(hin, 1, IN * NB);
  hipStream_t st[NS];
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev_in[NB], ev_k[NB];
  for (int i = 0; i < NB; i++) {
    CK(hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_k[i], hipEventDisableTiming));
  }
  auto kern = [&](int b, hipStream_t s) {
    hipLaunchKernelGGL(half_copy, dim3(1024), dim3(256), 0, s,
                       reinterpret_cast<const uint4 *>(din[b % NS]),
                       reinterpret_cast<uint4 *>(dout[b % NS]), OUT / 16);
  };
  struct V {
    std::string name;
    std::function<void()> run;
    std::vector<double> gbs;
  };
  std::vector<V> vs;
  vs.push_back({"A: H2D stream 0 || D2H stream 1, no kernels", [&] {
                  for (int b = 0; b < NB; b++) {
                    CK(hipMemcpyAsync(din[b % NS], hin + b * IN, IN, hipMemcpyHostToDevice, st[0]));
                    CK(hipMemcpyAsync(hout + b * OUT, dout[b % NS], OUT, hipMemcpyDeviceToHost, st[1]));
                  }
                }, {}});
  for (int ns : {2, 4})
    vs.push_back({"B/D: batch i on stream i % " + std::to_string(ns) + ": H2D, kernel, D2H", [&, ns] {
                    for (int b = 0; b < NB; b++) {
                      hipStream_t s = st[b % ns];
                      CK(hipMemcpyAsync(din[b % NS], hin + b * IN, IN, hipMemcpyHostToDevice, s));
                      kern(b, s);
                      CK(hipMemcpyAsync(hout + b * OUT, dout[b % NS], OUT, hipMemcpyDeviceToHost, s));
                    }
                  }, {}});
  vs.push_back({"C: in-stream H2D, compute stream kernel, out-stream D2H", [&] {
                  for (int b = 0; b < NB; b++) {
                    // buffer b % NS reused every NS batches: the in-stream waits
                    // for the kernel that last read it (ev_k of b - NS)
                    if (b >= NS) CK(hipStreamWaitEvent(st[0], ev_k[b - NS], 0));
                    CK(hipMemcpyAsync(din[b % NS], hin + b * IN, IN, hipMemcpyHostToDevice, st[0]));
                    CK(hipEventRecord(ev_in[b], st[0]));
                    CK(hipStreamWaitEvent(st[1], ev_in[b], 0));
                    kern(b, st[1]);
                    CK(hipEventRecord(ev_k[b], st[1]));
                    CK(hipStreamWaitEvent(st[2], ev_k[b], 0));
                    CK(hipMemcpyAsync(hout + b * OUT, dout[b % NS], OUT, hipMemcpyDeviceToHost, st[2]));
                  }
                }, {}});
  for (auto &v : vs) {  // warm
    v.run();
    CK(hipDeviceSynchronize());
  }
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs) {
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      v.run();
      CK(hipDeviceSynchronize());
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      v.gbs.push_back(static_cast<double>(NB) * (IN + OUT) / s / 1e9);
    }
  for (auto &v : vs) {
    std::sort(v.gbs.begin(), v.gbs.end());
    std::printf("%-60s median %6.1f GB/s (max %6.1f)  = %5.1f GiB/s of RS(4,2) user data\n",
                v.name.c_str(), v.gbs[v.gbs.size() / 2], v.gbs.back(),
                v.gbs[v.gbs.size() / 2] * 1e9 / 1.5 / (1u << 30));
  }
  return 0;
}
