// rs_jit.cpp -- bit-sliced kernels for matrices known only at run time.
//
// Decode (Fec::decode, piece.rs:384-386) and repair apply rows of the
// inverted survivor matrix, which depend on which shares survived. The
// v_perm table kernel takes any matrix but spends ~5.6 VALU ops per
// (input, output, dword); from ~3 missing rows at k = 16 (the loss of 3+
// miners per chunk for objects of 1 GiB and up) it is VALU-bound at 27-50 %
// of HBM peak (profiles/r1_bsbench.txt); at k = 32 the table kernel loses
// from 2 missing rows on. The bit-sliced method needs the
// matrix as compile-time constants (rs_bitslice_core.h), so here the host
// writes the matrix out as a constexpr table and compiles the same core
// header with hipRTC, once per (matrix, copy mask), on a background thread.
// Calls that arrive while a kernel compiles run the table kernel
// (STORB_RS_JIT=sync waits instead). A matrix is compiled only once it has
// been asked for twice (a pattern one chunk of a download uses is not worth
// a compile); at most STORB_RS_JIT_MAX kernels (default 256) are loaded, the
// least recently used one unloaded for a new one once every launch of it
// has completed (per-stream launch events), so no queued launch can outlive
// its code object. One compile thread.
#include <hip/hip_runtime_api.h>
#include <hip/hiprtc.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>


#include "../../include/storb_rs.h"
#include "gf256.hpp"
#include "rs_jit.hpp"
#include "rs_kernels.hpp"

namespace storb_rs {
namespace jit {
namespace {

// The header texts hipRTC compiles (generated from rs_args.h and
// rs_bitslice_core.h by the Makefile, so they cannot drift from the
// ahead-of-time kernels).
#include "jit_headers.inc"

enum class Mode { Off, Async, Sync, Always };

// STORB_RS_JIT (read once): unset / 1 = async, sync, 0 = off; "always"
// (measurements only) = sync and every k >= 8 matrix, VALU-bound on the
// table kernel or not.
Mode raw_mode() {
  static const Mode m = [] {
    const char *e = std::getenv("STORB_RS_JIT");
    if (!e || !*e) return Mode::Async;
    if (std::strcmp(e, "always") == 0) return Mode::Always;
    if (std::strcmp(e, "sync") == 0) return Mode::Sync;
    return std::atoi(e) ? Mode::Async : Mode::Off;
  }();
  return m;
}
Mode mode() { return raw_mode() == Mode::Always ? Mode::Sync : raw_mode(); }
bool always() { return raw_mode() == Mode::Always; }

// STORB_RS_JIT_DUMP=dir: write every compiled kernel's source and code
// object there (and a failed compile's log to stderr).
const char *dump_dir() {
  static const char *d = std::getenv("STORB_RS_JIT_DUMP");
  return d && *d ? d : nullptr;
}

// STORB_RS_JIT_TEST_CALL=1: every generated kernel gets an out-of-line call
// (tests/test_abi_host.py checks that the compile thread refuses it).
bool test_call() {
  static const bool v = [] {
    const char *e = std::getenv("STORB_RS_JIT_TEST_CALL");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// STORB_RS_JIT_STREAM=1: single calls with k > 16 run the matrix's compiled
// kernel in its streamed form (one launch gated per slice) once it is ready.
// Off by default: measured slower than the sliced path it replaces
// (tools/stream_jit_ab.py, profiles/r6r_stream_jit_ab.jsonl, pageable
// buffers, caller on the GPU's node, three interleaved pairs: (32, 48) 32 MiB
// decode, 2 lost, 1.57-1.60 ms streamed against 0.89-1.19 ms sliced; (24, 36)
// 6 MiB 226-245 against 196-199 us). The sliced path's compiled launches
// start on packed slices at full width; the gated launch holds its later
// slices' workgroups resident and polling while the host packs.
bool stream_enabled() {
  static const bool v = [] {
    const char *e = std::getenv("STORB_RS_JIT_STREAM");
    return e && *e && std::atoi(e) != 0;
  }();
  return v;
}

size_t max_kernels() {
  static const size_t v = [] {
    const char *e = std::getenv("STORB_RS_JIT_MAX");
    return e && *e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : size_t{256};
  }();
  return v;
}

struct Entry {
  enum State { Pending, Ready, Failed };
  std::atomic<State> state{Pending};  // read by launching threads without the lock
  std::string src;
  std::string name;  // kernel symbol: storb_bs_jit_k<k>_r<rows>_{ip,asm}
  int opt = 3;       // -O level (opt_level())
  std::vector<char> code;
  std::string log;
  std::map<int, hipFunction_t> fn;  // per device
  std::vector<std::pair<int, hipModule_t>> modules;  // (device, module)
  // Last launch on each (device, stream): the entry may be unloaded once all
  // have completed.
  struct Use {
    int device;
    hipStream_t stream;
    hipEvent_t done;
  };
  std::vector<Use> uses;
  uint64_t tick = 0;  // LRU clock
};

class Jit;
Jit &jit();

class Jit {
 public:
  ~Jit() { shutdown(); }

  // Stop compiling: queued entries fail, the compile in flight finishes,
  // the worker is joined. Runs at process exit from an atexit handler
  // registered after hipRTC / comgr have built their static state (a
  // warm-up compile before the worker starts, and again after every
  // compile), so -- exit handlers run in reverse order of registration --
  // before that state is torn down. Without it a compile still running at
  // exit used comgr's destroyed state: "LLVM ERROR: Invalid size request on
  // a scalable vector" + abort on the GPU box (tools/fuzz.py), a hang here.
  void shutdown() {
    std::thread w;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      for (auto &e : queue_) {
        e->state = Entry::Failed;
        failed_++;
        pending_--;
      }
      queue_.clear();
      if (worker_.joinable() && worker_.get_id() != std::this_thread::get_id())
        w = std::move(worker_);
    }
    cv_.notify_all();
    if (w.joinable()) w.join();
  }

  // The entry for key, created and queued for compilation if new; src()
  // writes the kernel source (symbol `name`), only for a new entry. nullptr
  // (the caller runs the table kernel): a matrix asked for the first time
  // (unless `force`, or in Sync mode), or no room -- STORB_RS_JIT_MAX loaded
  // and none of them idle. In Sync mode waits for the compile.
  template <typename Src>
  std::shared_ptr<Entry> get(const std::string &key, const std::string &name, int opt, Src &&src,
                             bool force) {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = entries_.find(key);
    std::shared_ptr<Entry> e;
    if (it != entries_.end()) {
      e = it->second;
      e->tick = ++tick_;
    } else {
      if (stop_) return nullptr;
      if (!force && mode() != Mode::Sync) {
        if (seen_.size() > (1u << 16)) seen_.clear();
        if (++seen_[key] < 2) return nullptr;
      }
      if (entries_.size() >= max_kernels() && !evict_one_locked()) return nullptr;
      seen_.erase(key);
      e = std::make_shared<Entry>();
      e->tick = ++tick_;
      e->src = src();
      e->name = name;
      e->opt = opt;
      entries_.emplace(key, e);
      queue_.push_back(e);
      pending_++;
      if (!worker_.joinable() && !stop_) {
        warm_up();
        worker_ = std::thread([this] { run(); });
      }
      cv_.notify_all();
    }
    if (mode() == Mode::Sync) cv_.wait(lk, [&] { return e->state != Entry::Pending; });
    return e;
  }

  // Device function of a ready entry (module loaded on first use per device;
  // the caller has made `device` current).
  hipError_t function(Entry &e, int device, hipFunction_t *f) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = e.fn.find(device);
    if (it != e.fn.end()) {
      *f = it->second;
      return hipSuccess;
    }
    hipModule_t m = nullptr;
    hipError_t r = hipModuleLoadData(&m, e.code.data());
    if (r != hipSuccess) return r;
    r = hipModuleGetFunction(f, m, e.name.c_str());
    if (r != hipSuccess) return r;
    e.modules.emplace_back(device, m);
    e.fn[device] = *f;
    return hipSuccess;
  }

  // After launching e on stream s of `device` (current): record the launch.
  hipError_t used(Entry &e, int device, hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &u : e.uses)
      if (u.device == device && u.stream == s) return hipEventRecord(u.done, s);
    Entry::Use u{device, s, nullptr};
    // ordering only (the module is unloaded after it): no system-scope fence
    hipError_t r = hipEventCreateWithFlags(&u.done, hipEventDisableTiming | hipEventDisableSystemFence);
    if (r != hipSuccess) return r;
    e.uses.push_back(u);
    return hipEventRecord(u.done, s);
  }



  void wait_for(const Entry &e) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return e.state != Entry::Pending; });
  }

  void wait_idle() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return pending_ == 0; });
  }

  void stats(storb_rs_jit_stats_t *s) {
    std::lock_guard<std::mutex> lk(mu_);
    s->compiled = compiled_;
    s->failed = failed_;
    s->pending = pending_;
    s->launches = launches;
    s->fallbacks = fallbacks;
    s->compile_ms = compile_ms_;
    s->evicted = evicted_;
    s->loaded = entries_.size();
    s->refused = refused_;
  }

  std::atomic<uint64_t> launches{0}, fallbacks{0};

 private:
  // Unload the least recently used compiled kernel that nobody holds and
  // whose launches have all completed. Under mu_.
  bool evict_one_locked() {
    auto victim = entries_.end();
    for (auto it = entries_.begin(); it != entries_.end(); ++it) {
      const Entry &e = *it->second;
      if (e.state == Entry::Pending || it->second.use_count() > 1) continue;
      if (victim != entries_.end() && victim->second->tick <= e.tick) continue;
      bool idle = true;
      for (const auto &u : e.uses) idle = idle && hipEventQuery(u.done) == hipSuccess;
      if (idle) victim = it;
    }
    if (victim == entries_.end()) return false;
    Entry &e = *victim->second;
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (auto &dm : e.modules) {
      (void)hipSetDevice(dm.first);
      (void)hipModuleUnload(dm.second);
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    for (auto &u : e.uses) (void)hipEventDestroy(u.done);
    entries_.erase(victim);
    evicted_++;
    return true;
  }

  void run() {
    // (A nice-10 compile thread starved on the GPU box: 0 of 32 queued
    // compiles done after 4 s of decode calls, tools/jit_fuzz.py,
    // profiles/r3_jit_fuzz_nice10.jsonl. One thread at normal priority.)
    for (;;) {
      std::shared_ptr<Entry> e;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
        if (stop_) return;
        e = queue_.front();
        queue_.pop_front();
      }
      const auto t0 = std::chrono::steady_clock::now();
      std::vector<char> code;
      std::string log;
      bool ok = compile(e->src, e->opt, code, log);
      register_exit_hook();
      // Never load a kernel that makes a function call (code_object_check.cpp:
      // the round-4 hang was an out-of-line callee that lost its return
      // address); its matrix keeps the table kernel.
      bool refused = false;
      if (ok) {
        std::string why;
        if (code_object_calls(code.data(), code.size(), why) != 0) {
          ok = false;
          refused = true;
          log = "refused: " + why;
        }
      }
      const double ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      {
        std::lock_guard<std::mutex> lk(mu_);
        e->code = std::move(code);
        e->log = std::move(log);
        e->state = ok ? Entry::Ready : Entry::Failed;
        (ok ? compiled_ : failed_)++;
        if (refused) refused_++;
        compile_ms_ += ms;
        pending_--;
      }
      if (refused) std::fprintf(stderr, "storb_rs jit: %s\n", e->log.c_str());
      if (const char *dir = dump_dir()) {  // inspect with hipcc -S
        if (!ok) std::fprintf(stderr, "storb_rs jit: compile failed:\n%s\n", e->log.c_str());
        const std::string path = std::string(dir) + "/storb_bs_jit_" +
                                 std::to_string(compiled_ + failed_) + ".hip";
        if (FILE *f = std::fopen(path.c_str(), "w")) {
          std::fputs(e->src.c_str(), f);
          std::fclose(f);
        }
        // the code object too (llvm-readelf --notes: .vgpr_count, .sgpr_count)
        if (ok || refused)
          if (FILE *f = std::fopen((path + ".co").c_str(), "wb")) {
            std::fwrite(e->code.data(), 1, e->code.size(), f);
            std::fclose(f);
          }
      }
      cv_.notify_all();
    }
  }

  // Once per process (it was registered again after every compile).
  static void register_exit_hook() {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit([] { jit().shutdown(); }); });
  }

  // One tiny hipRTC compile in the calling thread before the first worker
  // starts (once per process, ~0.1-0.3 s): comgr builds its static state
  // here, then the exit hook is registered after it.
  void warm_up() {
    std::vector<char> code;
    std::string log;
    compile("extern \"C\" __global__ void storb_jit_warm(unsigned *p) { p[threadIdx.x] = 1u; }\n",
            3, code, log);
    register_exit_hook();
  }

  static bool compile(const std::string &src, int opt, std::vector<char> &code, std::string &log) {
    hiprtcProgram prog = nullptr;
    const char *hdrs[] = {kRsArgsH, kRsBitsliceCoreH, kRsStreamH};
    const char *names[] = {"rs_args.h", "rs_bitslice_core.h", "rs_stream.hpp"};
    if (hiprtcCreateProgram(&prog, src.c_str(), "storb_bs_jit.hip", 3, hdrs, names) !=
        HIPRTC_SUCCESS)
      return false;
    const std::string o = "-O" + std::to_string(opt);
    const char *opts[] = {"--offload-arch=gfx950", o.c_str(), "-std=c++17"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
    size_t n = 0;
    if (hiprtcGetProgramLogSize(prog, &n) == HIPRTC_SUCCESS && n > 1) {
      log.resize(n);
      hiprtcGetProgramLog(prog, &log[0]);
    }
    bool ok = r == HIPRTC_SUCCESS && hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n > 0;
    if (ok) {
      code.resize(n);
      ok = hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS;
    }
    hiprtcDestroyProgram(&prog);
    return ok;
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::shared_ptr<Entry>> entries_;
  std::unordered_map<std::string, uint32_t> seen_;  // asked-for counts of keys not compiled
  uint64_t tick_ = 0, evicted_ = 0, refused_ = 0;
  std::deque<std::shared_ptr<Entry>> queue_;
  std::thread worker_;
  bool stop_ = false;
  uint64_t compiled_ = 0, failed_ = 0, pending_ = 0;
  double compile_ms_ = 0;
};

Jit &jit() {
  static Jit j;
  return j;
}

// Launch shape (rs_args.h bs_shape, shared with the ahead-of-time
// encoders); the resident-workgroup cap is an LDS reservation
// (rs_kernels.hpp cap_lds, see dynamic_lds()).
// (Round 2 swept it on the real decode path with a run-time override,
// a removed A/B script, profiles/r2_shape_ab/; the override is gone.)
bs::BsShape shape(uint32_t k, uint32_t r) {
  return bs::bs_shape(static_cast<int>(k), static_cast<int>(r));
}

bool split_rows(uint32_t k, uint32_t rows);

// The row-split kernels' shape (rs_args.h bs_split_cap), or shape().
bs::BsShape split_or_shape(uint32_t k, uint32_t r) {
  if (!split_rows(k, r)) return shape(k, r);
  return bs::BsShape{bs::kSplitThreads, 0, bs::bs_split_cap(static_cast<int>(r))};
}

// The input-split form (rs_args.h ks_shape) where it measured faster: k <=
// 16 with 4 or 8 rows, k > 16 with 16 rows (c = 0: not used).
// (Not with fused assembly at k > 16: the k = 32 16-row kernel that also
// stores its inputs spilled 171 VGPRs at -O1 in the input-split form; the
// in-place one took 249, none spilled.)
bs::KsShape ks_of(uint32_t k, uint32_t r, uint64_t copy_mask) {
  if (split_rows(k, r) || (copy_mask && k > 16)) return bs::KsShape{0, 0, 0, 0};
  return bs::ks_shape(static_cast<int>(k), static_cast<int>(r));
}

// Threads, 16-B columns per tile and LDS reservation of a JIT launch.
struct LaunchShape {
  int threads;
  uint64_t cpt;
  size_t lds;
};
LaunchShape launch_shape(uint32_t k, uint32_t r, uint64_t copy_mask) {
  const bs::KsShape ks = ks_of(k, r, copy_mask);
  if (ks.c)
    return {64 * ks.c * ks.w, 128u * static_cast<uint64_t>(ks.c),
            cap_lds(ks.cap, bs::ksplit_lds_bytes(ks.c, ks.w, static_cast<int>(r)))};
  const bool split = split_rows(k, r);
  const bs::BsShape sh = split_or_shape(k, r);
  return {sh.threads, split ? bs::kSplitColsPerTile : bs::bs_cols_per_tile(sh.threads),
          cap_lds(sh.cap, split ? bs::split_lds_bytes(bs::kSplitGroup) : 0)};
}

// The cap's LDS reservation is requested at launch (dynamic LDS) when it is
// at most 64 KiB (caps >= 3; above that a kernel must opt in) and baked into
// the source as a static array otherwise. Static LDS that limits occupancy
// to 2 waves per SIMD told the register allocator it could use all 256
// VGPRs, and it did: the k = 64 row-split encode took 256 VGPRs with 7
// spilled (0.535 ms in bench --config 7) against 197 and none with the same
// reservation made at launch (0.349 ms in the removed k64split probe, profiles/r2_k64/k64split.txt); likewise the
// 16-row blocks 229 vs 196 (profiles/r2_k64/split_dynlds_ab.txt).
size_t dynamic_lds(size_t lds) { return lds <= (64u << 10) ? lds : 0; }

// -O level of a k-input kernel. -O3 up to k = 16 (sub-second compiles); -O1
// above, where -O3's middle end costs seconds per new pattern (the calls
// meanwhile run the table kernel) and buys nothing: the kernels are one
// straight-line, fully unrolled body whose order the source fixes
// (static_for, ordering fences), and the backend emits the same code -- k =
// 64 32-row split 26,507 vs 26,513 instructions, 197 VGPRs both; k = 32 16
// rows 8,237 vs 8,191, 193 VGPRs. GPU A/B (bench, profiles/r2_jit_opt_ab.txt):
// k = 32 16-lost and k = 64 32-lost decodes equal (0.2720 / 0.2717 ms, 0.370
// / 0.368), compiles 1.1 vs 2.8 s and 5-6 vs 11.3 s; at k = 16 -O1 was 1.4-2.3 %
// slower (decode 0.1910 vs 0.1867 ms) for 0.4 s of compile saved, so -O3 there.
int opt_level(uint32_t k) { return k > 16 ? 1 : 3; }

// Kernel symbol, so profiles tell the compiled kernels apart (bench.py and
// profiles/summarize.py match on the "storb_bs_jit_k<k>_r<rows>_" prefix).
std::string kernel_name(uint32_t k, uint32_t rows, uint64_t copy_mask, bool streamed = false) {
  return "storb_bs_jit_k" + std::to_string(k) + "_r" + std::to_string(rows) +
         (copy_mask ? "_asm" : "_ip") + (streamed ? "_st" : "");
}

// Matrices of 17-32 rows run as ONE row-split launch (rs_bitslice_core.h
// bs_split_body: each input read and bit-sliced once, its planes shared by
// the two row-half waves through LDS) instead of row blocks of <= kSlotR
// that each re-read every input (rs_args.h bs_split). Needs an even k (one
// input per wave per load group). Row blocks measured 0.49 vs 0.35 ms for
// the k = 64 encode (profiles/r2_k64/k64split.txt).
bool split_rows(uint32_t k, uint32_t rows) {
  return rows <= kMaxRows && bs::bs_split(static_cast<int>(k), static_cast<int>(rows));
}

// The kernel source for a (rows x k) matrix: bit b' of row[p][j][b] is bit b
// of coef[p][j] * 2^b' (the GF(2) matrix of multiplication by coef[p][j]).
std::string source(uint32_t k, uint32_t rows, const uint8_t *coef, uint64_t copy_mask,
                   int group, const bs::BsShape &sh, size_t lds, bool split,
                   const bs::KsShape &ks, bool streamed = false) {
  const GF256 &g = gf();
  std::string s;
  s.reserve(64 + static_cast<size_t>(rows) * k * 40);
  s += "#include \"rs_bitslice_core.h\"\n";
  if (streamed) s += "#include \"rs_stream.hpp\"\n";
  s += "namespace {\nstruct JitMat {\n";
  s += "  static constexpr int K = " + std::to_string(k) + ", R = " + std::to_string(rows) + ";\n";
  s += "  static constexpr unsigned long long copy_mask = " + std::to_string(copy_mask) + "ull;\n";
  s += "  struct Net { unsigned char row[R][K][8]; };\n  static constexpr Net net = {{";
  for (uint32_t p = 0; p < rows; p++) {
    s += p ? ",{" : "{";
    for (uint32_t j = 0; j < k; j++) {
      const uint8_t c = coef[static_cast<size_t>(p) * k + j];
      s += j ? ",{" : "{";
      for (int b = 0; b < 8; b++) {
        unsigned m = 0;
        for (int bp = 0; bp < 8; bp++)
          if ((g.mul(c, static_cast<uint8_t>(1u << bp)) >> b) & 1u) m |= 1u << bp;
        if (b) s += ',';
        s += std::to_string(m);
      }
      s += '}';
    }
    s += '}';
  }
  s += "}};\n};\n}  // namespace\n";
  if (test_call()) {
    // STORB_RS_JIT_TEST_CALL=1 (tests only): a body with an out-of-line call,
    // which code_object_calls must refuse before anything loads it.
    s += "__attribute__((noinline)) __device__ void storb_jit_test_callee(const storb_rs::ApplyArgs &a) {\n"
         "  if (a.k == 0xFFFFu) reinterpret_cast<unsigned *>(a.out[0])[threadIdx.x] = 1u;\n}\n";
  }
  // 2 waves per SIMD (<= 256 registers): without the hint, 64- and 128-lane
  // workgroups let the allocator take 257 at k = 32 (1 wave per SIMD)
  const int threads = ks.c ? 64 * ks.c * ks.w : sh.threads;
  s += "extern \"C\" __global__ __launch_bounds__(" + std::to_string(threads) +
       ") __attribute__((amdgpu_waves_per_eu(2))) void " +
       kernel_name(k, rows, copy_mask, streamed) + "(const storb_rs::ApplyArgs a" +
       (streamed ? ", const storb_rs::StreamArgs st" : "") + ") {\n";
  if (streamed) {
    // The streamed single call's gate (rs_stream.hpp): a workgroup waits for
    // its slice's host-written ready word, runs its tile, reports the slice.
    // One wave per tile only (the caller sizes slices in these tiles).
    s += "  const unsigned slice = static_cast<unsigned>(blockIdx.x * " +
         std::to_string(bs::bs_cols_per_tile(sh.threads)) + "u / st.slice_cols);\n";
    s += "  if (!storb_rs::stream_gate(st, slice)) return;\n";
    s += "  storb_rs::bs::bs_kernel_body<JitMat, " + std::to_string(group) + ", " +
         std::to_string(sh.threads) + ", " + std::to_string(sh.swz) + ">(a);\n";
    s += "  storb_rs::stream_report(st, slice);\n}\n";
    return s;
  }
  if (test_call()) s += "  storb_jit_test_callee(a);\n";
  if (lds >= 4 && dynamic_lds(lds) == 0) {
    // Static LDS reserving 160 KiB / cap per workgroup (occupancy cap).
    s += "  __shared__ unsigned occ_pad[" + std::to_string(lds / 4) + "];\n";
    s += "  asm volatile(\"\" :: \"s\"(occ_pad));  // keeps the unused array allocated\n";
  }
  if (ks.c)
    s += "  storb_rs::bs::bs_ksplit_body<JitMat, " + std::to_string(ks.c) + ", " +
         std::to_string(ks.w) + ", " + std::to_string(ks.g) + ", 1>(a);\n}\n";
  else if (split)
    s += "  storb_rs::bs::bs_split_body<JitMat, " + std::to_string(group) + ", " +
         std::to_string(sh.swz) + ">(a);\n}\n";
  else
    s += "  storb_rs::bs::bs_kernel_body<JitMat, " + std::to_string(group) + ", " +
         std::to_string(sh.threads) + ", " + std::to_string(sh.swz) + ">(a);\n}\n";
  return s;
}

}  // namespace

bool enabled() { return mode() != Mode::Off; }

// Worth a compiled kernel where it beats the table kernel -- measured A/B on
// the GPU with the launch shapes of rs_args.h bs_shape (a removed A/B script,
// STORB_RS_JIT=0 vs =always, profiles/r2_jit_policy_ab2/; bench decode leg
// ms, table / compiled): k = 16: r = 2 0.195 / 0.189, r = 3 0.219 / 0.204,
// r = 4 0.235 / 0.218, r = 8 0.397 / 0.256; k = 32: r = 2 0.230 / 0.187,
// r = 4 0.295 / 0.202, r = 16 0.732 / 0.269; k = 8 (config 3, r = 3) 0.236 /
// 0.235-0.246 over six launch shapes (profiles/r2_shape_ab/), so the table
// kernel keeps it. Before the launch-shape sweep the table kernel won at k =
// 16 up to 4 rows (profiles/r2_jit_policy_ab.jsonl). One row (repair of a
// single share): 0.193 / 0.191 at k = 32, left to the table kernel. k = 8..11
// with r >= 6 is the VALU model's guess (~5.5 ops per HBM byte), not
// measured. Only for batches large enough to matter (>= 4 MiB).
static bool valu_bound(uint32_t k, uint32_t rows) {
  if (k < 8 || k > static_cast<uint32_t>(kMaxIn) || rows == 0 || rows > kMaxRows) return false;
  const uint32_t min_rows = k >= 12 ? 2 : 6;
  return always() || rows >= min_rows;
}

bool wanted(uint32_t k, uint32_t rows, uint64_t bytes) {
  return enabled() && bytes >= (4ull << 20) && valu_bound(k, rows);
}

// The cache entry of a (k x r) matrix with the given copy mask: looked up,
// or created and queued. wait: block until its compile has finished.
static std::shared_ptr<Entry> entry_for(uint32_t k, uint32_t r, const uint8_t *coef,
                                        uint64_t copy_mask, bool wait, bool force,
                                        bool streamed = false) {
  // the streamed form: one wave per tile, no row split, no input split
  const bool split = !streamed && split_rows(k, r);
  const int group = split ? bs::kSplitGroup : bs::bs_group(static_cast<int>(k), static_cast<int>(r));
  const bs::BsShape sh = streamed ? shape(k, r) : split_or_shape(k, r);
  const bs::KsShape ks = streamed ? bs::KsShape{0, 0, 0, 0} : ks_of(k, r, copy_mask);
  const size_t lds = streamed ? cap_lds(sh.cap, 0) : launch_shape(k, r, copy_mask).lds;
  std::string key(32 + static_cast<size_t>(r) * k, '\0');
  const uint64_t hdr[4] = {(static_cast<uint64_t>(k) << 32) | r, copy_mask,
                           (static_cast<uint64_t>(group) << 32) | lds,
                           (static_cast<uint64_t>(sh.threads) << 32) | static_cast<uint32_t>(sh.swz) |
                               (split ? 1ull << 16 : 0) |
                               (static_cast<uint64_t>(ks.c * 16 + ks.w) << 20) |
                               (static_cast<uint64_t>(ks.g) << 26) |
                               (streamed ? 1ull << 31 : 0)};
  std::memcpy(&key[0], hdr, sizeof(hdr));
  std::memcpy(&key[32], coef, static_cast<size_t>(r) * k);
  Jit &J = jit();
  auto e = J.get(key, kernel_name(k, r, copy_mask, streamed), opt_level(k),
                 [&] { return source(k, r, coef, copy_mask, group, sh, lds, split, ks, streamed); },
                 force);
  if (e && wait) J.wait_for(*e);
  return e;
}

// Row blocks of at most kSlotR rows (the accumulators of one launch), as
// even as possible: 20 rows -> 10 + 10. Block b covers rows [r0(b), r0(b+1)).
// A row-split matrix is one block of all its rows.
static uint32_t row_blocks(uint32_t k, uint32_t rows) {
  return split_rows(k, rows) ? 1 : (rows + kSlotR - 1) / kSlotR;
}
static uint32_t row_start(uint32_t k, uint32_t rows, uint32_t b) {
  const uint32_t nb = row_blocks(k, rows);
  return static_cast<uint32_t>(static_cast<uint64_t>(rows) * b / nb);
}

hipError_t try_launch(int device, const ApplyArgs &a, uint8_t *const *d_out,
                      const size_t *out_stride, const uint8_t *coef, hipStream_t s,
                      bool *launched) {
  *launched = false;
  if (a.k == 0 || a.k > static_cast<uint32_t>(kMaxIn) || a.r == 0 || a.r > kMaxRows ||
      a.accumulate)
    return hipSuccess;
  {  // 16-B aligned slots (the dwordx4 kernels); outputs come from d_out
    ApplyArgs in_only = a;
    in_only.r = 0;
    if (!vector_ok(in_only)) return hipSuccess;
    for (uint32_t i = 0; i < a.r; i++)
      if ((reinterpret_cast<uintptr_t>(d_out[i]) | out_stride[i]) % 16) return hipSuccess;
  }
  const uint64_t cols = a.block >> 4;
  if (cols == 0 || (cols + 127) / 128 * a.nstripes > 0x7FFFFFFFull) return hipSuccess;
  uint64_t copy_mask = 0;
  for (uint32_t j = 0; a.ncopy && j < a.k; j++)
    if (a.copy[j]) copy_mask |= 1ull << j;
  // Every row block's kernel must be ready (all or none: a matrix is never
  // split between the compiled and the table kernels); the first block
  // also does the fused-assembly copies.
  Jit &J = jit();
  const uint32_t nb = row_blocks(a.k, a.r);
  std::vector<std::shared_ptr<Entry>> es(nb);
  bool ready = true;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t r0 = row_start(a.k, a.r, b), rr = row_start(a.k, a.r, b + 1) - r0;
    es[b] = entry_for(a.k, rr, coef + static_cast<size_t>(r0) * a.k, b == 0 ? copy_mask : 0,
                      false, false);
    ready = ready && es[b] && es[b]->state == Entry::Ready;
  }
  if (!ready) {
    J.fallbacks++;
    return hipSuccess;
  }
  std::vector<hipFunction_t> fs(nb);
  for (uint32_t b = 0; b < nb; b++) {
    hipError_t r = J.function(*es[b], device, &fs[b]);
    if (r != hipSuccess) return r;
  }
  // One launch per row block, each over the whole batch: a.r rows in nb > 1
  // blocks read every input nb times. (Going block after block over ranges
  // small enough for the later blocks to re-read the inputs from the 256 MiB
  // Infinity Cache measured slower -- 0.49 -> 0.77 ms at 128 MiB ranges --
  // as a k = 64 range that fits leaves too few workgroups per launch;
  // profiles/r2_k64/.)
  hipError_t r = hipSuccess;
  for (uint32_t b = 0; b < nb && r == hipSuccess; b++) {
    const uint32_t r0 = row_start(a.k, a.r, b), rr = row_start(a.k, a.r, b + 1) - r0;
    const LaunchShape ls = launch_shape(a.k, rr, b == 0 ? copy_mask : 0);
    const uint64_t blocks = ((cols + ls.cpt - 1) / ls.cpt) * a.nstripes;
    if (blocks == 0 || blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    ApplyArgs arg = a;
    arg.r = rr;
    if (b > 0) {
      arg.ncopy = 0;
      for (uint32_t j = 0; j < a.k; j++) arg.copy[j] = nullptr;
    }
    for (uint32_t i = 0; i < rr; i++) {
      arg.out[i] = d_out[r0 + i];
      arg.out_stride[i] = out_stride[r0 + i];
    }
    void *params[] = {&arg};
    r = hipModuleLaunchKernel(fs[b], static_cast<unsigned>(blocks), 1, 1,
                              static_cast<unsigned>(ls.threads), 1, 1,
                              static_cast<unsigned>(dynamic_lds(ls.lds)), s, params, nullptr);
    if (r == hipSuccess) r = J.used(*es[b], device, s);
    if (r == hipSuccess) J.launches++;
  }
  if (r != hipSuccess) return r;
  *launched = true;
  return hipSuccess;
}

// The streamed form of a matrix's kernel (single calls with k > 16, whose
// table-kernel stream measured slower than the sliced compiled kernels):
// one wave per tile, no fused assembly, up to 8 rows -- a download's chunks
// lose a few data shares; the one-wave 16-row k = 32 form spilled 6 VGPRs,
// and those keep the sliced path.
bool stream_form(uint32_t k, uint32_t rows) {
  return stream_enabled() && k > 16 && k <= static_cast<uint32_t>(kMaxIn) && rows >= 1 &&
         rows <= 8;
}

uint32_t stream_cols_per_tile(uint32_t k, uint32_t rows) {
  return bs::bs_cols_per_tile(shape(k, rows).threads);
}

hipError_t try_launch_stream(int device, const ApplyArgs &a, const uint8_t *coef,
                             const StreamArgs &st, hipStream_t s, bool *launched) {
  *launched = false;
  if (!stream_form(a.k, a.r) || a.ncopy || a.accumulate || a.nstripes != 1 ||
      !wanted(a.k, a.r, static_cast<uint64_t>(a.k + a.r) * a.block) || !vector_ok(a))
    return hipSuccess;
  auto e = entry_for(a.k, a.r, coef, 0, false, false, true);
  Jit &J = jit();
  if (!e || e->state != Entry::Ready) {
    J.fallbacks++;
    return hipSuccess;
  }
  hipFunction_t f = nullptr;
  hipError_t r = J.function(*e, device, &f);
  if (r != hipSuccess) return r;
  const bs::BsShape sh = shape(a.k, a.r);
  const uint64_t cpt = bs::bs_cols_per_tile(sh.threads);
  const uint64_t blocks = ((a.block >> 4) + cpt - 1) / cpt;
  if (blocks == 0 || blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  ApplyArgs arg = a;
  StreamArgs sa = st;
  void *params[] = {&arg, &sa};
  r = hipModuleLaunchKernel(f, static_cast<unsigned>(blocks), 1, 1,
                            static_cast<unsigned>(sh.threads), 1, 1,
                            static_cast<unsigned>(dynamic_lds(cap_lds(sh.cap, 0))), s, params,
                            nullptr);
  if (r == hipSuccess) r = J.used(*e, device, s);
  if (r != hipSuccess) return r;
  J.launches++;
  *launched = true;
  return hipSuccess;
}

int prepare(uint32_t k, uint32_t rows, const uint8_t *coef, uint64_t copy_mask, bool wait) {
  if (!enabled() || !valu_bound(k, rows)) return 0;
  if (!copy_mask && stream_form(k, rows)) {  // the single calls' streamed form too
    auto e = entry_for(k, rows, coef, 0, wait, true, true);
    if (!e || e->state == Entry::Failed) return e ? -1 : 0;
  }
  int res = 1;
  for (uint32_t b = 0; b < row_blocks(k, rows); b++) {
    const uint32_t r0 = row_start(k, rows, b), rr = row_start(k, rows, b + 1) - r0;
    auto e = entry_for(k, rr, coef + static_cast<size_t>(r0) * k, b == 0 ? copy_mask : 0, wait,
                       true);
    if (!e) return 0;
    if (e->state == Entry::Failed) return -1;
    if (e->state != Entry::Ready) res = 0;
  }
  return res;
}

}  // namespace jit
}  // namespace storb_rs

extern "C" {

int storb_rs_jit_wait(void) {
  storb_rs::jit::jit().wait_idle();
  return STORB_RS_OK;
}

int storb_rs_jit_stats(storb_rs_jit_stats_t *out) {
  if (!out) return STORB_RS_EINVAL;
  storb_rs::jit::jit().stats(out);
  return STORB_RS_OK;
}

}  // extern "C"
