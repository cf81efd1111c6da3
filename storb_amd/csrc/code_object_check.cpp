// code_object_check.cpp -- refuse gfx950 code objects whose kernels make
// function calls (storb_rs_code_object_calls, include/storb_rs.h).
//
// Every kernel of this library is meant to be one inlined body. An
// out-of-line call is what hung the round-4 descriptor decode (tools/fuzz.py
// seed 4242): the callee was larger than a short branch can
// span, the backend relaxed three of its branches through s[30:31] -- the
// register the caller's s_swappc_b64 had put the return address in -- and the
// callee's final s_setpc_b64 s[30:31] jumped back into its own body instead
// of returning (profiles/r5_hang_isa_excerpt.txt). The run-time compiled
// kernels (rs_jit.cpp) are the largest bodies in the library and are built
// where no test sees their ISA, so every one is checked here before it is
// loaded; one that calls is refused and its matrix runs the table kernel.
//
// Checks, per kernel (an STT_FUNC symbol `name` with a `name.kd` descriptor):
//  * the code object holds no other function with a body (a call target);
//  * the descriptor does not ask for a dynamic stack (kernel_code_properties
//    bit 11, USES_DYNAMIC_STACK: recursion or indirect calls);
//  * its instructions, disassembled with comgr, contain no s_swappc /
//    s_call (a kernel's own long branches, s_getpc + s_setpc, are fine: a
//    kernel has no return address to lose).
#include <amd_comgr/amd_comgr.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/storb_rs.h"

namespace {

template <typename T>
bool rd(const uint8_t *p, size_t len, size_t off, T *out) {
  if (off > len || sizeof(T) > len - off) return false;
  std::memcpy(out, p + off, sizeof(T));
  return true;
}

struct Sym {
  std::string name;
  uint8_t type = 0;
  uint16_t shndx = 0;
  uint64_t value = 0, size = 0;
};

struct Sec {
  uint32_t type = 0;
  uint64_t addr = 0, off = 0, size = 0;
  uint32_t link = 0;
};

struct Disasm {
  const uint8_t *base;
  size_t len;
  std::string last;
};

uint64_t read_mem(uint64_t from, char *to, uint64_t size, void *user) {
  auto *d = static_cast<Disasm *>(user);
  if (from >= d->len) return 0;
  const uint64_t n = std::min<uint64_t>(size, d->len - from);
  std::memcpy(to, d->base + from, n);
  return n;
}
void print_insn(const char *insn, void *user) { static_cast<Disasm *>(user)->last = insn; }
void print_addr(uint64_t, void *) {}

// 0 clean, 1 a call (why says where), -1 unreadable (why says what).
int check(const uint8_t *co, size_t len, std::string &why) {
  static const uint8_t kMagic[4] = {0x7f, 'E', 'L', 'F'};
  if (len < 64 || std::memcmp(co, kMagic, 4) != 0 || co[4] != 2 || co[5] != 1) {
    why = "not a 64-bit little-endian ELF";
    return -1;
  }
  uint64_t shoff = 0;
  uint16_t shentsize = 0, shnum = 0;
  if (!rd(co, len, 0x28, &shoff) || !rd(co, len, 0x3A, &shentsize) || !rd(co, len, 0x3C, &shnum) ||
      shentsize < 64) {
    why = "bad ELF header";
    return -1;
  }
  std::vector<Sec> secs(shnum);
  for (uint16_t i = 0; i < shnum; i++) {
    const size_t o = shoff + static_cast<size_t>(i) * shentsize;
    if (!rd(co, len, o + 4, &secs[i].type) || !rd(co, len, o + 16, &secs[i].addr) ||
        !rd(co, len, o + 24, &secs[i].off) || !rd(co, len, o + 32, &secs[i].size) ||
        !rd(co, len, o + 40, &secs[i].link)) {
      why = "bad section header";
      return -1;
    }
  }
  std::vector<Sym> syms;
  for (const Sec &s : secs) {
    if (s.type != 2 /* SHT_SYMTAB */) continue;
    if (s.link >= secs.size()) continue;
    const Sec &str = secs[s.link];
    for (uint64_t o = 24; o + 24 <= s.size; o += 24) {  // entry 0 is the null symbol
      uint32_t name = 0;
      uint8_t info = 0;
      Sym y;
      if (!rd(co, len, s.off + o, &name) || !rd(co, len, s.off + o + 4, &info) ||
          !rd(co, len, s.off + o + 6, &y.shndx) || !rd(co, len, s.off + o + 8, &y.value) ||
          !rd(co, len, s.off + o + 16, &y.size)) {
        why = "bad symbol";
        return -1;
      }
      y.type = info & 0xF;
      if (name < str.size && str.off + name < len) {
        const char *c = reinterpret_cast<const char *>(co + str.off + name);
        y.name.assign(c, strnlen(c, len - str.off - name));
      }
      syms.push_back(std::move(y));
    }
  }
  auto has_kd = [&](const std::string &n) {
    for (const Sym &y : syms)
      if (y.name == n + ".kd") return true;
    return false;
  };
  std::vector<const Sym *> kernels;
  for (const Sym &y : syms) {
    if (y.type != 2 /* STT_FUNC */ || y.size == 0) continue;
    if (has_kd(y.name)) {
      kernels.push_back(&y);
    } else {
      why = "out-of-line function " + y.name;
      return 1;
    }
  }
  if (kernels.empty()) {
    why = "no kernel symbols";
    return -1;
  }
  amd_comgr_disassembly_info_t info;
  Disasm d{co, len, {}};
  if (amd_comgr_create_disassembly_info("amdgcn-amd-amdhsa--gfx950", read_mem, print_insn,
                                        print_addr, &info) != AMD_COMGR_STATUS_SUCCESS) {
    why = "comgr disassembler unavailable";
    return -1;
  }
  int res = 0;
  for (const Sym *k : kernels) {
    // descriptor: kernel_code_properties (u16 at byte 56), bit 11
    for (const Sym &y : syms)
      if (y.name == k->name + ".kd" && y.shndx < secs.size()) {
        const Sec &s = secs[y.shndx];
        uint16_t props = 0;
        if (rd(co, len, s.off + (y.value - s.addr) + 56, &props) && (props & (1u << 11))) {
          why = k->name + ": descriptor asks for a dynamic stack";
          res = 1;
        }
      }
    if (res) break;
    if (k->shndx >= secs.size()) continue;
    const Sec &s = secs[k->shndx];
    const uint64_t begin = s.off + (k->value - s.addr), end = begin + k->size;
    if (end > len || begin > end) {
      why = k->name + ": body outside the file";
      res = -1;
      break;
    }
    for (uint64_t pc = begin; pc < end;) {
      uint64_t n = 0;
      d.last.clear();
      if (amd_comgr_disassemble_instruction(info, pc, &d, &n) != AMD_COMGR_STATUS_SUCCESS ||
          n == 0) {
        pc += 4;  // undecodable word (padding): skip it
        continue;
      }
      const size_t p = d.last.find_first_not_of(" \t");
      if (p != std::string::npos && (d.last.compare(p, 8, "s_swappc") == 0 ||
                                     d.last.compare(p, 6, "s_call") == 0)) {
        why = k->name + ": " + d.last.substr(p) + " at +" + std::to_string(pc - begin);
        res = 1;
        break;
      }
      pc += n;
    }
    if (res) break;
  }
  amd_comgr_destroy_disassembly_info(info);
  return res;
}

}  // namespace

namespace storb_rs {
int code_object_calls(const void *co, size_t len, std::string &why) {
  return check(static_cast<const uint8_t *>(co), len, why);
}
}  // namespace storb_rs

extern "C" int storb_rs_code_object_calls(const void *code, size_t len, char *why,
                                          size_t why_len) {
  if (!code) return -1;
  std::string w;
  const int r = check(static_cast<const uint8_t *>(code), len, w);
  if (why && why_len) {
    const size_t n = std::min(w.size(), why_len - 1);
    std::memcpy(why, w.data(), n);
    why[n] = '\0';
  }
  return r;
}
