// CPU unit test of the single calls' sequence numbers (storb_amd/csrc/
// seq.hpp): the counter never hands out 0, also across the 2^32 wrap.
#include <cstdio>

#include "../../storb_amd/csrc/seq.hpp"

int main() {
  uint32_t c = 0;
  if (storb_rs::next_seq(c) != 1) return 1;
  c = 0xFFFFFFFDu;
  const uint32_t want[] = {0xFFFFFFFEu, 0xFFFFFFFFu, 1u, 2u};
  for (uint32_t w : want) {
    const uint32_t s = storb_rs::next_seq(c);
    if (s != w || s == 0) {
      std::printf("next_seq gave %u, want %u\n", s, w);
      return 1;
    }
  }
  std::printf("seq ok\n");
  return 0;
}
