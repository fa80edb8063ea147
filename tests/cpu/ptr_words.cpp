// Host check of se::ptr_from_words (csrc/common.hpp), the join behind every buffer-resource
// base the conv GEMMs build from readfirstlane'd pointer words (se::uniform_ptr). Built and
// run by tests/test_uniform_ptr_cpu.py (host-only compile, no GPU).
#include <cstdio>
#include "../../speech-enhancement_amd/csrc/common.hpp"

int main() {
  int bad = 0;
  const unsigned long long cases[] = {0x00007f1280001000ull, 0x00007fffffffff00ull, 0x0000000180000000ull,
                                      0x00007f1200001000ull, 0x0000000000000000ull};
  for (unsigned long long p : cases) {
    // readfirstlane returns int: the words arrive as signed 32-bit values
    const int lo = (int)(unsigned)p, hi = (int)(unsigned)(p >> 32);
    const unsigned long long got = se::ptr_from_words((unsigned)lo, (unsigned)hi);
    // the pre-d630867 stencil form: widening the signed low word directly
    const unsigned long long old = ((unsigned long long)(unsigned)hi << 32) | (unsigned long long)(long long)lo;
    const bool high = ((unsigned)p) >= 0x80000000u;
    std::printf("%016llx -> %016llx (old form %016llx)%s\n", p, got, old, high ? "  low word >= 2^31" : "");
    if (got != p) ++bad;
    if (high != (old != p)) ++bad;   // the old form breaks exactly when the low word is >= 2^31
  }
  std::printf(bad ? "FAIL\n" : "OK\n");
  return bad;
}
