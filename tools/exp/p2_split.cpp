// time split of the host permutation: full rounds vs partial rounds (transcript.cpp's own code)
#include <chrono>
#include <cstdio>
#include "../../latticeum_amd/csrc/transcript.cpp"
namespace {
void full_only(uint64_t *s) {
  mds16_rc(s, EXT_INIT);
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox7(s[i]);
    mds16_rc(s, r < 3 ? EXT_INIT + 16 * (r + 1) : nullptr);
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox7(s[i]);
    mds16_rc(s, r < 3 ? EXT_TERM + 16 * (r + 1) : nullptr);
  }
}
void partial_only(uint64_t *s) {
  for (int r = 0; r < 22; r++) {
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
    for (int i = 0; i < 16; i++) s[i] = wmuladd(s[i], DIAG_M1[i], sum);
  }
}
template <class F>
double timeit(F f) {
  uint64_t s[16];
  for (int i = 0; i < 16; i++) s[i] = i * 0x1234567ull;
  const int n = 200000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) f(s);
  auto t1 = std::chrono::steady_clock::now();
  volatile uint64_t sink = s[0];
  (void)sink;
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}
}  // namespace
int main() {
  for (int k = 0; k < 3; k++)
    printf("permute %.3f us  full rounds %.3f  partial rounds %.3f\n", timeit(permute), timeit(full_only), timeit(partial_only));
}
