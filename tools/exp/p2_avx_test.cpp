// transcript.cpp's AVX-512 permutation (and its lane ops) against the scalar form: equality and time
// build: hipcc -O3 -std=c++17 -x hip --offload-arch=gfx950 --offload-host-only p2_avx_test.cpp -L../../latticeum_amd -llatticeum_amd
#include <chrono>
#include <cstdio>
#include <random>
#include "../../latticeum_amd/csrc/transcript.cpp"
namespace {
using namespace p2avx;
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
LF_AVX512 uint64_t check_ops(std::mt19937_64 &g) {
  uint64_t badop = 0;
  // lane ops on extreme and random weak values
  const uint64_t ext[] = {0, 1, 2, gl::EPS, gl::EPS + 1, gl::P - 1, gl::P, gl::P + 1, ~0ull, ~0ull - 1, 1ull << 63,
                          (1ull << 63) - 1, 0xFFFFFFFF00000000ull, 0x00000001FFFFFFFFull};
  for (int it = 0; it < 400000; it++) {
    alignas(64) uint64_t a[8], b[8], m[8], w[8];
    for (int i = 0; i < 8; i++) {
      a[i] = (it % 4 == 0) ? ext[g() % 14] : g();
      b[i] = (it % 3 == 0) ? ext[g() % 14] : g();
    }
    _mm512_store_si512(m, wmul8(_mm512_load_si512(a), _mm512_load_si512(b)));
    _mm512_store_si512(w, wadd8(_mm512_load_si512(a), _mm512_load_si512(b)));
    alignas(64) uint64_t q[8];
    _mm512_store_si512(q, wsqr8(_mm512_load_si512(a)));
    for (int i = 0; i < 8; i++) badop += gl::canon(q[i]) != gl::mul(gl::canon(a[i]), gl::canon(a[i]));
    for (int i = 0; i < 8; i++) {
      badop += gl::canon(m[i]) != gl::canon(wmul(a[i], b[i])) ||
               gl::canon(m[i]) != gl::mul(gl::canon(a[i]), gl::canon(b[i]));
      badop += gl::canon(w[i]) != gl::add(gl::canon(a[i]), gl::canon(b[i]));
    }
  }
  return badop;
}
int main() {
  std::mt19937_64 g(1);
  uint64_t bad = 0, badop = check_ops(g);
  for (int it = 0; it < 100000; it++) {
    uint64_t a[16], b[16];
    for (int i = 0; i < 16; i++) {
      uint64_t v = g();
      if (it % 3 == 0) v = gl::P - 1 - (uint64_t)(i % 3);
      if (it % 7 == 0) v = i;
      a[i] = b[i] = gl::canon(v);
    }
    permute_scalar(a);
    permute_avx512(b);
    for (int i = 0; i < 16; i++) bad += a[i] != b[i];
  }
  printf("op mismatches %llu, permutation mismatches %llu\n", (unsigned long long)badop, (unsigned long long)bad);
  for (int k = 0; k < 3; k++) printf("scalar %.3f us  avx512 %.3f us\n", timeit(permute_scalar), timeit(permute_avx512));
}
