// Probe (diagnostic only, not part of the library): issue throughput of the
// VALU instructions the Goldilocks arithmetic is built from, on gfx950.
// Each thread runs 8 independent dependency chains of one instruction; the
// result is wave-instructions per cycle per CU (1.0 = one wave64 instruction
// per cycle per CU, i.e. full rate on 4 SIMDs x 16 lanes).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

constexpr int ITERS = 2048;

#define CHAIN8(BODY) BODY(0) BODY(1) BODY(2) BODY(3) BODY(4) BODY(5) BODY(6) BODY(7)

template <int OP>
__global__ void __launch_bounds__(256) k_op(unsigned *out, unsigned seed) {
  unsigned a[8], b[8];
  unsigned long long w[8];
  for (int i = 0; i < 8; i++) {
    a[i] = seed * (threadIdx.x + 1) + i;
    b[i] = a[i] ^ 0x9e3779b9u;
    w[i] = ((unsigned long long)b[i] << 32) | a[i];
  }
  for (int it = 0; it < ITERS; it++) {
    if constexpr (OP == 0) {  // v_add_u32
#define B(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 1) {  // v_mad_u64_u32
#define B(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(b[i]) : "vcc");
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 2) {  // v_mul_lo_u32
#define B(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 3) {  // v_mul_hi_u32
#define B(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 4) {  // v_lshl_add_u64
#define B(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[i]) : "v"(w[(i + 1) & 7]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 5) {  // v_add_co_u32 (carry out to vcc)
#define B(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b[i]) : "vcc");
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 6) {  // v_cmp_lt_u64 + v_cndmask_b32
#define B(i)                                                                                      \
  asm volatile("v_cmp_lt_u64 vcc, %0, %2\n\tv_cndmask_b32 %1, %1, 0, vcc" : "+v"(w[i]), "+v"(a[i]) \
               : "v"(w[(i + 3) & 7]) : "vcc");
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 7) {  // v_alignbit_b32
#define B(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 8) {  // v_lshlrev_b64
#define B(i) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(w[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 9) {  // v_mul_u32_u24
#define B(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 10) {  // v_cndmask_b32 alone
#define B(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 11) {  // v_cmp_lt_u64 alone (result to a SGPR pair)
#define B(i) asm volatile("v_cmp_lt_u64 vcc, %0, %1" : : "v"(w[i]), "v"(w[(i + 1) & 7]) : "vcc");
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 12) {  // v_mad_u32_u24
#define B(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 13) {  // v_pk_add_u16 (packed)
#define B(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 14) {  // v_add_f64 (reference point for 64-bit datapath)
#define B(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(w[i]) : "v"(w[(i + 1) & 7]));
      CHAIN8(B)
#undef B
    } else if constexpr (OP == 15) {  // v_addc_co_u32 (carry in + out)
#define B(i) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(b[i]) : "vcc");
      CHAIN8(B)
#undef B
    }
  }
  unsigned s = 0;
  for (int i = 0; i < 8; i++) s += a[i] + (unsigned)w[i] + (unsigned)(w[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char *name, unsigned *out, int cus, double ghz, int instrs_per_chain_step) {
  const int blocks = cus * 16;  // 16 blocks x 4 waves = 64 waves per CU (8 per SIMD) max
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, out, 3u);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double waves = blocks * 4.0;
  const double winstr = waves * ITERS * 8.0 * instrs_per_chain_step;
  const double per_cu_cycle = winstr / (ms * 1e-3 * ghz * 1e9 * cus);
  printf("%-22s %8.3f ms  %.3f wave-instr/cycle/CU\n", name, ms, per_cu_cycle);
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;
  printf("%s  CUs %d  clock %.2f GHz\n", p.gcnArchName, cus, ghz);
  unsigned *out;
  CK(hipMalloc(&out, (size_t)cus * 16 * 256 * 4));
  run<0>("v_add_u32", out, cus, ghz, 1);
  run<1>("v_mad_u64_u32", out, cus, ghz, 1);
  run<2>("v_mul_lo_u32", out, cus, ghz, 1);
  run<3>("v_mul_hi_u32", out, cus, ghz, 1);
  run<4>("v_lshl_add_u64", out, cus, ghz, 1);
  run<5>("v_add_co_u32", out, cus, ghz, 1);
  run<15>("v_addc_co_u32", out, cus, ghz, 1);
  run<6>("v_cmp_lt_u64+cndmask", out, cus, ghz, 2);
  run<11>("v_cmp_lt_u64", out, cus, ghz, 1);
  run<10>("v_cndmask_b32", out, cus, ghz, 1);
  run<7>("v_alignbit_b32", out, cus, ghz, 1);
  run<8>("v_lshlrev_b64", out, cus, ghz, 1);
  run<9>("v_mul_u32_u24", out, cus, ghz, 1);
  run<12>("v_mad_u32_u24", out, cus, ghz, 1);
  run<13>("v_pk_add_u16", out, cus, ghz, 1);
  run<14>("v_add_f64", out, cus, ghz, 1);
  CK(hipFree(out));
  return 0;
}
