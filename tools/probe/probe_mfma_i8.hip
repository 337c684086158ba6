// Probe (diagnostic only, not part of the library): on gfx950
//  (1) verify the lane map of v_mfma_i32_32x32x32_i8 with exact integer data,
//  (2) measure 64x64->128-bit multiply-accumulate throughput on the VALU
//      (C version vs. a v_mad_u64_u32 carry-chain version),
//  (3) measure i8 MFMA throughput.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

// hypothesis: lane l (r = l&31, h = l>>5) holds A[r][16h + j], B[16h + j][r], j = 0..15;
// D reg i of lane l is D[row = (i&3) + 8(i>>2) + 4h][col = r]
__global__ void k_layout(const signed char *A, const signed char *B, int *D) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  signed char a[16], b[16];
  for (int j = 0; j < 16; j++) {
    a[j] = A[r * 32 + 16 * h + j];
    b[j] = B[(16 * h + j) * 32 + r];
  }
  v4i fa, fb;
  memcpy(&fa, a, 16);
  memcpy(&fb, b, 16);
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, c, 0, 0, 0);
  for (int i = 0; i < 16; i++) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

__device__ __forceinline__ void mad_c(uint64_t &lo, uint64_t &hi, uint32_t &top, uint64_t a, uint64_t b) {
  uint64_t pl = a * b, ph = __umul64hi(a, b);
  uint64_t nlo = lo + pl;
  ph += nlo < pl;
  lo = nlo;
  uint64_t nhi = hi + ph;
  top += nhi < ph;
  hi = nhi;
}

// carry-chain: S0 += a0*b0, S1 += a0*b1 + a1*b0, S2 += a1*b1, carries counted
__device__ __forceinline__ void mad_asm(uint64_t &s0, uint64_t &s1, uint64_t &s2, uint32_t &c0, uint32_t &c1,
                                        uint32_t &c2, uint64_t a, uint64_t b) {
  uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t cc;
  asm volatile(
      "v_mad_u64_u32 %0, %6, %7, %9, %0\n\t"
      "v_addc_co_u32_e64 %3, %6, 0, %3, %6\n\t"
      "v_mad_u64_u32 %1, %6, %7, %10, %1\n\t"
      "v_addc_co_u32_e64 %4, %6, 0, %4, %6\n\t"
      "v_mad_u64_u32 %1, %6, %8, %9, %1\n\t"
      "v_addc_co_u32_e64 %4, %6, 0, %4, %6\n\t"
      "v_mad_u64_u32 %2, %6, %8, %10, %2\n\t"
      "v_addc_co_u32_e64 %5, %6, 0, %5, %6"
      : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(c0), "+v"(c1), "+v"(c2), "=&s"(cc)
      : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
}

template <int NACC>
__global__ void k_bench_c(const uint64_t *in, uint64_t *out, int iters) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a[NACC], b = in[t] | 1;
  uint64_t lo[NACC], hi[NACC];
  uint32_t top[NACC];
  for (int i = 0; i < NACC; i++) {
    a[i] = in[t + i + 1];
    lo[i] = hi[i] = 0;
    top[i] = 0;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) mad_c(lo[i], hi[i], top[i], a[i], b);
    b = b * 0x9e3779b97f4a7c15ull + 1;
  }
  uint64_t s = 0;
  for (int i = 0; i < NACC; i++) s += lo[i] ^ hi[i] ^ top[i];
  out[t] = s;
}

template <int NACC>
__global__ void k_bench_asm(const uint64_t *in, uint64_t *out, int iters) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a[NACC], b = in[t] | 1;
  uint64_t s0[NACC], s1[NACC], s2[NACC];
  uint32_t c0[NACC], c1[NACC], c2[NACC];
  for (int i = 0; i < NACC; i++) {
    a[i] = in[t + i + 1];
    s0[i] = s1[i] = s2[i] = 0;
    c0[i] = c1[i] = c2[i] = 0;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) mad_asm(s0[i], s1[i], s2[i], c0[i], c1[i], c2[i], a[i], b);
    b = b * 0x9e3779b97f4a7c15ull + 1;
  }
  uint64_t s = 0;
  for (int i = 0; i < NACC; i++) s += s0[i] ^ s1[i] ^ s2[i] ^ c0[i] ^ c1[i] ^ c2[i];
  out[t] = s;
}

__global__ void k_bench_mfma(const v4i *in, v16i *out, int iters) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  v4i a = in[t & 1023], b = in[(t + 7) & 1023];
  v16i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int it = 0; it < iters; it++) {
    c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
  }
  out[t] = c0 + c1 + c2 + c3;
}

int main() {
  // (1) layout
  std::vector<signed char> A(1024), B(1024);
  for (int i = 0; i < 1024; i++) {
    A[i] = (signed char)((i * 37 + 11) % 251 - 125);
    B[i] = (signed char)((i * 53 + 5) % 241 - 120);
  }
  signed char *dA, *dB;
  int *dD;
  CK(hipMalloc(&dA, 1024));
  CK(hipMalloc(&dB, 1024));
  CK(hipMalloc(&dD, 4096));
  CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  std::vector<int> D(1024);
  CK(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      int s = 0;
      for (int k = 0; k < 32; k++) s += A[i * 32 + k] * B[k * 32 + j];
      if (s != D[i * 32 + j]) bad++;
    }
  printf("mfma_i32_32x32x32_i8 layout hypothesis: %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);

  // (2)/(3) throughput
  const int blocks = 256 * 8, threads = 256, iters = 4096;
  const size_t n = (size_t)blocks * threads + 64;
  uint64_t *din, *dout;
  CK(hipMalloc(&din, n * 8));
  CK(hipMalloc(&dout, n * 8));
  std::vector<uint64_t> h(n);
  for (size_t i = 0; i < n; i++) h[i] = 0x123456789abcdefull * (i + 1);
  CK(hipMemcpy(din, h.data(), n * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  double macs = (double)blocks * threads * iters * 8;
#define TIME(label, launch, work, unit)                                             \
  launch;                                                                           \
  CK(hipDeviceSynchronize());                                                       \
  CK(hipEventRecord(e0));                                                           \
  launch;                                                                           \
  CK(hipEventRecord(e1));                                                           \
  CK(hipEventSynchronize(e1));                                                      \
  CK(hipEventElapsedTime(&ms, e0, e1));                                             \
  printf("%-40s %8.3f ms  %8.3f T%s/s\n", label, ms, (work) / (ms * 1e-3) / 1e12, unit);
  TIME("VALU 64x64 mac, C (8 acc)", hipLaunchKernelGGL(k_bench_c<8>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters), macs, "MAC");
  TIME("VALU 64x64 mac, asm carry chain (8 acc)", hipLaunchKernelGGL(k_bench_asm<8>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters), macs, "MAC");
  v16i *dmf;
  CK(hipMalloc(&dmf, (size_t)blocks * threads * sizeof(v16i)));
  double mf = (double)blocks * (threads / 64) * iters * 4 * 32.0 * 32 * 32 * 2;
  TIME("MFMA i32_32x32x32_i8 (4 acc)", hipLaunchKernelGGL(k_bench_mfma, dim3(blocks), dim3(threads), 0, 0, (const v4i *)din, dmf, iters), mf, "OP");
  return 0;
}
