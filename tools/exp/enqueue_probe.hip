// host enqueue cost vs commands in flight on one stream: kernels only, kernels +
// async D2H copies into pinned memory, kernels + event records
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

struct Big {
  int v[330];
};
__global__ void spin_big(unsigned long long cycles, int *out, Big b) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = b.v[7];
}
__global__ void spin(unsigned long long cycles, int *out) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

int main() {
  hipStream_t st;
  hipStreamCreate(&st);
  int *d;
  hipMalloc(&d, 64 << 20);
  void *h;
  hipHostMalloc(&h, 64 << 20, hipHostMallocDefault);
  Big big{};
  std::vector<hipEvent_t> ev(400);
  for (auto &e : ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  const unsigned long long cyc = 240000;  // about 100 us of shader clock
  for (int mode = 0; mode < 7; mode++) {
    hipStreamSynchronize(st);
    std::vector<double> us;
    for (int i = 0; i < 300; i++) {
      auto a = std::chrono::steady_clock::now();
      if (mode == 0 || i % 2 == 0) {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, cyc, d);
      } else if (mode == 1) {
        hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, st);
      } else if (mode == 2) {
        hipEventRecord(ev[i], st);
      } else if (mode == 3) {
        hipMemcpyAsync(d + 1024, d, 4096, hipMemcpyDeviceToDevice, st);
      } else if (mode == 4) {
        hipMemcpyAsync(h, d, 49152, hipMemcpyDeviceToHost, st);
      } else if (mode == 5) {
        hipMemcpyAsync(d + (8 << 20), d, 4 << 20, hipMemcpyDeviceToDevice, st);
      } else {
        hipLaunchKernelGGL(spin_big, dim3(1), dim3(64), 0, st, cyc, d, big);
      }
      auto b = std::chrono::steady_clock::now();
      us.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    hipStreamSynchronize(st);
    const char *nm[] = {"kernels", "kernel+d2h", "kernel+event", "kernel+d2d", "kernel+d2h48K", "kernel+d2d4M",
                        "kernel+bigarg"};
    printf("%-14s", nm[mode]);
    for (int i = 0; i < 300; i += 20) printf(" [%d]%.0f", i, us[i] + us[i + 1]);
    double tot = 0;
    for (double x : us) tot += x;
    printf("  total %.0f us\n", tot);
  }
  return 0;
}
