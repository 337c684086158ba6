// probe: what ds_read_b64_tr_b8 (__builtin_amdgcn_ds_read_tr8_b64_v2i32) delivers to each
// lane on gfx950. LDS bytes hold their own index (mod 256); lane l supplies byte address
// addr(l) = 8 l (variant 0) or a permuted map (variant 1); each lane writes its 8 bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;
__global__ void k(unsigned char *out, int variant) {
  __shared__ unsigned char buf[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) buf[i] = (unsigned char)(i & 255);
  __syncthreads();
  const int l = threadIdx.x;
  int addr = 8 * l;
  if (variant == 1) addr = 8 * ((l & 15) ^ 5) + 128 * (l >> 4);
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i *)(buf + addr));
  *(v2i *)(out + 8 * l) = r;
}
int main() {
  unsigned char *d, h[512];
  (void)hipMalloc(&d, 512);
  for (int v = 0; v < 2; v++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, v);
    (void)hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("variant %d\n", v);
    for (int l = 0; l < 64; l++) {
      printf("lane %2d:", l);
      for (int b = 0; b < 8; b++) printf(" %3d", h[8 * l + b]);
      printf("\n");
    }
  }
  return 0;
}
