// merkle.hip -- width-8 Poseidon2 Merkle trees of VM memory (SURVEY.md 8(f)
// rank 3): the zkvm's ZkVmCommitter hashes every memory page (a row of the
// memory matrix) with PaddingFreeSponge<Poseidon2Goldilocks<8>, 8, 4, 4> and
// joins digests with TruncatedPermutation<.., 2, 4, 8> up to the root
// (zkvm/src/commitments.rs:192-262, poseidon2.rs:31-49). Every page hash is an
// independent sponge chain (one thread each); every tree level is one launch
// of independent compressions.
//
// One permutation state spreads over 8 lanes (permute8_lane) in the tree
// kernels; the batched permutation keeps one state per thread.
//
// Constants: the width-8 external rounds from the reference
// (crypto_consts.rs:9-96), the 22 internal constants shared with width 16;
// the internal diagonal is Plonky3's MATRIX_DIAG_8_GOLDILOCKS, which the
// reference does not vendor (restated; parity unpinned).
#include "gl.hpp"
#include "kernels.hpp"
#include "p2_consts.inc"

namespace lfk {

namespace {

__constant__ uint64_t W8_EXT_INIT[32] = LF_P2W8_EXT_INIT;
__constant__ uint64_t W8_EXT_TERM[32] = LF_P2W8_EXT_TERM;
__constant__ uint64_t W8_INTERNAL[22] = LF_P2_INTERNAL;
__constant__ uint64_t W8_DIAG_M1[8] = LF_P2W8_DIAG_M1;

__device__ __forceinline__ uint64_t sbox7(uint64_t x) {
  const uint64_t x2 = gl::mul(x, x), x4 = gl::mul(x2, x2);
  return gl::mul(gl::mul(x4, x2), x);
}
// MDS light (poseidon2.rs:243-268 at width 8): MDSMat4 on each 4-chunk, then
// each word plus the sum of its column over the chunks
__device__ __forceinline__ void mds8(uint64_t *s) {
#pragma unroll
  for (int c = 0; c < 8; c += 4) {
    const uint64_t x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    const uint64_t t = gl::add(gl::add(x0, x1), gl::add(x2, x3));
    s[c + 0] = gl::add(t, gl::add(x0, gl::add(x1, x1)));
    s[c + 1] = gl::add(t, gl::add(x1, gl::add(x2, x2)));
    s[c + 2] = gl::add(t, gl::add(x2, gl::add(x3, x3)));
    s[c + 3] = gl::add(t, gl::add(x3, gl::add(x0, x0)));
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t sum = gl::add(s[k], s[4 + k]);
    s[k] = gl::add(s[k], sum);
    s[4 + k] = gl::add(s[4 + k], sum);
  }
}
__device__ void permute8(uint64_t *s) {
  mds8(s);
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = sbox7(gl::add(s[i], W8_EXT_INIT[8 * r + i]));
    mds8(s);
  }
#pragma unroll 1
  for (int r = 0; r < 22; r++) {
    s[0] = sbox7(gl::add(s[0], W8_INTERNAL[r]));
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) sum = gl::add(sum, s[i]);
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = gl::add(gl::mul(s[i], W8_DIAG_M1[i]), sum);
  }
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = sbox7(gl::add(s[i], W8_EXT_TERM[8 * r + i]));
    mds8(s);
  }
}

__global__ void __launch_bounds__(256) k_p2w8_permute(uint64_t *states, size_t n) {
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e >= n) return;
  uint64_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = gl::canon(states[e * 8 + i]);
  permute8(s);
#pragma unroll
  for (int i = 0; i < 8; i++) states[e * 8 + i] = s[i];
}

// ---------------------------------------------------------------- one state over 8 lanes
// A sponge chain is sequential, so a tree over P pages has only P independent
// chains (8 MB of memory: 8192, an eighth of the chip's SIMDs at one lane
// each). Here lane i of an 8-lane group holds state word i: the s-boxes of a
// full round run in parallel, the MDS mixing and the partial rounds' sum use
// cross-lane reads (ds_swizzle / bpermute), and 8x as many waves run.
__device__ __forceinline__ uint64_t shfl64(uint64_t x, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, src), hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), src);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t shfl64_xor(uint64_t x, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), m);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
// mds8 with word i in lane i of the group (lane = the thread's lane in the wave)
__device__ __forceinline__ uint64_t mds8_lane(uint64_t x, int lane) {
  const uint64_t s1 = gl::add(x, shfl64_xor(x, 1));
  const uint64_t t = gl::add(s1, shfl64_xor(s1, 2));                 // the 4-chunk's sum
  const uint64_t xn = shfl64(x, (lane & ~3) | ((lane + 1) & 3));     // x_(i+1 mod 4) of the chunk
  const uint64_t y = gl::add(t, gl::add(x, gl::add(xn, xn)));
  return gl::add(y, gl::add(y, shfl64_xor(y, 4)));                   // + the column sum over the two chunks
}
__device__ uint64_t permute8_lane(uint64_t x, int lane) {
  const int i = lane & 7;
  x = mds8_lane(x, lane);
#pragma unroll 1
  for (int r = 0; r < 4; r++) x = mds8_lane(sbox7(gl::add(x, W8_EXT_INIT[8 * r + i])), lane);
  const uint64_t dg = W8_DIAG_M1[i];
#pragma unroll 1
  for (int r = 0; r < 22; r++) {
    if (i == 0) x = sbox7(gl::add(x, W8_INTERNAL[r]));
    uint64_t sum = gl::add(x, shfl64_xor(x, 1));
    sum = gl::add(sum, shfl64_xor(sum, 2));
    sum = gl::add(sum, shfl64_xor(sum, 4));
    x = gl::add(gl::mul(x, dg), sum);
  }
#pragma unroll 1
  for (int r = 0; r < 4; r++) x = mds8_lane(sbox7(gl::add(x, W8_EXT_TERM[8 * r + i])), lane);
  return x;
}

// leaf e = PaddingFreeSponge hash of row e: overwrite state[0..4) with the next
// four words, permute; a partial last block is permuted too; no padding. One
// 8-lane group per row (groups past nrows run on a clamped row, store nothing:
// every lane of a wave takes part in the cross-lane reads)
__global__ void __launch_bounds__(256) k_merkle_leaves(const uint64_t *rows, size_t nrows, size_t width,
                                                      uint64_t *leaves) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, i = lane & 7;
  const size_t e = t >> 3;
  const bool ok = e < nrows;
  const uint64_t *row = rows + (ok ? e : 0) * width;
  uint64_t x = 0;
  for (size_t pos = 0; pos < width; pos += 4) {
    const size_t take = width - pos < 4 ? width - pos : 4;
    if ((size_t)i < take) x = gl::canon(row[pos + i]);
    x = permute8_lane(x, lane);
  }
  if (ok && i < 4) leaves[e * 4 + i] = x;
}

// parent e = permute(child 2e || child 2e + 1)[0..4): the 8 words are contiguous
__global__ void __launch_bounds__(256) k_merkle_level(const uint64_t *children, size_t nparents, uint64_t *parents) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, i = lane & 7;
  const size_t e = t >> 3;
  const bool ok = e < nparents;
  uint64_t x = children[(ok ? e : 0) * 8 + i];
  x = permute8_lane(x, lane);
  if (ok && i < 4) parents[e * 4 + i] = x;
}

unsigned nb(size_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

hipError_t p2w8_permute(uint64_t *states, size_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_p2w8_permute, dim3(nb(n)), dim3(256), 0, st, states, n);
  return hipGetLastError();
}

// Plonky3 MerkleTree::new over one matrix (p3-merkle-tree merkle_tree.rs at
// git 33e58c7787f9; not vendored): every layer but the root is padded to an even
// length with the zero digest (first_digest_layer: max_height + max_height % 2;
// compress: prev == 2 ? 1 : (prev / 2 + 1) & ~1), so any number of rows works
// (vm_code_comm, commitments.rs:314-340, commits a width-1 matrix of the code's
// half-words). nodes: the padded layers, leaves first, root last.
size_t merkle_nodes(size_t nrows) {
  size_t n = nrows <= 1 ? 1 : nrows + nrows % 2, tot = n;
  while (n > 1) {
    n = n == 2 ? 1 : ((n / 2 + 1) & ~(size_t)1);
    tot += n;
  }
  return tot;
}

hipError_t merkle_tree(const uint64_t *rows, size_t nrows, size_t width, uint64_t *nodes, hipStream_t st) {
  if (!nrows || !width) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_merkle_leaves, dim3(nb(8 * nrows)), dim3(256), 0, st, rows, nrows, width, nodes);
  size_t off = 0, n = nrows <= 1 ? 1 : nrows + nrows % 2;
  hipError_t e;
  if (n > nrows && (e = hipMemsetAsync(nodes + 4 * nrows, 0, 32 * (n - nrows), st)) != hipSuccess) return e;
  while (n > 1) {
    const size_t nn = n == 2 ? 1 : ((n / 2 + 1) & ~(size_t)1);
    hipLaunchKernelGGL(k_merkle_level, dim3(nb(8 * (n / 2))), dim3(256), 0, st, nodes + 4 * off, n / 2,
                       nodes + 4 * (off + n));
    if (nn > n / 2 && (e = hipMemsetAsync(nodes + 4 * (off + n + n / 2), 0, 32 * (nn - n / 2), st)) != hipSuccess)
      return e;
    off += n;
    n = nn;
  }
  return hipGetLastError();
}

// independent PaddingFreeSponge hashes of nrows rows (the leaf layer alone)
hipError_t hash_w8_rows(const uint64_t *rows, size_t nrows, size_t width, uint64_t *out, hipStream_t st) {
  if (!nrows) return hipSuccess;
  if (!width) return hipMemsetAsync(out, 0, 32 * nrows, st);  // the empty input's digest is the zero state
  hipLaunchKernelGGL(k_merkle_leaves, dim3(nb(8 * nrows)), dim3(256), 0, st, rows, nrows, width, out);
  return hipGetLastError();
}

}  // namespace lfk
