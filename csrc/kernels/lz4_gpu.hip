// GPU LZ4 codec for activations (gfx950), producing / consuming STANDARD LZ4
// frames so a GPU-compressed activation can be decoded by any LZ4 frame
// decoder (our host codec in csrc/runtime/lz4.cpp, python-lz4, lz4 CLI).
//
// The reference compresses every activation on the CPU before each TCP hop
// (`src/node.py:178`, `src/dispatcher.py:92-98`).  Here compression runs on a
// side HIP stream right after the producing slice, overlapped with the next
// micro-batch's compute (parallel/gpu_codec.py).
//
// Layout: the input is cut into CHUNK-byte chunks; each chunk is one
// independent LZ4 block (frame FLG: independent blocks, content size, no
// checksums; BD: 64 KiB max block).  One thread compresses one chunk with a
// greedy single-probe hash matcher (a private 512-entry u16 table in LDS);
// incompressible chunks are stored raw (block size high bit).  A single
// workgroup prefix-sums the block sizes and a pack kernel scatters the
// blocks after the 15-byte frame header.  Decoding is one thread per block,
// with block offsets parsed from the headers on the host.
#include "kernels.h"

namespace adapt {

namespace {
constexpr int CHUNK = 1024;                          // bytes per LZ4 block
constexpr int BOUND = CHUNK + CHUNK / 255 + 16;      // worst-case compressed block
constexpr int HBITS = 9;
constexpr int ENC_THREADS = 128;                     // 128 x 1 KiB of hash tables = 128 KiB LDS
constexpr int MINMATCH = 4, LASTLIT = 5, MFLIMIT = 12;

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t hsh(uint32_t v) { return (v * 2654435761u) >> (32 - HBITS); }

__device__ __forceinline__ uint8_t* put_len(uint8_t* op, int len) {
  while (len >= 255) { *op++ = 255; len -= 255; }
  *op++ = (uint8_t)len;
  return op;
}
}  // namespace

// scratch[c * BOUND ...] <- compressed chunk c; sizes[c] = LZ4 block-size word
__global__ __launch_bounds__(ENC_THREADS) void lz4_enc_chunks(const uint8_t* __restrict__ in, size_t n,
                                                              uint8_t* __restrict__ scratch,
                                                              uint32_t* __restrict__ sizes, int nchunks) {
  __shared__ uint16_t tables[ENC_THREADS][1 << HBITS];
  const int c = blockIdx.x * ENC_THREADS + threadIdx.x;
  if (c >= nchunks) return;
  uint16_t* tab = tables[threadIdx.x];
  for (int i = 0; i < (1 << HBITS); ++i) tab[i] = 0;
  const uint8_t* src = in + (size_t)c * CHUNK;
  const int len = (int)min((size_t)CHUNK, n - (size_t)c * CHUNK);
  uint8_t* dst = scratch + (size_t)c * BOUND;
  uint8_t* op = dst;
  int ip = 0, anchor = 0;
  if (len > MFLIMIT) {
    const int mflimit = len - MFLIMIT, matchlimit = len - LASTLIT;
    ip = 1;
    while (ip < mflimit) {
      uint32_t seq = ld32(src + ip);
      uint32_t h = hsh(seq);
      int ref = tab[h];
      tab[h] = (uint16_t)ip;
      if (ref >= ip || ld32(src + ref) != seq) {
        ++ip;
        continue;
      }
      // backwards extension
      while (ip > anchor && ref > 0 && src[ip - 1] == src[ref - 1]) { --ip; --ref; }
      int p = ip + MINMATCH, m = ref + MINMATCH;
      while (p < matchlimit && src[p] == src[m]) { ++p; ++m; }
      const int lit = ip - anchor, ml = p - ip - MINMATCH;
      uint8_t* token = op++;
      *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
      if (lit >= 15) op = put_len(op, lit - 15);
      for (int i = 0; i < lit; ++i) op[i] = src[anchor + i];
      op += lit;
      const int off = ip - ref;
      op[0] = (uint8_t)(off & 0xFF);
      op[1] = (uint8_t)(off >> 8);
      op += 2;
      *token |= (uint8_t)(ml >= 15 ? 15 : ml);
      if (ml >= 15) op = put_len(op, ml - 15);
      ip = anchor = p;
      if (p - 2 > 0 && p - 2 < mflimit) tab[hsh(ld32(src + p - 2))] = (uint16_t)(p - 2);
    }
  }
  {  // last literals
    const int lit = len - anchor;
    uint8_t* token = op++;
    *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
    if (lit >= 15) op = put_len(op, lit - 15);
    for (int i = 0; i < lit; ++i) op[i] = src[anchor + i];
    op += lit;
  }
  const int csize = (int)(op - dst);
  sizes[c] = csize < len ? (uint32_t)csize : ((uint32_t)len | 0x80000000u);
}

// single-workgroup exclusive scan of (4 + payload) over the blocks -> offsets; total in *total
__global__ __launch_bounds__(1024) void lz4_scan(const uint32_t* __restrict__ sizes, uint32_t* __restrict__ offs,
                                                 int nchunks, uint64_t* __restrict__ total) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int per = (nchunks + 1023) / 1024;
  const int b0 = t * per, b1 = min(nchunks, b0 + per);
  uint32_t s = 0;
  for (int i = b0; i < b1; ++i) s += 4 + (sizes[i] & 0x7FFFFFFFu);
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {        // Hillis-Steele inclusive scan
    uint32_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = t ? part[t - 1] : 0;
  for (int i = b0; i < b1; ++i) {
    offs[i] = run;
    run += 4 + (sizes[i] & 0x7FFFFFFFu);
  }
  if (t == 1023) *total = 15ull + part[1023] + 4;   // header + blocks + end mark
}

__global__ __launch_bounds__(256) void lz4_pack(const uint8_t* __restrict__ in, size_t n,
                                                const uint8_t* __restrict__ scratch,
                                                const uint32_t* __restrict__ sizes, const uint32_t* __restrict__ offs,
                                                int nchunks, uint8_t* __restrict__ out, const uint64_t* total) {
  const int c = blockIdx.x;   // one workgroup per block: cooperative byte copy
  if (c == 0 && threadIdx.x == 0) {
    // frame header: magic, FLG (v01, B.Indep, C.Size), BD (64 KiB), content size, HC
    uint8_t h[15] = {0x04, 0x22, 0x4D, 0x18, (1u << 6) | (1u << 5) | (1u << 3), 4u << 4};
    uint64_t cs = n;
    for (int i = 0; i < 8; ++i) h[6 + i] = (uint8_t)(cs >> (8 * i));
    // xxh32(h+4, 10, 0) >> 8 & 0xFF computed inline
    const uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U, P5 = 374761393U;
    uint32_t acc = P5 + 10u;
    const uint8_t* q = h + 4;
    for (int i = 0; i < 2; ++i) {
      uint32_t v = (uint32_t)q[4 * i] | ((uint32_t)q[4 * i + 1] << 8) | ((uint32_t)q[4 * i + 2] << 16) |
                   ((uint32_t)q[4 * i + 3] << 24);
      acc += v * P3;
      acc = ((acc << 17) | (acc >> 15)) * P4;
    }
    for (int i = 8; i < 10; ++i) {
      acc += q[i] * P5;
      acc = ((acc << 11) | (acc >> 21)) * P1;
    }
    acc ^= acc >> 15; acc *= P2; acc ^= acc >> 13; acc *= P3; acc ^= acc >> 16;
    h[14] = (uint8_t)((acc >> 8) & 0xFF);
    for (int i = 0; i < 15; ++i) out[i] = h[i];
    const uint64_t tot = *total;
    for (int i = 0; i < 4; ++i) out[tot - 4 + i] = 0;   // end mark
  }
  if (c >= nchunks) return;
  const uint32_t w = sizes[c];
  uint8_t* o = out + 15 + offs[c];
  if (threadIdx.x < 4) o[threadIdx.x] = (uint8_t)(w >> (8 * threadIdx.x));
  const uint32_t len = w & 0x7FFFFFFFu;
  const uint8_t* src = (w & 0x80000000u) ? in + (size_t)c * CHUNK : scratch + (size_t)c * BOUND;
  for (uint32_t i = threadIdx.x; i < len; i += blockDim.x) o[4 + i] = src[i];
}

// one thread per block: decode block c (payload at frame+offs[c], size word sizes[c]) into out + c*CHUNK
__global__ __launch_bounds__(256) void lz4_dec_chunks(const uint8_t* __restrict__ frame,
                                                      const uint32_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ sizes, int nchunks,
                                                      uint8_t* __restrict__ out, size_t n, int* __restrict__ err) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const uint32_t w = sizes[c];
  const uint32_t len = w & 0x7FFFFFFFu;
  const uint8_t* ip = frame + offs[c];
  const uint8_t* iend = ip + len;
  uint8_t* dst = out + (size_t)c * CHUNK;
  const int cap = (int)min((size_t)CHUNK, n - (size_t)c * CHUNK);
  if (w & 0x80000000u) {
    if ((int)len != cap) { atomicOr(err, 1); return; }
    for (uint32_t i = 0; i < len; ++i) dst[i] = ip[i];
    return;
  }
  int o = 0;
  while (ip < iend) {
    const unsigned token = *ip++;
    int lit = token >> 4;
    if (lit == 15) { unsigned b; do { b = *ip++; lit += b; } while (b == 255 && ip < iend); }
    if (o + lit > cap || ip + lit > iend) { atomicOr(err, 2); return; }
    for (int i = 0; i < lit; ++i) dst[o + i] = ip[i];
    o += lit;
    ip += lit;
    if (ip >= iend) break;
    const int off = ip[0] | (ip[1] << 8);
    ip += 2;
    int ml = token & 15;
    if (ml == 15) { unsigned b; do { b = *ip++; ml += b; } while (b == 255 && ip < iend); }
    ml += MINMATCH;
    if (off == 0 || off > o || o + ml > cap) { atomicOr(err, 4); return; }
    for (int i = 0; i < ml; ++i) dst[o + i] = dst[o - off + i];
    o += ml;
  }
  if (o != cap) atomicOr(err, 8);
}

// ---------------------------------------------------------------- launchers
int lz4_gpu_chunk() { return CHUNK; }
size_t lz4_gpu_scratch_bytes(size_t n) {
  const size_t nch = (n + CHUNK - 1) / CHUNK;
  return nch * BOUND;
}
size_t lz4_gpu_max_frame(size_t n) {
  const size_t nch = (n + CHUNK - 1) / CHUNK;
  return 15 + nch * (4 + CHUNK) + 4;
}

// sizes/offs: >= nchunks u32 each; total: one u64 (frame bytes)
hipError_t lz4_gpu_compress(const uint8_t* in, size_t n, uint8_t* scratch, uint32_t* sizes, uint32_t* offs,
                            uint8_t* out, uint64_t* total, hipStream_t s) {
  const int nch = (int)((n + CHUNK - 1) / CHUNK);
  if (nch == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lz4_enc_chunks, dim3((nch + ENC_THREADS - 1) / ENC_THREADS), dim3(ENC_THREADS), 0, s, in, n,
                     scratch, sizes, nch);
  hipLaunchKernelGGL(lz4_scan, dim3(1), dim3(1024), 0, s, sizes, offs, nch, total);
  hipLaunchKernelGGL(lz4_pack, dim3(nch), dim3(256), 0, s, in, n, scratch, sizes, offs, nch, out, total);
  return hipGetLastError();
}

hipError_t lz4_gpu_decompress(const uint8_t* frame, const uint32_t* offs, const uint32_t* sizes, int nchunks,
                              uint8_t* out, size_t n, int* err, hipStream_t s) {
  hipLaunchKernelGGL(lz4_dec_chunks, dim3((nchunks + 255) / 256), dim3(256), 0, s, frame, offs, sizes, nchunks, out,
                     n, err);
  return hipGetLastError();
}

}  // namespace adapt
